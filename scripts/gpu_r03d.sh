set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03d; mkdir -p $O; export TMPDIR=/tmp
for a in "reduce --w 1920 --h 1080 --b 3 --n 64 --s 1.6" "reduce --w 1920 --h 1080 --b 3 --n 64 --s 2.4" "reduce --w 500 --h 375 --b 3 --n 128 --s 1.46484375" "reduce --w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333"; do
  MIPX_RCOL_STAMPS=1 timeout -k 5 60 python3 scripts/op_bench.py $a --iters 2 > $O/stamps.log 2>&1 || { cat $O/stamps.log; exit 1; }
  grep k_rcol_stamps $O/stamps.log | tail -1
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc1 -o run -- python3 scripts/op_bench.py reduce --w 1920 --h 1080 --b 3 --n 64 --s 1.6 --iters 3 > $O/pmc1.log 2>&1 || { tail $O/pmc1.log; exit 1; }
python3 - $O/pmc1 <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for fn in f:
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"][:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    n = max(cnt[(k, c)] for c in d)
    print(k, {c: round(v / n) for c, v in d.items()})
PY
