#!/bin/bash
# k_rchain (v1, direct-load front) PMC on C3, k_reduce2d batched-MFMA A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05d}"; mkdir -p "$O"
timeout -k 10 200 python3 scripts/op_bench.py reduce --w 3840 --h 2160 --b 3 --n 256 --s 2 --iters 20 --ab MIPX_R2D=0,1 > "$O/r2d_batched_ab.jsonl" || exit 1
cat "$O/r2d_batched_ab.jsonl"
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
            "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  MIPX_CHAIN=1 timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$O/pc$i" -o run -- \
    python3 bench_configs.py --configs C3 --steps 3 --warmup 1 --warm-ms 0 > "$O/pc$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$O/pc$i.log"; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
vals = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/pc*/*counter_collection.csv"):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "mipx" not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void mipx::", "").split("(")[0]
        per[(k, r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (k, c, d), v in per.items():
        vals[(k, c)].append(v)
for (k, c), v in sorted(vals.items()):
    print(f"{k[:48]:48s} {c:26s} {sum(v)/len(v):18.1f}")
PY
