# k_bcol defaults (RGB 256-byte strips, 6-round segments): parity, shapes, C3 config
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zq; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_bcol_gpu.py tests/test_demand_gpu.py tests/test_parity_gpu.py tests/test_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "bcol or blur or demand or pipeline or c3" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
A="timeout -k 10 150 python3 -u scripts/op_bench.py"
{ $A blur --w 1920 --h 1080 --b 3 --n 64 --s 1 --ab MIPX_BCOL_SEGS=,4,6,9 &&
  $A blur --w 1920 --h 1080 --b 3 --n 64 --s 5 --ab MIPX_BCOL_SEGS=,4,6,9 &&
  $A blur --w 3840 --h 2160 --b 3 --n 16 --s 5 --ab MIPX_BCOL_SEGS=,8,12,17 &&
  $A blur --w 4000 --h 3000 --b 3 --n 16 --s 3 --ab MIPX_BCOL_SEGS=,8,12,16 &&
  $A blur --w 1920 --h 1080 --b 4 --n 32 --s 2 --ab MIPX_BCOL_SEGS=,4,8; } > $O/ab.jsonl 2>&1 || { tail $O/ab.jsonl; exit 1; }
python3 - $O/ab.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d=json.loads(l); k=[x for x in d if x.startswith("MIPX")][0]
    if d["round"]==1: print(d["op"], d["w"], d["h"], d["b"], d["s"], k, repr(d[k]), d["ms"], d["alg_GBps"])
PY
timeout -k 10 300 python3 -u bench_configs.py --configs C3,C5 --steps 10 --warmup 2 > $O/configs.jsonl 2> $O/configs.err || { tail $O/configs.err; exit 1; }
cut -c1-250 $O/configs.jsonl
