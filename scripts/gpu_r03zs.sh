# zoom with non-temporal row stores: parity, A/B
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zs; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "zoom" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
A="timeout -k 10 150 python3 -u scripts/op_bench.py"
{ $A zoom --w 1920 --h 1080 --b 3 --n 16 --s 2 --ab MIPX_ZOOM_NT=0,1 &&
  $A zoom --w 1024 --h 768 --b 4 --n 16 --s 3 --ab MIPX_ZOOM_NT=0,1 &&
  $A zoom --w 640 --h 480 --b 3 --n 64 --s 2 --ab MIPX_ZOOM_NT=0,1; } > $O/ab.jsonl 2>&1 || { tail $O/ab.jsonl; exit 1; }
python3 - $O/ab.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d=json.loads(l); k=[x for x in d if x.startswith("MIPX")][0]
    if d["round"]==1: print(d["op"], d["w"], d["h"], d["b"], d["s"], k, repr(d[k]), d["ms"], d["alg_GBps"])
PY
