# k_bcol byte strips + segment rule: parity, then the r03zl shapes, RGB256 A/B
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zp; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_bcol_gpu.py tests/test_demand_gpu.py tests/test_parity_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "bcol or blur or demand or pipeline" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
A="timeout -k 10 150 python3 -u scripts/op_bench.py"
{ $A blur --w 1920 --h 1080 --b 3 --n 64 --s 1 --ab MIPX_BCOL_RGB256=0,1 &&
  $A blur --w 1920 --h 1080 --b 3 --n 64 --s 3 --ab MIPX_BCOL_RGB256=0,1 &&
  $A blur --w 1920 --h 1080 --b 3 --n 64 --s 5 --ab MIPX_BCOL_RGB256=0,1 &&
  $A blur --w 3840 --h 2160 --b 3 --n 16 --s 5 --ab MIPX_BCOL_RGB256=0,1 &&
  $A blur --w 4000 --h 3000 --b 3 --n 16 --s 3 --ab MIPX_BCOL_RGB256=0,1 &&
  $A blur --w 768 --h 512 --b 4 --n 512 --s 5 --ab MIPX_BCOL_SEGS=,1,2,3 &&
  $A blur --w 1920 --h 1080 --b 4 --n 32 --s 2 --ab MIPX_BCOL_SEGS=,2,4,8; } > $O/ab.jsonl 2>&1 || { tail $O/ab.jsonl; exit 1; }
python3 - $O/ab.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d=json.loads(l); k=[x for x in d if x.startswith("MIPX")][0]
    if d["round"]==1: print(d["op"], d["w"], d["h"], d["b"], d["s"], k, repr(d[k]), d["ms"], d["alg_GBps"])
PY
for s in 1 5; do MIPX_BCOL_DBG=1 timeout -k 10 60 python3 -u scripts/op_bench.py blur --w 1920 --h 1080 --b 3 --n 64 --s $s --warm-ms 0 --iters 1 2>&1 | grep k_bcol | head -1; done
MIPX_BCOL_DBG=1 timeout -k 10 60 python3 -u scripts/op_bench.py blur --w 768 --h 512 --b 4 --n 512 --s 5 --warm-ms 0 --iters 1 2>&1 | grep k_bcol | head -1
