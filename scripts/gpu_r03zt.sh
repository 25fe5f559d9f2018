# extract rows with non-temporal stores: parity, A/B
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zt; mkdir -p $O; export TMPDIR=/tmp
MIPX_EXTRACT_NT=1 timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "extract" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
A="timeout -k 10 150 python3 -u scripts/op_bench.py"
{ $A extract --w 3840 --h 2160 --b 3 --n 32 --ow 2000 --oh 1500 --ab MIPX_EXTRACT_NT=0,1 &&
  $A extract --w 4000 --h 3000 --b 3 --n 16 --ow 3000 --oh 2000 --ab MIPX_EXTRACT_NT=0,1 &&
  $A extract --w 1920 --h 1080 --b 4 --n 32 --ow 1280 --oh 720 --ab MIPX_EXTRACT_NT=0,1; } > $O/ab.jsonl 2>&1 || { tail $O/ab.jsonl; exit 1; }
python3 - $O/ab.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d=json.loads(l); k=[x for x in d if x.startswith("MIPX")][0]
    if d["round"]==1: print(d["op"], d["w"], d["h"], d["b"], d["out"], k, repr(d[k]), d["ms"], d["alg_GBps"], d.get("same_as_first"))
PY
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; exit $rc
