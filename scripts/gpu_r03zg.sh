# non-temporal stores: parity of the touched kernels, then same-process A/Bs (MIPX_NT, reduce2x2 variants)
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zg; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_parity_gpu.py tests/test_rcol_gpu.py tests/test_bcol_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
A="timeout -k 10 120 python3 -u scripts/op_bench.py"
{ $A rot --w 3840 --h 2160 --b 3 --n 32 --s 90 --ab MIPX_NT=0,1 &&
  $A rot --w 4000 --h 3000 --b 3 --n 16 --s 270 --ab MIPX_NT=0,1 &&
  $A blur --w 1920 --h 1080 --b 3 --n 64 --s 3 --ab MIPX_NT=0,1 &&
  $A blur --w 768 --h 512 --b 4 --n 512 --s 5 --ab MIPX_NT=0,1 &&
  $A blur --w 3840 --h 2160 --b 3 --n 16 --s 5 --ab MIPX_NT=0,1 &&
  $A reduce --w 1920 --h 1080 --b 3 --n 64 --s 1.6 --ab MIPX_NT=0,1 &&
  $A reduce --w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333 --ab MIPX_NT=0,1 &&
  $A reduce --w 480 --h 270 --b 3 --n 256 --s 1.6 --ab MIPX_NT=0,1 &&
  $A reduce --w 3840 --h 2160 --b 3 --n 256 --s 2 --ab MIPX_R2_VARIANT=66,82,98,114 &&
  $A reduce --w 2048 --h 2048 --b 4 --n 512 --s 2 --ab MIPX_R2_VARIANT=66,82,98,114; } > $O/nt_ab2.jsonl 2>&1 || { tail $O/nt_ab2.jsonl; exit 1; }
python3 - $O/nt_ab2.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d=json.loads(l); k=[x for x in d if x.startswith("MIPX")][0]
    print(d["op"], d["w"], d["h"], d["b"], d["s"], k, d[k], d["round"], d["ms"], d["alg_GBps"], d["same_as_first"])
PY
