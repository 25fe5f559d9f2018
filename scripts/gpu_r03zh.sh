# k_rot90_px on RGBA and non-temporal shrink loads: parity, then same-process A/Bs
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zh; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_parity_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "rot or shrink" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
A="timeout -k 10 120 python3 -u scripts/op_bench.py"
{ $A rot --w 3840 --h 2160 --b 4 --n 16 --s 90 --ab MIPX_ROT_PX4=0,1 &&
  $A rot --w 1920 --h 1080 --b 4 --n 32 --s 270 --ab MIPX_ROT_PX4=0,1 &&
  $A rot --w 4000 --h 3000 --b 4 --n 8 --s 90 --ab MIPX_ROT_PX4=0,1 &&
  $A shrink --w 4000 --h 3000 --b 3 --n 64 --s 8 --ab MIPX_SHRINK_NTL=0,1 &&
  $A shrink --w 4000 --h 3000 --b 3 --n 64 --s 11 --ab MIPX_SHRINK_NTL=0,1 &&
  $A shrink --w 3840 --h 2160 --b 3 --n 64 --s 4 --ab MIPX_SHRINK_NTL=0,1 &&
  $A shrink --w 1920 --h 1080 --b 3 --n 64 --s 3 --ab MIPX_SHRINK_NTL=0,1 &&
  $A shrink --w 3840 --h 2160 --b 3 --n 32 --s 2 --ab MIPX_SHRINK_NTL=0,1 &&
  $A shrink --w 4000 --h 3000 --b 3 --n 32 --s 3 --ab MIPX_SHRINK_NTL=0,1; } > $O/ab.jsonl 2>&1 || { tail $O/ab.jsonl; exit 1; }
python3 - $O/ab.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d=json.loads(l); k=[x for x in d if x.startswith("MIPX")][0]
    print(d["op"], d["w"], d["h"], d["b"], d["s"], k, d[k], d["round"], d["ms"], d["alg_GBps"], d["same_as_first"])
PY
