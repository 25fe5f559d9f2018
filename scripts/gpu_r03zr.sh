# k_rcol segment rule A/B (old rounds x steps model vs ~6 rounds) on the reduce shapes
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zr; mkdir -p $O; export TMPDIR=/tmp
A="timeout -k 10 150 python3 -u scripts/op_bench.py"
{ $A reduce --w 480 --h 270 --b 3 --n 256 --s 1.6 --ab MIPX_RCOL_SEGRULE=0,1 &&
  $A reduce --w 500 --h 375 --b 3 --n 128 --s 1.46484375 --ab MIPX_RCOL_SEGRULE=0,1 &&
  $A reduce --w 1920 --h 1080 --b 3 --n 64 --s 1.6 --ab MIPX_RCOL_SEGRULE=0,1 &&
  $A reduce --w 1920 --h 1080 --b 3 --n 64 --s 2.4 --ab MIPX_RCOL_SEGRULE=0,1 &&
  $A reduce --w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333 --ab MIPX_RCOL_SEGRULE=0,1 &&
  MIPX_RCOL_SEGRULE=1 $A reduce --w 480 --h 270 --b 3 --n 256 --s 1.6 --ab MIPX_RCOL_ROUNDS=2,3,4,6,8 &&
  MIPX_RCOL_SEGRULE=1 $A reduce --w 1920 --h 1080 --b 3 --n 64 --s 1.6 --ab MIPX_RCOL_ROUNDS=2,3,4,6,8; } > $O/ab.jsonl 2>&1 || { tail $O/ab.jsonl; exit 1; }
python3 - $O/ab.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d=json.loads(l); k=[x for x in d if x.startswith("MIPX")][0]
    if d["round"]==1: print(d["op"], d["w"], d["h"], d["b"], d["s"], k, repr(d[k]), d["ms"], d["alg_GBps"])
PY
for r in 0 1; do MIPX_RCOL_DBG=1 MIPX_RCOL_SEGRULE=$r timeout -k 10 60 python3 -u scripts/op_bench.py reduce --w 480 --h 270 --b 3 --n 256 --s 1.6 --warm-ms 0 --iters 1 2>&1 | grep k_rcol | head -1; done
