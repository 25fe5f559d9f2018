# k_bcol segment counts (MIPX_BCOL_SEGS) for RGB 64-px / 256-byte strips and RGBA
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zo; mkdir -p $O; export TMPDIR=/tmp
A="timeout -k 10 150 python3 -u scripts/op_bench.py"
{ $A blur --w 1920 --h 1080 --b 3 --n 64 --s 1 --ab MIPX_BCOL_SEGS=,1,2,3,4,6,8,12 &&
  $A blur --w 1920 --h 1080 --b 3 --n 64 --s 5 --ab MIPX_BCOL_SEGS=,1,2,3,4,6,8,12 &&
  MIPX_BCOL_RGB256=1 $A blur --w 1920 --h 1080 --b 3 --n 64 --s 1 --ab MIPX_BCOL_SEGS=,2,3,4,6,8,12 &&
  $A blur --w 3840 --h 2160 --b 3 --n 16 --s 5 --ab MIPX_BCOL_SEGS=,1,2,3,4,6,8,12 &&
  $A blur --w 768 --h 512 --b 4 --n 512 --s 5 --ab MIPX_BCOL_SEGS=,1,2,3,4 &&
  $A blur --w 4000 --h 3000 --b 3 --n 16 --s 3 --ab MIPX_BCOL_SEGS=,2,3,4,6,8,12,16; } > $O/ab.jsonl 2>&1 || { tail $O/ab.jsonl; exit 1; }
python3 - $O/ab.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d=json.loads(l); k=[x for x in d if x.startswith("MIPX")][0]
    if d["round"]==1: print(d["op"], d["w"], d["h"], d["b"], d["s"], k, repr(d[k]), d["ms"], d["alg_GBps"])
PY
