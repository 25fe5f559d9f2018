#!/bin/bash
# k_rcol segments per strip (MIPX_RCOL_SEGS; 0 = the cost model) on the survey reduce shapes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05seg}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
: > "$O/seg_ab.jsonl"
for args in "--w 480 --h 270 --b 3 --n 256 --s 1.6" "--w 500 --h 375 --b 3 --n 128 --s 1.465" "--w 1333 --h 1000 --b 3 --n 48 --s 1.6666666666666667" \
            "--w 1920 --h 1080 --b 3 --n 64 --s 1.6" "--w 1920 --h 1080 --b 3 --n 64 --s 2.4" "--w 1024 --h 1024 --b 4 --n 512 --s 1.333"; do
  run 200 python3 scripts/op_bench.py reduce $args --iters 20 --ab MIPX_RCOL_SEGS=0,1,2,3,4,6,8 >> "$O/seg_ab.jsonl"
done
python3 - "$O/seg_ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    if d["round"] == 0: print(d["w"], d["h"], d["b"], round(d["s"], 3), "segs", d["MIPX_RCOL_SEGS"], d["ms"], round(d["alg_GBps"] / 8000, 3), d["same_as_first"])
PY
