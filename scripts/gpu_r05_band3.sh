#!/bin/bash
# k_reduce2x2 bands (MIPX_R2_BAND) on C3's 2x2 stage (2048^2 RGBA x512) and 2048^2 RGB, same-process A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05band3}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
: > "$O/r2_band_rgba_ab.jsonl"
run 200 python3 scripts/op_bench.py reduce --w 2048 --h 2048 --b 4 --n 512 --s 2 --iters 20 --ab MIPX_R2_BAND=2,4,5,6,8,4 >> "$O/r2_band_rgba_ab.jsonl"
run 200 python3 scripts/op_bench.py reduce --w 1920 --h 1080 --b 3 --n 512 --s 2 --iters 20 --ab MIPX_R2_BAND=1,2,3,2 >> "$O/r2_band_rgba_ab.jsonl"
python3 - "$O/r2_band_rgba_ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["w"], d["b"], "MIPX_R2_BAND", d["MIPX_R2_BAND"], "r", d["round"], d["ms"], round(d["alg_GBps"] / 8000, 4), d["same_as_first"])
PY
