#!/bin/bash
# k_enlm band-height sweep on the op-survey enlarge shapes (MIPX_ENLM_BR; 0 = the heuristic)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05br}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
: > "$O/br_sweep.jsonl"
export MIPX_ENLM=2
sweep() { run 150 python3 scripts/op_bench.py affine $1 --iters 20 --ab MIPX_ENLM_BR=$2 >> "$O/br_sweep.jsonl"; }
sweep "--w 550 --h 740 --b 3 --n 64 --s 2" 0,112,144,160,176,192,208
sweep "--w 1024 --h 768 --b 4 --n 16 --s 1.5" 0,48,64,80,96
sweep "--w 1920 --h 1080 --b 3 --n 16 --s 2" 0,96,112,144,160
sweep "--w 1024 --h 768 --b 4 --n 16 --s 2" 0,48,64,96,128
sweep "--w 1280 --h 720 --b 3 --n 16 --s 3" 0,96,144,176,208
sweep "--w 960 --h 540 --b 3 --n 16 --s 4" 0,96,144,176,208
python3 - "$O/br_sweep.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    if d["round"] == 0: print(d["w"], d["h"], d["b"], d["s"], "br", d["MIPX_ENLM_BR"], d["ms"], round(d["alg_GBps"] / 8000, 3))
PY
