#!/bin/bash
# k_enlm two-group emission: affine parity (pair on by default), same-process A/B of
# MIPX_ENLM_PAIR on the op-survey enlarge shapes, then the C5 A/B of this round's switches
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05v}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 400 python3 -u -m pytest tests/test_affine_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_affine.log" 2>&1
tail -3 "$O/pytest_affine.log"
: > "$O/pair_ab.jsonl"
export MIPX_ENLM=2
for args in "--w 1920 --h 1080 --b 3 --n 16 --s 2" "--w 550 --h 740 --b 3 --n 64 --s 2" "--w 1024 --h 768 --b 4 --n 16 --s 1.5" \
            "--w 1280 --h 720 --b 3 --n 16 --s 3" "--w 960 --h 540 --b 3 --n 16 --s 4" "--w 1024 --h 768 --b 4 --n 16 --s 2"; do
  run 120 python3 scripts/op_bench.py affine $args --iters 20 --ab MIPX_ENLM_PAIR=0,1 >> "$O/pair_ab.jsonl"
done
python3 - "$O/pair_ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); print(d["w"], d["h"], d["b"], d["s"], "pair", d["MIPX_ENLM_PAIR"], "r", d["round"], d["ms"], round(d["alg_GBps"] / 8000, 3), d["same_as_first"])
PY
unset MIPX_ENLM
: > "$O/c5_ab.jsonl"
for k in MIPX_RCOL_UNAL=0,1 MIPX_ENLM=0,1 MIPX_RCOL_SWZ=0,1; do
  run 300 python3 scripts/cfg_ab.py --config C5 --ab $k --rounds 2 >> "$O/c5_ab.jsonl"
done
cut -c1-220 "$O/c5_ab.jsonl"
