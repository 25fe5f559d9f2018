#!/bin/bash
# k_enlm 5 waves/SIMD + LDS-aware bands; k_rcol realigning build for unaligned RGB rows
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05n}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 600 python3 -u -m pytest tests/test_rcol_gpu.py tests/test_parity_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_rcol.log" 2>&1
tail -2 "$O/pytest_rcol.log"
OUT=${OUT:-r05n} run 600 bash scripts/gpu_r05_enlm.sh
: > "$O/unal_ab.jsonl"
for args in "--w 1333 --h 1000 --b 3 --n 48 --s 1.6666666666666667" "--w 1331 --h 999 --b 3 --n 48 --s 1.6"; do
  run 120 python3 scripts/op_bench.py reduce $args --iters 20 --ab MIPX_RCOL_UNAL=0,1 >> "$O/unal_ab.jsonl"
done
python3 - "$O/unal_ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); print(d["w"], d["h"], d["b"], d["s"], "unal", d["MIPX_RCOL_UNAL"], "r", d["round"], d["ms"], round(d["alg_GBps"] / 8000, 3), d["same_as_first"])
PY
