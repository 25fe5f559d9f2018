#!/bin/bash
# k_rcol: ring load batches no lane of the wave needs not issued (MIPX_RCOL_SKIPL)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05sl}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
MIPX_RCOL_SKIPL=1 run 500 python3 -u -m pytest tests/test_rcol_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_rcol.log" 2>&1
tail -2 "$O/pytest_rcol.log"
: > "$O/sl_ab.jsonl"
for args in "--w 480 --h 270 --b 3 --n 256 --s 1.6" "--w 500 --h 375 --b 3 --n 128 --s 1.465" "--w 1333 --h 1000 --b 3 --n 48 --s 1.6666666666666667" \
            "--w 1920 --h 1080 --b 3 --n 64 --s 1.6" "--w 1920 --h 1080 --b 3 --n 64 --s 2.4" "--w 1024 --h 1024 --b 4 --n 512 --s 1.333"; do
  run 200 python3 scripts/op_bench.py reduce $args --iters 20 --ab MIPX_RCOL_SKIPL=0,1 >> "$O/sl_ab.jsonl"
done
python3 - "$O/sl_ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["w"], d["h"], d["n"], round(d["s"], 3), "skipl", d["MIPX_RCOL_SKIPL"], "r", d["round"], d["ms"], round(d["alg_GBps"] / 8000, 3), d["same_as_first"])
PY
