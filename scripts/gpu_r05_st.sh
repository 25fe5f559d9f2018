#!/bin/bash
# k_rcol: edge-piece dword stores only in the last strip (MIPX_RCOL_ALLST=1: every strip, as before)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05st}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 500 python3 -u -m pytest tests/test_rcol_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_rcol.log" 2>&1
tail -2 "$O/pytest_rcol.log"
run 500 python3 -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "reduce or C1 or c1" > "$O/pytest_reduce.log" 2>&1
tail -2 "$O/pytest_reduce.log"
: > "$O/st_ab.jsonl"
for args in "--w 480 --h 270 --b 3 --n 256 --s 1.6" "--w 480 --h 270 --b 3 --n 1024 --s 1.6" "--w 500 --h 300 --b 3 --n 256 --s 1.6666666666666667" \
            "--w 1920 --h 1080 --b 3 --n 64 --s 1.6"; do
  run 200 python3 scripts/op_bench.py reduce $args --iters 20 --ab MIPX_RCOL_ALLST=1,0 >> "$O/st_ab.jsonl"
done
python3 - "$O/st_ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["w"], d["h"], d["n"], round(d["s"], 3), d["out"], "allst", d["MIPX_RCOL_ALLST"], "r", d["round"], d["ms"], round(d["alg_GBps"] / 8000, 3), d["same_as_first"])
PY
run 300 python3 scripts/cfg_ab.py --config C5 --ab MIPX_RCOL_ALLST=1,0 --rounds 2 > "$O/c5_st_ab.jsonl"
cut -c1-200 "$O/c5_st_ab.jsonl"
