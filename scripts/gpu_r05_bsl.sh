#!/bin/bash
# k_bcol: load batches no lane of the wave needs not issued (MIPX_BCOL_SKIPL)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05bsl}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 500 python3 -u -m pytest tests/test_bcol_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_bcol.log" 2>&1
tail -2 "$O/pytest_bcol.log"
: > "$O/bsl_ab.jsonl"
for args in "--w 768 --h 512 --b 4 --n 512 --s 5" "--w 1920 --h 1080 --b 3 --n 64 --s 1" "--w 1920 --h 1080 --b 3 --n 64 --s 3" "--w 3840 --h 2160 --b 3 --n 16 --s 5"; do
  run 200 python3 scripts/op_bench.py blur $args --iters 20 --ab MIPX_BCOL_SKIPL=0,1 >> "$O/bsl_ab.jsonl"
done
python3 - "$O/bsl_ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["w"], d["h"], d["b"], d["n"], d["s"], "skipl", d["MIPX_BCOL_SKIPL"], "r", d["round"], d["ms"], round(d["alg_GBps"] / 8000, 3), d["same_as_first"])
PY
run 300 python3 scripts/cfg_ab.py --config C3 --ab MIPX_BCOL_SKIPL=0,1 --rounds 2 > "$O/c3_bsl_ab.jsonl"
run 300 python3 scripts/cfg_ab.py --config C5 --ab MIPX_BCOL_SKIPL=0,1 --rounds 2 > "$O/c5_bsl_ab.jsonl"
cut -c1-200 "$O/c3_bsl_ab.jsonl" "$O/c5_bsl_ab.jsonl"
