#!/bin/bash
# k_reduce2m prime: both row batches in flight (MIPX_R2M_PP) — 2x2 parity, same-process A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05x}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 400 python3 -u -m pytest tests/test_parity_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "reduce2x2_variants or 4k_to_1080p" > "$O/pytest_r2.log" 2>&1
tail -2 "$O/pytest_r2.log"
: > "$O/pp_ab.jsonl"
for args in "--w 3840 --h 2160 --b 3 --n 256 --s 2" "--w 2048 --h 2048 --b 4 --n 512 --s 2"; do
  run 150 python3 scripts/op_bench.py reduce $args --sampling centre --iters 20 --ab MIPX_R2M_PP=0,1,0,1 >> "$O/pp_ab.jsonl"
  run 150 python3 scripts/op_bench.py reduce $args --sampling centre --iters 20 --ab MIPX_R2M_VBF=0,1,0,1 >> "$O/pp_ab.jsonl"
done
python3 - "$O/pp_ab.jsonl" <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        d = json.loads(l); k = [x for x in d if x.startswith("MIPX_")][0]
        print(d["w"], d["h"], d["b"], k, d[k], "r", d["round"], d["ms"], round(d["alg_GBps"] / 8000, 4), d["same_as_first"])
PY
