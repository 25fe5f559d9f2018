#!/bin/bash
# k_enlm_fx (fixed per-tile memory schedule, interior groups): parity, A/B vs k_enlm, NU 4 / 8
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05u}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 400 python3 -u -m pytest tests/test_affine_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_affine.log" 2>&1
MIPX_ENLM_NU=4 run 400 python3 -u -m pytest tests/test_affine_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k enlm > "$O/pytest_affine_nu4.log" 2>&1
MIPX_ENLM_NU=8 run 400 python3 -u -m pytest tests/test_affine_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k enlm > "$O/pytest_affine_nu8.log" 2>&1
for f in pytest_affine pytest_affine_nu4 pytest_affine_nu8; do tail -n 1 "$O/$f.log"; done
: > "$O/fx_ab.jsonl"; : > "$O/fxnu_ab.jsonl"
export MIPX_ENLM=2
for args in "--w 1920 --h 1080 --b 3 --n 16 --s 2" "--w 550 --h 740 --b 3 --n 64 --s 2" "--w 1024 --h 768 --b 4 --n 16 --s 1.5" \
            "--w 1280 --h 720 --b 3 --n 16 --s 3" "--w 960 --h 540 --b 3 --n 16 --s 4" "--w 1024 --h 768 --b 4 --n 16 --s 2"; do
  run 120 python3 scripts/op_bench.py affine $args --iters 20 --ab MIPX_ENLM_FX=0,1 >> "$O/fx_ab.jsonl"
  run 120 python3 scripts/op_bench.py affine $args --iters 20 --ab MIPX_ENLM_NU=4,8 >> "$O/fxnu_ab.jsonl"
done
python3 - "$O/fx_ab.jsonl" "$O/fxnu_ab.jsonl" <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        d = json.loads(l)
        k = [x for x in d if x.startswith("MIPX_") and x != "MIPX_ENLM"][0]
        if d["round"] == 0: print(d["w"], d["h"], d["b"], d["s"], k, d[k], d["ms"], round(d["alg_GBps"] / 8000, 3), d["same_as_first"])
PY
