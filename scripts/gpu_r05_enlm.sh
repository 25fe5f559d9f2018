#!/bin/bash
# k_enlm: affine parity suite, then same-process A/B against the VALU kernels on the
# op-survey enlarge shapes (MIPX_ENLM=0: k_enlarge2 / k_affine_sep; 2: k_enlm or an error)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05h}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 400 python3 -u -m pytest tests/test_affine_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_affine.log" 2>&1
tail -3 "$O/pytest_affine.log"
: > "$O/enlm_ab.jsonl"
for args in "--w 1920 --h 1080 --b 3 --n 16 --s 2" "--w 550 --h 740 --b 3 --n 64 --s 2" "--w 1024 --h 768 --b 4 --n 16 --s 1.5" \
            "--w 1280 --h 720 --b 3 --n 16 --s 3" "--w 960 --h 540 --b 3 --n 16 --s 4" "--w 1024 --h 768 --b 4 --n 16 --s 2"; do
  run 120 python3 scripts/op_bench.py affine $args --iters 20 --ab MIPX_ENLM=0,2 >> "$O/enlm_ab.jsonl"
done
python3 - "$O/enlm_ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); print(d["w"], d["h"], d["b"], d["s"], "enlm", d["MIPX_ENLM"], "r", d["round"], d["ms"], d["alg_GBps"], round(d["alg_GBps"] / 8000, 3), d["same_as_first"])
PY
