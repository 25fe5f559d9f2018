#!/bin/bash
# r06: k_enlm's set-up with the row records and the first tile issued in the first memory
# round trip: the affine suite, then the base build (imaginary_amd/libmipx_base.so, the tree
# before the change) against this one, alternating processes, on the survey's enlarge shapes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r06_enlpre}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 400 python3 -u -m pytest tests/test_affine_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_affine.log" 2>&1
tail -1 "$O/pytest_affine.log"
: > "$O/ab.jsonl"
for args in "--w 550 --h 740 --b 3 --n 64 --s 2" "--w 1920 --h 1080 --b 3 --n 16 --s 2" "--w 1024 --h 768 --b 4 --n 16 --s 1.5" \
            "--w 1280 --h 720 --b 3 --n 16 --s 3" "--w 960 --h 540 --b 3 --n 16 --s 4" "--w 1024 --h 768 --b 4 --n 16 --s 2"; do
  for r in 0 1; do
    for lib in base new; do
      if [ $lib = base ]; then export MIPX_LIB_PATH="$R/imaginary_amd/libmipx_base.so"; else unset MIPX_LIB_PATH; fi
      run 120 python3 scripts/op_bench.py affine $args --iters 30 | sed "s/^{/{\"lib\": \"$lib\", \"r\": $r, /" >> "$O/ab.jsonl"
    done
  done
done
unset MIPX_LIB_PATH
python3 - "$O/ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["w"], d["h"], d["b"], d["s"], d["lib"], d["r"], round(d["ms"], 4), f'{d["alg_GBps"] / 8000:.1%}')
PY
