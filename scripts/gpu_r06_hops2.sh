#!/bin/bash
# r06: k_rcol's host-built operands extended to the two-K-step RGB builds (1080p / 2.4):
# the rcol / chain / parity tests, then the specialised builds against the argument-driven
# ones (MIPX_RCOL_SPEC=0,1) on the reduce shapes with two K steps and the survey's others
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r06_hops2}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
[ "${TESTS:-1}" = 1 ] && run 600 python3 -u -m pytest tests/test_rcol_gpu.py tests/test_chain_gpu.py tests/test_parity_gpu.py \
  -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1
[ "${TESTS:-1}" = 1 ] && tail -1 "$O/pytest.log"
ab() { run 150 python3 scripts/op_bench.py "$@" --iters 20 >> "$O/ab.jsonl" 2>> "$O/ab.err"; }
# SHAPES=2: the RGBA and RGB-rows-off-a-dword builds (second pass)
# KNOB: the A/B switch (default MIPX_RCOL_SPEC=0,1); TESTS=0 skips the tests
# SHAPES=3: every geometry specialised (one K step with 6 chunks, RGBA with 4-byte K origins)
if [ "${SHAPES:-1}" = 3 ]; then
  set -- "--w 1920 --h 1080 --b 3 --n 64 --s 1.9" "--w 1920 --h 1080 --b 3 --n 64 --s 1.8" "--w 1333 --h 1000 --b 3 --n 48 --s 1.9" \
    "--w 1024 --h 1024 --b 4 --n 128 --s 1.7" "--w 1024 --h 1024 --b 4 --n 128 --s 1.8" "--w 1024 --h 1024 --b 4 --n 128 --s 1.9" \
    "--w 800 --h 600 --b 4 --n 128 --s 1.6666666666666667" "--w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333" \
    "--w 1920 --h 1080 --b 3 --n 64 --s 1.6" "--w 500 --h 375 --b 3 --n 128 --s 1.46484375" \
    "--w 364 --h 273 --b 3 --n 128 --s 1.421875" "--w 1920 --h 1080 --b 3 --n 64 --s 2.4"
elif [ "${SHAPES:-1}" = 2 ]; then
  set -- "--w 1024 --h 1024 --b 4 --n 128 --s 2.4" "--w 1024 --h 1024 --b 4 --n 128 --s 2.2" "--w 800 --h 600 --b 4 --n 128 --s 2.25" \
    "--w 1333 --h 1000 --b 3 --n 48 --s 2.4" "--w 1366 --h 768 --b 3 --n 64 --s 2.2" "--w 999 --h 750 --b 3 --n 128 --s 2.25" \
    "--w 1920 --h 1080 --b 3 --n 64 --s 2.4"
else
  set -- "--w 1920 --h 1080 --b 3 --n 64 --s 2.4" "--w 1920 --h 1080 --b 3 --n 64 --s 2.0" "--w 1920 --h 1080 --b 3 --n 64 --s 2.2" \
    "--w 3840 --h 2160 --b 3 --n 16 --s 2.4" "--w 1000 --h 750 --b 3 --n 128 --s 2.25" "--w 640 --h 480 --b 3 --n 256 --s 2.5" \
    "--w 480 --h 270 --b 3 --n 256 --s 1.6 --s2 1.5976331360946747" "--w 1333 --h 1000 --b 3 --n 48 --s 1.6666666666666667"
fi
for a in "$@"; do
  ab reduce $a --ab ${KNOB:-MIPX_RCOL_SPEC=0,1}
done
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for l in open(O + "/ab.jsonl"):
    if l.startswith("{"):
        d = json.loads(l)
        knob = [k for k in d if k.startswith("MIPX_")][0]
        print(f'{d["op"]} {d["w"]}x{d["h"]}x{d["b"]} s{d["s"]:.4g} {knob}={d[knob]} r{d["round"]} {d["ms"]:.4f} ms {d["alg_GBps"]/8000:.1%} same={d["same_as_first"]}')
PY
