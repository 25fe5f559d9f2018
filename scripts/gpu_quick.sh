#!/bin/bash
# parity tests, then the C3/C4/C5 (+ optional) config lines; stops at the first failure
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=${TAG:-q}
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} ${KEXPR:+-k "$KEXPR"} > "$OUT/pytest_$TAG.log" 2>&1; rc=$?
tail -15 "$OUT/pytest_$TAG.log"; [ $rc -ne 0 ] && exit $rc
if [ -n "${CONFIGS:-C3,C4,C5}" ]; then
  timeout -k 10 300 python3 -u bench_configs.py --configs ${CONFIGS:-C3,C4,C5} > "$OUT/cfg_$TAG.log" 2>&1 || { tail "$OUT/cfg_$TAG.log"; exit 1; }
  grep '^{' "$OUT/cfg_$TAG.log" | cut -c1-400
fi
