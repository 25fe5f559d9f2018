#!/bin/bash
# One GPU session: parity tests -> bench -> rocprofv3 kernel trace.
# Stops at the first fault / abort / timeout (exit >= 2 or a signal).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT="$R/gpurun_out"
mkdir -p "$OUT"
TAG=${TAG:-r01}
export TMPDIR=/tmp
stop_if_fatal() {  # $1 = exit code, $2 = step name; pytest 1 = failed tests (not fatal)
    if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL in $2 (exit $1), stopping"; exit "$1"; fi
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python3 -m pytest tests -m gpu -x -q -p no:cacheprovider ${PYTEST_ARGS:-} > "$OUT/pytest_gpu_$TAG.log" 2>&1
  rc=$?; tail -25 "$OUT/pytest_gpu_$TAG.log"; stop_if_fatal $rc pytest
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
  rc=$?; cat "$OUT/bench_$TAG.json"; tail -5 "$OUT/bench_$TAG.err"; stop_if_fatal $rc bench
  [ $rc -ne 0 ] && exit $rc
fi
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
      python3 "$R/bench.py" --steps 100 --warmup 20 --no-cpu --no-verify > "$OUT/prof_$TAG.log" 2>&1
  rc=$?; tail -5 "$OUT/prof_$TAG.log"; stop_if_fatal $rc rocprof
  find "$OUT/prof_$TAG" -name "*stats*" | head
fi
echo "gpu_round done"
