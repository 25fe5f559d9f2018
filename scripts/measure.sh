#!/bin/bash
# Full measurement pass for one tree: GPU parity tests -> bench.py line ->
# rocprofv3 kernel stats of the bench -> FETCH_SIZE / WRITE_SIZE passes of the
# C2 kernel -> traffic json -> config lines (C3/C4/C5/E2E) with kernel stats.
# Stops at the first failure.  Outputs under gpurun_out/*_$TAG.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=${TAG:-m}
KERNEL=${KERNEL:-k_reduce2x2<3, 66>}
SKIP_TESTS=${SKIP_TESTS:-0} SKIP_BENCH=0 SKIP_PROF=0 TAG=$TAG PYTEST_ARGS="--timeout 120 --timeout-method thread" bash scripts/gpu_round.sh || exit $?
TAG=$TAG PMC_LIST=$'FETCH_SIZE\nWRITE_SIZE' bash scripts/pmc.sh || exit $?
ALG_BYTES=7962624000 timeout -k 5 60 python3 scripts/traffic_json.py "$OUT/pmc_$TAG" "$KERNEL" "$OUT/traffic_$TAG.json" \
    "256 x 3840x2160x3 -> 1920x1080x3" || exit $?
CONFIGS="C3 C4 C5" TAG=$TAG bash scripts/prof_configs.sh > /dev/null || exit $?
timeout -k 10 300 python3 -u bench_configs.py --configs E2E > "$OUT/e2e_$TAG.log" 2>&1 || exit $?
grep '^{' "$OUT"/profcfg_$TAG/*.log "$OUT/e2e_$TAG.log" | cut -c1-300
echo "measure done"
