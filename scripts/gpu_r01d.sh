#!/bin/bash
# request-path tests + E2E line + PMC traffic of the C2 kernel
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_r01d.log" 2>&1; rc=$?
tail -5 "$OUT/pytest_r01d.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench_configs.py --configs E2E > "$OUT/e2e_r01d.log" 2>&1 || { tail "$OUT/e2e_r01d.log"; exit 1; }
grep '^{' "$OUT/e2e_r01d.log"
TAG=r01d PMC_LIST=$'FETCH_SIZE\nWRITE_SIZE' bash scripts/pmc.sh || exit $?
ALG_BYTES=7962624000 python3 scripts/traffic_json.py "$OUT/pmc_r01d" "k_reduce2x2<3, 2>" "$OUT/traffic_r01d.json" "256 x 3840x2160x3 -> 1920x1080x3, band 24 rows"
