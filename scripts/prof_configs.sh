#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out/profcfg_${TAG:-r01}"; mkdir -p "$OUT"; export TMPDIR=/tmp
for c in ${CONFIGS:-C3 C4 C5}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$c" -o run -- python3 "$R/bench_configs.py" --configs $c --steps 3 --warmup 1 > "$OUT/$c.log" 2>&1 || exit $?
  echo "== $c"; head -12 "$OUT/$c/run_kernel_stats.csv" | cut -d, -f1-4 | sed 's/(anonymous namespace):://g' | cut -c1-160
done
