#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out/calib"; mkdir -p "$OUT"; export TMPDIR=/tmp
[ -x "$R/scripts/calib_traffic" ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 "$R/scripts/calib_traffic.hip" -o "$R/scripts/calib_traffic" || exit $?
timeout -k 10 120 "$R/scripts/calib_traffic" > "$OUT/plain.log" 2>&1 || exit $?
cat "$OUT/plain.log"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/$c" -o run -- "$R/scripts/calib_traffic" > "$OUT/$c.log" 2>&1 || exit $?
done
echo calib done
