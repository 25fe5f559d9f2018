#!/bin/bash
# r06: stage pipelining across sub-batches (MIPX_PIPE = chunks): the chain tests with it on,
# then C3 at both conventions with MIPX_PIPE off / 2 / 4 / 8, alternating in separate processes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r06_pipe}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
if [ "${TESTS:-1}" = 1 ]; then
  MIPX_PIPE=2 run 600 python3 -u -m pytest tests/test_pipe_gpu.py tests/test_chain_gpu.py tests/test_demand_gpu.py tests/test_pipeline.py \
    -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_pipe.log" 2>&1
  tail -2 "$O/pytest_pipe.log"
fi
for rep in 1 2; do
  for k in 0 2 4 8; do
    for smp in corner centre; do
      MIPX_PIPE=$k timeout -k 10 300 python3 -u bench_configs.py --configs C3 --steps 20 --warmup 2 --sampling $smp \
        | sed "s/^{/{\"pipe\": $k, /" >> "$O/configs.jsonl" 2>> "$O/configs.err" || { echo "configs failed"; exit 1; }
    done
  done
done
python3 - "$O" <<'PY'
import json, sys
for l in open(sys.argv[1] + "/configs.jsonl"):
    d = json.loads(l); print(d["pipe"], d["config"], d["sampling"], d["ms_per_step"], d["hbm_frac"], d["verified_vs_oracle"])
PY
