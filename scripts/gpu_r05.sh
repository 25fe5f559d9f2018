#!/bin/bash
# r05 step runner: chain tests first, then the evidence steps (each under its own limit)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05}"; mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests/test_chain_gpu.py tests/test_sampling_gpu.py -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$O/pytest_chain.log" 2>&1; rc=$?
tail -30 "$O/pytest_chain.log"
[ $rc -eq 0 ] || exit $rc
OUT=${OUT:-r05} STEPS="${STEPS:-tests smoke bench}" bash scripts/gpu_evidence.sh
