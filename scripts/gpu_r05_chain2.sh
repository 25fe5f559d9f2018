#!/bin/bash
# chain v2 (FRONT 1): parity tests, then C3 A/B (unfused / FRONT 0 / FRONT 1)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05e}"; mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_chain_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest_chain.log" 2>&1
rc=$?; tail -15 "$O/pytest_chain.log"; [ $rc -eq 0 ] || exit $rc
MIPX_CHAIN=1 timeout -k 10 300 python3 scripts/cfg_ab.py --config C3 --ab MIPX_CHAIN_FRONT=0,1 --rounds 2 > "$O/c3_front_ab.jsonl" || exit 1
timeout -k 10 300 python3 scripts/cfg_ab.py --config C3 --ab MIPX_CHAIN=0,1 --rounds 3 >> "$O/c3_front_ab.jsonl" || exit 1
cat "$O/c3_front_ab.jsonl"
