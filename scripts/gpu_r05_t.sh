#!/bin/bash
# C5 same-process A/B of this round's kernel switches; k_enlm timing probes and band heights
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05t}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
: > "$O/c5_ab.jsonl"
for k in MIPX_RCOL_UNAL=0,1 MIPX_ENLM=0,1 MIPX_RCOL_SWZ=0,1; do
  run 300 python3 scripts/cfg_ab.py --config C5 --ab $k --rounds 2 >> "$O/c5_ab.jsonl"
done
cat "$O/c5_ab.jsonl" | cut -c1-200
OUT=${OUT:-r05t} run 600 bash scripts/gpu_r05_s.sh
