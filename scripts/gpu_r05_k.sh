#!/bin/bash
# k_enlm v3 parity + A/B; v_cvt_pk_u8_f32 semantics probe
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05k}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
run 60 scripts/probe/cvt_pk_u8 > "$O/cvt_pk_u8.txt" 2>&1
cat "$O/cvt_pk_u8.txt"
OUT=${OUT:-r05k} run 600 bash scripts/gpu_r05_enlm.sh
