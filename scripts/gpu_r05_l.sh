#!/bin/bash
# k_enlm v4 (cvt_pk_u8 epilogue): parity + A/B, PMC on 1080p x2 RGB and 1024x768 RGBA x2
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05l}"; mkdir -p "$O"
run() { local lim=$1; shift; timeout -k 10 "$lim" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step failed rc=$rc: $*"; exit $rc; }; }
OUT=${OUT:-r05l} run 600 bash scripts/gpu_r05_enlm.sh
export MIPX_ENLM=2
P="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS
FETCH_SIZE
WRITE_SIZE"
TAG=enlm4_1080p OP_ARGS="affine --w 1920 --h 1080 --b 3 --n 16 --s 2" PMC_LIST="$P" run 300 bash scripts/pmc_op.sh > "$O/pmc_enlm_1080p.txt" 2>&1
TAG=enlm4_rgba OP_ARGS="affine --w 1024 --h 768 --b 4 --n 16 --s 2" PMC_LIST="$P" run 300 bash scripts/pmc_op.sh > "$O/pmc_enlm_rgba.txt" 2>&1
grep "^k_enlm" "$O/pmc_enlm_1080p.txt" "$O/pmc_enlm_rgba.txt"
