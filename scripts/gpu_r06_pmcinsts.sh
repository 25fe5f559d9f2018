#!/bin/bash
# r06: instruction mix of k_rcol (C1 shape, C3's window shape) and k_reduce2m (C2 centre):
# per-wave VALU / SALU / LDS / VMEM instruction counts and the issue-active / wait split
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
L="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA"
TAG=insts_rcol480 PMC_LIST="$L" OP_ARGS="reduce --w 480 --h 270 --b 3 --n 256 --s 1.6 --s2 1.5976331360946747" bash scripts/pmc_op.sh > gpurun_out/pmc_insts_rcol480.txt 2>&1 || exit 1
TAG=insts_rcol1024 PMC_LIST="$L" OP_ARGS="reduce --w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333" bash scripts/pmc_op.sh > gpurun_out/pmc_insts_rcol1024.txt 2>&1 || exit 1
TAG=insts_r2m PMC_LIST="$L" OP_ARGS="reduce --w 3840 --h 2160 --b 3 --n 256 --s 2 --sampling centre" bash scripts/pmc_op.sh > gpurun_out/pmc_insts_r2m.txt 2>&1 || exit 1
cat gpurun_out/pmc_insts_*.txt
