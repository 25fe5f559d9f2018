#!/bin/bash
# k_reduce2d: A/B of the SGPR row offsets, then SQ counters of k_reduce2d vs k_reduce2x2 on C2
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
O="$R/gpurun_out/${OUT:-r05c}"; mkdir -p "$O"
timeout -k 10 200 python3 scripts/op_bench.py reduce --w 3840 --h 2160 --b 3 --n 256 --s 2 --iters 20 --ab MIPX_R2D=0,1 > "$O/r2d_ab.jsonl" || exit 1
MIPX_R2D=1 timeout -k 10 200 python3 scripts/op_bench.py reduce --w 3840 --h 2160 --b 3 --n 256 --s 2 --iters 20 --ab MIPX_R2D_SOFF=0,1 >> "$O/r2d_ab.jsonl" || exit 1
cat "$O/r2d_ab.jsonl"
MIPX_R2D=1 TAG=r2d OP_ARGS="reduce --w 3840 --h 2160 --b 3 --n 256 --s 2" PMC_LIST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES
FETCH_SIZE
TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" timeout -k 10 400 bash scripts/pmc_op.sh > "$O/pmc_r2d.txt" 2>&1; tail -40 "$O/pmc_r2d.txt"
