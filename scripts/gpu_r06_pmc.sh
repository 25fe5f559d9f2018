#!/bin/bash
# r06 PMC passes: k_bcol on C3's blur (L2 hit rate: is the strips' halo re-read served by
# L2?; LDS conflicts), k_enlm at the survey's Enlarge shapes (LDS conflicts after the
# read-back lane order), k_rcol at the C1 shape (waits)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
SQL="SQ_WAVES SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
go() {  # go TAG "op args" "pass list"
  TAG=$1 OP_ARGS=$2 PMC_LIST=$3 timeout -k 10 700 bash scripts/pmc_op.sh > "gpurun_out/pmcop_$1.txt" 2>&1
  local rc=$?; [ $rc -eq 0 ] || { echo "pmc $1 failed rc=$rc"; tail -5 "gpurun_out/pmcop_$1.txt"; exit $rc; }
  cat "gpurun_out/pmcop_$1.txt"
}
for v in 0 1; do
  MIPX_BCOL_VPERM=$v MIPX_BCOL_WSW=$v go "bcol_c3_k$v" "blur --w 768 --h 512 --b 4 --n 512 --s 5" "$SQL
TCC_HIT_sum TCC_MISS_sum
FETCH_SIZE
WRITE_SIZE"
done
for v in 0 1; do
  MIPX_ENLM_OSW=$v go "enlm_1080p_k$v" "affine --w 1920 --h 1080 --b 3 --n 16 --s 2" "$SQL"
  MIPX_ENLM_OSW=$v go "enlm_550_k$v" "affine --w 550 --h 740 --b 3 --n 64 --s 2" "$SQL"
done
go "rcol_480" "reduce --w 480 --h 270 --b 3 --n 256 --s 1.6 --s2 1.5976331360946747" "$SQL
TCC_HIT_sum TCC_MISS_sum"
