# full GPU suite, k_rcol v4 PMC at two shapes, op survey
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03g; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
PL='SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM
FETCH_SIZE
WRITE_SIZE'
PMC_LIST="$PL" TAG=rc16 OP_ARGS="reduce --w 1920 --h 1080 --b 3 --n 64 --s 1.6" timeout -k 10 400 bash scripts/pmc_op.sh > $O/pmc_rc16.txt 2>&1 || { tail $O/pmc_rc16.txt; exit 1; }
cat $O/pmc_rc16.txt
PMC_LIST="$PL" TAG=rc500 OP_ARGS="reduce --w 500 --h 375 --b 3 --n 128 --s 1.46484375" timeout -k 10 400 bash scripts/pmc_op.sh > $O/pmc_rc500.txt 2>&1 || { tail $O/pmc_rc500.txt; exit 1; }
cat $O/pmc_rc500.txt
bash scripts/op_survey.sh > $O/op_survey.txt 2>&1; rc=$?; cp gpurun_out/op_survey.jsonl $O/; cat $O/op_survey.txt; exit $rc
