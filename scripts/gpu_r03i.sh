# k_rcol: software-pipelined vertical pass (VP) parity + A/B
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03i; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_rcol_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_rcol.log 2>&1; rc=$?; tail -3 $O/pytest_rcol.log; [ $rc -eq 0 ] || exit $rc
MIPX_RCOL_VP=1 timeout -k 10 400 python3 -u -m pytest tests/test_rcol_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "rcol" > $O/pytest_rcol_vp1.log 2>&1; rc=$?; tail -3 $O/pytest_rcol_vp1.log; [ $rc -eq 0 ] || exit $rc
VARIANTS='MIPX_RCOL_VP=1;MIPX_RCOL_VP=0;MIPX_RCOL=0' timeout -k 10 400 python3 -u scripts/ab_rcol.py > $O/ab_rcol.jsonl 2> $O/ab_rcol.err || { tail $O/ab_rcol.err; exit 1; }
cat $O/ab_rcol.jsonl
PL='SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE
FETCH_SIZE'
PMC_LIST="$PL" TAG=b2d OP_ARGS="blur --w 768 --h 512 --b 4 --n 512 --s 5" timeout -k 10 300 bash scripts/pmc_op.sh > $O/pmc_b2d.txt 2>&1 || { tail $O/pmc_b2d.txt; exit 1; }
cat $O/pmc_b2d.txt
PMC_LIST="$PL" TAG=bmf OP_ARGS="blur --w 1920 --h 1080 --b 3 --n 64 --s 3" timeout -k 10 300 bash scripts/pmc_op.sh > $O/pmc_bmf.txt 2>&1 || { tail $O/pmc_bmf.txt; exit 1; }
cat $O/pmc_bmf.txt
