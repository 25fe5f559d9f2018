# k_rcol horizontal reads as ds_read2_b64: parity, A/B vs k_rmf2, PMC (verdict r2 item 1 counters)
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03o; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_rcol_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_rcol.log 2>&1; rc=$?; tail -3 $O/pytest_rcol.log; [ $rc -eq 0 ] || exit $rc
VARIANTS='MIPX_RCOL_WST=1;MIPX_RCOL=0' timeout -k 10 400 python3 -u scripts/ab_rcol.py > $O/ab_rcol.jsonl 2> $O/ab_rcol.err || { tail $O/ab_rcol.err; exit 1; }
cat $O/ab_rcol.jsonl
PL='SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD
FETCH_SIZE
WRITE_SIZE'
PMC_LIST="$PL" TAG=rc16w OP_ARGS="reduce --w 1920 --h 1080 --b 3 --n 64 --s 1.6" timeout -k 10 300 bash scripts/pmc_op.sh > $O/pmc_rc16.txt 2>&1 || { tail $O/pmc_rc16.txt; exit 1; }
cat $O/pmc_rc16.txt
PMC_LIST="$PL" TAG=rc133w OP_ARGS="reduce --w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333" timeout -k 10 300 bash scripts/pmc_op.sh > $O/pmc_rc133.txt 2>&1 || { tail $O/pmc_rc133.txt; exit 1; }
cat $O/pmc_rc133.txt
timeout -k 10 120 ./scripts/strip_probe > $O/tile_probe.jsonl 2>&1; rc=$?; cat $O/tile_probe.jsonl; exit $rc
