# rot 90 RGB: memory-only ceilings of the tile pattern (scripts/strip_probe.hip PROBE_ROT) and PMC of the engine kernel
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03za; mkdir -p $O; export TMPDIR=/tmp
PROBE_ROT=1 timeout -k 10 240 ./scripts/strip_probe > $O/rot_probe.jsonl 2>&1 || { tail $O/rot_probe.jsonl; exit 1; }
PMC_LIST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU
FETCH_SIZE
WRITE_SIZE" TAG=rot OP_ARGS="rot --w 3840 --h 2160 --b 3 --n 32 --s 90" timeout -k 10 400 bash scripts/pmc_op.sh > $O/pmc_rot.txt 2>&1 || { tail $O/pmc_rot.txt; exit 1; }
cat $O/pmc_rot.txt
