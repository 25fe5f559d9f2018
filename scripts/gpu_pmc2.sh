set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
export OP_ARGS="reduce --w 1920 --h 1080 --b 3 --n 64 --s 1.6"
export PMC_LIST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM
GRBM_GUI_ACTIVE GRBM_COUNT
FETCH_SIZE
WRITE_SIZE"
TAG=${TAG:-vf} bash scripts/pmc_op.sh > gpurun_out/pmc_${TAG:-vf}.txt 2>&1 || { tail gpurun_out/pmc_${TAG:-vf}.txt; exit 1; }
cat gpurun_out/pmc_${TAG:-vf}.txt
