# k_bcol PMC: RGB sigma 3 (1 K step) vs sigma 5 (2 K steps), RGBA sigma 5 (C3)
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zi; mkdir -p $O; export TMPDIR=/tmp
PL="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
SQ_INSTS_VALU_MFMA_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_IDX_ACTIVE
GRBM_GUI_ACTIVE GRBM_COUNT"
PMC_LIST="$PL" TAG=b3 OP_ARGS="blur --w 1920 --h 1080 --b 3 --n 64 --s 3" timeout -k 10 300 bash scripts/pmc_op.sh > $O/pmc_bcol_rgb_s3.txt 2>&1 || { tail $O/pmc_bcol_rgb_s3.txt; exit 1; }
PMC_LIST="$PL" TAG=b5 OP_ARGS="blur --w 1920 --h 1080 --b 3 --n 64 --s 5" timeout -k 10 300 bash scripts/pmc_op.sh > $O/pmc_bcol_rgb_s5.txt 2>&1 || { tail $O/pmc_bcol_rgb_s5.txt; exit 1; }
PMC_LIST="$PL" TAG=b45 OP_ARGS="blur --w 768 --h 512 --b 4 --n 512 --s 5" timeout -k 10 300 bash scripts/pmc_op.sh > $O/pmc_bcol_rgba_s5.txt 2>&1 || { tail $O/pmc_bcol_rgba_s5.txt; exit 1; }
A="timeout -k 10 120 python3 -u scripts/op_bench.py"
$A blur --w 1920 --h 1080 --b 3 --n 64 --s 5 > $O/t.jsonl && $A blur --w 1920 --h 1080 --b 3 --n 64 --s 3 >> $O/t.jsonl && $A blur --w 3840 --h 2160 --b 3 --n 16 --s 3 >> $O/t.jsonl && $A blur --w 3840 --h 2160 --b 3 --n 16 --s 1 >> $O/t.jsonl
cat $O/t.jsonl
paste $O/pmc_bcol_rgb_s3.txt $O/pmc_bcol_rgb_s5.txt $O/pmc_bcol_rgba_s5.txt | awk '{print $2, $3, $6, $9}'
