#!/bin/bash
# PMC passes (separate rocprofv3 runs, counters only + kernel-trace) over a short bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT="$R/gpurun_out/pmc_${TAG:-r01}"
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="$R/bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu --no-verify ${BENCH_ARGS:-}"
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$OUT/p$i" -o run -- python3 $BENCH > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($ctrs): rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done <<LIST
${PMC_LIST:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT}
LIST
echo pmc done
