#!/bin/bash
# PMC passes (one rocprofv3 run each) over scripts/op_bench.py with OP_ARGS;
# prints per-kernel averages.  TAG names the output dir under gpurun_out/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out/pmcop_${TAG:-x}"; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/scripts/op_bench.py" $OP_ARGS --iters 3 --warm-ms 0 > "$OUT/p$i.log" 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -5 "$OUT/p$i.log"; exit $rc; fi
done <<LIST
${PMC_LIST:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
FETCH_SIZE
WRITE_SIZE
GRBM_GUI_ACTIVE GRBM_COUNT}
LIST
python3 - "$OUT" <<'EOF'
import csv, glob, sys, collections
vals = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/*counter_collection.csv"):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "mipx" not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void mipx::", "").split("(")[0]
        per[(k, r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (k, c, d), v in per.items():
        vals[(k, c)].append(v)
for (k, c), v in sorted(vals.items()):
    print(f"{k[:48]:48s} {c:22s} {sum(v)/len(v):16.1f}")
EOF
