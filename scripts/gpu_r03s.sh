# k_bcol operand chunks (128-px strips) parity + A/B; C5 kernel-time split
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03s; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_bcol_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_bcol.log 2>&1; rc=$?; tail -3 $O/pytest_bcol.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/blur_ab.py "MIPX_BCOL=,MIPX_BCOL_PX=64" "MIPX_BCOL=,MIPX_BCOL_PX=128" "MIPX_BCOL=0,MIPX_BCOL_PX=64" > $O/blur_ab.jsonl 2> $O/blur_ab.err || { tail $O/blur_ab.err; exit 1; }
cat $O/blur_ab.jsonl
CONFIGS=C5 TAG=r03s timeout -k 10 400 bash scripts/prof_configs.sh > $O/prof_c5.txt 2>&1 || { tail $O/prof_c5.txt; exit 1; }
python3 - gpurun_out/profcfg_r03s/C5/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows if "mipx" in r["Name"])
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:20]:
    if "mipx" not in r["Name"]: continue
    nm = r["Name"].replace("(anonymous namespace)::", "").replace("void mipx::", "").split("(")[0]
    print(f'{nm[:60]:60s} calls {r["Calls"]:>5s} avg {float(r["AverageNs"])/1e3:9.1f} us  share {float(r["TotalDurationNs"])/tot:6.1%}')
PY
