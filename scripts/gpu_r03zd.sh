# C3 stages one at a time (scripts/c3_stage_probe.py), then its kernel trace
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zd; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/c3_stage_probe.py > $O/c3_stages.jsonl 2>&1 || { tail $O/c3_stages.jsonl; exit 1; }
cut -c1-120 $O/c3_stages.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/c3_stage_probe.py > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cut -c1-150 {} \; | grep -v distribution
