set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
S=$(date +%s); timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo "bench wall $(( $(date +%s) - S )) s"; cut -c1-300 $O/bench.json; tail -1 $O/bench.err
timeout -k 10 600 bash scripts/op_survey.sh > $O/op_survey.log 2>&1 || exit $?; cp gpurun_out/op_survey.jsonl $O/; cat $O/op_survey.log
