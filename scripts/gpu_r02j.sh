set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r02j; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit $?
cut -c1-200 $O/bench.json
timeout -k 10 300 python3 bench_configs.py --configs C3,C4,C5 > $O/configs.jsonl 2> $O/configs.err || exit $?
cut -c1-200 $O/configs.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_C5 -o run -- python3 bench_configs.py --configs C5 --steps 3 --warmup 1 > $O/prof_C5.log 2>&1 || exit $?
echo done
timeout -k 10 600 bash scripts/op_survey.sh > $O/op_survey.log 2>&1 || exit $?; cp gpurun_out/op_survey.jsonl $O/; echo done3
