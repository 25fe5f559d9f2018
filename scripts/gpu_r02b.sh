set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r02b; export TMPDIR=/tmp
O=gpurun_out/r02b
timeout -k 10 300 python3 bench_configs.py --configs C3,C4,C5 > $O/configs.jsonl 2> $O/configs.err; rc=$?; cut -c1-200 $O/configs.jsonl; [ $rc -eq 0 ] || exit $rc
for c in C3 C4 C5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 bench_configs.py --configs $c --steps 3 --warmup 1 > $O/prof_$c.log 2>&1 || exit $?
done
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json; exit $rc
