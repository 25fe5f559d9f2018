# r02 final: smoke, torchrun bench (1 rank), full GPU suite, bench + rocprof, configs + rocprof, op survey
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r02d; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_torchrun.json 2> $O/bench_torchrun.err || { tail $O/bench_torchrun.err; exit 1; }
cut -c1-200 $O/bench_torchrun.json
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit $?
cut -c1-300 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 bench.py --steps 100 --warmup 20 --no-cpu --no-verify > $O/prof_bench.log 2>&1 || exit $?
timeout -k 10 300 python3 bench_configs.py --configs C3,C4,C5 > $O/configs.jsonl 2> $O/configs.err || exit $?
cut -c1-200 $O/configs.jsonl
for c in C3 C4 C5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 bench_configs.py --configs $c --steps 3 --warmup 1 > $O/prof_$c.log 2>&1 || exit $?
done
timeout -k 10 600 bash scripts/op_survey.sh > $O/op_survey.log 2>&1 || exit $?
cp gpurun_out/op_survey.jsonl $O/op_survey.jsonl
echo done
