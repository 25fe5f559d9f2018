# r03 final checkpoint: rot px tiles, batch copy, NT embed/flip, bcol A16 + byte strips: smoke, torchrun bench, full GPU suite, configs, op survey,
# rocprofv3 kernel stats of the bench
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zz; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 100 --warmup 20 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
timeout -k 10 300 python3 -u bench_configs.py --configs C3,C4,C5 --steps 10 --warmup 2 > $O/configs.jsonl 2> $O/configs.err || { tail $O/configs.err; exit 1; }
cut -c1-300 $O/configs.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 100 --warmup 20 --no-cpu --no-verify > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec head -5 {} \;
bash scripts/op_survey.sh > $O/op_survey.txt 2>&1; rc=$?; cp gpurun_out/op_survey.jsonl $O/; cat $O/op_survey.txt; exit $rc
