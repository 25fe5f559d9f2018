# r03 checkpoint on the k_rcol v4 tree: smoke, torchrun bench, full GPU suite, op survey
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03f; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 50 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/op_survey.sh > $O/op_survey.txt 2>&1; rc=$?; cp gpurun_out/op_survey.jsonl $O/; cat $O/op_survey.txt; exit $rc
