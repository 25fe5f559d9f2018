# round-end rehearsal: smoke(), the torchrun launch path of bench.py (1 rank), full GPU suite
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_torchrun.json 2> gpurun_out/bench_torchrun.err || { tail gpurun_out/bench_torchrun.err; exit 1; }
cut -c1-300 gpurun_out/bench_torchrun.json
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_rehearsal.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_rehearsal.log; exit $rc
