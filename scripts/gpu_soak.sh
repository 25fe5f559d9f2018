set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
MIPX_FUZZ_SEEDS=200 timeout -k 10 900 python3 -u -m pytest tests/test_fuzz_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/fuzz200.log 2>&1; rc=$?; tail -3 gpurun_out/fuzz200.log; exit $rc
