# k_bcol (64-px only) parity + 200-seed whole-plan fuzz on the r03 kernels
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03t; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_bcol_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_bcol.log 2>&1; rc=$?; tail -3 $O/pytest_bcol.log; [ $rc -eq 0 ] || exit $rc
MIPX_FUZZ_SEEDS=200 timeout -k 10 900 python3 -u -m pytest tests/test_fuzz_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/fuzz200.log 2>&1; rc=$?; tail -5 $O/fuzz200.log; exit $rc
