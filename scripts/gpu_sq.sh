set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py tests/test_demand_gpu.py tests/test_configs_gpu.py -k "shrink or c5 or C5" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_sq.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_sq.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/shrink_ab.py > gpurun_out/sq_ab.jsonl 2>gpurun_out/sq_ab.err; rc=$?; cut -c1-150 gpurun_out/sq_ab.jsonl; exit $rc
