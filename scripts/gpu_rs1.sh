set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_rstrip_gpu.py tests/test_parity_gpu.py -k "reduce or rstrip or plan" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_rs.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_rs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/rs_ab.py > gpurun_out/rs_ab.jsonl 2>gpurun_out/rs_ab.err; rc=$?; cat gpurun_out/rs_ab.jsonl; tail -3 gpurun_out/rs_ab.err; exit $rc
