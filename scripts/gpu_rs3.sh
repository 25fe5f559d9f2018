set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_rstrip_gpu.py tests/test_parity_gpu.py tests/test_configs_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_rs.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_rs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/rs_ab.py MIPX_RSTRIP= MIPX_RSTRIP=1 MIPX_RSTRIP=0 > gpurun_out/rstrip_ab.jsonl 2>gpurun_out/rs_ab3.err; rc=$?; cut -c1-160 gpurun_out/rstrip_ab.jsonl; tail -3 gpurun_out/rs_ab3.err; exit $rc
