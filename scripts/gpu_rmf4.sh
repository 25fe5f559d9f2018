set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py -k "rmfma_fused" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_rmf4.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_rmf4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/rs_ab.py MIPX_RMF4=1 MIPX_RMF4=2 MIPX_RMF4=0 > gpurun_out/rmf4_ab.jsonl 2>gpurun_out/rmf4_ab.err; rc=$?; cut -c1-170 gpurun_out/rmf4_ab.jsonl; exit $rc
