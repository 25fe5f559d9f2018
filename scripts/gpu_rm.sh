set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "rmfma" > gpurun_out/pytest_rm.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_rm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/rs_ab.py ${RM_VARIANTS:-MIPX_RMFMA=3 MIPX_RMFMA=2 MIPX_RMFMA=0} > gpurun_out/rm_ab.jsonl 2>gpurun_out/rm_ab.err; rc=$?; cut -c1-140 gpurun_out/rm_ab.jsonl; exit $rc
