set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "reduceh_paths" > gpurun_out/pytest_hm.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_hm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_parity_gpu.py tests/test_rstrip_gpu.py tests/test_configs_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_hm2.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_hm2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/rs_ab.py MIPX_HP_MFMA=1,MIPX_HM_XW=1 MIPX_HP_MFMA=1,MIPX_HM_XW=2 MIPX_HP_MFMA=0 > gpurun_out/hm_ab.jsonl 2>gpurun_out/hm_ab.err; rc=$?; cut -c1-150 gpurun_out/hm_ab.jsonl; exit $rc
