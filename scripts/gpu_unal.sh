set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_demand_gpu.py -k "rmfma_fused or reduce or C5 or c5 or crop" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_unal.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_unal.log; [ $rc -eq 0 ] || exit $rc
RS_SHAPES="1333,1000,3,48,1.6666666666666667,1.6666666666666667;1331,999,3,48,1.6666666666666667,1.6666666666666667;1026,770,3,64,1.5,1.5" timeout -k 10 300 python3 scripts/rs_ab.py MIPX_RMF2_UNALIGNED=1 MIPX_RMF2_UNALIGNED=0 > gpurun_out/unal_ab.jsonl 2>gpurun_out/unal_ab.err; rc=$?; cut -c1-170 gpurun_out/unal_ab.jsonl; exit $rc
