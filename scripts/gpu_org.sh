set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_demand_gpu.py tests/test_pipeline.py -k "rmfma_fused or reduce or C3 or C4 or C5 or c3 or c4 or c5 or crop or fused" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_org.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_org.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/rs_ab.py MIPX_RMF2_ORG=4 MIPX_RMF2_ORG=16 > gpurun_out/org_ab.jsonl 2>gpurun_out/org_ab.err; rc=$?; cut -c1-170 gpurun_out/org_ab.jsonl; exit $rc
