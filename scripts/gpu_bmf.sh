set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_pipeline.py -k "blur or C5 or c5 or fused" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_bmf.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_bmf.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/blur_ab.py MIPX_BMF_RG=2 MIPX_BMF_RG=1 MIPX_BMF=1,MIPX_BMF_RG=2 MIPX_BMF=0,MIPX_BMF_RG= > gpurun_out/bmf_rg_ab.jsonl 2>gpurun_out/bmf_rg_ab.err; rc=$?; cut -c1-150 gpurun_out/bmf_rg_ab.jsonl; exit $rc
