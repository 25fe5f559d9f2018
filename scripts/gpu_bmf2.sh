set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py -k "blur_mfma" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_bmf3.log 2>&1 || { tail -20 gpurun_out/pytest_bmf3.log; exit 1; }
timeout -k 10 300 python3 scripts/blur_ab.py MIPX_BMF=1,MIPX_BMF_RG=2 MIPX_BMF=1,MIPX_BMF_RG=3 MIPX_BMF=0,MIPX_BMF_RG=2 > gpurun_out/bmf_rg3_ab.jsonl 2>gpurun_out/bmf_rg_ab.err; rc=$?; cut -c1-150 gpurun_out/bmf_rg3_ab.jsonl; exit $rc
