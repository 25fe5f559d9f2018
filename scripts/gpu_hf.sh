set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_parity_gpu.py tests/test_rstrip_gpu.py tests/test_configs_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_hf.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_hf.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/rs_ab.py MIPX_HP_FAST=1 MIPX_HP_FAST=0 MIPX_HP_FAST=1,MIPX_HP_PACK3=1 > gpurun_out/hf_ab.jsonl 2>gpurun_out/hf_ab.err; rc=$?; cut -c1-170 gpurun_out/hf_ab.jsonl; exit $rc
