set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/repro_fuzz75.py || exit 1
MIPX_FUZZ_SEEDS=200 timeout -k 10 600 python3 -u -m pytest tests/test_fuzz_gpu.py tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_demand_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/fix.log 2>&1; rc=$?; tail -3 gpurun_out/fix.log; [ $rc -eq 0 ] || exit $rc
ANGLES=180 timeout -k 10 300 python3 scripts/rot_ab.py MIPX_FLIP_RPB=4 MIPX_FLIP_RPB=1 MIPX_FLIP_RPB=8 > gpurun_out/flip_ab.jsonl 2>gpurun_out/flip_ab.err; rc=$?; cut -c1-170 gpurun_out/flip_ab.jsonl; exit $rc
