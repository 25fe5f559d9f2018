set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_fuzz_gpu.py tests/test_demand_gpu.py -k "embed or extract or C5 or c5 or C4 or c4 or smartcrop or random or crop" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_embed.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_embed.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/embed_ab.py MIPX_EMBED_RPB=4 MIPX_EMBED_RPB=1 MIPX_EMBED_RPB=8 > gpurun_out/embed_ab.jsonl 2>gpurun_out/embed_ab.err; rc=$?; cut -c1-170 gpurun_out/embed_ab.jsonl; exit $rc
