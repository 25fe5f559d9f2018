# batch device copy (k_copy16): parity, A/B vs hipMemcpyAsync, then the configs with the 200 ms warm-up
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03ze; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_parity_gpu.py tests/test_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/copy_ab.py > $O/copy_ab.jsonl 2>&1 || { tail $O/copy_ab.jsonl; exit 1; }
cat $O/copy_ab.jsonl
timeout -k 10 300 python3 -u bench_configs.py --configs C3,C4,C5 --steps 10 --warmup 2 > $O/configs.jsonl 2> $O/configs.err || { tail $O/configs.err; exit 1; }
cut -c1-300 $O/configs.jsonl
