set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/voff; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
MIPX_FUZZ_SEEDS=200 timeout -k 10 600 python3 -u -m pytest tests/test_fuzz_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/fuzz200.log 2>&1; rc=$?; tail -2 $O/fuzz200.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/rs_ab.py MIPX_RSTRIP=1 MIPX_RSTRIP=0 > $O/rs_ab.jsonl 2>&1; cut -c1-150 $O/rs_ab.jsonl | head -8
timeout -k 10 300 python3 scripts/blur_ab.py MIPX_BMF=1 > $O/blur_ab.jsonl 2>&1; cut -c1-150 $O/blur_ab.jsonl
