# k_rcol on unaligned input rows: parity (incl. fuzz, probe-fallback cases), A/B
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03y; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_rcol_gpu.py tests/test_configs_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_rcol.log 2>&1; rc=$?; tail -3 $O/pytest_rcol.log; [ $rc -eq 0 ] || exit $rc
VARIANTS='MIPX_RCOL=;MIPX_RCOL=0' timeout -k 10 400 python3 -u scripts/ab_rcol.py > $O/ab_rcol.jsonl 2> $O/ab_rcol.err || { tail $O/ab_rcol.err; exit 1; }
cat $O/ab_rcol.jsonl
