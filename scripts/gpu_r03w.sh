# k_bcol: skip the last K step's reads past the taps; parity + A/B
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03w; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_bcol_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_bcol.log 2>&1; rc=$?; tail -3 $O/pytest_bcol.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/blur_ab.py "MIPX_BCOL=" "MIPX_BCOL=0" > $O/blur_ab.jsonl 2> $O/blur_ab.err || { tail $O/blur_ab.err; exit 1; }
cat $O/blur_ab.jsonl
