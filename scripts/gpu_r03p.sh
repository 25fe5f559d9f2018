# k_bcol (column-walking gaussblur): parity, A/B vs k_bmf / k_blur2d
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03p; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_bcol_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_bcol.log 2>&1; rc=$?; tail -15 $O/pytest_bcol.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/blur_ab.py "MIPX_BCOL=,MIPX_BCOL_PX=64" "MIPX_BCOL=,MIPX_BCOL_PX=128" "MIPX_BCOL=0,MIPX_BCOL_PX=64" > $O/blur_ab.jsonl 2> $O/blur_ab.err || { tail $O/blur_ab.err; exit 1; }
cat $O/blur_ab.jsonl
