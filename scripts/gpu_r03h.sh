# k_rcol row cap (narrow strips, 2.4) + 128-VGPR variant + unaligned rows: parity, A/B
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_rcol_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_rcol.log 2>&1; rc=$?; tail -5 $O/pytest_rcol.log; [ $rc -eq 0 ] || exit $rc
VARIANTS='MIPX_RCOL_ONEB=1;MIPX_RCOL_ONEB=0;MIPX_RCOL_ONEB=0,MIPX_RCOL_W4=0;MIPX_RCOL=0' timeout -k 10 400 python3 -u scripts/ab_rcol.py > $O/ab_rcol.jsonl 2> $O/ab_rcol.err || { tail $O/ab_rcol.err; exit 1; }
cat $O/ab_rcol.jsonl
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "rot" > $O/pytest_rot.log 2>&1; rc=$?; tail -3 $O/pytest_rot.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/rot_ab.py "MIPX_ROT_ST16=1" "MIPX_ROT_ST16=0" > $O/rot_ab.jsonl 2> $O/rot_ab.err || { tail $O/rot_ab.err; exit 1; }
cat $O/rot_ab.jsonl
