# rot 90/270: 128 x 128 tiles for RGB: parity + A/B
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03v; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "rot" > $O/pytest_rot.log 2>&1; rc=$?; tail -3 $O/pytest_rot.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/rot_ab.py "MIPX_ROT_T=,MIPX_ROT_TH=,MIPX_ROT_ORDER=" "MIPX_ROT_T=128,MIPX_ROT_TH=128,MIPX_ROT_ORDER=1" "MIPX_ROT_T=128,MIPX_ROT_TH=128,MIPX_ROT_ORDER=0" > $O/rot_ab.jsonl 2> $O/rot_ab.err || { tail $O/rot_ab.err; exit 1; }
cat $O/rot_ab.jsonl
