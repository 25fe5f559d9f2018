# k_rot90_px (3-band rot through the pixel-major LDS tile): parity, then A/B vs k_rot90_lds
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03zb; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_parity_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "rot or extract_rot" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/rot_ab.py MIPX_ROT_PX=0,MIPX_ROT_PXH=128,MIPX_ROT_ORDER= MIPX_ROT_PX=1,MIPX_ROT_PXH=32,MIPX_ROT_ORDER=1 MIPX_ROT_PX=1,MIPX_ROT_PXH=64,MIPX_ROT_ORDER=1 MIPX_ROT_PX=1,MIPX_ROT_PXH=128,MIPX_ROT_ORDER=1 MIPX_ROT_PX=1,MIPX_ROT_PXH=128,MIPX_ROT_ORDER=0 MIPX_ROT_PX=1,MIPX_ROT_PXH=32,MIPX_ROT_ORDER=0 > $O/rot_px_ab.jsonl 2>&1 || { tail $O/rot_px_ab.jsonl; exit 1; }
cat $O/rot_px_ab.jsonl
