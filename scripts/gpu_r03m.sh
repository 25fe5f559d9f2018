# k_bmf VALU diet: fp32 rounding + p-128 flip once in LDS: parity + A/B (RGB and forced RGBA)
set -u; cd $GRAFT_REPO_ROOT; O=gpurun_out/r03m; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_parity_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "blur" > $O/pytest_blur.log 2>&1; rc=$?; tail -3 $O/pytest_blur.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/blur_ab.py "MIPX_BMF=1,MIPX_BMF_FP=1,MIPX_BMF_X1=1" "MIPX_BMF=1,MIPX_BMF_FP=0,MIPX_BMF_X1=1" "MIPX_BMF=1,MIPX_BMF_FP=1,MIPX_BMF_X1=0" "MIPX_BMF=1,MIPX_BMF_FP=0,MIPX_BMF_X1=0" "MIPX_BMF=,MIPX_BMF_FP=1,MIPX_BMF_X1=1" > $O/blur_ab.jsonl 2> $O/blur_ab.err || { tail $O/blur_ab.err; exit 1; }
cat $O/blur_ab.jsonl
