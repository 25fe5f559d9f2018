set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "blur or plan_execution" > gpurun_out/pt_blur2d.log 2>&1; rc=$?; tail -5 gpurun_out/pt_blur2d.log; [ $rc -ne 0 ] && exit $rc
ENVS="MIPX_BLUR2D_FROUND=0;MIPX_BLUR2D_FROUND=1;MIPX_BLUR2D_FROUND=1 MIPX_BLUR2D_ROWS=256;MIPX_BLUR2D_FROUND=1 MIPX_BLUR2D_ROWS=64" OP="blur --w 768 --h 512 --b 4 --n 512 --s 5" timeout -k 10 200 bash scripts/ab_env.sh > gpurun_out/ab_blur2d_fround_c3.log 2>&1 || exit 1
ENVS="MIPX_BLUR2D_FROUND=0;MIPX_BLUR2D_FROUND=1;MIPX_BLUR2D_FROUND=1 MIPX_BLUR2D_ROWS=256" OP="blur --w 1920 --h 1080 --b 3 --n 64 --s 3" timeout -k 10 200 bash scripts/ab_env.sh > gpurun_out/ab_blur2d_fround_rgb.log 2>&1 || exit 1
cut -c1-200 gpurun_out/ab_blur2d_fround_*.log
