set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "reduce or plan_execution or hpass" > gpurun_out/pt_reduce2d.log 2>&1; rc=$?; tail -5 gpurun_out/pt_reduce2d.log; [ $rc -ne 0 ] && exit $rc
ENVS="MIPX_REDUCE2D=0;MIPX_REDUCE2D=1 MIPX_REDUCE2D_ROWS=4;MIPX_REDUCE2D=1 MIPX_REDUCE2D_ROWS=8;MIPX_REDUCE2D=1 MIPX_REDUCE2D_ROWS=16" OP="reduce --w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333" timeout -k 10 200 bash scripts/ab_env.sh > gpurun_out/ab_reduce2d_c3.log 2>&1 || exit 1
ENVS="MIPX_REDUCE2D=0;MIPX_REDUCE2D=1 MIPX_REDUCE2D_ROWS=8;MIPX_REDUCE2D=1 MIPX_REDUCE2D_ROWS=16" OP="reduce --w 1920 --h 1080 --b 3 --n 64 --s 2.466666666666667" timeout -k 10 200 bash scripts/ab_env.sh > gpurun_out/ab_reduce2d_rgb.log 2>&1 || exit 1
ENVS="MIPX_REDUCE2D=0;MIPX_REDUCE2D=1 MIPX_REDUCE2D_ROWS=8;MIPX_REDUCE2D=1 MIPX_REDUCE2D_ROWS=16" OP="reduce --w 1280 --h 720 --b 3 --n 64 --s 1.6" timeout -k 10 200 bash scripts/ab_env.sh > gpurun_out/ab_reduce2d_rgb2.log 2>&1 || exit 1
cut -c1-250 gpurun_out/ab_reduce2d_*.log
