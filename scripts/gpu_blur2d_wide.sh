# fused blur at wide masks (NQ 9..12): parity, then A/B vs the two passes
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py tests/test_fuzz_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "blur or plan_execution or fuzz" > gpurun_out/pt_blur2d_wide.log 2>&1; rc=$?; tail -3 gpurun_out/pt_blur2d_wide.log; [ $rc -ne 0 ] && exit $rc
ENVS="MIPX_BLUR2D=0;MIPX_BLUR2D=1" OP="blur --w 768 --h 512 --b 4 --n 512 --s 9" timeout -k 10 200 bash scripts/ab_env.sh > gpurun_out/ab_blur2d_s9.log 2>&1 || exit 1
ENVS="MIPX_BLUR2D=0;MIPX_BLUR2D=1" OP="blur --w 1920 --h 1080 --b 3 --n 64 --s 12.5" timeout -k 10 200 bash scripts/ab_env.sh > gpurun_out/ab_blur2d_s12.log 2>&1 || exit 1
python3 - << 'PY'
import json
for f in ("gpurun_out/ab_blur2d_s9.log", "gpurun_out/ab_blur2d_s12.log"):
    for l in open(f):
        d = json.loads(l); print(f[-16:], d["round"], f'{d["env"]:16s}', d["r"]["ms"], d["r"]["alg_GBps"])
PY
