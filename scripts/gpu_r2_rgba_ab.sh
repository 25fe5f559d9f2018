# A/B of the fused 2x2 reduce geometry knobs on C3's RGBA shape (2048^2 -> 1024^2, x512)
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
ENVS="MIPX_R2_BAND=2;MIPX_R2_BAND=1;MIPX_R2_BAND=3;MIPX_R2_BAND=4;MIPX_R2_ORDER=1;MIPX_R2_REMAP=0;MIPX_R2_VARIANT=0;MIPX_R2_VARIANT=130" OP="reduce --w 2048 --h 2048 --b 4 --n 512 --s 2" timeout -k 10 400 bash scripts/ab_env.sh > gpurun_out/ab_r2_rgba.log 2>&1 || exit 1
ENVS="MIPX_R2_BAND=2;MIPX_R2_BAND=3;MIPX_R2_ORDER=1" OP="reduce --w 3840 --h 2160 --b 3 --n 256 --s 2" timeout -k 10 300 bash scripts/ab_env.sh > gpurun_out/ab_r2_rgb.log 2>&1 || exit 1
python3 - << 'PY'
import json
for f in ("gpurun_out/ab_r2_rgba.log", "gpurun_out/ab_r2_rgb.log"):
    for l in open(f):
        d = json.loads(l); print(f[-12:], d["round"], f'{d["env"]:24s}', d["r"]["ms"], d["r"]["alg_GBps"])
PY
