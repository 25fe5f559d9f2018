import os, sys, json
sys.path.insert(0, os.getcwd())
import numpy as np
import imaginary_amd as ia
from oracle import oracle
opts = {'width': 0, 'height': 17, 'crop': 0, 'embed': 1, 'force': 0, 'enlarge': 0, 'gravity': 3, 'extend': 4, 'rotate': 0, 'flip': 0, 'flop': 0, 'sigma': 1.2, 'zoom': 0, 'interpretation': 0, 'background': [0, 0, 0]}
w, h, b, orient = 13, 258, 3, 4
p = ia.plan_make(ia.make_opts(**opts), ia.make_input(w, h, b, "png", orient))
e, rp = oracle.plan(opts, dict(w=w, h=h, bands=b, type=3, orientation=orient))
r = np.random.default_rng(5)
imgs = r.integers(0, 256, (2, h, w, b), dtype=np.uint8)
for env in [{}, {"MIPX_RMF2_UNALIGNED": "0"}, {"MIPX_RMF2_ORG": "16"}, {"MIPX_RMFMA": "0"}, {"MIPX_RMF2_HT": "1"}]:
    for k in ("MIPX_RMF2_UNALIGNED", "MIPX_RMF2_ORG", "MIPX_RMFMA", "MIPX_RMF2_HT"):
        os.environ.pop(k, None)
    os.environ.update(env)
    ia.lib.mipx_tuning_reload()  # the library snapshots MIPX_* knobs
    got = ia.execute(p, imgs)
    bad = [int((got[i] != oracle.execute(rp, imgs[i])).sum()) for i in range(2)]
    print(json.dumps({"env": env, "bytes_differ": bad}))
# the reduce alone on 1 x 23
x = r.integers(0, 256, (3, 23, 1, 3), dtype=np.uint8)
for env in [{}, {"MIPX_RMF2_UNALIGNED": "0"}, {"MIPX_RMF2_ORG": "16"}]:
    for k in ("MIPX_RMF2_UNALIGNED", "MIPX_RMF2_ORG"):
        os.environ.pop(k, None)
    os.environ.update(env)
    ia.lib.mipx_tuning_reload()  # the library snapshots MIPX_* knobs
    g = ia.run_op("reduce", x, hshrink=1.3529411764705883, vshrink=1.3529411764705883)
    bad = [int((g[i] != oracle.reduce(x[i], 1.3529411764705883, 1.3529411764705883)).sum()) for i in range(3)]
    print(json.dumps({"reduce_1x23": env, "bytes_differ": bad}))
