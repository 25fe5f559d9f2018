"""Replay one whole-plan fuzz seed case by case on the GPU and report the case that
fails (error code or first differing byte); used to pin down fuzz failures."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import imaginary_amd as gpu  # noqa: E402
from oracle import oracle  # noqa: E402
from test_fuzz_gpu import random_case  # noqa: E402

seed = int(sys.argv[1])
r = np.random.default_rng(1000 + seed)
for k in range(40):
    w, h, b, opts, orient = random_case(r)
    try:
        p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(w, h, b, "png", orient))
    except gpu.MipxError:
        continue
    if p.out_w * p.out_h > 4_000_000:
        continue
    e, rp = oracle.plan(opts, dict(w=w, h=h, bands=b, type=3, orientation=orient))
    imgs = r.integers(0, 256, (2, h, w, b), dtype=np.uint8)
    try:
        got = gpu.execute(p, imgs)
    except gpu.MipxError as ex:
        print("FAIL", k, w, h, b, orient, opts, p.describe(), ex, flush=True)
        break
    ok = all(np.array_equal(got[i], oracle.execute(rp, imgs[i])) for i in range(2))
    print("ok" if ok else "MISMATCH", k, w, h, b, p.describe()[-1][0], flush=True)
