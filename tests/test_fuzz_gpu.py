"""Randomised whole-plan parity: bimg option combinations the planner accepts,
executed by libmipx on the GPU and by the oracle (ref_execute) on the same
seeded images, must agree bit for bit.  Covers op sequences no hand-written
case lists (rotate + shrink + reduce + embed + blur + flatten + B_W ...)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
# MIPX_FUZZ_SEEDS widens the run (e.g. 400 for a long soak on the GPU box)
SEEDS = int(os.environ.get("MIPX_FUZZ_SEEDS", "24"))


def random_case(r):
    w, h = int(r.integers(8, 420)), int(r.integers(8, 420))
    b = int(r.choice([1, 2, 3, 4]))
    opts = dict(width=int(r.choice([0, r.integers(4, 600)])), height=int(r.choice([0, r.integers(4, 600)])),
                crop=int(r.integers(0, 2)), embed=int(r.integers(0, 2)), force=int(r.integers(0, 2)),
                enlarge=int(r.integers(0, 2)), gravity=int(r.integers(0, 5)), extend=int(r.integers(0, 7)),
                rotate=int(r.choice([0, 0, 90, 180, 270])), flip=int(r.integers(0, 2)), flop=int(r.integers(0, 2)),
                sigma=float(r.choice([0, 0, 0, 0.7, 1.2, 3.0, 5.0, 9.0])), zoom=int(r.choice([0, 0, 0, 0, 1])),
                interpretation=int(r.choice([0, 0, 26])),
                background=[int(v) for v in r.choice([[0, 0, 0], [240, 30, 7]])])
    if opts["zoom"]:
        opts.update(width=0, height=0)
    orient = int(r.integers(0, 9))
    return w, h, b, opts, orient


@pytest.mark.parametrize("seed", range(SEEDS))
def test_random_plans_match_oracle(gpu, oracle, seed):
    r = np.random.default_rng(1000 + seed)
    ran = 0
    for _ in range(40):
        w, h, b, opts, orient = random_case(r)
        try:
            p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(w, h, b, "png", orient))
        except gpu.MipxError:
            continue
        if p.out_w * p.out_h > 4_000_000:
            continue
        e, rp = oracle.plan(opts, dict(w=w, h=h, bands=b, type=3, orientation=orient))
        assert e == 0
        imgs = r.integers(0, 256, (2, h, w, b), dtype=np.uint8)
        got = gpu.execute(p, imgs)
        for i in range(2):
            want = oracle.execute(rp, imgs[i])
            if not np.array_equal(got[i], want):
                d = np.argwhere(got[i] != want)
                raise AssertionError(f"{opts} {w}x{h}x{b} o{orient} {p.describe()}: {len(d)} bytes differ at {d[0]}")
        ran += 1
    assert ran >= 15
