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


def random_jpeg_case(r):
    """A JPEG header large enough for shrink-on-load; the host codec's decoded size
    is ceil(w / s) (libjpeg DCT scaling) or one pixel less (another codec's rounding)."""
    w, h = int(r.integers(200, 2400)), int(r.integers(200, 2400))
    opts = dict(width=int(r.choice([0, r.integers(16, 400)])), height=int(r.choice([0, r.integers(16, 400)])),
                crop=int(r.integers(0, 2)), embed=int(r.integers(0, 2)), gravity=int(r.integers(0, 6)),
                extend=int(r.integers(0, 7)), rotate=int(r.choice([0, 0, 90, 180, 270])),
                flip=int(r.integers(0, 2)), sigma=float(r.choice([0, 0, 0, 1.2, 3.0])))
    if opts["width"] == 0 and opts["height"] == 0:
        opts["width"] = int(r.integers(16, 400))
    return w, h, opts, int(r.integers(0, 9)), int(r.choice([0, 0, 1]))


def _jpeg_plans(gpu, oracle, w, h, opts, orient, delta):
    p0 = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(w, h, 3, "jpeg", orient))
    s = p0.load_shrink
    if s == 1:
        delta = 0                      # no shrink-on-load: the codec decodes the header size
    dw, dh = max(1, -(-w // s) - delta), max(1, -(-h // s) - delta)
    p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(w, h, 3, "jpeg", orient, dw, dh))
    e, rp = oracle.plan(opts, dict(w=w, h=h, bands=3, type=1, orientation=orient, decoded_w=dw, decoded_h=dh))
    assert e == 0 and rp.load_shrink == s and (rp.in_w, rp.in_h) == (p.in_w, p.in_h) == (dw, dh)
    return p, rp


@pytest.mark.parametrize("seed", range(max(2, SEEDS // 4)))
def test_random_jpeg_shrink_on_load_plans(gpu, oracle, seed):
    """JPEG-typed plans: the planner picks the codec shrink-on-load, the engine runs
    the rest of the plan on the decoded-size image."""
    r = np.random.default_rng(5000 + seed)
    ran = sol = 0
    for _ in range(12):
        w, h, opts, orient, delta = random_jpeg_case(r)
        try:
            p, rp = _jpeg_plans(gpu, oracle, w, h, opts, orient, delta)
        except gpu.MipxError:
            continue
        img = r.integers(0, 256, (1, p.in_h, p.in_w, 3), dtype=np.uint8)
        got = gpu.execute(p, img)[0]
        want = oracle.execute(rp, img[0])
        if not np.array_equal(got, want):
            d = np.argwhere(got != want)
            raise AssertionError(f"{opts} {w}x{h} o{orient} sol{p.load_shrink} {p.describe()}: "
                                 f"{len(d)} bytes differ at {d[0]}")
        ran += 1
        sol += p.load_shrink > 1
    assert ran >= 6 and sol >= 3


@pytest.mark.parametrize("opts", [dict(width=300), dict(width=1280, height=720, crop=1, sigma=3.0),
                                  dict(width=800, height=800, embed=1, extend=3, rotate=90)])
def test_4k_jpeg_plan(gpu, oracle, opts):
    """A 4K JPEG header (3840x2160) through shrink-on-load + the rest of the plan."""
    p, rp = _jpeg_plans(gpu, oracle, 3840, 2160, opts, 0, 0)
    img = np.random.default_rng(4096).integers(0, 256, (1, p.in_h, p.in_w, 3), dtype=np.uint8)
    assert np.array_equal(gpu.execute(p, img)[0], oracle.execute(rp, img[0])), p.describe()
