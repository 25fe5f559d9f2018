"""k_rstrip (fused streaming Lanczos3 reduce, any shrink pair) against the
oracle: every band count, aligned and skewed rows (odd widths), every strip
width, edge strips, windows (reduce -> extract), the config shapes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = [  # h, w, b, hs, vs
    (270, 480, 3, 1.6, 1.6), (101, 131, 4, 4 / 3, 4 / 3), (300, 200, 3, 2.4666666666666666, 2.4666666666666666),
    (60, 90, 3, 3.7, 1.2), (375, 500, 3, 1.46484375, 1.46484375), (273, 364, 3, 1.421875, 1.06640625),
    (77, 301, 1, 1.33, 2.9), (29, 31, 2, 1.25, 1.6), (41, 43, 3, 1.7, 1.7), (128, 96, 3, 7.3, 7.3),
    (1080, 1920, 3, 2.4, 2.4), (9, 13, 4, 1.1, 1.9), (333, 1001, 4, 2.5, 1.01),
]


@pytest.mark.parametrize("tw", ["", "64", "128", "256"])
@pytest.mark.parametrize("h,w,b,hs,vs", CASES)
def test_rstrip_matches_oracle(gpu, oracle, monkeypatch, h, w, b, hs, vs, tw):
    monkeypatch.setenv("MIPX_RSTRIP", "1")
    monkeypatch.setenv("MIPX_RSTRIP_TW", tw)
    rng = np.random.default_rng(h * 7 + w)
    imgs = rng.integers(0, 256, (3, h, w, b), dtype=np.uint8)
    got = gpu.run_op("reduce", imgs, hshrink=hs, vshrink=vs)
    for i in range(3):
        want = oracle.reduce(imgs[i], hs, vs)
        assert got[i].shape == want.shape
        if not np.array_equal(got[i], want):
            d = np.argwhere(got[i] != want)
            raise AssertionError(f"{len(d)} bytes differ, first {d[0].tolist()}")


@pytest.mark.parametrize("band", ["4", "8", "64"])
def test_rstrip_bands(gpu, oracle, monkeypatch, band):
    monkeypatch.setenv("MIPX_RSTRIP_BAND", band)
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (1, 203, 301, 3), dtype=np.uint8)
    got = gpu.run_op("reduce", img, hshrink=1.6, vshrink=2.2)[0]
    assert np.array_equal(got, oracle.reduce(img[0], 1.6, 2.2))


@pytest.mark.parametrize("opts,hdr", [
    (dict(width=300, height=200, crop=1), (640, 480, 3)),
    (dict(width=251, height=99, crop=1, gravity=3), (1001, 333, 3)),
    (dict(width=768, height=512, crop=1), (1024, 1024, 4)),
    (dict(width=97, height=61, crop=1), (301, 203, 4)),
])
def test_rstrip_window_plans(gpu, oracle, opts, hdr):
    """reduce -> extract (the window reduce) runs k_rstrip over the window."""
    w, h, b = hdr
    p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(w, h, b, "png"))
    e, rp = oracle.plan(opts, dict(w=w, h=h, bands=b, type=3))
    assert e == 0
    imgs = np.random.default_rng(9).integers(0, 256, (2, h, w, b), dtype=np.uint8)
    got = gpu.execute(p, imgs)
    for i in range(2):
        assert np.array_equal(got[i], oracle.execute(rp, imgs[i])), p.describe()
