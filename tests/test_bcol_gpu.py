"""k_bcol, the column-walking gaussblur (both convsep passes on the i8 matrix cores,
input rows staged once per segment, a ring of filtered rows, 16-byte row-piece
stores), against the oracle: RGB and RGBA, sigma from 0.3 to 8 (masks of 3 to 33
taps: one to three horizontal K steps, 32- and 64-row rings), images narrower than a
strip and shorter than a step, strips at both window edges, segment boundaries in
tall images, windows (resize -> crop -> blur) at every gravity, output rows that are
not a multiple of 16 bytes.  Every case also through the kernels behind it
(MIPX_BCOL=0: k_blur2d, then the separable passes)."""
import numpy as np
import pytest

from test_parity_gpu import assert_same, rand_img, smooth_img

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["bcol", "bcol192", "bcol192_dw", "nobcol"])
def route(request, monkeypatch):
    """k_bcol (the default: 256-byte strips, RGB ones starting mid-pixel, 16-byte-aligned
    horizontal operands), RGB on 64-pixel strips (MIPX_BCOL_RGB192=1), the same with the
    dword-aligned operands (+ MIPX_BCOL_A16=0; RGBA too) and the kernels behind it
    (MIPX_BCOL=0: k_blur2d, then the separable passes)."""
    monkeypatch.setenv("MIPX_BCOL", "0" if request.param == "nobcol" else "")
    monkeypatch.setenv("MIPX_BCOL_RGB192", "1" if request.param.startswith("bcol192") else "")
    monkeypatch.setenv("MIPX_BCOL_A16", "0" if request.param == "bcol192_dw" else "")
    yield request.param


SHAPES = [(64, 76, 3), (130, 516, 3), (9, 600, 4), (50, 260, 4), (3, 8, 4), (33, 20, 3), (17, 132, 3), (200, 388, 4),
          (47, 140, 3), (95, 300, 4), (300, 64, 3), (1, 128, 4), (700, 96, 3), (37, 1028, 3), (20, 88, 3), (19, 84, 3),
          (40, 172, 3), (12, 256, 3)]


@pytest.mark.parametrize("sigma", [0.3, 1.0, 2.2, 3.0, 5.0, 7.5])
def test_bcol_matches_oracle(gpu, oracle, rng, sigma):
    for h, w, b in SHAPES:
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b), rand_img(rng, h, w, b)])
        got = gpu.run_op("gaussblur", imgs, sigma=sigma, min_ampl=0.2)
        for i in range(len(imgs)):
            assert_same(got[i], oracle.gaussblur(imgs[i], sigma, 0.2), f"bcol {sigma} {h}x{w}x{b} img{i}")


@pytest.mark.parametrize("b", [3, 4])
@pytest.mark.parametrize("g", [0, 1, 2, 3, 4])
def test_bcol_windows(gpu, oracle, rng, b, g):
    """resize -> crop -> blur: the blur reads the crop window in place, its COPY edge at
    the window edge."""
    for sigma in (1.0, 5.0):
        opts = dict(width=300, height=200, crop=1, gravity=g, sigma=sigma)
        p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(1200, 700, b, "png"))
        e, rp = oracle.plan(opts, dict(w=1200, h=700, bands=b, type=3))
        assert e == 0
        imgs = rng.integers(0, 256, (2, 700, 1200, b), dtype=np.uint8)
        got = gpu.execute(p, imgs)
        for i in range(2):
            assert_same(got[i], oracle.execute(rp, imgs[i]), f"bcol window gravity {g} bands {b} sigma {sigma}")


def test_bcol_fuzz(gpu, oracle):
    r = np.random.default_rng(20261017)
    for case in range(40):
        b = int(r.choice([3, 4]))
        w = int(r.integers(1, 700))
        if b == 3:
            w = max(4, w & ~3)  # dword-aligned rows (k_bcol's domain; the rest leave it)
        h = int(r.integers(1, 400))
        sigma = float(r.uniform(0.3, 8.0))
        n = int(r.integers(1, 4))
        imgs = r.integers(0, 256, (n, h, w, b), dtype=np.uint8)
        got = gpu.run_op("gaussblur", imgs, sigma=sigma, min_ampl=0.2)
        for i in range(n):
            assert_same(got[i], oracle.gaussblur(imgs[i], sigma, 0.2), f"fuzz {case}: {h}x{w}x{b} sigma {sigma} img{i}")
