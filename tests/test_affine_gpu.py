"""vips_affine bicubic (bimg Enlarge, reference image.go:202-211) at multi-tile sizes:
the staged separable kernel (k_affine_sep, default) and the per-pixel gather kernel
(MIPX_AFFINE_SEP=0) against the oracle — interior tiles (dword staging) and border
tiles (extend mode per byte), every extend mode, unaligned output rows, scales below
1 and per-axis scales, RGB / RGBA / grey."""
import numpy as np
import pytest

from test_parity_gpu import assert_same, rand_img, smooth_img

pytestmark = pytest.mark.gpu

CASES = [  # h, w, b, xs, ys, extend
    (740, 550, 3, 2.0, 2.0, 1),             # C5-like Enlarge of imaginary.jpg's size
    (270, 480, 3, 1.5, 1.5, 1),
    (131, 257, 4, 3.3, 3.3, 0),
    (61, 403, 3, 1.2, 5.0, 3),
    (200, 300, 1, 2.5, 1.7, 2),
    (97, 203, 4, 1.75, 1.75, 4),
    (64, 640, 3, 2.0, 2.0, 5),
    (150, 150, 3, 0.8, 1.6, 1),
    (33, 1201, 2, 1.01, 1.3, 1),
]


@pytest.mark.parametrize("sep", ["1", "0"])
@pytest.mark.parametrize("h,w,b,xs,ys,extend", CASES)
def test_affine_tiles_match_oracle(gpu, oracle, rng, monkeypatch, sep, h, w, b, xs, ys, extend):
    monkeypatch.setenv("MIPX_AFFINE_SEP", sep)
    imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
    got = gpu.run_op("affine", imgs, xscale=xs, yscale=ys, extend=extend)
    for i in range(2):
        assert_same(got[i], oracle.affine(imgs[i], xs, ys, extend), f"affine sep={sep} {h}x{w}x{b} {xs}x{ys} e{extend} img{i}")


def test_enlarge_plans(gpu, oracle, rng):
    """Enlarge through whole plans (planner + affine), as image.go:202 builds them."""
    for (iw, ih, b, opts) in ((550, 740, 3, dict(width=1100, height=1480, enlarge=1)),
                              (400, 300, 4, dict(width=1000, enlarge=1)),
                              (640, 360, 3, dict(width=1920, height=1080, enlarge=1, crop=1))):
        p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(iw, ih, b, "png"))
        e, rp = oracle.plan(opts, dict(w=iw, h=ih, bands=b, type=3))
        assert e == 0
        imgs = rng.integers(0, 256, (2, ih, iw, b), dtype=np.uint8)
        got = gpu.execute(p, imgs)
        for i in range(2):
            assert_same(got[i], oracle.execute(rp, imgs[i]), f"enlarge plan {iw}x{ih}x{b} {opts}")


E2_CASES = [  # h, w, b, extend: exactly 2 x 2 on the VALU kernels at every band count and edge
    (740, 550, 3, 1), (33, 1201, 4, 0), (97, 203, 1, 2), (61, 130, 2, 3), (64, 640, 3, 4),
    (5, 7, 3, 5), (1, 1, 4, 1), (2, 3, 3, 0), (70, 129, 4, 1), (129, 128, 3, 3),
    # a 16-byte chunk ending exactly at the image's last byte with in_img % 4 != 0
    # (w = 14 mod 16 pixels for B = 1, odd h): its tail dword straddled the descriptor's range and read 0
    (1151, 1150, 3, 1), (31, 30, 1, 1), (31, 30, 1, 3),
]


@pytest.mark.parametrize("sep", ["1", "0"])
@pytest.mark.parametrize("h,w,b,extend", E2_CASES)
def test_enlarge2_matches_oracle(gpu, oracle, rng, monkeypatch, sep, h, w, b, extend):
    """vips_affine at exactly 2 x 2 with k_enlm off: k_affine_sep (MIPX_AFFINE_SEP=1) and the
    per-pixel k_affine (0), strips and bands that end at the image edges, images narrower
    than the 6-pixel window, every extend mode, all bands.  (r04's fixed-pattern
    k_enlarge2, shadowed by k_enlm since r05, was removed in r06.)"""
    monkeypatch.setenv("MIPX_ENLM", "0")
    monkeypatch.setenv("MIPX_AFFINE_SEP", sep)
    imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
    got = gpu.run_op("affine", imgs, xscale=2.0, yscale=2.0, extend=extend)
    for i in range(2):
        assert_same(got[i], oracle.affine(imgs[i], 2.0, 2.0, extend), f"enlarge sep={sep} {h}x{w}x{b} e{extend} img{i}")


@pytest.mark.parametrize("dbg", ["1", "2", "3", "4", "7"])
def test_enlm_probe_knob_is_compiled_out(gpu, oracle, rng, monkeypatch, dbg):
    """the timing probes (MIPX_ENLM_DBG: skip the staging loads / the
    stores, wrong pixels) exist only in a `make PROBES=1` library; the shipped one ignores
    the variable, so Enlarge stays oracle-exact whatever the environment says."""
    monkeypatch.setenv("MIPX_ENLM", "2")
    monkeypatch.setenv("MIPX_ENLM_DBG", dbg)
    img = np.stack([rand_img(rng, 61, 130, 3), smooth_img(rng, 61, 130, 3)])
    got = gpu.run_op("affine", img, xscale=2.0, yscale=2.0, extend=1)
    for i in range(2):
        assert_same(got[i], oracle.affine(img[i], 2.0, 2.0, 1), f"MIPX_ENLM_DBG={dbg} img{i}")


# k_enlm (both passes on the matrix cores): integer and fractional scales, per-axis mixes,
# every extend mode, every band count, ragged last column groups and bands, images smaller
# than a tile, the op-survey shapes
ENLM_SCALES = [(2.0, 2.0), (3.0, 3.0), (4.0, 4.0), (1.5, 1.5), (2.5, 2.5), (3.0, 2.0), (2.0, 4.0), (1.5, 3.0),
               (1.4, 1.4), (5.0, 5.0), (8.0, 8.0)]
ENLM_SHAPES = [(740, 550, 3, 1), (33, 1201, 4, 0), (97, 203, 1, 2), (61, 130, 2, 3), (64, 640, 3, 4),
               (5, 7, 3, 5), (1, 1, 4, 1), (2, 3, 3, 0), (70, 129, 4, 1), (129, 128, 3, 3), (31, 30, 1, 1),
               (1151, 1150, 3, 1)]


@pytest.mark.parametrize("xs,ys", ENLM_SCALES, ids=[f"{x}x{y}" for x, y in ENLM_SCALES])
def test_enlm_matches_oracle(gpu, oracle, rng, monkeypatch, xs, ys):
    monkeypatch.setenv("MIPX_ENLM", "2")  # k_enlm or an error, never a fallback
    for h, w, b, extend in ENLM_SHAPES:
        if h * w * xs * ys > 3e6:
            continue
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
        got = gpu.run_op("affine", imgs, xscale=xs, yscale=ys, extend=extend)
        for i in range(2):
            assert_same(got[i], oracle.affine(imgs[i], xs, ys, extend), f"enlm {h}x{w}x{b} {xs}x{ys} e{extend} img{i}")


def test_enlm_extremes(gpu, oracle, monkeypatch):
    """Saturating content (0 / 255 steps: the bicubic over- and undershoot, H outside
    0..255 before the vertical pass) at 2 x, 3 x and 1.5 x."""
    monkeypatch.setenv("MIPX_ENLM", "2")
    h, w = 90, 130
    y, x = np.mgrid[0:h, 0:w]
    for b in (1, 3, 4):
        chans = [(((x // 3 + y // 3) % 2) * 255), ((x % 2) * 255), ((y % 2) * 255), np.full((h, w), 255)]
        img = np.stack(chans[:b], -1).astype(np.uint8)
        for s in (2.0, 3.0, 1.5):
            got = gpu.run_op("affine", img[None], xscale=s, yscale=s, extend=1)
            assert_same(got[0], oracle.affine(img, s, s, 1), f"enlm extremes b{b} x{s}")


def test_enlm_declines_outside_its_tiles(gpu, rng, monkeypatch):
    """Scales below 1 or too close to 1 are outside k_enlm's tiles: with MIPX_ENLM=2 an
    error, by default the other kernels (checked against the oracle elsewhere)."""
    monkeypatch.setenv("MIPX_ENLM", "2")
    img = rng.integers(0, 256, (1, 40, 50, 3), dtype=np.uint8)
    for xs, ys in ((0.8, 2.0), (2.0, 1.0), (1.2, 1.1)):
        with pytest.raises(Exception):
            gpu.run_op("affine", img, xscale=xs, yscale=ys, extend=1)
