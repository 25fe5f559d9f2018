"""The oracle itself (CPU, no GPU): pinned against the committed golden vectors
and the known-answer facts of the restated libvips tables, plus the structural
identities the ops must satisfy.  Pixel values remain "parity unpinned" against
real libvips (none exists here); these checks pin the restatement."""
import numpy as np
import pytest

from conftest import load_golden


def test_golden_ops_reproduced(oracle):
    g = load_golden("ops.npz")
    n = 0
    for key in g.files:
        if not key.endswith("__in"):
            continue
        name = key[:-4]
        src, want = g[key], g[name + "__out"]
        op, *args = name.split("__")
        if op == "reduce":
            got = oracle.reduce(src, float(args[0]), float(args[1]))
        elif op == "shrink":
            got = oracle.shrink(src, int(args[0]), int(args[1]))
        elif op == "blur":
            got = oracle.gaussblur(src, float(args[0]))
        else:
            continue
        assert np.array_equal(got, want), name
        n += 1
    assert n >= 8


def test_golden_smartcrop_reproduced(oracle):
    g = load_golden("smartcrop.npz")
    assert oracle.smartcrop_origin(g["smart_quarter"], 100, 100) == tuple(g["smart_quarter_100x100"])
    assert oracle.smartcrop_origin(g["large_crop"], 64, 64) == tuple(g["large_crop_64x64"])


def test_gaussmat_sigma5_known_answer(oracle):
    """vips_gaussmat(5, 0.2, integer): 17 taps, rint(20 exp(-x^2/50)), scale = sum."""
    mask, scale = oracle.gaussmat(5.0)
    assert mask == [6, 8, 10, 12, 15, 17, 18, 20, 20, 20, 18, 17, 15, 12, 10, 8, 6]
    assert scale == 232
    assert np.array_equal(load_golden("tables.npz")["gauss_5_0"], mask)


def test_reduce_table_shrink2_known_answer(oracle):
    """Lanczos3 at shrink 2, phase 0: 13 taps, zeros at the odd integer lobe
    positions, symmetric, truncated to 12 bits (sum 4093, not 4096)."""
    t = oracle.reduce_table(2.0)
    assert t.shape == (129, 13)
    assert t[0].tolist() == [49, 0, -277, 0, 1248, 2053, 1248, 0, -277, 0, 49, 0, 0]
    assert t[0].sum() == 4093
    assert np.array_equal(load_golden("tables.npz")["reduce_2_0"], t)
    # every phase stays normalised within truncation error
    assert np.all(np.abs(t.sum(1) - 4096) <= 13)
    # phase 64 (x = 0.5): every output of a shrink-2 reduce under the centre sampling
    # convention; 12 non-zero taps symmetric about 5.5, tap 12 (at 3.25) zero
    assert t[64].tolist() == [15, 61, -139, -272, 555, 1828, 1828, 555, -272, -139, 61, 15, 0]
    assert t[64].sum() == 4096


@pytest.mark.parametrize("s,n", [(1.6, 11), (2.0, 13), (2.4666, 15), (1.3333, 9), (8.0, 49)])
def test_reduce_points(oracle, s, n):
    assert oracle.lib().ref_reduce_points(s) == n


def test_reduce_constant_image_is_stable(oracle):
    """A flat image stays flat (up to the 4093/4096 truncation of libvips' taps)."""
    for v in (0, 1, 128, 254, 255):
        img = np.full((50, 70, 3), v, np.uint8)
        out = oracle.reduce(img, 1.6, 1.6)
        assert out.shape == (31, 44, 3)
        assert np.all(np.abs(out.astype(int) - v) <= 1)


def test_geometry_identities(oracle, rng):
    img = rng.integers(0, 256, (21, 34, 3), dtype=np.uint8)
    assert np.array_equal(oracle.rot(oracle.rot(img, 90), 270), img)
    assert np.array_equal(oracle.rot(img, 180), oracle.flip(oracle.flip(img, 0), 1))
    assert np.array_equal(oracle.flip(oracle.flip(img, 1), 1), img)
    e = oracle.embed(img, 5, 7, 60, 40, 0)
    assert np.array_equal(oracle.extract(e, 5, 7, 34, 21), img)
    assert e[:7].max() == 0 and e[:, :5].max() == 0
    w = oracle.embed(img, 5, 7, 60, 40, 4)
    assert w[:7].min() == 255
    c = oracle.embed(img, -3, -2, 40, 30, 1)
    assert np.array_equal(c[0, 0], img[2, 3]) and np.array_equal(c[-1, -1], img[-1, -1])
    r = oracle.embed(img, 0, 0, 68, 42, 2)
    assert np.array_equal(r[21:, 34:], img)
    m = oracle.embed(img, 0, 0, 68, 21, 3)
    assert np.array_equal(m[:, 34:], img[:, ::-1])


def test_shrink_is_two_stage_rounded_mean(oracle, rng):
    img = rng.integers(0, 256, (8, 8, 1), dtype=np.uint8)
    out = oracle.shrink(img, 2, 2)
    col = (img.reshape(4, 2, 8).astype(int).sum(1) + 1) // 2           # shrinkv
    want = (col.reshape(4, 4, 2).sum(2) + 1) // 2                      # shrinkh
    assert np.array_equal(out[..., 0], want)


def test_watermark_blend_formula(oracle):
    base = np.full((4, 4, 3), 100, np.uint8)
    wm = np.zeros((2, 2, 4), np.uint8)
    wm[..., :3] = 200
    wm[..., 3] = 255
    out = oracle.watermark(base, wm, 1, 1, 0.5)
    assert out.shape == (4, 4, 4)
    m = int(255 * 0.5)  # 127: vips_cast truncates
    want_in = (m * 200 + (255 - m) * 100 + 128) // 255
    assert out[1, 1, 0] == want_in and out[0, 0, 0] == 100 and out[0, 0, 3] == 255
    assert out[1, 1, 3] == (m * 255 + (255 - m) * 255 + 128) // 255


def test_blur_preserves_flat_and_is_separable_order(oracle, rng):
    img = np.full((30, 30, 4), 77, np.uint8)
    assert np.array_equal(oracle.gaussblur(img, 5.0), img)
    x = rng.integers(0, 256, (30, 40, 3), dtype=np.uint8)
    y = oracle.gaussblur(x, 2.0)
    assert y.shape == x.shape and y.std() < x.std()


def test_cpu_baseline_batch_matches_single(oracle, rng):
    imgs = [rng.integers(0, 256, (48, 64, 3), dtype=np.uint8) for _ in range(5)]
    outs = oracle.reduce_batch(imgs, 2.0, 2.0, 3)
    for a, b in zip(imgs, outs):
        assert np.array_equal(oracle.reduce(a, 2.0, 2.0), b)


@pytest.mark.parametrize("h,w,b,hs,vs", [(216, 384, 3, 2.0, 2.0), (270, 480, 3, 1.6, 1.5976331360946747),
                                         (101, 131, 4, 4 / 3, 4 / 3), (37, 53, 1, 2.4, 1.0), (29, 31, 2, 1.0, 1.7),
                                         (9, 7, 3, 3.7, 2.9), (64, 300, 4, 14.2, 1.3)])
@pytest.mark.parametrize("centre", [0, 1])
def test_fast_cpu_baseline_is_the_oracle(oracle, h, w, b, hs, vs, centre):
    """bench.py times vips_fast.c as the CPU baseline; it must compute exactly the
    oracle's reduce (interior, clamped edges, one-axis and tiny images) under both
    sampling conventions (PARITY_ASSUMPTIONS.md row 1)."""
    prev = oracle.get_switch("reduce_centre")
    oracle.set_switch("reduce_centre", centre)
    try:
        _fast_vs_oracle(oracle, h, w, b, hs, vs)
    finally:
        oracle.set_switch("reduce_centre", prev)


def _fast_vs_oracle(oracle, h, w, b, hs, vs):
    rng = np.random.default_rng(h * w + b)
    img = rng.integers(0, 256, (h, w, b), dtype=np.uint8)
    assert np.array_equal(oracle.reduce_fast(img, hs, vs), oracle.reduce(img, hs, vs))
    outs = oracle.reduce_fast_batch([img, img[::-1].copy()], hs, vs, 2)
    assert np.array_equal(outs[1], oracle.reduce(img[::-1].copy(), hs, vs))
