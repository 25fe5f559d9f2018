"""vips_reduce 2 x 2 followed by a second vips_reduce (and its extract window): the
/pipeline resize -> crop chain of C3 (reference image.go:379-410).

The merged plan (mipx_plan_chain) of a 2 x 2 resize stage and a resize / crop stage runs
k_reduce2x2 / k_reduce2m (only the rows and columns the second reduce reads, plan_demand)
then k_rcol over the window; each case is checked against the oracle run stage by stage
(o.reduce twice, then the extract), under both sampling conventions.  (r05's one-launch
k_rchain, measured slower, was removed in r06: profiles/r05/c3_chain_ab.jsonl.)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# (w, h, bands, stage-2 opts): the C3 shape scaled down, full-output windows (rows above
# and below the 2 x 2 output: the COPY edge of the second reduce), crops at the gravities,
# narrow / short images, one strip and partial last strips, RGB and RGBA
CASES = [
    (512, 512, 4, dict(width=192, height=128, crop=1)),
    (512, 512, 3, dict(width=192, height=128, crop=1)),
    (600, 400, 4, dict(width=225, height=150, embed=1)),     # 2 x 2 -> 300x200 -> 1.333: whole output
    (600, 400, 3, dict(width=225, height=150, embed=1)),
    (1000, 752, 4, dict(width=300, height=200, crop=1, gravity=1)),
    (1000, 752, 4, dict(width=300, height=200, crop=1, gravity=3)),
    (1000, 752, 3, dict(width=300, height=200, crop=1, gravity=2)),
    (1000, 752, 3, dict(width=300, height=200, crop=1, gravity=4)),
    (132, 90, 4, dict(width=40, height=27, embed=1)),        # 66x45 -> 40x27: one strip
    (132, 90, 3, dict(width=40, height=27, embed=1)),
    (200, 40, 4, dict(width=60, height=12, embed=1)),        # fewer 2 x 2 rows than a front step
    (2048, 2048, 4, dict(width=768, height=512, crop=1)),    # C3's own geometry
    (1540, 300, 3, dict(width=481, height=94, embed=1)),     # shrink 1.6: 16 taps
]


def _chain_plan(gpu, w, h, b, opts2):
    p1 = gpu.plan_make(gpu.make_opts(width=w // 2, embed=1), gpu.make_input(w, h, b, "png"))
    assert [s[0] for s in p1.describe()] == ["reduce"] and p1.describe()[0][2][:2] == (2.0, 2.0), p1.describe()
    p2 = gpu.plan_make(gpu.make_opts(**opts2), gpu.make_input(p1.out_w, p1.out_h, b, "png"))
    assert p2.describe()[0][0] == "reduce", p2.describe()
    return p1, p2, gpu.plan_chain([p1, p2])


def _oracle(oracle, p1, p2, px):
    d1 = p1.describe()[0][2]
    mid = oracle.reduce(px, d1[0], d1[1])
    out = mid
    for op, a, d, _ in p2.describe():
        if op == "reduce":
            out = oracle.reduce(out, d[0], d[1])
        elif op == "extract":
            out = out[a[1]:a[1] + a[3], a[0]:a[0] + a[2]]
        else:
            raise AssertionError(op)
    return np.ascontiguousarray(out)


@pytest.mark.parametrize("w,h,b,opts2", CASES, ids=[f"{c[0]}x{c[1]}x{c[2]}-{i}" for i, c in enumerate(CASES)])
def test_chain_matches_oracle(gpu, oracle, convention, w, h, b, opts2):
    r = np.random.default_rng(w * 7 + h * 3 + b)
    px = r.integers(0, 256, (2, h, w, b), dtype=np.uint8)
    p1, p2, plan = _chain_plan(gpu, w, h, b, opts2)
    got = gpu.execute(plan, px, junk=0xA5)
    for i in range(2):
        want = _oracle(oracle, p1, p2, px[i])
        assert got[i].shape == want.shape
        d = np.argwhere(got[i] != want)
        assert len(d) == 0, f"{convention} {w}x{h}x{b} {opts2}: {len(d)} bytes differ, first at {d[0]}"


def test_chain_smooth_images_and_extremes(gpu, oracle, convention):
    """Saturating inputs (0 / 255 blocks, ramps) through both products' rounding and clamping."""
    h, w, b = 300, 420, 4
    y, x = np.mgrid[0:h, 0:w]
    px = np.stack([((x * 255) // (w - 1)).astype(np.uint8), ((y // 7) % 2 * 255).astype(np.uint8),
                   (((x // 5 + y // 5) % 2) * 255).astype(np.uint8), np.full((h, w), 255, np.uint8)], -1)
    p1, p2, plan = _chain_plan(gpu, w, h, b, dict(width=150, height=100, crop=1))
    got = gpu.execute(plan, px[None])
    assert np.array_equal(got[0], _oracle(oracle, p1, p2, px))


# ------------------------------------------------- the default 2 x 2 kernels at edge shapes
R2D_SHAPES = ((270, 480, 3), (130, 260, 4), (37, 52, 3), (61, 1000, 4), (200, 648, 3), (8, 8, 4), (9, 12, 3),
              (25, 164, 3), (131, 1000, 4), (1081, 324, 3), (16, 3840, 3), (47, 226, 4), (2160, 3840, 3))


def test_reduce2x2_edge_shapes_exact(gpu, oracle, convention):
    """k_reduce2x2 / k_reduce2m (the generic reduce where rows are off a dword) at both
    conventions: strips ending at the image edges, images shorter than a step, widths
    past one strip, full 4K (r05's shapes for the removed ring-less k_reduce2d)."""
    r = np.random.default_rng(11)
    for h, w, b in R2D_SHAPES:
        imgs = r.integers(0, 256, (2, h, w, b), dtype=np.uint8)
        got = gpu.run_op("reduce", imgs, hshrink=2.0, vshrink=2.0)
        for i in range(2):
            want = oracle.reduce(imgs[i], 2.0, 2.0)
            d = np.argwhere(got[i] != want)
            assert len(d) == 0, f"{convention} {h}x{w}x{b} img{i}: {len(d)} differ, first {d[0]}"


def test_reduce2x2_windows(gpu, oracle, convention):
    """The 2 x 2 kernels computing only a reduce's demanded region (reduce -> crop plans)."""
    r = np.random.default_rng(12)
    for (w, h, b), (left, top, cw, ch) in (((1200, 800, 3), (150, 100, 300, 200)), ((1200, 800, 4), (0, 280, 500, 120)),
                                           ((640, 960, 3), (0, 0, 320, 100)), ((640, 960, 4), (219, 0, 100, 480))):
        px = r.integers(0, 256, (1, h, w, b), dtype=np.uint8)
        opts = dict(width=w // 2, height=h // 2, embed=1)
        p1 = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(w, h, b, "png"))
        p2 = gpu.plan_make(gpu.make_opts(left=left, top=top, area_width=cw, area_height=ch),
                           gpu.make_input(p1.out_w, p1.out_h, b, "png"))
        plan = gpu.plan_chain([p1, p2])
        got = gpu.execute(plan, px)[0]
        mid = oracle.reduce(px[0], 2.0, 2.0)
        (op, a, _d, _o), = p2.describe()
        assert op == "extract"
        want = mid[a[1]:a[1] + a[3], a[0]:a[0] + a[2]]
        assert np.array_equal(got, want), (w, h, b, left, top, cw, ch)
