"""GPU parity: every libmipx kernel against the CPU oracle on the same seeded
inputs, through the C-ABI.  The bar is BIT-EXACT for every op (the integer
libvips C paths are reproduced exactly; the north star's ±1 LSB allowance for
resize/blur/composite covers libvips' ORC vector paths, which the oracle does
not model — see PARITY_ASSUMPTIONS.md)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def rand_img(rng, h, w, b):
    return rng.integers(0, 256, (h, w, b), dtype=np.uint8)


def smooth_img(rng, h, w, b):
    """Band-limited content (exercises mid-range sums rather than noise)."""
    y, x = np.mgrid[0:h, 0:w]
    out = np.empty((h, w, b), np.uint8)
    for c in range(b):
        f = rng.uniform(0.01, 0.2, 2)
        out[..., c] = (127.5 + 127.5 * np.sin(x * f[0] + c) * np.cos(y * f[1] - c)).astype(np.uint8)
    return out


def assert_same(got, want, what=""):
    got = np.asarray(got)
    want = np.asarray(want)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    if not np.array_equal(got, want):
        d = np.argwhere(got != want)
        raise AssertionError(f"{what}: {len(d)} bytes differ, first at {d[0].tolist()} "
                             f"got {got[tuple(d[0])]} want {want[tuple(d[0])]}")


# ---------------------------------------------------------------- Lanczos3 reduce
REDUCE_CASES = [
    # (h, w, bands, hshrink, vshrink) — the first group takes the fused 2x2 kernel
    (64, 64, 3, 2.0, 2.0), (270, 480, 3, 2.0, 2.0), (37, 52, 3, 2.0, 2.0), (130, 260, 4, 2.0, 2.0),
    (9, 12, 3, 2.0, 2.0), (100, 300, 4, 2.0, 2.0),
    # generic path
    (64, 65, 3, 2.0, 2.0), (50, 77, 1, 2.0, 2.0), (40, 40, 2, 2.0, 2.0),
    (270, 480, 3, 1.6, 1.6), (300, 200, 3, 2.4666666666666666, 2.4666666666666666),
    (101, 131, 4, 1.3333333333333333, 1.3333333333333333), (60, 90, 3, 3.7, 1.2), (33, 17, 3, 1.0, 2.5),
    (64, 64, 3, 2.5, 1.0), (128, 96, 3, 7.3, 7.3),
    # large shrink: the horizontal pass falls back from LDS staging to gathers
    (300, 420, 3, 14.2, 14.2), (90, 700, 4, 20.0, 3.0),
]


@pytest.mark.parametrize("h,w,b,hs,vs", REDUCE_CASES)
def test_reduce_matches_oracle(gpu, oracle, rng, convention, h, w, b, hs, vs):
    imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
    got = gpu.run_op("reduce", imgs, hshrink=hs, vshrink=vs)
    for i in range(len(imgs)):
        assert_same(got[i], oracle.reduce(imgs[i], hs, vs), f"reduce {h}x{w}x{b} {hs}x{vs} img{i}")


@pytest.mark.parametrize("h,w,b,hs,vs", [(41, 43, 3, 1.7, 1.7), (29, 31, 2, 1.25, 1.6), (77, 301, 1, 1.33, 2.9),
                                         (240, 427, 3, 1.4233, 1.4233), (61, 97, 4, 3.1, 1.1)])
def test_reduce_unaligned_batches(gpu, oracle, rng, h, w, b, hs, vs):
    """Batches of odd-sized images: every image after the first starts at an
    unaligned address, rows have odd pitches (the any-alignment DMA paths)."""
    imgs = np.stack([rand_img(rng, h, w, b) for _ in range(3)])
    got = gpu.run_op("reduce", imgs, hshrink=hs, vshrink=vs)
    for i in range(3):
        assert_same(got[i], oracle.reduce(imgs[i], hs, vs), f"reduce {h}x{w}x{b} img{i}")
    blur = gpu.run_op("gaussblur", imgs, sigma=1.7, min_ampl=0.2)
    for i in range(3):
        assert_same(blur[i], oracle.gaussblur(imgs[i], 1.7, 0.2), f"blur {h}x{w}x{b} img{i}")


@pytest.mark.parametrize("band", ["", "1", "16"])
def test_reduce2x2_variants_exact(gpu, oracle, rng, convention, band, monkeypatch):
    """The fused 2x2 kernels (corner: k_reduce2x2 variant 66, the r01/r02 A/B builds are
    recorded under profiles/ and no longer compiled; centre: k_reduce2m, both passes on
    the matrix cores, at its default band and at 1 / 16 steps per band) are bit-exact,
    including strips that end at the image edge, images shorter than a band and the
    smallest eligible sizes."""
    monkeypatch.setenv("MIPX_R2M_BAND", band)
    for h, w, b in ((270, 480, 3), (130, 260, 4), (37, 52, 3), (61, 1001 * 4 // 4 - 1, 4), (200, 646, 3),
                    (8, 8, 4), (9, 12, 3), (25, 164, 3), (131, 1000, 4), (1081, 324, 3), (16, 3840, 3)):
        if (w * b) % 4:
            continue
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
        got = gpu.run_op("reduce", imgs, hshrink=2.0, vshrink=2.0)
        for i in range(2):
            assert_same(got[i], oracle.reduce(imgs[i], 2.0, 2.0), f"{convention} band={band} {h}x{w}x{b} img{i}")


@pytest.mark.parametrize("fused", ["0", "1"])
def test_reduce_fused_and_two_pass_paths(gpu, oracle, rng, fused, monkeypatch):
    """Both generic reduce paths (one fused launch / two DMA-staged passes) on the
    same shapes, including output windows (reduce -> extract plans).  "0" turns
    the small-image fused kernel off."""
    monkeypatch.setenv("MIPX_FUSED_REDUCE", fused)
    monkeypatch.setenv("MIPX_RCOL", "0")   # k_rcol and k_rmf2 have their own tests
    monkeypatch.setenv("MIPX_RMFMA", "0")
    for h, w, b, hs, vs in ((240, 427, 3, 1.4233, 1.4233), (273, 364, 3, 1.421875, 1.06640625),
                            (97, 130, 4, 1.3333333333333333, 1.3333333333333333), (45, 61, 1, 2.9, 1.7),
                            (60, 90, 2, 1.05, 3.3), (300, 200, 3, 2.4666666666666666, 2.4666666666666666)):
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
        got = gpu.run_op("reduce", imgs, hshrink=hs, vshrink=vs)
        for i in range(2):
            assert_same(got[i], oracle.reduce(imgs[i], hs, vs), f"fused={fused} {h}x{w}x{b} {hs}x{vs}")
    opts = dict(width=251, height=99, crop=1, gravity=3)
    p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(401, 333, 3, "png"))
    e, rp = oracle.plan(opts, dict(w=401, h=333, bands=3, type=3))
    img = rand_img(rng, 333, 401, 3)
    assert_same(gpu.execute(p, img)[0], oracle.execute(rp, img), f"fused={fused} window plan")


@pytest.mark.parametrize("h,w,b,s", [(50, 60, 3, 1.6), (31, 45, 4, 2.0), (20, 33, 1, 3.3)])
def test_reducev_reduceh_separately(gpu, oracle, rng, h, w, b, s):
    img = rand_img(rng, h, w, b)
    assert_same(gpu.run_op("reducev", img, vshrink=s)[0], oracle.reducev(img, s), "reducev")
    assert_same(gpu.run_op("reduceh", img, hshrink=s)[0], oracle.reduceh(img, s), "reduceh")


def test_reduce_extremes(gpu, oracle):
    """All-0 / all-255 / checkerboard: clip paths and negative lobes."""
    h, w = 40, 64
    cases = [np.zeros((h, w, 3), np.uint8), np.full((h, w, 3), 255, np.uint8),
             ((np.indices((h, w)).sum(0) % 2) * 255).astype(np.uint8)[..., None].repeat(3, 2)]
    for img in cases:
        for s in (2.0, 1.6):
            assert_same(gpu.run_op("reduce", img, hshrink=s, vshrink=s)[0], oracle.reduce(img, s, s), f"reduce {s}")


@pytest.mark.slow
def test_reduce_4k_to_1080p_full_size(gpu, oracle, rng, convention):
    """BASELINE C2 geometry at full size (3840x2160x3 -> 1920x1080x3), bit-exact."""
    imgs = np.stack([rand_img(rng, 2160, 3840, 3), smooth_img(rng, 2160, 3840, 3)])
    got = gpu.run_op("reduce", imgs, hshrink=2.0, vshrink=2.0)
    for i in range(2):
        assert_same(got[i], oracle.reduce(imgs[i], 2.0, 2.0), f"4k img{i}")


# ---------------------------------------------------------------- box shrink
@pytest.mark.parametrize("h,w,b,hs,vs", [(64, 64, 3, 2, 2), (100, 75, 3, 8, 8), (31, 47, 4, 3, 5),
                                         (3000 // 10, 4000 // 10, 3, 11, 11), (9, 9, 1, 4, 4), (20, 20, 2, 1, 3),
                                         (37, 1001, 3, 7, 3), (40, 3000, 4, 33, 2), (16, 4096, 1, 200, 8)])
def test_shrink_matches_oracle(gpu, oracle, rng, h, w, b, hs, vs):
    img = rand_img(rng, h, w, b)
    assert_same(gpu.run_op("shrink", img, hshrink=hs, vshrink=vs)[0], oracle.shrink(img, hs, vs), "shrink")


# ---------------------------------------------------------------- geometry (bit-exact by definition)
@pytest.mark.parametrize("extend", range(7))
@pytest.mark.parametrize("x,y,W,H", [(10, 5, 100, 60), (-7, -3, 40, 30), (0, 0, 64, 48), (30, 40, 50, 50),
                                     (-100, 60, 300, 200)])
def test_embed_matches_oracle(gpu, oracle, rng, extend, x, y, W, H):
    for b in (3, 4):
        img = rand_img(rng, 48, 64, b)
        got = gpu.run_op("embed", img, x=x, y=y, width=W, height=H, extend=extend, background=(12, 200, 77))
        assert_same(got[0], oracle.embed(img, x, y, W, H, extend, (12, 200, 77)), f"embed mode {extend} b{b}")


@pytest.mark.parametrize("b", [1, 2, 3])
@pytest.mark.parametrize("extend", [0, 1, 2, 3, 5])
def test_embed_odd_sizes_all_bands(gpu, oracle, rng, b, extend):
    """Row embed kernel: unaligned pixel offsets, odd row lengths, 1-3 bands."""
    img = rand_img(rng, 37, 53, b)
    for x, y, W, H in ((3, 2, 61, 40), (-5, -7, 33, 29), (0, 5, 53, 47), (13, 0, 101, 37), (-60, -40, 71, 45)):
        got = gpu.run_op("embed", img, x=x, y=y, width=W, height=H, extend=extend, background=(9, 250, 31))
        assert_same(got[0], oracle.embed(img, x, y, W, H, extend, (9, 250, 31)), f"embed {x},{y} {W}x{H} b{b}")


@pytest.mark.parametrize("ver", ["0", "1", "2"])
def test_embed_and_flip_row_kernels(gpu, oracle, rng, monkeypatch, ver):
    """The embed row kernels (MIPX_EMBED_V: 0 one row at a time, 1 every row of the block
    fetched first, 2 the same with non-temporal stores) and flip / rot 180 with plain or
    non-temporal stores (MIPX_FLIP_NT), on batches with ragged row blocks, every extend mode."""
    monkeypatch.setenv("MIPX_EMBED_V", ver)
    monkeypatch.setenv("MIPX_FLIP_NT", "1" if ver == "2" else "0")
    for h, w, b in ((37, 53, 3), (64, 96, 4), (130, 1100, 3), (7, 2000, 1)):
        imgs = np.stack([rand_img(rng, h, w, b) for _ in range(2)])
        for ext in range(6):
            W, H = w + 37, h + 6
            got = gpu.run_op("embed", imgs, x=17, y=3, width=W, height=H, extend=ext, background=(9, 250, 31))
            for i in range(2):
                assert_same(got[i], oracle.embed(imgs[i], 17, 3, W, H, ext, (9, 250, 31)), f"embed {ext} {h}x{w}x{b}")
        for v in (0, 1):
            got = gpu.run_op("flip", imgs, vertical=v)
            for i in range(2):
                assert_same(got[i], oracle.flip(imgs[i], v), f"flip{v} {h}x{w}x{b}")
        got = gpu.run_op("rot", imgs, angle=180)
        for i in range(2):
            assert_same(got[i], oracle.rot(imgs[i], 180), f"rot180 {h}x{w}x{b}")


@pytest.mark.parametrize("b", [1, 2, 3, 4])
def test_extract_rot_flip(gpu, oracle, rng, b):
    img = rand_img(rng, 37, 53, b)
    assert_same(gpu.run_op("extract", img, left=5, top=7, width=31, height=20)[0],
                oracle.extract(img, 5, 7, 31, 20), "extract")
    for a in (0, 90, 180, 270):
        assert_same(gpu.run_op("rot", img, angle=a)[0], oracle.rot(img, a), f"rot{a}")
    for v in (0, 1):
        assert_same(gpu.run_op("flip", img, vertical=v)[0], oracle.flip(img, v), f"flip{v}")
    r = img
    for _ in range(4):
        r = gpu.run_op("rot", r, angle=90)[0]
    assert_same(r, img, "rot90^4 == identity")


@pytest.mark.parametrize("nt", ["0", "1"])
@pytest.mark.parametrize("b", [1, 2, 3, 4])
def test_extract_batches_any_alignment(gpu, oracle, rng, monkeypatch, b, nt):
    """Extract over batches of odd-size images (later images start unaligned) and odd
    windows: the dword copy, the embed-interior path and the per-pixel remap, with plain
    and non-temporal row stores (MIPX_EXTRACT_NT)."""
    monkeypatch.setenv("MIPX_EXTRACT_NT", nt)
    for h, w, left, top, ow, oh in ((37, 53, 5, 7, 31, 20), (40, 64, 4, 3, 32, 16), (29, 301, 101, 2, 157, 25)):
        imgs = np.stack([rand_img(rng, h, w, b) for _ in range(3)])
        got = gpu.run_op("extract", imgs, left=left, top=top, width=ow, height=oh)
        for i in range(3):
            assert_same(got[i], oracle.extract(imgs[i], left, top, ow, oh), f"extract {h}x{w}x{b} img{i}")


@pytest.mark.parametrize("h,w,b", [(33, 65, 3), (64, 96, 4), (100, 31, 1), (70, 71, 2), (128, 256, 4)])
def test_rot_tiles_and_aligned_extract(gpu, oracle, rng, h, w, b):
    img = rand_img(rng, h, w, b)
    for a in (90, 180, 270):
        assert_same(gpu.run_op("rot", img, angle=a)[0], oracle.rot(img, a), f"rot{a} {h}x{w}x{b}")
    for left, top, ew, eh in ((4, 3, w - 8, h - 5), (0, 0, w, h), (w // 2, h // 3, w // 2, h // 2)):
        assert_same(gpu.run_op("extract", img, left=left, top=top, width=ew, height=eh)[0],
                    oracle.extract(img, left, top, ew, eh), f"extract {left},{top}")


@pytest.mark.parametrize("th,tc,order", [("64", "64", "0"), ("128", "64", "0"), ("64", "128", "0"), ("64", "64", "1"),
                                          ("64", "128", "1")])
@pytest.mark.parametrize("xcd", ["1", "0"])
def test_rot90_tile_orders(gpu, oracle, rng, monkeypatch, xcd, th, tc, order):
    """The LDS-tile rotation on its flat grid, XCD-contiguous (default for odd band counts) or x-fastest
    round robin (MIPX_ROT_XCD=0), 64 or 128 input rows per tile (MIPX_ROT_TH), 64 or 128
    input columns per tile (MIPX_ROT_T), tiles x- or y-fastest (MIPX_ROT_ORDER): a batch of
    3 with ragged edge tiles, every band count."""
    monkeypatch.setenv("MIPX_ROT_XCD", xcd)
    monkeypatch.setenv("MIPX_ROT_TH", th)
    monkeypatch.setenv("MIPX_ROT_T", tc)
    monkeypatch.setenv("MIPX_ROT_ORDER", order)
    for h, w, b in ((130, 197, 3), (65, 300, 4), (200, 129, 1), (67, 131, 2), (261, 70, 4), (128, 160, 3), (96, 64, 3)):
        imgs = np.stack([rand_img(rng, h, w, b) for _ in range(3)])
        for a in (90, 270):
            got = gpu.run_op("rot", imgs, angle=a)
            for i in range(3):
                assert_same(got[i], oracle.rot(imgs[i], a), f"rot{a} {h}x{w}x{b} img{i} xcd={xcd}")


@pytest.mark.parametrize("pxh,order", [("32", "1"), ("64", "1"), ("128", "1"), ("128", "0"), ("off", "1")])
def test_rot90_rgb_pixel_tiles(gpu, oracle, rng, monkeypatch, pxh, order):
    """k_rot90_px (3-band 90 / 270 through the pixel-major LDS tile): 32 / 64 / 128 input
    rows per tile (MIPX_ROT_PXH), tiles y- or x-fastest; images whose rows are not on a
    dword (b128 + de-skew staging) and batches of odd-size images (unaligned image bases),
    ragged edge tiles with row counts that are not a multiple of 4, images of one row or
    column.  "off": the same cases through k_rot90_lds (MIPX_ROT_PX=0)."""
    if pxh == "off":
        monkeypatch.setenv("MIPX_ROT_PX", "0")
    else:
        monkeypatch.setenv("MIPX_ROT_PXH", pxh)
    monkeypatch.setenv("MIPX_ROT_ORDER", order)
    for h, w in ((130, 197), (128, 160), (96, 64), (1, 77), (77, 1), (3, 5), (257, 63), (66, 129), (200, 300)):
        imgs = np.stack([rand_img(rng, h, w, 3) for _ in range(3)])
        for a in (90, 270):
            got = gpu.run_op("rot", imgs, angle=a)
            for i in range(3):
                assert_same(got[i], oracle.rot(imgs[i], a), f"rot{a} {h}x{w}x3 img{i} pxh={pxh} order={order}")


@pytest.mark.parametrize("route", ["1", "2", "0"])
def test_batch_device_copy(gpu, rng, monkeypatch, route):
    """The batch copy behind rot 0, flatten without alpha, a 1.0 reduce and B_W of 1-2
    bands (k_copy16, non-temporal or plain; MIPX_COPY=0: hipMemcpyAsync): byte counts
    below one chunk, not a multiple of 16, and past one 16 KB block."""
    monkeypatch.setenv("MIPX_COPY", route)
    for h, w, b, n in ((1, 1, 1, 1), (1, 5, 3, 1), (3, 7, 3, 2), (37, 53, 3, 3), (64, 64, 4, 2), (333, 251, 3, 5)):
        imgs = rng.integers(0, 256, (n, h, w, b), dtype=np.uint8)
        assert np.array_equal(gpu.run_op("rot", imgs, angle=0), imgs), f"rot 0 {n}x{h}x{w}x{b}"
        if b == 3:
            assert np.array_equal(gpu.run_op("flatten", imgs, background=(1, 2, 3)), imgs), f"flatten {h}x{w}"


@pytest.mark.parametrize("pxh", ["64", "128"])
def test_rot90_rgba_pixel_tiles(gpu, oracle, rng, monkeypatch, pxh):
    """k_rot90_px on 4-band images (the default; MIPX_ROT_PX4=0 keeps them on k_rot90_lds):
    one b128 load and store per 4 pixels, ragged edge tiles, one-row / one-column images,
    batches."""
    monkeypatch.setenv("MIPX_ROT_PXH", pxh)
    for h, w in ((130, 197), (128, 160), (1, 77), (77, 1), (3, 5), (257, 63), (66, 129)):
        imgs = np.stack([rand_img(rng, h, w, 4) for _ in range(3)])
        for a in (90, 270):
            got = gpu.run_op("rot", imgs, angle=a)
            for i in range(3):
                assert_same(got[i], oracle.rot(imgs[i], a), f"rot{a} {h}x{w}x4 img{i} pxh={pxh}")


@pytest.mark.parametrize("x4", ["1", "0"])
def test_shrink_x4_and_dword_kernels(gpu, oracle, rng, monkeypatch, x4):
    """Box shrink: the 16-byte-per-lane kernel (dword-aligned rows, vs <= 257) and
    the dword kernel (MIPX_SHRINK_X4=0, and any odd row), vs above one load batch,
    spans past the row end (COPY border), every band count."""
    monkeypatch.setenv("MIPX_SHRINK_X4", x4)
    for h, w, b, hs, vs in ((64, 400, 3, 8, 8), (70, 333, 3, 3, 11), (300, 64, 4, 7, 260), (45, 1000, 1, 9, 5),
                            (33, 66, 2, 5, 17), (100, 1024, 4, 16, 3), (50, 4000 // 8, 3, 11, 11)):
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
        got = gpu.run_op("shrink", imgs, hshrink=hs, vshrink=vs)
        for i in range(2):
            assert_same(got[i], oracle.shrink(imgs[i], hs, vs), f"shrink {h}x{w}x{b} {hs}x{vs} x4={x4}")


@pytest.mark.parametrize("q", ["1", "0"])
@pytest.mark.parametrize("s", [2, 3, 4])
def test_shrink_quad_kernel(gpu, oracle, rng, monkeypatch, q, s):
    """Small equal factors (k_shrink_q: registers only, 4 output pixels per lane)
    against the oracle and against the LDS kernels (MIPX_SHRINK_Q=0): widths that end
    inside a quad and past the last whole box (COPY border), odd heights, output rows
    that are not dword aligned (byte stores), RGB and RGBA, batches of 2."""
    monkeypatch.setenv("MIPX_SHRINK_Q", q)
    for h, w, b in ((64, 400, 3), (37, 1000, 3), (9, 4000 // 3 * 3 // 4 * 4, 3), (33, 84, 3), (5, 12, 3), (70, 333 * 4, 4),
                    (41, 52, 4), (3, 4, 4), (17, 1276, 3)):
        if (w * b) % 4:
            continue
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
        got = gpu.run_op("shrink", imgs, hshrink=s, vshrink=s)
        for i in range(2):
            assert_same(got[i], oracle.shrink(imgs[i], s, s), f"shrink q={q} {h}x{w}x{b} /{s}")


@pytest.mark.parametrize("p1", ["1", "0"])
@pytest.mark.parametrize("s", [5, 6, 7, 8, 9, 10, 11, 12])
def test_shrink_p1_kernel(gpu, oracle, rng, monkeypatch, s, p1):
    """Equal factors 5-12 on the one-pixel-per-lane register kernel (MIPX_SHRINK_P1=1,
    RGBA up to 11) and on k_shrink_x4 / k_shrink_lds (=0): rows of any byte alignment,
    widths ending inside a box (COPY border), heights past the last whole box, RGB and
    RGBA, batches of 2."""
    monkeypatch.setenv("MIPX_SHRINK_P1", p1)
    for h, w, b in ((64, 400, 3), (37, 1001, 3), (s, s, 3), (2 * s + 1, 13 * s - 1, 3), (70, 333, 4),
                    (41, 52, 4), (s + 3, 5 * s + 2, 4), (17, 1277, 3)):
        if b == 4 and s > 11:
            continue
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
        got = gpu.run_op("shrink", imgs, hshrink=s, vshrink=s)
        for i in range(2):
            assert_same(got[i], oracle.shrink(imgs[i], s, s), f"shrink p1 {h}x{w}x{b} /{s}")


# ---------------------------------------------------------------- gaussian blur
@pytest.mark.parametrize("sigma", [0.8, 1.0, 3.0, 5.0, 12.5])
@pytest.mark.parametrize("b", [1, 3, 4])
def test_gaussblur_matches_oracle(gpu, oracle, rng, sigma, b):
    img = rand_img(rng, 45, 301 if b == 1 else 70, b)
    assert_same(gpu.run_op("gaussblur", img, sigma=sigma, min_ampl=0.2)[0], oracle.gaussblur(img, sigma, 0.2),
                f"blur {sigma}")


@pytest.mark.parametrize("dot", ["1", "0"])
@pytest.mark.parametrize("sigma", [0.6, 2.2, 5.0, 9.0])
def test_gaussblur_dot4_and_float_paths(gpu, oracle, rng, monkeypatch, dot, sigma):
    """Conv passes: the packed-u8 v_dot4 path (default) and the float path
    (MIPX_SEP_DOT=0) on every band count, odd widths and unaligned batches
    (3 images of an odd byte size: the DMA=0 vertical staging)."""
    monkeypatch.setenv("MIPX_SEP_DOT", dot)
    monkeypatch.setenv("MIPX_BLUR2D", "0")  # the two separable passes, not the fused kernels
    for h, w, b in ((37, 53, 1), (29, 41, 2), (64, 77, 3), (50, 260, 4), (33, 19, 3)):
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b), rand_img(rng, h, w, b)])
        got = gpu.run_op("gaussblur", imgs, sigma=sigma, min_ampl=0.2)
        for i in range(3):
            assert_same(got[i], oracle.gaussblur(imgs[i], sigma, 0.2), f"blur {sigma} {h}x{w}x{b} dot={dot} img{i}")


@pytest.mark.parametrize("fround", ["1", "0"])
@pytest.mark.parametrize("rows", ["4", "64"])
@pytest.mark.parametrize("sigma", [0.3, 1.0, 2.2, 5.0, 7.5, 9.0, 12.5])
def test_blur2d_fused_matches_oracle(gpu, oracle, rng, monkeypatch, rows, sigma, fround):
    """Fused gaussblur (k_blur2d: horizontal pass into a per-lane register ring,
    vertical pass from it) for masks up to 45 taps: every band count, odd sizes,
    unaligned batches (odd image byte sizes), several column blocks, images
    shorter than the mask, band heights of 4 and 64 rows (MIPX_BLUR2D_ROWS), integer
    mul-hi (default) and fp32 rounding (MIPX_BLUR2D_FROUND=1)."""
    monkeypatch.setenv("MIPX_BLUR2D_ROWS", rows)
    monkeypatch.setenv("MIPX_BLUR2D_FROUND", fround)
    monkeypatch.setenv("MIPX_BCOL", "0")
    for h, w, b in ((37, 53, 1), (29, 41, 2), (64, 77, 3), (50, 260, 4), (33, 19, 3), (9, 600, 4), (130, 513, 3),
                    (3, 5, 4), (70, 257, 2)):
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b), rand_img(rng, h, w, b)])
        got = gpu.run_op("gaussblur", imgs, sigma=sigma, min_ampl=0.2)
        for i in range(3):
            assert_same(got[i], oracle.gaussblur(imgs[i], sigma, 0.2), f"blur2d {sigma} {h}x{w}x{b} rows={rows} fr={fround} img{i}")


@pytest.mark.parametrize("sigma", [0.3, 1.0, 2.2, 5.0, 7.5, 9.0, 12.5])
def test_blur_fallback_matches_oracle(gpu, oracle, rng, monkeypatch, sigma):
    """The gaussblur chain behind the column walker (MIPX_BCOL=0: k_blur2d, then the two
    separable passes; r02's k_bmf was removed in r04, k_bcol serves every image it could)
    against the oracle: RGB / RGBA, images narrower than a block and shorter than the
    mask, both edges of every window, windowed plans (resize -> crop -> blur) at every
    gravity, unaligned rows, 1-2 bands, > 33 taps."""
    monkeypatch.setenv("MIPX_BCOL", "0")  # the column walker itself: tests/test_bcol_gpu.py
    for h, w, b in ((64, 76, 3), (130, 516, 3), (9, 600, 4), (50, 260, 4), (3, 8, 4), (33, 20, 3), (17, 132, 3),
                    (200, 388, 4), (33, 19, 3), (29, 41, 2), (41, 57, 1), (47, 140, 3), (95, 300, 4)):
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
        got = gpu.run_op("gaussblur", imgs, sigma=sigma, min_ampl=0.2)
        for i in range(2):
            assert_same(got[i], oracle.gaussblur(imgs[i], sigma, 0.2), f"fallback {sigma} {h}x{w}x{b} img{i}")
    if sigma in (1.0, 5.0):
        for g, b in ((0, 3), (2, 3), (3, 4), (1, 4)):
            opts = dict(width=300, height=200, crop=1, gravity=g, sigma=sigma)
            p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(1200, 700, b, "png"))
            e, rp = oracle.plan(opts, dict(w=1200, h=700, bands=b, type=3))
            assert e == 0
            imgs = rng.integers(0, 256, (2, 700, 1200, b), dtype=np.uint8)
            got = gpu.execute(p, imgs)
            for i in range(2):
                assert_same(got[i], oracle.execute(rp, imgs[i]), f"fallback window gravity {g} bands {b}")


@pytest.mark.parametrize("hdma", ["16", "4"])
def test_hpass_dma_widths(gpu, oracle, rng, monkeypatch, hdma):
    """Horizontal passes on RGBA with 16-byte-aligned rows stage through dwordx4
    DMA by default (MIPX_HP_DMA=4 caps it at dword DMA): reduceh at several
    shrinks, blur, and a whole reduce -> extract plan (window origin off the
    16-byte grid), each against the oracle, with both image edges inside a block."""
    monkeypatch.setenv("MIPX_HP_DMA", hdma)
    monkeypatch.setenv("MIPX_BLUR2D", "0")
    for h, w, s in ((23, 256, 1.3333333333333333), (19, 300, 2.5), (11, 1028, 1.1), (9, 64, 3.0)):
        imgs = np.stack([rand_img(rng, h, w, 4), smooth_img(rng, h, w, 4)])
        got = gpu.run_op("reduceh", imgs, hshrink=s)
        for i in range(2):
            assert_same(got[i], oracle.reduceh(imgs[i], s), f"reduceh {w} {s} dma={hdma}")
        got = gpu.run_op("gaussblur", imgs, sigma=2.4, min_ampl=0.2)
        for i in range(2):
            assert_same(got[i], oracle.gaussblur(imgs[i], 2.4, 0.2), f"blur {w} dma={hdma}")
    opts = dict(width=300, height=200, crop=1)
    p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(640, 520, 4, "png"))
    e, rp = oracle.plan(opts, dict(w=640, h=520, bands=4, type=3))
    assert e == 0
    imgs = rng.integers(0, 256, (2, 520, 640, 4), dtype=np.uint8)
    got = gpu.execute(p, imgs)
    for i in range(2):
        assert_same(got[i], oracle.execute(rp, imgs[i]), f"reduce+extract dma={hdma}")


@pytest.mark.parametrize("dot", ["1", "0"])
@pytest.mark.parametrize("s", [1.1, 1.3333333333333333, 2.5, 3.7])
def test_reduce_passes_dot2_and_float_paths(gpu, oracle, rng, monkeypatch, dot, s):
    """Generic reduce passes: the int16 v_dot2 path (default) and the float path
    (MIPX_SEP_DOT=0), every band count, odd sizes, unaligned batches."""
    monkeypatch.setenv("MIPX_SEP_DOT", dot)
    for h, w, b in ((41, 57, 1), (37, 43, 2), (64, 90, 3), (50, 128, 4), (31, 17, 3)):
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b), rand_img(rng, h, w, b)])
        gv = gpu.run_op("reducev", imgs, vshrink=s)
        gh = gpu.run_op("reduceh", imgs, hshrink=s)
        for i in range(3):
            assert_same(gv[i], oracle.reducev(imgs[i], s), f"reducev {s} {h}x{w}x{b} dot={dot}")
            assert_same(gh[i], oracle.reduceh(imgs[i], s), f"reduceh {s} {h}x{w}x{b} dot={dot}")


@pytest.mark.parametrize("path", ["unrolled", "loop"])
@pytest.mark.parametrize("s", [1.02, 1.3333333333333333, 1.6, 2.4, 2.7, 3.7, 5.9])
def test_reducev_paths(gpu, oracle, rng, monkeypatch, path, s):
    """Vertical reduce kernels: k_vreduce with the tap pairs unrolled (default for
    <= 16 taps on 4-byte rows), k_vpass's generic loop (MIPX_VP_FAST=0, and every
    case k_vreduce does not take): 16- and 4-byte-aligned
    batches (DMA 16 / 4), odd row bytes and an unaligned batch (DMA 0), many row
    blocks, both pair alignments of each row, short images, windowed plans."""
    monkeypatch.setenv("MIPX_VP_FAST", "0" if path == "loop" else "1")
    monkeypatch.setenv("MIPX_RCOL", "0")
    monkeypatch.setenv("MIPX_RMFMA", "0")
    monkeypatch.setenv("MIPX_FUSED_REDUCE", "0")
    monkeypatch.setenv("MIPX_RSTRIP", "0")
    for h, w, b in ((301, 64, 4), (257, 100, 3), (97, 1030, 4), (45, 301, 1), (7, 80, 4), (333, 33, 3),
                    (120, 1111, 3), (64, 2, 2)):
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
        gv = gpu.run_op("reducev", imgs, vshrink=s)
        for i in range(2):
            assert_same(gv[i], oracle.reducev(imgs[i], s), f"reducev {s} {h}x{w}x{b} {path}")
    opts = dict(width=301, height=173, crop=1, gravity=3)  # south; reduce -> extract: window row offset
    p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(640, 1020, 4, "png"))
    e, rp = oracle.plan(opts, dict(w=640, h=1020, bands=4, type=3))
    assert e == 0
    imgs = rng.integers(0, 256, (2, 1020, 640, 4), dtype=np.uint8)
    got = gpu.execute(p, imgs)
    for i in range(2):
        assert_same(got[i], oracle.execute(rp, imgs[i]), f"reduce+extract {path}")


@pytest.mark.parametrize("kernel,pack3", [("hreduce", "0"), ("hreduce", "1"), ("hpass", "0"), ("hpass", "1")])
@pytest.mark.parametrize("s", [1.02, 1.3333333333333333, 1.6, 2.4, 2.7, 3.7, 6.3])
def test_reduceh_paths(gpu, oracle, rng, monkeypatch, kernel, pack3, s):
    """Horizontal reduce kernels: k_hreduce (default: compile-time tap pairs, up to 16 taps) and k_hpass
    (MIPX_HP_FAST=0 as well, and 1 / 2 bands, longer masks): RGBA rows 16- / 4-byte
    aligned and unaligned (DW 16 / 4 / 0), RGB with and without the 3-dword group
    stores (MIPX_HP_PACK3), rows that end inside a 4-pixel group, images narrower
    than a group, several column blocks, windowed plans (reduce -> extract)."""
    monkeypatch.setenv("MIPX_HP_FAST", "0" if kernel == "hpass" else "1")
    monkeypatch.setenv("MIPX_RCOL", "0")
    monkeypatch.setenv("MIPX_RMFMA", "0")
    monkeypatch.setenv("MIPX_HP_PACK3", pack3)
    monkeypatch.setenv("MIPX_FUSED_REDUCE", "0")
    monkeypatch.setenv("MIPX_RSTRIP", "0")
    for h, w, b in ((19, 1100, 4), (23, 1027, 4), (21, 641, 3), (17, 2000, 3), (9, 64, 3), (5, 13, 4), (11, 301, 2),
                    (7, 250, 1), (40, 333, 3), (33, 7, 3), (3, 7, 4)):
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b), rand_img(rng, h, w, b)])
        gh = gpu.run_op("reduceh", imgs, hshrink=s)
        for i in range(3):
            assert_same(gh[i], oracle.reduceh(imgs[i], s), f"reduceh {s} {h}x{w}x{b} {kernel} pack3={pack3} img{i}")
    for b in (3, 4):
        opts = dict(width=333, height=120, crop=1, gravity=2)  # east: window column offset
        p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(1500, 400, b, "png"))
        e, rp = oracle.plan(opts, dict(w=1500, h=400, bands=b, type=3))
        assert e == 0
        imgs = rng.integers(0, 256, (2, 400, 1500, b), dtype=np.uint8)
        got = gpu.execute(p, imgs)
        for i in range(2):
            assert_same(got[i], oracle.execute(rp, imgs[i]), f"reduce+extract b={b} {kernel}")


@pytest.mark.parametrize("on", ["", "2n", "2t", "0"])
@pytest.mark.parametrize("hs,vs", [(1.6, 1.6), (1.3333333333333333, 1.3333333333333333), (2.4, 2.4), (1.02, 1.9),
                                   (2.7, 1.5), (1.46484375, 1.46484375), (1.1, 1.05)])
def test_reduce_rmfma_fused(gpu, oracle, rng, monkeypatch, on, hs, vs):
    """k_rmf2 (both passes on the i8 matrix cores, channel-planar horizontal operands)
    against the oracle, with k_rcol off so it takes every case it can: RGB / RGBA, rows
    of any alignment, blocks at both image edges, images narrower than a block and
    shorter than 16 rows, windowed plans (reduce -> extract), and the cases it leaves to
    other kernels (17 taps).  "2n" forces its 64-pixel columns, "2t" its tap loads
    after the barriers; "0" turns it off (the strip walker / two passes take over)."""
    monkeypatch.setenv("MIPX_RCOL", "0")
    monkeypatch.setenv("MIPX_RMFMA", "0" if on == "0" else "")
    monkeypatch.setenv("MIPX_RMF2_HT", "0" if on == "2t" else "1")
    monkeypatch.setenv("MIPX_RMF2_XW", "64" if on == "2n" else "0")
    monkeypatch.setenv("MIPX_RSTRIP", "0")
    monkeypatch.setenv("MIPX_FUSED_REDUCE", "0")
    for h, w, b in ((301, 1100, 3), (97, 640, 3), (13, 200, 3), (40, 36, 3), (270, 480, 3), (37, 1026, 3),
                    (150, 97, 3), (201, 700, 4), (19, 333, 4), (64, 1024, 4), (101, 1333, 3), (99, 1331, 3)):
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
        got = gpu.run_op("reduce", imgs, hshrink=hs, vshrink=vs)
        for i in range(2):
            assert_same(got[i], oracle.reduce(imgs[i], hs, vs), f"rmfma={on} {h}x{w}x{b} {hs}x{vs} img{i}")
    for g, b in ((0, 3), (2, 3), (3, 3), (0, 4), (3, 4)):
        opts = dict(width=333, height=171, crop=1, gravity=g)
        p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(1500, 1000, b, "png"))
        e, rp = oracle.plan(opts, dict(w=1500, h=1000, bands=b, type=3))
        assert e == 0
        imgs = rng.integers(0, 256, (2, 1000, 1500, b), dtype=np.uint8)
        got = gpu.execute(p, imgs)
        for i in range(2):
            assert_same(got[i], oracle.execute(rp, imgs[i]), f"rmfma={on} window gravity {g} bands {b}")


@pytest.mark.parametrize("w", [1, 2, 5, 7, 13])
def test_reduce_narrow_unaligned_rows(gpu, oracle, rng, w):
    """k_rmf2 on images a few pixels wide with rows that are not a multiple of 4 bytes
    (found by the 200-seed whole-plan fuzz, seed 75: a 1 x 23 RGB reduce).  A staged
    row then spans several image rows and the last image row's dwords end past the
    image; the row offset must ride in the range-checked VGPR offset."""
    for h, s in ((23, 1.3529411764705883), (17, 1.6), (40, 2.4), (9, 1.25)):
        if int(w / s + 0.5) < 1:  # libvips' reduce would make an empty image (EINVAL)
            continue
        imgs = np.stack([rand_img(rng, h, w, 3), smooth_img(rng, h, w, 3), rand_img(rng, h, w, 3)])
        got = gpu.run_op("reduce", imgs, hshrink=s, vshrink=s)
        for i in range(3):
            assert_same(got[i], oracle.reduce(imgs[i], s, s), f"reduce {h}x{w}x3 /{s} img{i}")


@pytest.mark.parametrize("repack", ["1", "0"])
def test_hpass_raw_repack_paths(gpu, oracle, rng, monkeypatch, repack):
    """Horizontal passes on rows that are not 16/4-byte aligned stage raw bytes and
    repack them per pixel: 4 pixels per item with v_alignbyte / v_perm (default) or
    one per item (MIPX_HP_REPACK=0); every band count, both image edges in a block."""
    monkeypatch.setenv("MIPX_HP_REPACK", repack)
    monkeypatch.setenv("MIPX_BLUR2D", "0")
    for h, w, b in ((9, 301, 3), (7, 517, 1), (6, 259, 2), (5, 263, 4), (11, 37, 3)):
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b), rand_img(rng, h, w, b)])
        for s in (1.6, 2.9):
            got = gpu.run_op("reduceh", imgs, hshrink=s)
            for i in range(3):
                assert_same(got[i], oracle.reduceh(imgs[i], s), f"reduceh {h}x{w}x{b} {s} repack={repack}")
        got = gpu.run_op("gaussblur", imgs, sigma=1.5, min_ampl=0.2)
        for i in range(3):
            assert_same(got[i], oracle.gaussblur(imgs[i], 1.5, 0.2), f"blur {h}x{w}x{b} repack={repack}")


@pytest.mark.parametrize("pack3", ["1", "0"])
def test_hpass_rgb_packed_stores(gpu, oracle, rng, monkeypatch, pack3):
    """3-band horizontal passes store each aligned 4-pixel group as 3 dwords (lanes
    exchange neighbours) or per byte (MIPX_HP_PACK3=0); output widths with and without
    dword-aligned rows, partial groups at the row end, several x blocks per row."""
    monkeypatch.setenv("MIPX_HP_PACK3", pack3)
    monkeypatch.setenv("MIPX_BLUR2D", "0")
    for h, w in ((5, 1280), (4, 1283), (3, 1922), (6, 17), (2, 1041)):
        imgs = np.stack([rand_img(rng, h, w, 3), smooth_img(rng, h, w, 3)])
        for s in (1.6, 2.4, 1.0 + 1.0 / 3.0):
            got = gpu.run_op("reduceh", imgs, hshrink=s)
            for i in range(2):
                assert_same(got[i], oracle.reduceh(imgs[i], s), f"reduceh {h}x{w} {s} pack3={pack3}")
        got = gpu.run_op("gaussblur", imgs, sigma=2.0, min_ampl=0.2)
        for i in range(2):
            assert_same(got[i], oracle.gaussblur(imgs[i], 2.0, 0.2), f"blur {h}x{w} pack3={pack3}")


# ---------------------------------------------------------------- affine (enlarge) / zoom / flatten / B_W
@pytest.mark.parametrize("h,w,b,xs,ys,extend", [(30, 40, 3, 2.0, 2.0, 1), (17, 23, 4, 3.004291845493562, 3.004291845493562, 1),
                                              (33, 29, 1, 1.7, 0.8, 1), (20, 20, 3, 2.5, 2.5, 0), (15, 31, 2, 1.3, 4.1, 3),
                                              (12, 9, 3, 7.0, 7.0, 2), (25, 25, 4, 1.5, 1.5, 4)])
def test_affine_matches_oracle(gpu, oracle, rng, h, w, b, xs, ys, extend):
    imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
    got = gpu.run_op("affine", imgs, xscale=xs, yscale=ys, extend=extend)
    for i in range(2):
        assert_same(got[i], oracle.affine(imgs[i], xs, ys, extend), f"affine {xs}x{ys} e{extend} img{i}")


@pytest.mark.parametrize("nt", ["1", "0"])
@pytest.mark.parametrize("b", [1, 2, 3, 4])
def test_zoom_flatten_bw_match_oracle(gpu, oracle, rng, monkeypatch, b, nt):
    monkeypatch.setenv("MIPX_ZOOM_NT", nt)  # zoom rows with non-temporal (default) or plain stores
    imgs = np.stack([rand_img(rng, 19, 23, b), smooth_img(rng, 19, 23, b)])
    for xf, yf in ((2, 2), (3, 1), (1, 4), (5, 3)):
        got = gpu.run_op("zoom", imgs, xfac=xf, yfac=yf)
        for i in range(2):
            assert_same(got[i], oracle.zoom(imgs[i], xf, yf), f"zoom {xf}x{yf}")
    # r03 row-staged zoom: rows of several 4 KiB output chunks, unaligned output rows, tall factors
    big = np.stack([rand_img(rng, 37, 1500, b), smooth_img(rng, 37, 1500, b)])
    for xf, yf in ((2, 2), (3, 5), (7, 1), (1, 3)):
        got = gpu.run_op("zoom", big, xfac=xf, yfac=yf)
        for i in range(2):
            assert_same(got[i], oracle.zoom(big[i], xf, yf), f"zoom {xf}x{yf} 37x1500x{b}")
    got = gpu.run_op("flatten", imgs, background=(200, 17, 90))
    for i in range(2):
        assert_same(got[i], oracle.flatten(imgs[i], (200, 17, 90)), "flatten")
    got = gpu.run_op("bw", imgs)
    for i in range(2):
        assert_same(got[i], oracle.bw(imgs[i]), "bw")


def test_bw_every_colour(gpu, oracle):
    """Every one of the 2^24 sRGB colours through B_W (as a 4096 x 4096 image).
    The float LUT pipeline has exact .5 ties (e.g. RGB (206, 28, 113) -> 108.5 ->
    108), so one fused multiply-add anywhere in it shows up here."""
    v = np.arange(1 << 24, dtype=np.uint32)
    img = np.stack([(v >> 16) & 255, (v >> 8) & 255, v & 255], -1).astype(np.uint8).reshape(4096, 4096, 3)
    assert_same(gpu.run_op("bw", img)[0], oracle.bw(img), "bw all colours")


# ---------------------------------------------------------------- watermark composite
@pytest.mark.parametrize("bb,wb", [(3, 3), (3, 4), (4, 4), (4, 3), (1, 2), (2, 2)])
@pytest.mark.parametrize("opacity", [0.5, 1.0, 0.2])
def test_watermark_matches_oracle(gpu, oracle, rng, bb, wb, opacity):
    base = rand_img(rng, 40, 60, bb)
    wm = rand_img(rng, 16, 24, wb)
    for left, top in ((3, 4), (50, 30), (0, 0)):
        got = gpu.run_op("watermark", base, wm=wm, left=left, top=top, opacity=opacity)
        assert_same(got[0], oracle.watermark(base, wm, left, top, opacity), f"wm {bb}/{wb} at {left},{top}")


# ---------------------------------------------------------------- smartcrop
@pytest.mark.parametrize("h,w,cw,ch", [(256, 341, 256, 256), (300, 400, 100, 80), (240, 180, 100, 100),
                                       (512, 384, 200, 300)])
def test_smartcrop_origin_identical(gpu, oracle, rng, h, w, cw, ch):
    imgs = np.stack([smooth_img(rng, h, w, 3), rand_img(rng, h, w, 3)])
    got = gpu.smartcrop_origins(imgs, cw, ch)
    for i in range(len(imgs)):
        assert tuple(got[i]) == oracle.smartcrop_origin(imgs[i], cw, ch), f"smartcrop img{i}"


# ---------------------------------------------------------------- whole plans
PLANS = [
    # (opts, header (w, h, bands, type, orientation))
    (dict(width=300, height=300, embed=1), (550, 740, 3, "png", 0)),
    (dict(width=300, embed=1, crop=1), (550, 740, 3, "png", 0)),
    (dict(width=300, height=200, crop=1, gravity=5), (640, 480, 3, "png", 0)),
    (dict(width=256, height=256, crop=1, gravity=5), (1000, 750, 3, "png", 0)),
    (dict(width=256, height=256), (1000, 750, 3, "png", 6)),
    (dict(width=100, height=100, embed=1, extend=3), (320, 200, 4, "png", 0)),
    (dict(rotate=90, flip=1, flop=1), (123, 77, 3, "png", 0)),
    (dict(sigma=5.0), (200, 150, 4, "png", 0)),
    (dict(top=10, left=20, area_width=100, area_height=50), (200, 150, 3, "png", 0)),
    (dict(width=1024, embed=1), (2048, 2048, 4, "png", 0)),
    # peephole fusions: reduce -> extract (window reduce), extract -> blur (window blur)
    (dict(top=10, left=21, area_width=101, area_height=50, sigma=2.0), (200, 150, 3, "png", 0)),
    (dict(top=3, left=4, area_width=64, area_height=40, sigma=5.0), (97, 61, 4, "png", 0)),
    (dict(width=300, height=200, crop=1, sigma=1.5), (640, 480, 4, "png", 0)),
    (dict(width=251, height=99, crop=1, gravity=3), (1001, 333, 3, "png", 0)),
    (dict(width=768, height=512, crop=1), (1024, 1024, 4, "png", 0)),
    # Enlarge (affine bicubic), Zoom, flatten, colorspace=bw
    (dict(width=400, height=300, enlarge=1, crop=1), (200, 150, 3, "png", 0)),
    (dict(width=1000, height=700, enlarge=1, crop=1), (333, 233, 3, "png", 0)),
    (dict(width=500, enlarge=1, embed=1), (123, 77, 4, "png", 0)),
    (dict(zoom=1), (41, 29, 3, "png", 0)),
    (dict(zoom=2, top=5, left=7, area_width=30, area_height=20), (40, 30, 4, "png", 0)),
    (dict(width=150, background=(250, 20, 3)), (300, 200, 4, "png", 0)),
    (dict(width=150, interpretation=26), (300, 200, 3, "png", 0)),
    (dict(width=150, interpretation=26, background=(9, 9, 9)), (300, 200, 4, "png", 0)),
]


@pytest.mark.parametrize("opts,hdr", PLANS)
def test_plan_execution_matches_oracle(gpu, oracle, rng, opts, hdr):
    w, h, b, typ, orient = hdr
    p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(w, h, b, typ, orient))
    e, rp = oracle.plan(opts, dict(w=w, h=h, bands=b, type=3, orientation=orient))
    assert e == 0
    imgs = np.stack([smooth_img(rng, h, w, b), rand_img(rng, h, w, b)])
    got = gpu.execute(p, imgs)
    for i in range(2):
        assert_same(got[i], oracle.execute(rp, imgs[i]), f"plan {opts} img{i}")


def test_watermark_plan(gpu, oracle, rng):
    opts = dict(width=256, height=192, wm_enable=1, wm_left=16, wm_top=16, wm_opacity=0.5)
    img = smooth_img(rng, 300, 400, 3)
    wm = rand_img(rng, 128, 128, 4)
    p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(400, 300, 3, "png", 0, wm_w=128, wm_h=128, wm_bands=4))
    e, rp = oracle.plan(opts, dict(w=400, h=300, bands=3, type=3, wm_w=128, wm_h=128, wm_bands=4))
    assert e == 0
    assert_same(gpu.execute(p, img, wm)[0], oracle.execute(rp, img, wm), "thumbnail+watermark")


def test_request_path_batches_and_matches(gpu, oracle, rng):
    """mipx_submit/mipx_wait: pinned staging, queue, cross-request batching."""
    gpu.lib.mipx_shutdown()  # mipx_init refuses another configuration while one runs
    eng = gpu.Engine(max_batch=8)
    try:
        p = gpu.plan_make(gpu.make_opts(width=160, height=120, embed=1), gpu.make_input(320, 240, 3, "png"))
        e, rp = oracle.plan(dict(width=160, height=120, embed=1), dict(w=320, h=240, bands=3, type=3))
        imgs = [rand_img(rng, 240, 320, 3) for _ in range(12)]
        subs = [eng.submit(p, im) for im in imgs]
        for (t, out), im in zip(subs, imgs):
            eng.wait(t)
            assert_same(out, oracle.execute(rp, im), "request path")
    finally:
        eng.shutdown()


def test_request_path_concurrent_mixed_plans(gpu, oracle, rng):
    """Many submitting threads, two interleaved plans, strided host buffers: every
    result matches the oracle, batches fuse requests, the three-stream pipeline
    retires everything."""
    from concurrent.futures import ThreadPoolExecutor
    gpu.lib.mipx_shutdown()  # mipx_init refuses another configuration while one runs
    eng = gpu.Engine(max_batch=16, batch_wait_us=2000)
    try:
        specs = [(dict(width=160, height=120, embed=1), (320, 240, 3)),
                 (dict(sigma=2.0), (100, 80, 4)),
                 (dict(width=50, height=50, crop=1, gravity=5), (200, 150, 3))]
        plans = []
        for opts, (w, h, b) in specs:
            p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(w, h, b, "png"))
            e, rp = oracle.plan(opts, dict(w=w, h=h, bands=b, type=3))
            assert e == 0
            plans.append((p, rp, (h, w, b)))
        jobs = []
        for i in range(60):
            p, rp, (h, w, b) = plans[i % len(plans)]
            wide = rand_img(rng, h, w + 7, b)          # a row stride wider than the image
            jobs.append((p, rp, wide[:, :w]))

        def one(job):
            p, rp, img = job
            t, out = eng.submit(p, img)
            eng.wait(t)
            return out, oracle.execute(rp, np.ascontiguousarray(img))

        with ThreadPoolExecutor(6) as ex:
            results = list(ex.map(one, jobs))
        for k, (got, want) in enumerate(results):
            assert_same(got, want, f"request {k}")
        batches, requests = eng.stats(0)
        assert requests == len(jobs)
        assert batches < len(jobs)
    finally:
        eng.shutdown()


def test_golden_vectors_on_gpu(gpu):
    """The committed fixtures (oracle outputs) are reproduced by the kernels."""
    from conftest import load_golden
    g = load_golden("ops.npz")
    for key in g.files:
        if not key.endswith("__in"):
            continue
        name = key[:-4]
        src = g[key]
        want = g[name + "__out"]
        op, *args = name.split("__")
        if op == "reduce":
            got = gpu.run_op("reduce", src, hshrink=float(args[0]), vshrink=float(args[1]))[0]
        elif op == "shrink":
            got = gpu.run_op("shrink", src, hshrink=int(args[0]), vshrink=int(args[1]))[0]
        elif op == "blur":
            got = gpu.run_op("gaussblur", src, sigma=float(args[0]), min_ampl=0.2)[0]
        else:
            continue
        assert_same(got, want, name)
