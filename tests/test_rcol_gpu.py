"""k_rcol, the column-walking generic Lanczos3 reduce (LDS row ring, both passes on
the i8 matrix cores), against the oracle: strips at both image edges (the COPY edge
folded into the horizontal operands), images narrower than a strip and shorter than
a step, segment boundaries in tall images, RGB and RGBA, shrink pairs across
(1, 2.75), windows (reduce -> extract), unaligned output rows (byte stores) and a
seeded fuzz over shapes.  RGB input rows off a dword (r05) run k_rcol's realigning
build (MIPX_RCOL_UNAL=0 leaves them to k_rmf2, as the norcol route does); horizontal K
origins on 4 bytes where that saves a K step (r05, MIPX_RCOL_K4=0: 8 bytes).  RGBA store
tiles read back by tile_rd_lane (r06, MIPX_RCOL_TRL=0: lane / 4)."""
import numpy as np
import pytest

from test_parity_gpu import assert_same, rand_img, smooth_img

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["rcol", "rcol4b", "rcoltrl0", "norcol"])
def route(request, monkeypatch):
    """Every case through k_rcol (the default: 16-byte row pieces through a wave
    tile), k_rcol with 4-byte stores (MIPX_RCOL_WST=0), with r05's tile read-back order
    (MIPX_RCOL_TRL=0), and the kernels behind it (MIPX_RCOL=0: k_rmf2 and the strip
    walker)."""
    monkeypatch.setenv("MIPX_RCOL", "0" if request.param == "norcol" else "")
    monkeypatch.setenv("MIPX_RCOL_WST", "0" if request.param == "rcol4b" else "")
    monkeypatch.setenv("MIPX_RCOL_TRL", "0" if request.param == "rcoltrl0" else "")
    yield request.param

SHRINKS = [(1.6, 1.6), (1.3333333333333333, 1.3333333333333333), (2.4, 2.4), (1.02, 1.9), (2.7, 1.5),
           (1.46484375, 1.46484375), (1.1, 1.05), (1.6, 1.5976331360946747), (2.0, 1.25), (1.25, 2.0)]
SHAPES = [(301, 1100, 3), (97, 640, 3), (13, 200, 3), (40, 36, 3), (270, 480, 3), (37, 1028, 3), (150, 96, 3),
          (201, 700, 4), (19, 333, 4), (64, 1024, 4), (1000, 1500, 3), (9, 4, 3), (700, 64, 4), (101, 1333, 3)]


@pytest.mark.parametrize("hs,vs", SHRINKS)
def test_rcol_matches_oracle(gpu, oracle, rng, hs, vs):
    for h, w, b in SHAPES:
        if int(w / hs + 0.5) < 1 or int(h / vs + 0.5) < 1:
            continue
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b), rand_img(rng, h, w, b)])
        got = gpu.run_op("reduce", imgs, hshrink=hs, vshrink=vs)
        for i in range(len(imgs)):
            assert_same(got[i], oracle.reduce(imgs[i], hs, vs), f"rcol {h}x{w}x{b} {hs}x{vs} img{i}")


@pytest.mark.parametrize("b", [3, 4])
@pytest.mark.parametrize("g", [0, 1, 2, 3, 4])
def test_rcol_windows(gpu, oracle, rng, b, g):
    """reduce -> extract at every gravity: the window's rows and columns only."""
    for (iw, ih, opts) in ((1500, 1000, dict(width=333, height=171, crop=1)),
                           (1024, 1024, dict(width=768, height=512, crop=1)),
                           (1200, 800, dict(width=700, height=300, crop=1))):
        opts = dict(opts, gravity=g)
        p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(iw, ih, b, "png"))
        e, rp = oracle.plan(opts, dict(w=iw, h=ih, bands=b, type=3))
        assert e == 0
        imgs = rng.integers(0, 256, (2, ih, iw, b), dtype=np.uint8)
        got = gpu.execute(p, imgs)
        for i in range(2):
            assert_same(got[i], oracle.execute(rp, imgs[i]), f"rcol window {iw}x{ih} {opts} bands {b}")


def test_rcol_fuzz(gpu, oracle):
    r = np.random.default_rng(20241220)
    for case in range(60):
        b = int(r.choice([3, 4]))
        w = int(r.integers(1, 900))  # RGB rows off a dword: the realigning build
        h = int(r.integers(1, 500))
        hs, vs = float(r.uniform(1.01, 2.74)), float(r.uniform(1.01, 2.74))
        if int(w / hs + 0.5) < 1 or int(h / vs + 0.5) < 1:
            continue
        n = int(r.integers(1, 4))
        imgs = r.integers(0, 256, (n, h, w, b), dtype=np.uint8)
        got = gpu.run_op("reduce", imgs, hshrink=hs, vshrink=vs)
        for i in range(n):
            assert_same(got[i], oracle.reduce(imgs[i], hs, vs), f"fuzz {case}: {h}x{w}x{b} {hs}x{vs} img{i}")


@pytest.mark.parametrize("k4", ["0", "1"])
def test_rcol_k_origins(gpu, oracle, rng, monkeypatch, k4):
    """4-byte K origins (ds_read2_b32; the default where they save a K step, e.g. RGB /
    1.667, C5's 1333x1000 -> 800x600) and the 8-byte ones (MIPX_RCOL_K4=0)."""
    monkeypatch.setenv("MIPX_RCOL_K4", k4)
    for h, w, b, hs, vs in ((101, 1333, 3, 1.6666666666666667, 1.6666666666666667), (64, 1332, 3, 1.6666666666666667, 1.6),
                            (37, 700, 4, 1.7, 1.7), (50, 901, 3, 1.8, 1.25), (20, 96, 3, 1.66, 2.2), (33, 640, 4, 1.9, 1.9)):
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
        got = gpu.run_op("reduce", imgs, hshrink=hs, vshrink=vs)
        for i in range(2):
            assert_same(got[i], oracle.reduce(imgs[i], hs, vs), f"k4={k4} {h}x{w}x{b} {hs}x{vs} img{i}")


@pytest.mark.parametrize("probe", ["ok", "fail"])
def test_unaligned_rows_probe_fallback(gpu, oracle, rng, monkeypatch, probe):
    """Rows whose pitch is not a multiple of 4 bytes: k_rcol's realigning build (rcol
    routes) or k_rmf2 (norcol), whose staging relies on direct-to-LDS loads at unaligned
    byte offsets.  Each device
    runs a probe of that behaviour once; MIPX_LDS_PROBE=fail makes the engine act as
    on a device that fails it, so those rows take the aligned-only kernels.  Both
    routes must give the oracle's bytes."""
    monkeypatch.setenv("MIPX_LDS_PROBE", "fail" if probe == "fail" else "")
    for h, w, hs in ((101, 1333, 1.6666666666666667), (99, 1331, 1.6), (23, 1, 1.3529411764705883), (40, 7, 2.4),
                     (64, 333, 1.46484375)):
        if int(w / hs + 0.5) < 1:
            continue
        imgs = np.stack([rand_img(rng, h, w, 3), smooth_img(rng, h, w, 3)])
        got = gpu.run_op("reduce", imgs, hshrink=hs, vshrink=hs)
        for i in range(2):
            assert_same(got[i], oracle.reduce(imgs[i], hs, hs), f"probe={probe} {h}x{w}x3 /{hs} img{i}")


@pytest.fixture
def centre(oracle, gpu):
    """libvips' centre sampling convention (X = (o + 0.5) * shrink - 0.5, PARITY_ASSUMPTIONS.md
    row 1) in the engine (mipx_set_reduce_sampling) and the oracle."""
    prev_engine, prev_oracle = gpu.reduce_sampling(), oracle.get_switch("reduce_centre")
    gpu.set_reduce_sampling("centre")
    oracle.set_switch("reduce_centre", 1)
    yield
    gpu.set_reduce_sampling(prev_engine)
    oracle.set_switch("reduce_centre", prev_oracle)


def test_reduce_centre_c2_c1_shapes(gpu, oracle, rng, centre):
    """C2 (4K RGB -> 1080p, shrink 2: every output sits at phase 64, k_reduce2m) and
    C1's 480x270 -> 300x169, plus the kernels behind k_rcol (unaligned
    rows: k_rmf2; one axis: the separable passes) and a windowed plan."""
    for h, w, b, hs, vs in ((2160, 3840, 3, 2.0, 2.0), (270, 480, 3, 1.6, 1.5976331360946747),
                            (375, 500, 3, 1.46484375, 1.46484375), (301, 1333, 3, 1.6666666666666667, 1.6666666666666667),
                            (200, 300, 4, 1.3333333333333333, 1.3333333333333333), (97, 640, 3, 2.4, 1.0),
                            (33, 17, 3, 1.0, 2.5)):
        imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
        got = gpu.run_op("reduce", imgs, hshrink=hs, vshrink=vs)
        for i in range(2):
            assert_same(got[i], oracle.reduce(imgs[i], hs, vs), f"centre {h}x{w}x{b} {hs}x{vs} img{i}")
    for (iw, ih, b, opts) in ((1500, 1000, 3, dict(width=333, height=171, crop=1)),
                              (2048, 2048, 4, dict(width=1024)), (1920, 1080, 3, dict(width=300))):
        p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(iw, ih, b, "png"))
        e, rp = oracle.plan(opts, dict(w=iw, h=ih, bands=b, type=3))
        assert e == 0
        imgs = rng.integers(0, 256, (2, ih, iw, b), dtype=np.uint8)
        got = gpu.execute(p, imgs)
        for i in range(2):
            assert_same(got[i], oracle.execute(rp, imgs[i]), f"centre plan {iw}x{ih}x{b} {opts}")


def test_rcol_past_operand_table_cap(gpu, oracle, rng, monkeypatch):
    """Past the host-built operand tables' cap (MIPX_RCOL_HOPCAP_MB=0 here, 256 MiB by
    default) a new geometry runs the build that computes its operands; geometries whose
    tables exist keep them.  Every case must give the oracle's bytes."""
    cases = ((53, 611, 3, 1.55, 1.3), (47, 523, 4, 1.45, 1.7), (61, 739, 3, 2.2, 1.9), (29, 301, 3, 1.7, 1.7))
    for cap in ("0", ""):
        monkeypatch.setenv("MIPX_RCOL_HOPCAP_MB", cap)
        for h, w, b, hs, vs in cases:
            imgs = np.stack([rand_img(rng, h, w, b), smooth_img(rng, h, w, b)])
            got = gpu.run_op("reduce", imgs, hshrink=hs, vshrink=vs)
            for i in range(2):
                assert_same(got[i], oracle.reduce(imgs[i], hs, vs), f"cap={cap!r} {h}x{w}x{b} {hs}x{vs} img{i}")


@pytest.mark.parametrize("n", [128, 40, 3])
def test_rcol_four_wave_build(gpu, oracle, rng, n):
    """C4's thumbnail reduce (12 MP / 11 = 364x273 -> 256x256): with 40 or 128 images the
    whole launch fits one round of resident blocks at 4 waves per SIMD, so the launcher
    takes k_rcol<3, 1, 3>'s 4-wave build (2 segments per strip); 3 images stay on the
    default build.  Both must give the oracle's bytes."""
    h, w, hs, vs = 273, 364, 1.421875, 1.06640625
    imgs = np.stack([rand_img(rng, h, w, 3) if i % 2 else smooth_img(rng, h, w, 3) for i in range(n)])
    got = gpu.run_op("reduce", imgs, hshrink=hs, vshrink=vs)
    for i in range(n):
        assert_same(got[i], oracle.reduce(imgs[i], hs, vs), f"4-wave build n={n} img{i}")
