"""Planner known-answer tests — pinned by the reference's OWN dimension tests.

Every case below is an output size the reference asserts (image_test.go,
server_test.go) for an imaginary operation on one of its fixtures.  The
product planner (mipx_plan_make, host code, no GPU) and the oracle planner
(ref_plan_make) must both produce it, and must agree step for step.
"""
import pytest

import imaginary_amd as ia
from imaginary_amd import imaginary as im

# (label, fixture header, op wrapper, query, expected (w, h), reference line)
LARGE = dict(w=1920, h=1080, type="jpeg", orientation=0)       # testdata/large.jpg
IMAGINARY = dict(w=550, h=740, type="jpeg", orientation=1)     # testdata/imaginary.jpg

KAT = [
    ("resize 300x300", IMAGINARY, "Resize", {"width": 300, "height": 300}, (300, 300), "image_test.go:20"),
    ("resize w300", IMAGINARY, "Resize", {"width": 300}, (300, 404), "image_test.go:36"),
    ("resize w300 nocrop=false", IMAGINARY, "Resize", {"width": 300, "nocrop": "false"}, (300, 740),
     "image_test.go:54"),
    ("resize w300 nocrop=true", IMAGINARY, "Resize", {"width": 300, "nocrop": "true"}, (300, 404),
     "image_test.go:72"),
    ("fit 300x300", IMAGINARY, "Fit", {"width": 300, "height": 300}, (223, 300), "image_test.go:91"),
    ("autorotate (orientation 1)", IMAGINARY, "Thumbnail", {"width": 550}, (550, 740), "image_test.go:105"),
    ("pipeline crop 300x260", IMAGINARY, "Crop", {"width": 300, "height": 260}, (300, 260),
     "image_test.go:136-141"),
    ("crop w300", LARGE, "Crop", {"width": 300}, (300, 1080), "server_test.go:69"),
    ("resize w300 nocrop=false", LARGE, "Resize", {"width": 300, "nocrop": "false"}, (300, 1080),
     "server_test.go:102"),
    ("enlarge 300x200", LARGE, "Enlarge", {"width": 300, "height": 200}, (300, 200), "server_test.go:135"),
    ("extract 100,100 200x120", LARGE, "Extract",
     {"top": 100, "left": 100, "areawidth": 200, "areaheight": 120}, (200, 120), "server_test.go:168"),
    ("crop w300 type=auto", LARGE, "Crop", {"width": 300}, (300, 1080), "server_test.go:220"),
    ("fit 300x300", LARGE, "Fit", {"width": 300, "height": 300}, (300, 169), "server_test.go:267"),
    ("remote crop 200x200", LARGE, "Crop", {"width": 200, "height": 200}, (200, 200), "server_test.go:308"),
    ("mount crop 200x200", LARGE, "Crop", {"width": 200, "height": 200}, (200, 200), "server_test.go:366"),
]


def _opts_for(opname, hdr, query):
    """Run the image.go wrapper logic up to Process and capture the bimg options."""
    o = im.build_params_from_query({k: str(v) for k, v in query.items()})
    captured = {}

    def fake_process(img, opts, **kw):
        captured.update(opts)
        return None

    real = im.process
    im.process = fake_process
    try:
        getattr(im, opname)(im.Decoded(pixels=__import__("numpy").zeros((1, 1, 3), "uint8"), type=hdr["type"],
                                       orientation=hdr["orientation"], header_w=hdr["w"], header_h=hdr["h"]), o)
    finally:
        im.process = real
    return captured


def _product_plan(opts, hdr):
    return ia.plan_make(ia.make_opts(**opts), ia.make_input(hdr["w"], hdr["h"], 3, hdr["type"], hdr["orientation"]))


def _steps(p):
    return [(p.steps[i].op, tuple(p.steps[i].a), tuple(round(x, 12) for x in p.steps[i].d),
             p.steps[i].out_w, p.steps[i].out_h, p.steps[i].out_bands) for i in range(p.n_steps)]


@pytest.mark.parametrize("label,hdr,op,query,want,ref", KAT, ids=[f"{k[0]}@{k[5]}" for k in KAT])
def test_reference_dimension_kat(label, hdr, op, query, want, ref, oracle):
    opts = _opts_for(op, hdr, query)
    p = _product_plan(opts, hdr)
    assert (p.out_w, p.out_h) == want, (label, ref, p.describe())
    e, rp = oracle.plan(opts, dict(w=hdr["w"], h=hdr["h"], bands=3, type=1, orientation=hdr["orientation"]))
    assert e == 0
    assert (rp.out_w, rp.out_h) == want
    assert _steps(p) == _steps(rp)
    assert p.load_shrink == rp.load_shrink


def test_c1_resize_width_300_plan():
    """BASELINE config C1: POST /resize?width=300 on large.jpg -> JPEG shrink-on-load 4,
    Lanczos3 reduce by 1.6 on 480x270 -> 300x169."""
    opts = _opts_for("Resize", LARGE, {"width": 300})
    p = _product_plan(opts, LARGE)
    assert p.load_shrink == 4 and (p.in_w, p.in_h) == (480, 270)
    d = p.describe()
    assert d[0][0] == "reduce" and abs(d[0][2][0] - 1.6) < 1e-12 and d[0][3][:2] == (300, 169)
    assert (p.out_w, p.out_h) == (300, 169)


def test_c2_4k_to_1080p_plan():
    """BASELINE config C2: decoded 3840x2160 -> 1920x1080 is one Lanczos3 reduce by 2 x 2."""
    opts = _opts_for("Resize", dict(w=3840, h=2160, type="png", orientation=0), {"width": 1920, "height": 1080})
    p = ia.plan_make(ia.make_opts(**opts), ia.make_input(3840, 2160, 3, "png"))
    assert p.load_shrink == 1 and p.describe() == [("reduce", (0,) * 8, (2.0, 2.0, 0.0, 0.0), (1920, 1080, 3))]


def test_c3_pipeline_plans():
    """C3: resize w=1024 -> crop 768x512 -> blur sigma 5 on 2048^2 RGBA (PNG intermediates)."""
    p1 = ia.plan_make(ia.make_opts(**_opts_for("Resize", dict(w=2048, h=2048, type="png", orientation=0),
                                                  {"width": 1024})), ia.make_input(2048, 2048, 4, "png"))
    assert [s[0] for s in p1.describe()] == ["reduce"] and (p1.out_w, p1.out_h) == (1024, 1024)
    p2 = ia.plan_make(ia.make_opts(**_opts_for("Crop", dict(w=1024, h=1024, type="png", orientation=0),
                                                  {"width": 768, "height": 512})), ia.make_input(1024, 1024, 4, "png"))
    assert [s[0] for s in p2.describe()] == ["reduce", "extract"] and (p2.out_w, p2.out_h) == (768, 512)
    p3 = ia.plan_make(ia.make_opts(**_opts_for("GaussianBlur", dict(w=768, h=512, type="png", orientation=0),
                                                  {"sigma": 5})), ia.make_input(768, 512, 4, "png"))
    assert p3.describe() == [("blur", (0,) * 8, (5.0, 0.2, 0.0, 0.0), (768, 512, 4))]


FIT_KAT = [  # image_test.go:160-167
    (1280, 1000, 710, 9999, 710, 555),
    (1279, 1000, 710, 9999, 710, 555),
    (900, 500, 312, 312, 312, 173),
    (900, 500, 313, 313, 313, 174),
    (1299, 2000, 710, 999, 649, 999),
    (1500, 2000, 710, 999, 710, 947),
]


@pytest.mark.parametrize("iw,ih,fw,fh,ew,eh", FIT_KAT)
def test_calculate_destination_fit_dimension(iw, ih, fw, fh, ew, eh, oracle):
    assert ia.fit_dimension(iw, ih, fw, fh) == (ew, eh)
    assert oracle.fit_dimension(iw, ih, fw, fh) == (ew, eh)


@pytest.mark.parametrize("orientation,rot,flip", [(0, 0, 0), (1, 0, 0), (2, 0, 1), (3, 180, 0), (4, 180, 1),
                                                   (5, 90, 1), (6, 90, 0), (7, 270, 1), (8, 270, 0)])
def test_exif_autorotate_plan(orientation, rot, flip, oracle):
    p = ia.plan_make(ia.make_opts(), ia.make_input(64, 48, 3, "jpeg", orientation))
    ops = p.describe()
    want = ([("rot", rot)] if rot else []) + ([("flip", 0)] if flip else [])
    assert [(o[0], o[1][0]) for o in ops] == want
    assert (p.out_w, p.out_h) == ((48, 64) if rot in (90, 270) else (64, 48))
    e, rp = oracle.plan({}, dict(w=64, h=48, bands=3, type=1, orientation=orientation))
    assert e == 0 and _steps(p) == _steps(rp)


@pytest.mark.parametrize("rotate,angle", [(90, 90), (180, 180), (270, 270), (45, None), (360, 270), (100, 90)])
def test_rotate_angle_normalisation(rotate, angle):
    """bimg getAngle: remainder mod 90 dropped, capped at 270 (so 360 -> 270)."""
    p = ia.plan_make(ia.make_opts(rotate=rotate), ia.make_input(64, 48, 3, "png"))
    ops = p.describe()
    if angle is None:
        assert ops == []
    else:
        assert ops[0][0] == "rot" and ops[0][1][0] == angle


def test_enlarge_is_bicubic_affine(oracle):
    """Enlarge (image.go:202): residual > 1 -> vipsAffine(residual) with the bimg
    default bicubic interpolator; output = ceil(w * r) x ceil(h * r), then the
    crop/embed to the exact target (bimg transformImage / extractOrEmbedImage)."""
    cases = [(dict(width=800, height=600, enlarge=1, crop=1), (400, 300), [("affine", (800, 600))], (800, 600)),
             (dict(width=1000, height=700, enlarge=1, crop=1), (333, 233), None, (1000, 700)),
             (dict(width=500, enlarge=1, embed=1), (123, 77), None, (500, 313))]
    for opts, (w, h), want_steps, want_out in cases:
        p = ia.plan_make(ia.make_opts(**opts), ia.make_input(w, h, 3, "png"))
        e, rp = oracle.plan(opts, dict(w=w, h=h, bands=3, type=3))
        assert e == 0 and _steps(p) == _steps(rp), (opts, p.describe())
        assert p.describe()[0][0] == "affine"
        if want_steps:
            assert [(s[0], s[3][:2]) for s in p.describe()] == want_steps
        if want_out:
            assert (p.out_w, p.out_h) == want_out


def test_zoom_plans(oracle):
    """Zoom (image.go:286): vips_zoom(factor + 1) before the transform; with an
    area the extract reads the zoomed image (bimg zoomImage)."""
    for opts, (w, h), want in [(dict(zoom=1), (40, 30), (80, 60)), (dict(zoom=3), (17, 11), (68, 44)),
                               (dict(zoom=1, top=5, left=7, area_width=30, area_height=20), (40, 30), (30, 20))]:
        p = ia.plan_make(ia.make_opts(**opts), ia.make_input(w, h, 3, "png"))
        e, rp = oracle.plan(opts, dict(w=w, h=h, bands=3, type=3))
        assert e == 0 and _steps(p) == _steps(rp)
        assert p.describe()[0][0] == "zoom" and (p.out_w, p.out_h) == want


def test_flatten_and_bw_plans(oracle):
    """imageFlatten (PNG input, non-black background, alpha) drops the alpha band;
    colorspace=bw (params.go:392 -> Interpretation B_W) converts at save."""
    for opts, typ, bands, want_ops, want_bands in [
            (dict(width=250, background=(10, 20, 30)), "png", 4, ["reduce", "flatten"], 3),
            (dict(width=250, background=(10, 20, 30)), "jpeg", 4, ["reduce"], 4),
            (dict(width=250, background=(0, 0, 0)), "png", 4, ["reduce"], 4),
            (dict(width=250, background=(0, 0, 9)), "png", 2, ["reduce", "flatten"], 1),
            (dict(width=250, interpretation=26), "png", 3, ["reduce", "bw"], 1),
            (dict(width=250, interpretation=26), "png", 4, ["reduce", "bw"], 2),
            (dict(width=250, interpretation=22), "png", 3, ["reduce"], 3),
            (dict(width=250, interpretation=26, background=(5, 5, 5)), "png", 4, ["reduce", "flatten", "bw"], 1)]:
        p = ia.plan_make(ia.make_opts(**opts), ia.make_input(400, 300, bands, typ))
        e, rp = oracle.plan(opts, dict(w=400, h=300, bands=bands, type=ia.TYPES[typ]))
        assert e == 0 and _steps(p) == _steps(rp), opts
        assert [s[0] for s in p.describe()] == want_ops and p.out_bands == want_bands, (opts, p.describe())


def test_extract_out_of_bounds_is_einval():
    with pytest.raises(ia.MipxError) as e:
        ia.plan_make(ia.make_opts(top=100, left=100, area_width=400, area_height=10),
                     ia.make_input(400, 300, 3, "png"))
    assert e.value.code == -1


def test_shrunk_to_nothing_is_einval(oracle):
    """height=4 with force on a 16 x 368 image: bimg derives width floor(16 / 92) = 0,
    which libvips' resample ops refuse ("image has shrunk to nothing"); both planners
    return EINVAL (found by the 400-seed whole-plan GPU fuzz, seed 110)."""
    opts = dict(height=4, force=1)
    with pytest.raises(ia.MipxError) as e:
        ia.plan_make(ia.make_opts(**opts), ia.make_input(16, 368, 3, "png"))
    assert e.value.code == -1
    e2, _ = oracle.plan(opts, dict(w=16, h=368, bands=3, type=3))
    assert e2 != 0
    ok = ia.plan_make(ia.make_opts(height=4, force=1), ia.make_input(160, 368, 3, "png"))
    assert ok.out_w >= 1 and ok.out_h == 4


def test_embed_modes_and_background_mapping(oracle):
    for mode in range(7):
        opts = dict(width=100, height=100, embed=1, extend=mode, background=(10, 20, 30))
        p = ia.plan_make(ia.make_opts(**opts), ia.make_input(160, 40, 3, "png"))
        e, rp = oracle.plan(opts, dict(w=160, h=40, bands=3, type=3))
        assert e == 0 and _steps(p) == _steps(rp)
        emb = [s for s in p.describe() if s[0] == "embed"]
        assert emb and emb[0][1][4] == (5 if mode == 6 else mode)


def test_gravity_crop_origins(oracle):
    for g in range(5):
        opts = dict(width=50, height=50, crop=1, gravity=g)
        p = ia.plan_make(ia.make_opts(**opts), ia.make_input(120, 80, 3, "png"))
        e, rp = oracle.plan(opts, dict(w=120, h=80, bands=3, type=3))
        assert e == 0 and _steps(p) == _steps(rp)


def test_random_plans_agree_with_oracle(oracle):
    """Fuzz the option space: product and oracle planners agree on every field."""
    import numpy as np
    r = np.random.default_rng(7)
    agree = 0
    for _ in range(1500):
        w, h = int(r.integers(1, 5000)), int(r.integers(1, 5000))
        opts = dict(width=int(r.choice([0, r.integers(1, 3000)])), height=int(r.choice([0, r.integers(1, 3000)])),
                    crop=int(r.integers(0, 2)), embed=int(r.integers(0, 2)), force=int(r.integers(0, 2)),
                    gravity=int(r.integers(0, 6)), extend=int(r.integers(0, 7)),
                    rotate=int(r.choice([0, 0, 90, 180, 270, 45])), flip=int(r.integers(0, 2)),
                    flop=int(r.integers(0, 2)), sigma=float(r.choice([0, 0, 1.5, 5.0])),
                    enlarge=int(r.integers(0, 2)), zoom=int(r.choice([0, 0, 0, 1, 2])),
                    interpretation=int(r.choice([0, 22, 26])),
                    background=[int(v) for v in r.choice([[0, 0, 0], [255, 10, 3]])])
        typ = int(r.choice([1, 2, 3]))
        orient = int(r.integers(0, 9))
        inp = dict(w=w, h=h, bands=int(r.integers(1, 5)), type=typ, orientation=orient)
        try:
            p = ia.plan_make(ia.make_opts(**opts), ia.make_input(inp["w"], inp["h"], inp["bands"], typ, orient))
            pe = 0
        except ia.MipxError as ex:
            pe, p = ex.code, None
        e, rp = oracle.plan(opts, inp)
        assert pe == e, (opts, inp)
        if e == 0:
            assert _steps(p) == _steps(rp), (opts, inp)
            assert (p.out_w, p.out_h, p.load_shrink) == (rp.out_w, rp.out_h, rp.load_shrink)
            agree += 1
    assert agree > 500


def test_extract_area_branch_follows_bimg(oracle):
    """PARITY_ASSUMPTIONS #11: bimg 1.1.9's extract branch assigns `o.AreaHeight =
    o.Width` when AreaWidth is 0, so a zero AreaWidth is an error in both planners;
    the oracle switch `extract_area_fallback` gives the intended fallback."""
    hdr = dict(w=400, h=300, bands=3, type=3)
    zero_w = dict(width=200, top=5, area_height=100)       # Thumbnail-style: force -> reduce -> area
    with pytest.raises(ia.MipxError) as e:
        ia.plan_make(ia.make_opts(**zero_w), ia.make_input(400, 300, 3, "png"))
    assert e.value.code == -1 and b"Extract area" in ia.lib.mipx_last_error()
    assert oracle.plan(zero_w, hdr)[0] != 0
    assert oracle.plan(dict(zoom=1, top=5, left=7, area_height=20), dict(hdr, w=40, h=30))[0] != 0
    # AreaHeight 0 still falls back to Height, in both planners
    zero_h = dict(width=200, left=5, area_width=100)
    p = ia.plan_make(ia.make_opts(**zero_h), ia.make_input(400, 300, 3, "png"))
    e2, rp = oracle.plan(zero_h, hdr)
    assert e2 == 0 and _steps(p) == _steps(rp) and (p.out_w, p.out_h) == (100, 150)
    oracle.set_switch("extract_area_fallback", 1)
    try:
        e3, rp = oracle.plan(zero_w, hdr)
        assert e3 == 0 and (rp.out_w, rp.out_h) == (200, 100)
    finally:
        oracle.set_switch("extract_area_fallback", 0)


def test_webp_shrink_on_load_switch(oracle):
    """PARITY_ASSUMPTIONS #10: by default WEBP shrinks on load like JPEG (8/4/2
    ladder, factor divided); `webp_sol_bimg` loads at 1/shrink with the factor kept
    and the residual recomputed from the decoded size."""
    opts = dict(width=500)
    hdr = dict(w=4000, h=3000, bands=3, type=2)
    p = ia.plan_make(ia.make_opts(**opts), ia.make_input(4000, 3000, 3, "webp"))
    e, rp = oracle.plan(opts, hdr)
    assert e == 0 and _steps(p) == _steps(rp)
    assert p.load_shrink == rp.load_shrink == 4 and (p.out_w, p.out_h) == (500, 375)
    oracle.set_switch("webp_sol_bimg", 1)
    try:
        e, rp = oracle.plan(opts, hdr)
        assert e == 0 and rp.load_shrink == 6                       # floor(8 * 3/4)
        assert (rp.in_w, rp.in_h) == (667, 500)
        ops = [rp.steps[i].op for i in range(rp.n_steps)]
        assert ops[0] == 3 and (rp.out_w, rp.out_h) == (500, 375)   # shrinkImage again, then residual
    finally:
        oracle.set_switch("webp_sol_bimg", 0)
    assert oracle.plan(opts, hdr)[1].load_shrink == 4
