"""The reference's own operation tests, end to end over ENCODED bytes.

image_test.go and server_test.go call the image.go operations with the
testdata fixtures and assert output size and type.  Here the same operations
run through the drop-in: host codec decode (with the plan's JPEG shrink-on-load)
-> libmipx on the GPU -> host codec encode.  Fixtures are the reference's own
testdata files (tests/golden/testdata/, copied verbatim as data).
"""
import os

import numpy as np

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
TESTDATA = os.path.join(ROOT, "tests", "golden", "testdata")


def read(name):
    with open(os.path.join(TESTDATA, name), "rb") as f:
        return f.read()


def size_of(body):
    from imaginary_amd import codec
    h = codec.header(body)
    return h.w, h.h


@pytest.fixture(scope="module")
def im(gpu):
    from imaginary_amd import imaginary
    return imaginary


CASES = [
    # (reference line, operation, fixture, query, (w, h), type)
    ("image_test.go:10-23", "Resize", "imaginary.jpg", {"width": 300, "height": 300}, (300, 300), "jpeg"),
    ("image_test.go:25-38", "Resize", "imaginary.jpg", {"width": 300}, (300, 404), "jpeg"),
    ("image_test.go:40-56", "Resize", "imaginary.jpg", {"width": 300, "nocrop": "false"}, (300, 740), "jpeg"),
    ("image_test.go:58-74", "Resize", "imaginary.jpg", {"width": 300, "nocrop": "true"}, (300, 404), "jpeg"),
    ("image_test.go:78-94", "Fit", "imaginary.jpg", {"width": 300, "height": 300}, (223, 300), "jpeg"),
    ("image_test.go:96-108", "AutoRotate", "imaginary.jpg", {}, (550, 740), "jpeg"),
    ("server_test.go:42-77", "Crop", "large.jpg", {"width": 300}, (300, 1080), "jpeg"),
    ("server_test.go:79-109", "Resize", "large.jpg", {"width": 300, "nocrop": "false"}, (300, 1080), "jpeg"),
    ("server_test.go:111-142", "Enlarge", "large.jpg", {"width": 300, "height": 200}, (300, 200), "jpeg"),
    ("server_test.go:144-175", "Extract", "large.jpg",
     {"top": 100, "left": 100, "areawidth": 200, "areaheight": 120}, (200, 120), "jpeg"),
    ("server_test.go:244-275", "Fit", "large.jpg", {"width": 300, "height": 300}, (300, 169), "jpeg"),
    ("server_test.go:277-316", "Crop", "large.jpg", {"width": 200, "height": 200}, (200, 200), "jpeg"),
    ("BASELINE C1", "Resize", "large.jpg", {"width": 300}, (300, 169), "jpeg"),
]


@pytest.mark.parametrize("ref,op,fixture,query,want,typ", CASES, ids=[f"{c[1]}@{c[0]}" for c in CASES])
def test_reference_operation_sizes(im, ref, op, fixture, query, want, typ):
    from imaginary_amd import codec
    o = im.build_params_from_query({k: str(v) for k, v in query.items()})
    img = getattr(im, op)(read(fixture), o)
    assert img.mime == codec.mime_type(typ), (ref, img.mime)
    assert size_of(img.body) == want, (ref, size_of(img.body))


def test_pipeline_crop_then_convert_webp(im):
    """image_test.go:110-142: crop 300x260 then convert to webp."""
    o = im.build_params_from_query({})
    o.operations = [{"operation": "crop", "params": {"width": 300, "height": 260}},
                    {"operation": "convert", "params": {"type": "webp"}}]
    img = im.Pipeline(read("imaginary.jpg"), o)
    assert img.mime == "image/webp"
    assert size_of(img.body) == (300, 260)


def test_more_operations_over_bytes(im):
    """The remaining image.go operations through the byte-level drop-in."""
    q = im.build_params_from_query
    cases = [
        ("SmartCrop", "smart-crop.jpg", {"width": 300, "height": 300}, (300, 300), "image/jpeg"),
        ("Thumbnail", "large.jpg", {"width": 100}, (100, 56), "image/jpeg"),
        ("Rotate", "imaginary.jpg", {"rotate": 90}, (740, 550), "image/jpeg"),
        ("Flip", "test.png", {}, (400, 300), "image/png"),
        ("Flop", "test.webp", {}, (550, 368), "image/webp"),
        ("Zoom", "test.png", {"factor": 1}, (800, 600), "image/png"),
        ("GaussianBlur", "test.png", {"sigma": 3}, (400, 300), "image/png"),
        ("Convert", "test.png", {"type": "jpeg"}, (400, 300), "image/jpeg"),
        ("Resize", "test.png", {"width": 200, "background": "255,0,0"}, (200, 150), "image/png"),
        ("Enlarge", "imaginary.jpg", {"width": 1100, "height": 1480}, (1100, 1480), "image/jpeg"),
    ]
    for op, fixture, query, want, mime in cases:
        img = getattr(im, op)(read(fixture), q({k: str(v) for k, v in query.items()}))
        assert img.mime == mime, (op, img.mime)
        assert size_of(img.body) == want, (op, size_of(img.body))


def test_watermark_image_over_bytes(im):
    o = im.build_params_from_query({"left": "10", "top": "10", "opacity": "0.5", "image": "wm.png"})
    img = im.WatermarkImage(read("large.jpg"), o, wm=read("test.png"))
    assert size_of(img.body) == (1920, 1080)


def test_text_watermark_falls_back(im):
    with pytest.raises(im.EngineUnsupported):
        im.Watermark(read("imaginary.jpg"), im.build_params_from_query({"text": "hello"}))


def _drop_leading(p, k, w, h):
    """An oracle plan without its first k steps, taking a w x h input."""
    import ctypes
    from oracle import oracle as o
    rest = o.RefPlan()
    ctypes.memmove(ctypes.byref(rest), ctypes.byref(p), ctypes.sizeof(p))
    rest.in_w, rest.in_h, rest.load_shrink, rest.n_steps = w, h, 1, p.n_steps - k
    for i in range(rest.n_steps):
        rest.steps[i] = p.steps[i + k]
    return rest


ROTATED = [("orient6.jpg", {"width": 300}), ("orient6.jpg", {"width": 200, "height": 200}),
           ("imaginary.jpg", {"width": 200, "rotate": 90}), ("imaginary.jpg", {"width": 120, "flip": "true"})]


@pytest.mark.parametrize("fixture,query", ROTATED, ids=[f"{f}-{'-'.join(q)}" for f, q in ROTATED])
def test_rotated_jpeg_reencodes_before_shrink_on_load(im, oracle, fixture, query):
    """bimg's resizer for a JPEG that rotates or flips (EXIF orientation 6, or an explicit
    rotate / flip) and shrinks on load: rotate the FULL decode, re-encode it (JPEG Q 100,
    no EXIF), decode that at 1/s, run the rest of the plan (image.go:96, :255-265).
    imaginary.Resize over bytes must equal that chain run stage by stage on the host
    with the oracle's pixels and the same codec calls, byte for byte."""
    from imaginary_amd import codec
    buf = read(fixture)
    hdr = codec.header(buf)
    o = im.build_params_from_query({k: str(v) for k, v in query.items()})
    got = im.Resize(buf, o)
    opts = {k: v for k, v in im.bimg_options(o).items() if k not in ("type", "quality", "compression")}
    opts["embed"] = 1
    full = codec.decode(buf)
    rot = {k: opts[k] for k in ("rotate", "flip", "flop", "no_auto_rotate") if k in opts}
    e, rp = oracle.plan(rot, dict(w=hdr.w, h=hdr.h, bands=hdr.bands, type=3, orientation=hdr.orientation))
    assert e == 0 and rp.n_steps >= 1
    upright = oracle.execute(rp, full)
    buf2 = codec.encode(upright, "jpeg", 100)
    inp = dict(w=hdr.w, h=hdr.h, bands=hdr.bands, type=1, orientation=hdr.orientation)
    e, p0 = oracle.plan(opts, inp)
    assert e == 0 and p0.load_shrink > 1, "the case must shrink on load"
    px = codec.decode(buf2, p0.load_shrink)
    swap = upright.shape[:2] != full.shape[:2]
    dw, dh = (px.shape[0], px.shape[1]) if swap else (px.shape[1], px.shape[0])
    e, p1 = oracle.plan(opts, dict(inp, decoded_w=dw, decoded_h=dh))
    assert e == 0
    want_px = oracle.execute(_drop_leading(p1, rp.n_steps, px.shape[1], px.shape[0]), px)
    assert (want_px.shape[1], want_px.shape[0]) == (p1.out_w, p1.out_h)
    want = codec.encode(want_px, "jpeg")
    assert size_of(got.body) == (p1.out_w, p1.out_h)
    assert got.body == want, "engine output differs from the stage-by-stage chain"
    # the test tells the two sequences apart: rotating the shrink-on-load decode instead
    # (the pre-r04 engine) gives other pixels
    old = oracle.execute(p1, codec.decode(buf, p0.load_shrink))
    assert old.shape == want_px.shape and not np.array_equal(old, want_px)
