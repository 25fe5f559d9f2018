"""Host codec boundary (CPU): type sniffing, headers, JPEG DCT shrink-on-load,
encode round trips, and Info over the reference's testdata fixtures."""
import json
import os

import numpy as np
import pytest

from conftest import ROOT

TESTDATA = os.path.join(ROOT, "tests", "golden", "testdata")
codec = pytest.importorskip("imaginary_amd.codec")


def read(name):
    with open(os.path.join(TESTDATA, name), "rb") as f:
        return f.read()


@pytest.mark.parametrize("name,typ,w,h,bands,orient", [
    ("imaginary.jpg", "jpeg", 550, 740, 3, 1), ("large.jpg", "jpeg", 1920, 1080, 3, 0),
    ("test.png", "png", 400, 300, 4, 0), ("test.webp", "webp", 550, 368, 3, 0),
    ("smart-crop.jpg", "jpeg", 700, 1050, 3, 0)])
def test_headers_match_the_fixtures(name, typ, w, h, bands, orient):
    hd = codec.header(read(name))
    assert (hd.type, hd.w, hd.h, hd.bands, hd.orientation) == (typ, w, h, bands, orient)


@pytest.mark.parametrize("s", [2, 4, 8])
def test_jpeg_shrink_on_load_sizes(s):
    """libjpeg scale 1/s gives ceil(w/s) x ceil(h/s) — what the planner assumes."""
    px = codec.decode(read("large.jpg"), s)
    assert px.shape == (-(-1080 // s), -(-1920 // s), 3)


def test_encode_roundtrip_lossless_png():
    rng = np.random.default_rng(3)
    for b in (1, 2, 3, 4):
        px = rng.integers(0, 256, (17, 23, b), dtype=np.uint8)
        back = codec.decode(codec.encode(px, "png"))
        assert np.array_equal(back, px)


def test_sniff_and_mime():
    assert codec.sniff_type(read("test.webp")) == "webp"
    assert codec.mime_type("jpeg") == "image/jpeg"
    assert codec.sniff_type(b"nope") == "unknown"


def test_info_is_host_only():
    from imaginary_amd import imaginary as im
    info = json.loads(im.Info(read("test.png"), im.ImageOptions()).body)
    assert info == {"width": 400, "height": 300, "type": "png", "space": "srgb", "hasAlpha": True,
                    "hasProfile": False, "channels": 4, "orientation": 0}
