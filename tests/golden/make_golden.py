"""Regenerate tests/golden/*.npz (run in the build container, where
/root/reference exists; the GPU box only reads the committed .npz files).

Inputs: seeded random images plus small crops of the reference's own fixtures
(testdata/large.jpg, smart-crop.jpg, test.png) decoded with Pillow — data, not
source.  Expected outputs: the CPU oracle (oracle/vips_ref.c).  These pin the
oracle against regressions and give the GPU tests fixed vectors; they are NOT
libvips outputs (no libvips here: "parity unpinned" for pixel values).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle as o  # noqa: E402

TESTDATA = "/root/reference/testdata"


def natural():
    from PIL import Image
    out = {}
    im = Image.open(os.path.join(TESTDATA, "large.jpg")).convert("RGB")
    out["large_crop"] = np.asarray(im)[400:496, 800:928].copy()          # 96 x 128 x 3
    im = Image.open(os.path.join(TESTDATA, "smart-crop.jpg"))
    im.draft("RGB", (im.width // 4, im.height // 4))
    out["smart_quarter"] = np.asarray(im.convert("RGB")).copy()          # libjpeg 1/4 scale
    im = Image.open(os.path.join(TESTDATA, "test.png")).convert("RGBA")
    out["png_crop"] = np.asarray(im)[50:114, 100:180].copy()             # 64 x 80 x 4
    return out


def main():
    rng = np.random.default_rng(20241220)
    nat = natural()
    ops = {}

    def add(name, src, out):
        ops[name + "__in"] = np.ascontiguousarray(src)
        ops[name + "__out"] = out

    add("reduce__2.0__2.0__rand", rng.integers(0, 256, (40, 64, 3), dtype=np.uint8), None)
    ops["reduce__2.0__2.0__rand__out"] = o.reduce(ops["reduce__2.0__2.0__rand__in"], 2.0, 2.0)
    for s in (2.0, 1.6, 2.4666666666666666):
        add(f"reduce__{s}__{s}__large", nat["large_crop"], o.reduce(nat["large_crop"], s, s))
    add("reduce__2.0__2.0__png", nat["png_crop"], o.reduce(nat["png_crop"], 2.0, 2.0))
    add("shrink__4__4__large", nat["large_crop"], o.shrink(nat["large_crop"], 4, 4))
    add("shrink__3__5__png", nat["png_crop"], o.shrink(nat["png_crop"], 3, 5))
    add("blur__5.0__png", nat["png_crop"], o.gaussblur(nat["png_crop"], 5.0))
    add("blur__1.5__large", nat["large_crop"], o.gaussblur(nat["large_crop"], 1.5))
    np.savez_compressed(os.path.join(HERE, "ops.npz"), **ops)

    sc = nat["smart_quarter"]
    l, t = o.smartcrop_origin(sc, 100, 100)
    l2, t2 = o.smartcrop_origin(nat["large_crop"], 64, 64)
    np.savez_compressed(os.path.join(HERE, "smartcrop.npz"), smart_quarter=sc,
                        smart_quarter_100x100=np.array([l, t], np.int32), large_crop=nat["large_crop"],
                        large_crop_64x64=np.array([l2, t2], np.int32))
    # known-answer facts of the restated libvips tables
    np.savez_compressed(os.path.join(HERE, "tables.npz"),
                        reduce_2_0=o.reduce_table(2.0), reduce_1_6=o.reduce_table(1.6),
                        gauss_5_0=np.array(o.gaussmat(5.0)[0], np.int32))
    for f in ("ops.npz", "smartcrop.npz", "tables.npz"):
        print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
