"""Writes tests/golden/testdata/orient6.jpg: a synthetic 1200x900 JPEG (Q90) whose EXIF
orientation is 6 (rotate 90 clockwise to display), so bimg rotates it and, for a
downsizing request, re-encodes the upright image before shrink-on-load.  The
reference's own imaginary.jpg has orientation 1, so this fixture is generated here:
    python tests/golden/make_rotated_jpeg.py"""
import io
import os

import numpy as np
from PIL import Image

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "testdata", "orient6.jpg")


def make() -> bytes:
    h, w = 900, 1200
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    px = np.empty((h, w, 3), np.uint8)
    px[..., 0] = (127.5 + 127.5 * np.sin(x / 37.0) * np.cos(y / 53.0)).astype(np.uint8)
    px[..., 1] = (255.0 * x / (w - 1)).astype(np.uint8)
    px[..., 2] = ((x // 16 + y // 16) % 2 * 200 + 25).astype(np.uint8)  # hard edges
    px[100:140, 50:700] = (250, 20, 20)  # an asymmetric mark: a wrong rotation shows
    exif = Image.Exif()
    exif[274] = 6
    out = io.BytesIO()
    Image.fromarray(px, "RGB").save(out, "JPEG", quality=90, exif=exif.tobytes())
    return out.getvalue()


if __name__ == "__main__":
    with open(OUT, "wb") as f:
        f.write(make())
    print(OUT, os.path.getsize(OUT))
