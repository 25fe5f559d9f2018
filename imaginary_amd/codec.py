"""Host codec boundary: encoded bytes <-> decoded pixels.

The north star keeps decode/encode on the host (libvips in the Go service);
the engine only sees decoded pixels.  libvips is not installed in this image,
so this module is the host-side stand-in used by the byte-level operation
layer (imaginary.process_bytes) and its tests: Pillow decodes and encodes, and
JPEG shrink-on-load uses libjpeg's DCT-domain scaling (Pillow ``draft``), the
same mechanism libvips' jpegload ``shrink`` uses.  It never
touches pixels the engine computes — only the codec work either side of it.

Reference points: bimg.DetermineImageType / imaginary type.go:46-60 (MIME),
image.go:96-112 (encode fallback to JPEG for WEBP/HEIF/AVIF).
"""
from __future__ import annotations

import io
from dataclasses import dataclass
from typing import Optional

import numpy as np

try:
    from PIL import Image as _PIL
except ImportError:  # pragma: no cover - the codec is optional for the pixel engine
    _PIL = None

MIME = {"jpeg": "image/jpeg", "png": "image/png", "webp": "image/webp", "gif": "image/gif",
        "tiff": "image/tiff", "svg": "image/svg+xml", "pdf": "application/pdf", "heif": "image/heif",
        "avif": "image/avif"}
_PIL_FORMAT = {"jpeg": "JPEG", "png": "PNG", "webp": "WEBP", "gif": "GIF", "tiff": "TIFF"}
DEFAULT_QUALITY = 75  # bimg default Quality (libvips saver default Q)


class CodecError(Exception):
    pass


def sniff_type(buf: bytes) -> str:
    """bimg.DetermineImageType: magic bytes -> type name ("unknown" if none)."""
    b = bytes(buf[:16])
    if b[:3] == b"\xff\xd8\xff":
        return "jpeg"
    if b[:8] == b"\x89PNG\r\n\x1a\n":
        return "png"
    if b[:4] == b"RIFF" and b[8:12] == b"WEBP":
        return "webp"
    if b[:6] in (b"GIF87a", b"GIF89a"):
        return "gif"
    if b[:4] in (b"II*\x00", b"MM\x00*"):
        return "tiff"
    if b[:4] == b"%PDF":
        return "pdf"
    if b[4:8] == b"ftyp":
        return "avif" if b[8:12] in (b"avif", b"avis") else "heif"
    if b"<svg" in bytes(buf[:512]) or b[:5] == b"<?xml":
        return "svg"
    return "unknown"


def mime_type(t: str) -> str:
    """imaginary type.go GetImageMimeType."""
    return MIME.get(t, "application/octet-stream")


@dataclass
class Header:
    w: int
    h: int
    bands: int
    type: str
    orientation: int


_BANDS = {"L": 1, "LA": 2, "RGB": 3, "RGBA": 4}


def _open(buf: bytes):
    if _PIL is None:
        raise CodecError("no host codec (Pillow) available")
    try:
        return _PIL.open(io.BytesIO(buf))
    except Exception as e:  # noqa: BLE001 - any decoder failure is a bad request
        raise CodecError(f"cannot decode image: {e}") from e


def _target_mode(im) -> str:
    if im.mode in _BANDS:
        return im.mode
    if im.mode in ("P", "PA"):
        return "RGBA" if ("transparency" in im.info or im.mode == "PA") else "RGB"
    if im.mode in ("I;16", "I", "F", "1"):
        return "L"
    return "RGBA" if "A" in im.mode else "RGB"


def header(buf: bytes) -> Header:
    """What bimg reads before planning: size, bands, type, EXIF orientation."""
    im = _open(buf)
    orient = 0
    try:
        orient = int(im.getexif().get(274, 0) or 0)
    except Exception:  # noqa: BLE001
        orient = 0
    return Header(im.size[0], im.size[1], _BANDS[_target_mode(im)], sniff_type(buf), orient)


def decode(buf: bytes, shrink: int = 1) -> np.ndarray:
    """Decode to (h, w, bands) uint8.  shrink in (2, 4, 8) uses the JPEG DCT-domain
    downscale (libjpeg scale_denom), giving ceil(w / shrink) x ceil(h / shrink)."""
    im = _open(buf)
    mode = _target_mode(im)
    if shrink > 1 and im.format == "JPEG":
        w, h = im.size
        im.draft(mode if mode in ("L", "RGB") else "RGB", ((w + shrink - 1) // shrink, (h + shrink - 1) // shrink))
    if im.mode != mode:
        im = im.convert(mode)
    a = np.asarray(im, dtype=np.uint8)
    return a[:, :, None] if a.ndim == 2 else np.ascontiguousarray(a)


def encode(px: np.ndarray, t: str, quality: Optional[int] = None, compression: Optional[int] = None) -> bytes:
    """Encode (h, w, bands) uint8 pixels as type t."""
    if _PIL is None:
        raise CodecError("no host codec (Pillow) available")
    fmt = _PIL_FORMAT.get(t)
    if fmt is None:
        raise CodecError(f"cannot encode to {t}")
    px = px if px.ndim == 3 else px[:, :, None]
    mode = {1: "L", 2: "LA", 3: "RGB", 4: "RGBA"}[px.shape[2]]
    im = _PIL.fromarray(px[:, :, 0] if mode == "L" else px, mode)
    if fmt == "JPEG" and mode in ("LA", "RGBA"):  # JPEG has no alpha: libvips drops it
        im = im.convert("L" if mode == "LA" else "RGB")
    out = io.BytesIO()
    kw = {}
    if fmt in ("JPEG", "WEBP"):
        kw["quality"] = quality or DEFAULT_QUALITY
    if fmt == "JPEG":
        # libvips jpegsave's automatic chroma subsampling: 4:2:0 below Q 90, 4:4:4 from Q 90
        kw["subsampling"] = 0 if kw["quality"] >= 90 else 2
    if fmt == "PNG" and compression is not None:
        kw["compress_level"] = compression
    try:
        im.save(out, fmt, **kw)
    except Exception as e:  # noqa: BLE001
        raise CodecError(f"encode {t}: {e}") from e
    return out.getvalue()
