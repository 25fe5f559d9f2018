"""Host-side mirror of imaginary's operation layer over the MI355X engine.

Reference: image.go (OperationsMap 15-32, Process 81-113, Resize 115, Fit 139,
calculateDestinationFitDimension 190, Enlarge 202, Extract 213, Crop 226,
SmartCrop 236, Rotate 247, Flip 267, Flop 273, Thumbnail 279, Zoom 286,
WatermarkImage 343, GaussianBlur 372, Pipeline 379), options.go (ImageOptions
11-52, BimgOptions 128-172) and params.go (buildParamsFromQuery 354-366,
parseInt 376-390, parseExtendMode 421-437, parseGravity 439-453).

Same operation names, argument meaning and error behaviour; the one change is
the seam: Process() hands DECODED pixels to libmipx (mipx_plan_make +
mipx_process) instead of calling bimg.Resize on encoded bytes.  Codec decode /
encode stay with the host (here: a `Decoded` value carrying the pixels plus
the header facts bimg would read: type, EXIF orientation).  Operations the
engine does not implement raise EngineUnsupported — the Go shim falls back to
bimg.Resize there.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import json
import math
import re
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

import numpy as np

from . import _abi, codec
from .engine import Engine, fit_dimension, make_input, make_opts, plan_chain, plan_make

HTTP_BAD_REQUEST = 400
HTTP_NOT_ACCEPTABLE = 406


class ImaginaryError(Exception):
    """error.go NewError: message + HTTP status."""

    def __init__(self, message: str, code: int = HTTP_BAD_REQUEST):
        super().__init__(message)
        self.message = message
        self.code = code


class EngineUnsupported(ImaginaryError):
    """The plan needs an op libmipx lacks (MIPX_EUNSUPPORTED): caller falls back to bimg."""

    def __init__(self, message: str):
        super().__init__(message, 501)


@dataclass
class IsDefinedField:
    flip: bool = False
    flop: bool = False
    force: bool = False
    embed: bool = False
    no_crop: bool = False
    no_rotation: bool = False


@dataclass
class ImageOptions:
    """options.go:11-52 (pixel-relevant subset)."""
    width: int = 0
    height: int = 0
    area_width: int = 0
    area_height: int = 0
    rotate: int = 0
    top: int = 0
    left: int = 0
    factor: int = 0
    flip: bool = False
    flop: bool = False
    force: bool = False
    embed: bool = False
    no_crop: bool = False
    no_rotation: bool = False
    opacity: float = 0.0
    sigma: float = 0.0
    min_ampl: float = 0.0
    image: str = ""
    type: str = ""
    aspect_ratio: str = ""
    background: List[int] = field(default_factory=list)
    color: List[int] = field(default_factory=list)   # text watermark colour (not a pixel-engine op)
    extend: int = 1          # bimg.ExtendCopy default (params.go:342, 356)
    colorspace: int = 0      # bimg.Interpretation (params.go:260, parseColorspace 392)
    quality: int = 0
    compression: int = 0
    text: str = ""           # Watermark (text): pango rendering, not a pixel-engine op
    gravity: int = 0
    operations: List[Dict[str, Any]] = field(default_factory=list)
    is_defined: IsDefinedField = field(default_factory=IsDefinedField)


@dataclass
class Decoded:
    """What the host codec hands over: pixels (h, w, bands) + header facts."""
    pixels: np.ndarray
    type: str = "png"
    orientation: int = 0
    # full-resolution header size when `pixels` were decoded with shrink-on-load
    header_w: int = 0
    header_h: int = 0

    @property
    def w(self):
        return self.header_w or self.pixels.shape[1]

    @property
    def h(self):
        return self.header_h or self.pixels.shape[0]


# ---- params.go helpers -----------------------------------------------------------
# Go's strconv semantics restated exactly (params_test.go's tables pass byte for byte:
# tests/test_params.py).  The helpers return Go's (value, error) pair: Go returns a
# value even when it also returns an error, and the tables check both.
_GO_DEC = re.compile(r"[+-]?(?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][+-]?[0-9]+)?\Z")
_GO_HEX = re.compile(r"[+-]?0[xX](?:[0-9a-fA-F]+\.?[0-9a-fA-F]*|\.[0-9a-fA-F]+)[pP][+-]?[0-9]+\Z")
_GO_SPECIAL = {"inf": math.inf, "+inf": math.inf, "-inf": -math.inf, "infinity": math.inf,
               "+infinity": math.inf, "-infinity": -math.inf, "nan": math.nan}


class GoParseError(ValueError):
    """strconv.NumError: ErrSyntax / ErrRange."""


def _go_parse_float(v: str):
    """strconv.ParseFloat(v, 64): no surrounding space, no underscores in decimal
    literals; inf / infinity / nan in any case; hex floats need a p exponent.  A
    syntax error gives (0, err); a range error gives (+-Inf, err)."""
    low = v.lower()
    if low in _GO_SPECIAL:
        return _GO_SPECIAL[low], None
    if _GO_DEC.match(v):
        f = float(v)
    elif _GO_HEX.match(v):
        sign = -1.0 if v[0] == "-" else 1.0
        try:
            f = sign * float.fromhex(v.lstrip("+-"))
        except OverflowError:
            return sign * math.inf, GoParseError(f'strconv.ParseFloat: parsing "{v}": value out of range')
    else:
        return 0.0, GoParseError(f'strconv.ParseFloat: parsing "{v}": invalid syntax')
    if math.isinf(f):
        return f, GoParseError(f'strconv.ParseFloat: parsing "{v}": value out of range')
    return f, None


def parse_float(v: str):
    """params.go:384-390: |strconv.ParseFloat|; "" is (0, nil)."""
    if v == "":
        return 0.0, None
    f, err = _go_parse_float(v)
    return abs(f), err


def parse_int(v: str):
    """params.go:376-382: int(math.Floor(f + 0.5)) of parse_float; "" is (0, nil)."""
    if v == "":
        return 0, None
    f, err = parse_float(v)
    if math.isinf(f) or math.isnan(f):  # Go's int() of +Inf / NaN on amd64: the minimum int64
        return -(1 << 63), err
    return int(math.floor(f + 0.5)), err


_GO_BOOLS = {"1": True, "t": True, "T": True, "TRUE": True, "true": True, "True": True,
             "0": False, "f": False, "F": False, "FALSE": False, "false": False, "False": False}


def parse_bool(v: str):
    """params.go:369-374: "" is (false, nil), else strconv.ParseBool's exact set."""
    if v == "":
        return False, None
    if v in _GO_BOOLS:
        return _GO_BOOLS[v], None
    return False, GoParseError(f'strconv.ParseBool: parsing "{v}": invalid syntax')


def _go_trim_lower(v: str) -> str:
    return v.lower().strip()   # strings.TrimSpace(strings.ToLower(v))


def parse_extend_mode(v: str) -> int:
    """params.go:421-437: bimg.Extend, mirror by default."""
    m = {"white": 4, "black": 0, "copy": 1, "background": 5, "lastpixel": 6}
    return m.get(_go_trim_lower(v), 3)


def parse_gravity(v: str) -> int:
    """params.go:439-453: bimg.Gravity, centre by default."""
    m = {"south": 3, "north": 1, "east": 2, "west": 4, "smart": 5}
    return m.get(_go_trim_lower(v), 0)


def parse_colorspace(v: str) -> int:
    """params.go:392-397: exactly "bw" -> InterpretationBW, anything else sRGB."""
    return _abi.INTERPRETATION_BW if v == "bw" else _abi.INTERPRETATION_SRGB


def _go_parse_uint8(v: str) -> int:
    """strconv.ParseUint(v, 10, 8) with the error dropped, as params.go:404 does: a
    syntax error (signs, spaces, letters, "") gives 0, a range error gives 255."""
    if not v or not all("0" <= c <= "9" for c in v):
        return 0
    return min(int(v), 255)


def parse_color(v: str) -> List[int]:
    """params.go:399-409: comma-split, TrimSpace, ParseUint(.., 10, 8)."""
    return [_go_parse_uint8(x.strip()) for x in v.split(",")] if v != "" else []


def parse_json_operations(data: str) -> List[Dict[str, Any]]:
    """params.go:411-419: shorter than 2 bytes is no operations; otherwise a JSON array
    of {"operation", "ignore_failure", "params"} with unknown fields refused (Go's
    DisallowUnknownFields; encoding/json matches field names case-insensitively)."""
    if len(data) < 2:
        return []
    ops = json.loads(data)
    if ops is None:
        return []
    if not isinstance(ops, list):
        raise GoParseError("json: cannot unmarshal into Go value of type main.PipelineOperations")
    out = []
    for op in ops:
        if op is None:
            op = {}
        if not isinstance(op, dict):
            raise GoParseError("json: cannot unmarshal into Go struct field of type main.PipelineOperation")
        d: Dict[str, Any] = {"operation": "", "ignore_failure": False, "params": None}
        for k, val in op.items():
            key = {"operation": "operation", "ignore_failure": "ignore_failure", "params": "params"}.get(k.lower())
            if key is None:
                raise GoParseError(f'json: unknown field "{k}"')
            want = {"operation": str, "ignore_failure": bool, "params": dict}[key]
            if val is not None and not isinstance(val, want):
                raise GoParseError(f"json: cannot unmarshal into Go struct field PipelineOperation.{key}")
            if val is not None:
                d[key] = val
        out.append(d)
    return out


# coerceType* (params.go:62-102): a pipeline operation's params are JSON values
class UnsupportedValue(ValueError):
    """params.go:14 ErrUnsupportedValue."""


def coerce_type_int(p):
    if isinstance(p, bool):
        raise UnsupportedValue("unsupported value")
    if isinstance(p, int):
        return p
    if isinstance(p, float):
        return int(p)              # Go int(float64): truncation toward zero
    if isinstance(p, str):
        v, err = parse_int(p)
        if err:
            raise err
        return v
    raise UnsupportedValue("unsupported value")


def coerce_type_float(p):
    if isinstance(p, bool):
        raise UnsupportedValue("unsupported value")
    if isinstance(p, (int, float)):
        return float(p)            # as given: no abs() for numbers (params.go:75-85)
    if isinstance(p, str):
        v, err = parse_float(p)
        if err:
            raise err
        return v
    raise UnsupportedValue("unsupported value")


def coerce_type_bool(p):
    if isinstance(p, bool):
        return p
    if isinstance(p, str):
        v, err = parse_bool(p)
        if err:
            raise err
        return v
    raise UnsupportedValue("unsupported value")


def coerce_type_string(p):
    if isinstance(p, str):
        return p
    raise UnsupportedValue("unsupported value")


_INT_PARAMS = {"width": "width", "height": "height", "areawidth": "area_width", "areaheight": "area_height",
               "rotate": "rotate", "top": "top", "left": "left", "factor": "factor", "quality": "quality",
               "compression": "compression"}
_FLOAT_PARAMS = {"sigma": "sigma", "minampl": "min_ampl", "opacity": "opacity"}
_BOOL_PARAMS = {"flip": "flip", "flop": "flop", "force": "force", "embed": "embed", "nocrop": "no_crop",
                "norotation": "no_rotation"}
_STR_PARAMS = {"type": "type", "aspectratio": "aspect_ratio", "image": "image", "text": "text"}


def _coerce(o: ImageOptions, k: str, v) -> None:
    """paramTypeCoercions (params.go:20-60) for the pixel-relevant keys."""
    if k in _INT_PARAMS:
        setattr(o, _INT_PARAMS[k], coerce_type_int(v))
    elif k in _FLOAT_PARAMS:
        val = coerce_type_float(v)
        setattr(o, _FLOAT_PARAMS[k], float(np.float32(val)) if k == "opacity" else val)  # Opacity is float32
    elif k in _BOOL_PARAMS:
        setattr(o.is_defined, _BOOL_PARAMS[k], True)
        setattr(o, _BOOL_PARAMS[k], coerce_type_bool(v))
    elif k in _STR_PARAMS:
        setattr(o, _STR_PARAMS[k], coerce_type_string(v))
    elif k in ("extend", "gravity", "colorspace", "background", "color", "operations"):
        if not isinstance(v, str):
            if k == "operations" and isinstance(v, list):   # already decoded (the Python mirror's callers)
                o.operations = v
                return
            raise UnsupportedValue("unsupported value")
        if k == "extend":
            o.extend = parse_extend_mode(v)
        elif k == "gravity":
            o.gravity = parse_gravity(v)
        elif k == "colorspace":
            o.colorspace = parse_colorspace(v)
        elif k == "background":
            o.background = parse_color(v)
        elif k == "color":
            o.color = parse_color(v)
        else:
            o.operations = parse_json_operations(v)


def _build_params(items) -> ImageOptions:
    o = ImageOptions()   # Extend defaults to bimg.ExtendCopy (params.go:342, 356)
    for k, v in items:
        try:
            _coerce(o, k, v)
        except (ValueError, json.JSONDecodeError) as e:
            raise ImaginaryError(f"error processing parameter {k!r} with value {v!r}: {e}") from e
    return o


def build_params_from_query(query: Dict[str, Any]) -> ImageOptions:
    """params.go:354-366.  A query value is a string (url.Values.Get: the first of a
    list); a value that is already typed (the Python callers' dicts) coerces as a
    pipeline param would."""
    return _build_params((k, (v[0] if v else "") if isinstance(v, list) and k != "operations" else v)
                         for k, v in query.items())


def build_params_from_operation(op: Dict[str, Any]) -> ImageOptions:
    """params.go:340-352: a pipeline operation's JSON params."""
    return _build_params((op.get("params") or {}).items())


# ---- options.go BimgOptions ----------------------------------------------------------
def _aspect(o: ImageOptions, w: int, h: int):
    if (w != 0 and h != 0) or (w == 0 and h == 0) or not o.aspect_ratio:
        return w, h
    parts = o.aspect_ratio.strip().lower().split(":")
    if len(parts) < 2:
        return w, h
    ar = {"width": int(parts[0] or 0), "height": int(parts[1] or 0)}
    if w != 0:
        h = int(w / ar["width"]) * ar["height"]   # Go integer arithmetic
    else:
        w = int(h / ar["height"]) * ar["width"]
    return w, h


def bimg_options(o: ImageOptions) -> Dict[str, Any]:
    """options.go:128-172 -> the mipx_opts field dict."""
    b = dict(width=o.width, height=o.height, flip=int(o.flip), flop=int(o.flop),
             no_auto_rotate=int(o.no_rotation), force=int(o.force), gravity=o.gravity,
             embed=int(o.embed), extend=o.extend, rotate=o.rotate, interpretation=o.colorspace)
    if o.background:
        b["background"] = (list(o.background) + [0, 0, 0])[:3]
    b["width"], b["height"] = _aspect(o, o.width, o.height)
    if o.sigma > 0 or o.min_ampl > 0:
        b["sigma"], b["min_ampl"] = o.sigma, o.min_ampl
    if o.type:
        b["type"] = o.type            # encode-side: bimg Type (options.go:138)
    if o.quality:
        b["quality"] = o.quality
    if o.compression:
        b["compression"] = o.compression
    return b


# ---- Process (image.go:81) ------------------------------------------------------------
_ENGINE: Optional[Engine] = None


def engine() -> Engine:
    """The process-wide request engine.  An engine already running in this process is
    used as it is, whoever started it and with whatever configuration (mipx_init
    refuses a second, different configuration, so this never calls it then); after an
    mipx_shutdown, or before any engine, a default one is started."""
    global _ENGINE
    if _abi.lib.mipx_queue_count() > 0:
        if _ENGINE is None:
            _ENGINE = Engine.attach()
        return _ENGINE
    _ENGINE = Engine()
    return _ENGINE


Decoder = Callable[[Decoded, int], np.ndarray]


@dataclass
class Image:
    """image.go:34-37."""
    body: bytes
    mime: str


_ENCODE_ONLY = ("type", "quality", "compression")


def _placeholder(h: int, w: int, b: int) -> np.ndarray:
    """Stand-in pixels of a planned-but-not-run stage: only the shape is read."""
    return np.lib.stride_tricks.as_strided(np.zeros(1, np.uint8), (h, w, b), (0, 0, 0), writeable=False)


def _run(plan, px, wm):
    try:
        return engine().process(plan, px, wm)
    except _abi.MipxError as e:
        if e.code == _abi.MIPX_EUNSUPPORTED:
            raise EngineUnsupported(str(e)) from e
        raise ImaginaryError(f"image processing error: {e}", 500) from e


def process(img, opts: Dict[str, Any], wm=None, redecode: Optional[Decoder] = None, chain: Optional[list] = None):
    """image.go:81-113 Process with bimg.Resize's pixel work on the GPU.

    Encoded bytes in -> Image out (the drop-in: host codec, engine, host codec);
    a Decoded in -> pixels out (the engine alone, for callers that own the codec).
    `redecode(img, s)` is the host codec's shrink-on-load (libjpeg scale 1/s);
    without one, a plan that asks for load_shrink > 1 is rejected.
    With `chain` (a list), a Decoded input is planned but not run: (plan, pixels,
    watermark) is appended and placeholder pixels of the output shape returned
    (Pipeline fuses the stages into one device-resident plan)."""
    if isinstance(img, (bytes, bytearray, memoryview)):
        return process_bytes(bytes(img), opts, wm)
    opts = {k: v for k, v in opts.items() if k not in _ENCODE_ONLY}
    px = img.pixels if img.pixels.ndim == 3 else img.pixels[:, :, None]
    inp = make_input(img.w, img.h, px.shape[2], img.type, img.orientation)
    if wm is not None:
        wm = wm if wm.ndim == 3 else wm[:, :, None]
        opts = dict(opts, wm_enable=1)
        inp.wm_w, inp.wm_h, inp.wm_bands = wm.shape[1], wm.shape[0], wm.shape[2]
    try:
        plan = plan_make(make_opts(**opts), inp)
        if plan.load_shrink > 1:
            if redecode is None:
                raise ImaginaryError("shrink-on-load requested but no host decoder given", 500)
            px = redecode(img, plan.load_shrink)
            inp.decoded_w, inp.decoded_h = px.shape[1], px.shape[0]
            plan = plan_make(make_opts(**opts), inp)
        elif img.header_w and (img.header_w, img.header_h) != (px.shape[1], px.shape[0]):
            raise ImaginaryError("decoded size does not match the header", 500)
        if chain is not None:
            chain.append((plan, px, wm))
            return _placeholder(plan.out_h, plan.out_w, plan.out_bands)
        return engine().process(plan, px, wm)
    except _abi.MipxError as e:
        if e.code == _abi.MIPX_EUNSUPPORTED:
            raise EngineUnsupported(str(e)) from e
        raise ImaginaryError(f"image processing error: {e}", 500) from e


def process_bytes(buf: bytes, opts: Dict[str, Any], wm=None) -> Image:
    """Process(buf, opts) over encoded bytes: header -> plan -> decode (with the
    plan's shrink-on-load) -> engine -> encode; WEBP/HEIF/AVIF encode failures
    retry as JPEG (image.go:97-107); MIME from the output bytes (image.go:109-112)."""
    opts = dict(opts)
    out_type = str(opts.pop("type", "") or "")
    quality = int(opts.pop("quality", 0) or 0)
    compression = opts.pop("compression", 0) or None
    try:
        hdr = codec.header(buf)
        wm_px = codec.decode(bytes(wm)) if isinstance(wm, (bytes, bytearray)) else wm
    except codec.CodecError as e:
        raise ImaginaryError(str(e), HTTP_BAD_REQUEST) from e

    def redecode(_img: Decoded, s: int) -> np.ndarray:
        return codec.decode(buf, s)

    itype = hdr.type if hdr.type in _abi.TYPES else "unknown"
    if wm_px is not None:
        opts = dict(opts, wm_enable=1)
    # plan on the header first: the decode depends on the plan's shrink-on-load
    inp = make_input(hdr.w, hdr.h, hdr.bands, itype, hdr.orientation)
    if wm_px is not None:
        inp.wm_w, inp.wm_h, inp.wm_bands = wm_px.shape[1], wm_px.shape[0], (wm_px.shape[2] if wm_px.ndim == 3 else 1)
    try:
        plan = plan_make(make_opts(**opts), inp)
    except _abi.MipxError as e:
        if e.code == _abi.MIPX_EUNSUPPORTED:
            raise EngineUnsupported(str(e)) from e
        raise ImaginaryError(f"image processing error: {e}", 500) from e
    rotates = any(step[0] in ("rot", "flip") for step in plan.describe())
    if plan.load_shrink > 1 and itype == "jpeg" and rotates and not opts.get("no_auto_rotate"):
        px = _rotate_reencode_shrink_on_load(buf, hdr, itype, opts, wm_px)
    elif plan.load_shrink > 1:  # process() re-plans on the codec-shrunk size
        src = Decoded(np.zeros((1, 1, hdr.bands), np.uint8), itype, hdr.orientation, hdr.w, hdr.h)
        px = process(src, opts, wm=wm_px, redecode=redecode)
    else:
        px = process(Decoded(codec.decode(buf), itype, hdr.orientation), opts, wm=wm_px)
    t = out_type or (hdr.type if hdr.type in ("jpeg", "png", "webp", "gif", "tiff") else "png")
    try:
        body = codec.encode(px, t, quality or None, compression)
    except codec.CodecError as e:
        if t not in ("webp", "heif", "avif"):
            raise ImaginaryError(f"image processing error: {e}", 500) from e
        body = codec.encode(px, "jpeg", quality or None)
    return Image(body, codec.mime_type(codec.sniff_type(body)))


_ROTATION_KEYS = ("rotate", "flip", "flop", "no_auto_rotate")
JPEG_REENCODE_QUALITY = 100  # bimg getImageBuffer: vips_jpegsave_bridge(strip 1, Q 100, no interlace)


def _drop_leading_steps(plan, k: int, w: int, h: int):
    """The plan without its first k steps, taking a w x h input."""
    rest = _abi.MipxPlan()
    C.memmove(C.byref(rest), C.byref(plan), C.sizeof(plan))
    rest.in_w, rest.in_h, rest.load_shrink = w, h, 1
    rest.n_steps = plan.n_steps - k
    for i in range(rest.n_steps):
        rest.steps[i] = plan.steps[i + k]
    return rest


def _rotate_reencode_shrink_on_load(buf: bytes, hdr, itype: str, opts: Dict[str, Any], wm_px):
    """bimg 1.1.9 resizer() for a JPEG that rotates or flips (EXIF orientation or an
    explicit rotate / flip / flop) and then shrinks on load (image.go:96 -> bimg
    resizer.go): rotateAndFlipImage runs on the FULL-size decode, the rotated image is
    re-encoded (getImageBuffer: jpegsave, Q 100, metadata stripped) and that buffer is
    what shrinkOnLoad decodes at 1/s; every later step is the plan's own (bimg computes
    its factors before the re-encode, from the caller's options).
      1. decode at full size;
      2. rotate / flip on the engine (the plan's rotation steps, at full size);
      3. re-encode with the host codec (JPEG Q 100, no EXIF);
      4. decode that with the DCT shrink the plan asks for;
      5. run the rest of the plan on it."""
    full = codec.decode(buf)
    rot_opts = {k: opts[k] for k in _ROTATION_KEYS if k in opts}
    rot_plan = plan_make(make_opts(**rot_opts), make_input(full.shape[1], full.shape[0], full.shape[2], "png",
                                                           hdr.orientation))
    rot_ops = [step[0] for step in rot_plan.describe()]
    if not rot_ops or any(op not in ("rot", "flip") for op in rot_ops):
        raise ImaginaryError(f"rotation plan {rot_ops}: expected rot / flip steps only", 500)
    upright = _run(rot_plan, full, None)
    buf2 = codec.encode(upright, "jpeg", JPEG_REENCODE_QUALITY)
    inp = make_input(hdr.w, hdr.h, hdr.bands, itype, hdr.orientation)
    if wm_px is not None:
        wm_px = wm_px if wm_px.ndim == 3 else wm_px[:, :, None]
        opts = dict(opts, wm_enable=1)
        inp.wm_w, inp.wm_h, inp.wm_bands = wm_px.shape[1], wm_px.shape[0], wm_px.shape[2]
    try:
        plan = plan_make(make_opts(**opts), inp)
        px = codec.decode(buf2, plan.load_shrink)
        # the decode the plan was made for is the un-rotated image at 1/s: same size,
        # axes swapped by a quarter turn
        swap = upright.shape[:2] != full.shape[:2]
        inp.decoded_w, inp.decoded_h = (px.shape[0], px.shape[1]) if swap else (px.shape[1], px.shape[0])
        plan = plan_make(make_opts(**opts), inp)
    except _abi.MipxError as e:
        if e.code == _abi.MIPX_EUNSUPPORTED:
            raise EngineUnsupported(str(e)) from e
        raise ImaginaryError(f"image processing error: {e}", 500) from e
    steps = plan.describe()
    k = len(rot_ops)
    if [st[0] for st in steps[:k]] != rot_ops:
        raise ImaginaryError(f"plan {steps}: expected the rotation steps {rot_ops} first", 500)
    rest = _drop_leading_steps(plan, k, px.shape[1], px.shape[0])
    if rest.n_steps == 0:
        return px
    return _run(rest, px, wm_px)


# ---- image.go operations ----------------------------------------------------------------
def Resize(img, o: ImageOptions, **kw):
    if o.width == 0 and o.height == 0:
        raise ImaginaryError("Missing required param: height or width")
    opts = bimg_options(o)
    opts["embed"] = 1
    if o.is_defined.no_crop:
        opts["crop"] = int(not o.no_crop)
    return process(img, opts, **kw)


def calculate_destination_fit_dimension(iw, ih, fw, fh):
    return fit_dimension(iw, ih, fw, fh)


def Fit(img, o: ImageOptions, **kw):
    if o.width == 0 or o.height == 0:
        raise ImaginaryError("Missing required params: height, width")
    if isinstance(img, (bytes, bytearray, memoryview)):  # bimg.Metadata (image.go:144)
        try:
            m = codec.header(bytes(img))
        except codec.CodecError as e:
            raise ImaginaryError(str(e)) from e
        w, h, orientation = m.w, m.h, m.orientation
    else:
        w, h, orientation = img.w, img.h, img.orientation
    if w == 0 or h == 0:
        raise ImaginaryError("Width or height of requested image is zero", HTTP_NOT_ACCEPTABLE)
    o = dataclasses.replace(o)
    if o.no_rotation or orientation <= 4:
        o.width, o.height = calculate_destination_fit_dimension(w, h, o.width, o.height)
    else:  # width/height switched by auto rotation
        o.height, o.width = calculate_destination_fit_dimension(h, w, o.height, o.width)
    opts = bimg_options(o)
    opts["embed"] = 1
    return process(img, opts, **kw)


def Enlarge(img, o: ImageOptions, **kw):
    if o.width == 0 or o.height == 0:
        raise ImaginaryError("Missing required params: height, width")
    opts = bimg_options(o)
    opts["enlarge"] = 1
    opts["crop"] = int(not o.no_crop)
    return process(img, opts, **kw)


def Extract(img, o: ImageOptions, **kw):
    if o.area_width == 0 or o.area_height == 0:
        raise ImaginaryError("Missing required params: areawidth or areaheight")
    opts = bimg_options(o)
    opts.update(top=o.top, left=o.left, area_width=o.area_width, area_height=o.area_height)
    return process(img, opts, **kw)


def Crop(img, o: ImageOptions, **kw):
    if o.width == 0 and o.height == 0:
        raise ImaginaryError("Missing required param: height or width")
    opts = bimg_options(o)
    opts["crop"] = 1
    return process(img, opts, **kw)


def SmartCrop(img, o: ImageOptions, **kw):
    if o.width == 0 and o.height == 0:
        raise ImaginaryError("Missing required param: height or width")
    opts = bimg_options(o)
    opts["crop"] = 1
    opts["gravity"] = 5
    return process(img, opts, **kw)


def Rotate(img, o: ImageOptions, **kw):
    if o.rotate == 0:
        raise ImaginaryError("Missing required param: rotate")
    return process(img, bimg_options(o), **kw)


def AutoRotate(img, o: ImageOptions, **kw):
    """image.go:255-265: bimg AutoRotate = the EXIF rotation/flip alone, same type."""
    return process(img, dict(no_auto_rotate=0), **kw)


def Convert(img, o: ImageOptions, **kw):
    """image.go:312-320."""
    if o.type == "":
        raise ImaginaryError("Missing required param: type")
    if o.type not in ("jpeg", "png", "webp", "tiff", "gif", "heif", "avif", "pdf", "svg", "magick", "auto"):
        raise ImaginaryError("Invalid image type: " + o.type)
    return process(img, bimg_options(o), **kw)


def Watermark(img, o: ImageOptions, **kw):
    """image.go:322-341: text watermark (pango rendering) stays with libvips."""
    if o.text == "":
        raise ImaginaryError("Missing required param: text")
    raise EngineUnsupported("text watermark is rendered by libvips, not the pixel engine")


def Info(buf: bytes, o: ImageOptions, **kw) -> Image:
    """image.go:56-79: metadata only (host codec header), no pixel work."""
    try:
        h = codec.header(buf)
    except codec.CodecError as e:
        raise ImaginaryError("Cannot retrieve image metadata: " + str(e)) from e
    info = {"width": h.w, "height": h.h, "type": h.type, "space": "b-w" if h.bands <= 2 else "srgb",
            "hasAlpha": h.bands in (2, 4), "hasProfile": False, "channels": h.bands, "orientation": h.orientation}
    return Image(json.dumps(info).encode(), "application/json")


def Flip(img, o: ImageOptions, **kw):
    opts = bimg_options(o)
    opts["flip"] = 1
    return process(img, opts, **kw)


def Flop(img, o: ImageOptions, **kw):
    opts = bimg_options(o)
    opts["flop"] = 1
    return process(img, opts, **kw)


def Thumbnail(img, o: ImageOptions, **kw):
    if o.width == 0 and o.height == 0:
        raise ImaginaryError("Missing required params: width or height")
    return process(img, bimg_options(o), **kw)


def Zoom(img, o: ImageOptions, **kw):
    if o.factor == 0:
        raise ImaginaryError("Missing required param: factor")
    opts = bimg_options(o)
    if o.top > 0 or o.left > 0:
        if o.area_width == 0 and o.area_height == 0:
            raise ImaginaryError("Missing required params: areawidth, areaheight")
        opts.update(top=o.top, left=o.left, area_width=o.area_width, area_height=o.area_height)
        if o.is_defined.no_crop:
            opts["crop"] = int(not o.no_crop)
    opts["zoom"] = o.factor
    return process(img, opts, **kw)


def GaussianBlur(img, o: ImageOptions, **kw):
    if o.sigma == 0 and o.min_ampl == 0:
        raise ImaginaryError("Missing required param: sigma or minampl")
    return process(img, bimg_options(o), **kw)


def WatermarkImage(img, o: ImageOptions, wm: Optional[np.ndarray] = None, **kw):
    """image.go:343-370; the watermark bytes are fetched (and decoded) by the host."""
    if o.image == "" and wm is None:
        raise ImaginaryError("Missing required param: image")
    if wm is None or len(wm) == 0 or (isinstance(wm, np.ndarray) and wm.size == 0):
        raise ImaginaryError("Unable to read watermark image")
    opts = bimg_options(o)
    opts.update(wm_left=o.left, wm_top=o.top, wm_opacity=float(o.opacity))
    return process(img, opts, wm=wm, **kw)


OperationsMap: Dict[str, Callable] = {
    "crop": Crop, "resize": Resize, "enlarge": Enlarge, "extract": Extract, "rotate": Rotate,
    "autorotate": AutoRotate, "flip": Flip, "flop": Flop, "thumbnail": Thumbnail, "zoom": Zoom,
    "convert": Convert, "watermark": Watermark, "watermarkImage": WatermarkImage, "blur": GaussianBlur,
    "smartcrop": SmartCrop, "fit": Fit,
}


def _stage_kw(fn, kw):
    """The caller's watermark pixels belong to watermarkImage stages only."""
    return kw if fn is WatermarkImage else {k: v for k, v in kw.items() if k != "wm"}


def Pipeline(img, o: ImageOptions, **kw):
    """image.go:379-410.  On encoded bytes every stage decodes and re-encodes in
    the stage's output format, exactly as the reference; on a Decoded input the
    intermediates stay pixels (lossless, as PNG intermediates would be)."""
    if isinstance(img, (bytes, bytearray, memoryview)):
        if len(o.operations) == 0:
            raise ImaginaryError("Missing pipeline operations")
        if len(o.operations) > 10:
            raise ImaginaryError("Maximum pipeline operations (10) exceeded")
        out = Image(bytes(img), codec.mime_type(codec.sniff_type(img)))
        for op in o.operations:
            name = op.get("operation") or op.get("name")
            fn = OperationsMap.get(name)
            if fn is None:
                raise ImaginaryError(f"Unsupported operation: {name}")
            try:
                out = fn(out.body, build_params_from_operation(op), **_stage_kw(fn, kw))
            except ImaginaryError:
                if not op.get("ignore_failure"):
                    raise
        return out
    if len(o.operations) == 0:
        raise ImaginaryError("Missing pipeline operations")
    if len(o.operations) > 10:
        raise ImaginaryError("Maximum pipeline operations (10) exceeded")
    # plan every stage on the previous stage's output geometry, then run the chain
    # as ONE plan (mipx_plan_chain): one upload, intermediates stay in HBM, one
    # download, and the runtime's peepholes see across stage boundaries
    stages: list = []
    cur = img
    for i, op in enumerate(o.operations):
        name = op.get("operation")
        fn = OperationsMap.get(name)
        if fn is None:
            raise ImaginaryError(f"Unsupported operation: {name}")
        opts = build_params_from_operation(op)
        try:
            out = fn(cur, opts, chain=stages, **_stage_kw(fn, kw))
        except ImaginaryError:
            if not op.get("ignore_failure"):
                raise
            continue
        cur = Decoded(out, type="png", orientation=0)
    if not stages:
        return cur.pixels
    try:
        merged = plan_chain([s[0] for s in stages])
    except _abi.MipxError as e:
        if e.code != _abi.MIPX_EUNSUPPORTED:
            raise ImaginaryError(f"image processing error: {e}", 500) from e
        px = stages[0][1]
        for plan, _, wm in stages:  # too long or two watermarks: stage by stage
            px = _run(plan, px, wm)
        return px
    wms = [s[2] for s in stages if s[2] is not None]
    return _run(merged, stages[0][1], wms[0] if wms else None)
