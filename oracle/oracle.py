"""ctypes wrapper of liboracle.so — the CPU ORACLE (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, as the checker / CPU baseline; the product (imaginary_amd) never
does.  The C sources restate libvips 8.12.2 / bimg v1.1.9 (see vips_ref.c);
pixel parity is "parity unpinned" (no libvips here), the planner is pinned by
the reference's dimension tests.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


class RefImg(C.Structure):
    _fields_ = [("data", C.POINTER(C.c_uint8)), ("w", C.c_int), ("h", C.c_int), ("bands", C.c_int)]


class RefOpts(C.Structure):
    _fields_ = [
        ("width", C.c_int), ("height", C.c_int), ("area_width", C.c_int), ("area_height", C.c_int),
        ("top", C.c_int), ("left", C.c_int), ("crop", C.c_int), ("embed", C.c_int),
        ("enlarge", C.c_int), ("force", C.c_int), ("no_auto_rotate", C.c_int), ("rotate", C.c_int),
        ("flip", C.c_int), ("flop", C.c_int), ("gravity", C.c_int), ("extend", C.c_int),
        ("background", C.c_int * 3), ("zoom", C.c_int), ("sigma", C.c_double), ("min_ampl", C.c_double),
        ("smart_crop", C.c_int), ("wm_enable", C.c_int), ("wm_left", C.c_int), ("wm_top", C.c_int),
        ("wm_opacity", C.c_float), ("interpretation", C.c_int),
    ]


class RefInput(C.Structure):
    _fields_ = [("w", C.c_int), ("h", C.c_int), ("bands", C.c_int), ("type", C.c_int),
                ("orientation", C.c_int), ("decoded_w", C.c_int), ("decoded_h", C.c_int),
                ("wm_w", C.c_int), ("wm_h", C.c_int), ("wm_bands", C.c_int)]


class RefStep(C.Structure):
    _fields_ = [("op", C.c_int), ("a", C.c_int * 8), ("d", C.c_double * 4),
                ("out_w", C.c_int), ("out_h", C.c_int), ("out_bands", C.c_int)]


class RefPlan(C.Structure):
    _fields_ = [("load_shrink", C.c_int), ("in_w", C.c_int), ("in_h", C.c_int), ("in_bands", C.c_int),
                ("out_w", C.c_int), ("out_h", C.c_int), ("out_bands", C.c_int), ("n_steps", C.c_int),
                ("steps", RefStep * 16)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        sig = {
            "ref_plan_make": (C.c_int, [P(RefOpts), P(RefInput), P(RefPlan)]),
            "ref_fit_dimension": (C.c_int, [C.c_int] * 4 + [P(C.c_int), P(C.c_int)]),
            "ref_reduce_points": (C.c_int, [C.c_double]),
            "ref_reduce_table": (C.c_int, [C.c_double, P(C.c_int), C.c_int]),
            "ref_reducev": (C.c_int, [P(RefImg), P(RefImg), C.c_double]),
            "ref_reduceh": (C.c_int, [P(RefImg), P(RefImg), C.c_double]),
            "ref_reduce": (C.c_int, [P(RefImg), P(RefImg), C.c_double, C.c_double]),
            "ref_shrinkv": (C.c_int, [P(RefImg), P(RefImg), C.c_int]),
            "ref_shrinkh": (C.c_int, [P(RefImg), P(RefImg), C.c_int]),
            "ref_shrink": (C.c_int, [P(RefImg), P(RefImg), C.c_int, C.c_int]),
            "ref_out_size_reduce": (C.c_int, [C.c_int, C.c_double]),
            "ref_out_size_shrink": (C.c_int, [C.c_int, C.c_int]),
            "ref_embed": (C.c_int, [P(RefImg), P(RefImg)] + [C.c_int] * 5 + [P(C.c_int)]),
            "ref_extract": (C.c_int, [P(RefImg), P(RefImg)] + [C.c_int] * 4),
            "ref_rot": (C.c_int, [P(RefImg), P(RefImg), C.c_int]),
            "ref_flip": (C.c_int, [P(RefImg), P(RefImg), C.c_int]),
            "ref_gaussmat": (C.c_int, [C.c_double, C.c_double, P(C.c_int), C.c_int, P(C.c_int)]),
            "ref_gaussblur": (C.c_int, [P(RefImg), P(RefImg), C.c_double, C.c_double]),
            "ref_watermark": (C.c_int, [P(RefImg), P(RefImg), P(RefImg), C.c_int, C.c_int, C.c_float]),
            "ref_bicubic_table": (C.c_int, [P(C.c_int)]),
            "ref_affine": (C.c_int, [P(RefImg), P(RefImg), C.c_double, C.c_double, C.c_int]),
            "ref_zoom": (C.c_int, [P(RefImg), P(RefImg), C.c_int, C.c_int]),
            "ref_flatten": (C.c_int, [P(RefImg), P(RefImg), P(C.c_int)]),
            "ref_bw": (C.c_int, [P(RefImg), P(RefImg)]),
            "ref_smartcrop_origin": (C.c_int, [P(RefImg), C.c_int, C.c_int, P(C.c_int), P(C.c_int)]),
            "ref_execute": (C.c_int, [P(RefPlan), P(RefImg), P(RefImg), P(RefImg)]),
            "ref_reduce_batch": (C.c_int, [P(P(C.c_uint8)), P(P(C.c_uint8)), C.c_int, C.c_int, C.c_int,
                                           C.c_int, C.c_double, C.c_double, C.c_int]),
            "ref_reduce_fast": (C.c_int, [P(RefImg), P(RefImg), C.c_double, C.c_double]),
            "ref_reduce_fast_batch": (C.c_int, [P(P(C.c_uint8)), P(P(C.c_uint8)), C.c_int, C.c_int, C.c_int,
                                                C.c_int, C.c_double, C.c_double, C.c_int]),
            "ref_set_switch": (None, [C.c_char_p, C.c_int]),
            "ref_get_switch": (C.c_int, [C.c_char_p]),
            "ref_free": (None, [C.c_void_p]),
        }
        for n, (r, a) in sig.items():
            f = getattr(L, n)
            f.restype = r
            f.argtypes = a
        _lib = L
    return _lib


class OracleError(RuntimeError):
    def __init__(self, code, what):
        self.code = code
        super().__init__(f"{what}: oracle error {code}")


def _in(img: np.ndarray) -> RefImg:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    if img.ndim == 2:
        img = img[:, :, None]
    h, w, b = img.shape
    r = RefImg(img.ctypes.data_as(C.POINTER(C.c_uint8)), w, h, b)
    r._keep = img
    return r


def _out(r: RefImg) -> np.ndarray:
    n = r.w * r.h * r.bands
    a = np.ctypeslib.as_array(r.data, shape=(n,)).copy().reshape(r.h, r.w, r.bands)
    lib().ref_free(C.cast(r.data, C.c_void_p))
    return a


def _call(name, img, *args):
    o = RefImg()
    e = getattr(lib(), name)(C.byref(_in(img)), C.byref(o), *args)
    if e:
        raise OracleError(e, name)
    return _out(o)


def reduce(img, hshrink, vshrink):
    return _call("ref_reduce", img, hshrink, vshrink)


def reducev(img, vshrink):
    return _call("ref_reducev", img, vshrink)


def reduceh(img, hshrink):
    return _call("ref_reduceh", img, hshrink)


def shrink(img, hs, vs):
    return _call("ref_shrink", img, hs, vs)


def embed(img, x, y, w, h, extend, bg=(0, 0, 0)):
    return _call("ref_embed", img, x, y, w, h, extend, (C.c_int * 3)(*bg))


def extract(img, left, top, w, h):
    return _call("ref_extract", img, left, top, w, h)


def rot(img, angle):
    return _call("ref_rot", img, angle)


def flip(img, vertical):
    return _call("ref_flip", img, int(vertical))


def gaussblur(img, sigma, min_ampl=0.2):
    return _call("ref_gaussblur", img, sigma, min_ampl)


def gaussmat(sigma, min_ampl=0.2):
    m = (C.c_int * 10001)()
    s = C.c_int()
    n = lib().ref_gaussmat(sigma, min_ampl, m, 10001, C.byref(s))
    if n < 0:
        raise OracleError(n, "ref_gaussmat")
    return list(m[:n]), s.value


def reduce_table(shrink):
    n = lib().ref_reduce_points(shrink)
    t = (C.c_int * (n * 129))()
    lib().ref_reduce_table(shrink, t, n)
    return np.array(t[:], dtype=np.int32).reshape(129, n)


def bicubic_table():
    t = (C.c_int * (129 * 4))()
    lib().ref_bicubic_table(t)
    return np.array(t[:], dtype=np.int32).reshape(129, 4)


def affine(img, xscale, yscale, extend=1):
    return _call("ref_affine", img, xscale, yscale, extend)


def zoom(img, xfac, yfac):
    return _call("ref_zoom", img, xfac, yfac)


def flatten(img, bg):
    return _call("ref_flatten", img, (C.c_int * 3)(*bg))


def bw(img):
    return _call("ref_bw", img)


def watermark(base, wm, left, top, opacity):
    o = RefImg()
    e = lib().ref_watermark(C.byref(_in(base)), C.byref(_in(wm)), C.byref(o), left, top, opacity)
    if e:
        raise OracleError(e, "ref_watermark")
    return _out(o)


def smartcrop_origin(img, w, h):
    l, t = C.c_int(), C.c_int()
    e = lib().ref_smartcrop_origin(C.byref(_in(img)), w, h, C.byref(l), C.byref(t))
    if e:
        raise OracleError(e, "ref_smartcrop_origin")
    return l.value, t.value


def plan(opts: dict, inp: dict):
    """opts/inp: dicts with the RefOpts / RefInput field names. Returns (code, RefPlan)."""
    o, i, p = RefOpts(), RefInput(), RefPlan()
    for k, v in opts.items():
        if k == "background":
            o.background[:] = list(v)
        else:
            setattr(o, k, v)
    for k, v in inp.items():
        setattr(i, k, v)
    e = lib().ref_plan_make(C.byref(o), C.byref(i), C.byref(p))
    return e, p


def execute(p: RefPlan, img, wm=None):
    o = RefImg()
    wmr = C.byref(_in(wm)) if wm is not None else None
    e = lib().ref_execute(C.byref(p), C.byref(_in(img)), wmr, C.byref(o))
    if e:
        raise OracleError(e, "ref_execute")
    return _out(o)


def fit_dimension(iw, ih, fw, fh):
    a, b = C.c_int(), C.c_int()
    lib().ref_fit_dimension(iw, ih, fw, fh, C.byref(a), C.byref(b))
    return a.value, b.value


def reduce_batch(imgs, hshrink, vshrink, threads):
    """CPU baseline: list of HxWxB uint8 arrays, OpenMP across images."""
    n = len(imgs)
    h, w, b = imgs[0].shape
    oh, ow = lib().ref_out_size_reduce(h, vshrink), lib().ref_out_size_reduce(w, hshrink)
    outs = [np.empty((oh, ow, b), np.uint8) for _ in range(n)]
    PP = C.POINTER(C.c_uint8) * n
    ins = PP(*[np.ascontiguousarray(a).ctypes.data_as(C.POINTER(C.c_uint8)) for a in imgs])
    ous = PP(*[a.ctypes.data_as(C.POINTER(C.c_uint8)) for a in outs])
    e = lib().ref_reduce_batch(ins, ous, n, w, h, b, hshrink, vshrink, threads)
    if e:
        raise OracleError(e, "ref_reduce_batch")
    return outs


def reduce_fast(img, hshrink, vshrink):
    """The CPU baseline's reduce (vips_fast.c): same result as reduce(), fast loop order."""
    o = RefImg()
    e = lib().ref_reduce_fast(C.byref(_in(img)), C.byref(o), hshrink, vshrink)
    if e:
        raise OracleError(e, "ref_reduce_fast")
    return _out(o)


def reduce_fast_batch(imgs, hshrink, vshrink, threads):
    """CPU baseline (bench.py): list of HxWxB uint8 arrays, OpenMP across images."""
    n = len(imgs)
    h, w, b = imgs[0].shape
    oh, ow = lib().ref_out_size_reduce(h, vshrink), lib().ref_out_size_reduce(w, hshrink)
    outs = [np.empty((oh, ow, b), np.uint8) for _ in range(n)]
    PP = C.POINTER(C.c_uint8) * n
    ins = PP(*[np.ascontiguousarray(a).ctypes.data_as(C.POINTER(C.c_uint8)) for a in imgs])
    ous = PP(*[a.ctypes.data_as(C.POINTER(C.c_uint8)) for a in outs])
    e = lib().ref_reduce_fast_batch(ins, ous, n, w, h, b, hshrink, vshrink, threads)
    if e:
        raise OracleError(e, "ref_reduce_fast_batch")
    return outs


def set_switch(name: str, value: int):
    lib().ref_set_switch(name.encode(), int(value))


def get_switch(name: str) -> int:
    return int(lib().ref_get_switch(name.encode()))
