"""ctypes mirror of include/mipx.h and the loader for the in-tree libmipx.so.

The product path is the HIP library: importing this module fails loudly when
libmipx.so is missing (there is no CPU fallback anywhere in the package).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MIPX_LIB_PATH: load another build of the same library (same-box A/B of two builds);
# unset, the in-tree libmipx.so is the product
LIB_PATH = os.environ.get("MIPX_LIB_PATH") or os.path.join(_HERE, "libmipx.so")

MIPX_OK = 0
MIPX_EINVAL = -1
MIPX_EUNSUPPORTED = -2
MIPX_ENOMEM = -3
MIPX_ENODEV = -4
MIPX_EDEVICE = -5
MIPX_ETIMEOUT = -6
MIPX_ENOTINIT = -7
MIPX_ESTALE = -8
MIPX_EBUSY = -9

GRAVITY = {"centre": 0, "north": 1, "east": 2, "south": 3, "west": 4, "smart": 5}
EXTEND = {"black": 0, "copy": 1, "repeat": 2, "mirror": 3, "white": 4, "background": 5, "lastpixel": 6}
TYPES = {"unknown": 0, "jpeg": 1, "webp": 2, "png": 3, "tiff": 4, "gif": 5, "pdf": 6, "svg": 7,
         "magick": 8, "heif": 9, "avif": 10}

(OP_ROT, OP_FLIP, OP_SHRINK, OP_REDUCE, OP_EXTRACT, OP_EMBED, OP_SMARTCROP, OP_BLUR, OP_WATERMARK,
 OP_AFFINE, OP_ZOOM, OP_FLATTEN, OP_BW) = range(1, 14)
OP_NAMES = {OP_ROT: "rot", OP_FLIP: "flip", OP_SHRINK: "shrink", OP_REDUCE: "reduce",
            OP_EXTRACT: "extract", OP_EMBED: "embed", OP_SMARTCROP: "smartcrop",
            OP_BLUR: "blur", OP_WATERMARK: "watermark", OP_AFFINE: "affine", OP_ZOOM: "zoom",
            OP_FLATTEN: "flatten", OP_BW: "bw"}
INTERPRETATION_SRGB = 22
INTERPRETATION_BW = 26
MAX_STEPS = 64


class MipxOpts(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32),
        ("area_width", C.c_int32), ("area_height", C.c_int32),
        ("top", C.c_int32), ("left", C.c_int32),
        ("crop", C.c_int32), ("embed", C.c_int32), ("enlarge", C.c_int32), ("force", C.c_int32),
        ("no_auto_rotate", C.c_int32),
        ("rotate", C.c_int32),
        ("flip", C.c_int32), ("flop", C.c_int32),
        ("gravity", C.c_int32),
        ("extend", C.c_int32),
        ("background", C.c_int32 * 3),
        ("zoom", C.c_int32),
        ("sigma", C.c_double), ("min_ampl", C.c_double),
        ("smart_crop", C.c_int32),
        ("wm_enable", C.c_int32),
        ("wm_left", C.c_int32), ("wm_top", C.c_int32),
        ("wm_opacity", C.c_float),
        ("interpretation", C.c_int32),
    ]


class MipxInput(C.Structure):
    _fields_ = [
        ("w", C.c_int32), ("h", C.c_int32), ("bands", C.c_int32),
        ("type", C.c_int32), ("orientation", C.c_int32),
        ("decoded_w", C.c_int32), ("decoded_h", C.c_int32),
        ("wm_w", C.c_int32), ("wm_h", C.c_int32), ("wm_bands", C.c_int32),
    ]


class MipxStep(C.Structure):
    _fields_ = [
        ("op", C.c_int32), ("a", C.c_int32 * 8), ("d", C.c_double * 4),
        ("out_w", C.c_int32), ("out_h", C.c_int32), ("out_bands", C.c_int32),
    ]


class MipxPlan(C.Structure):
    _fields_ = [
        ("load_shrink", C.c_int32),
        ("in_w", C.c_int32), ("in_h", C.c_int32), ("in_bands", C.c_int32),
        ("out_w", C.c_int32), ("out_h", C.c_int32), ("out_bands", C.c_int32),
        ("n_steps", C.c_int32),
        ("steps", MipxStep * MAX_STEPS),
    ]

    def describe(self):
        out = []
        for i in range(self.n_steps):
            s = self.steps[i]
            out.append((OP_NAMES.get(s.op, s.op), tuple(s.a), tuple(s.d), (s.out_w, s.out_h, s.out_bands)))
        return out


class MipxImg(C.Structure):
    _fields_ = [("data", C.c_void_p), ("w", C.c_int32), ("h", C.c_int32), ("bands", C.c_int32),
                ("stride", C.c_int64)]


class MipxCfg(C.Structure):
    _fields_ = [("n_devices", C.c_int32), ("device_ids", C.c_int32 * 16),
                ("staging_bytes", C.c_int64), ("max_batch", C.c_int32), ("batch_wait_us", C.c_int32),
                ("queues_per_device", C.c_int32)]


# name -> (restype, argtypes): every symbol include/mipx.h declares
_P = C.c_void_p
_U8P = C.c_void_p
_I = C.c_int32
_SIG = {
    "mipx_version": (C.c_char_p, []),
    "mipx_build_id": (C.c_char_p, []),
    "mipx_cancel": (C.c_int, [C.c_uint64]),
    "mipx_queue_count": (C.c_int, []),
    "mipx_pick_queue": (C.c_int, [C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.c_int32]),
    "mipx_queue_stats": (C.c_int, [C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                   C.POINTER(C.c_int64)]),
    "mipx_abi_version": (C.c_int, []),
    "mipx_plan_chain": (C.c_int, [C.POINTER(MipxPlan), C.c_int32, C.POINTER(MipxPlan)]),
    "mipx_strerror": (C.c_char_p, [C.c_int]),
    "mipx_last_error": (C.c_char_p, []),
    "mipx_init": (C.c_int, [C.POINTER(MipxCfg)]),
    "mipx_shutdown": (None, []),
    "mipx_device_count": (C.c_int, []),
    "mipx_plan_make": (C.c_int, [C.POINTER(MipxOpts), C.POINTER(MipxInput), C.POINTER(MipxPlan)]),
    "mipx_fit_dimension": (C.c_int, [_I, _I, _I, _I, C.POINTER(_I), C.POINTER(_I)]),
    "mipx_submit": (C.c_int, [C.c_int, C.POINTER(MipxPlan), C.POINTER(MipxImg), C.POINTER(MipxImg),
                              C.POINTER(MipxImg), C.POINTER(C.c_uint64)]),
    "mipx_wait": (C.c_int, [C.c_uint64, C.c_int]),
    "mipx_process": (C.c_int, [C.POINTER(MipxPlan), C.POINTER(MipxImg), C.POINTER(MipxImg), C.POINTER(MipxImg)]),
    "mipx_stats": (C.c_int, [C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "mipx_workspace_bytes": (C.c_size_t, [C.POINTER(MipxPlan), _I]),
    "mipx_execute_dev": (C.c_int, [C.POINTER(MipxPlan), _I, _U8P, _U8P, _U8P, _P, C.c_size_t, _P]),
    "mipx_op_reduce": (C.c_int, [_U8P, _U8P, _I, _I, _I, _I, C.c_double, C.c_double, _P, C.c_size_t, _P]),
    "mipx_op_reducev": (C.c_int, [_U8P, _U8P, _I, _I, _I, _I, C.c_double, _P]),
    "mipx_op_reduceh": (C.c_int, [_U8P, _U8P, _I, _I, _I, _I, C.c_double, _P]),
    "mipx_op_shrink": (C.c_int, [_U8P, _U8P, _I, _I, _I, _I, _I, _I, _P]),
    "mipx_op_embed": (C.c_int, [_U8P, _U8P, _I, _I, _I, _I, _I, _I, _I, _I, _I, C.POINTER(_I), _P]),
    "mipx_op_extract": (C.c_int, [_U8P, _U8P, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "mipx_op_rot": (C.c_int, [_U8P, _U8P, _I, _I, _I, _I, _I, _P]),
    "mipx_op_flip": (C.c_int, [_U8P, _U8P, _I, _I, _I, _I, _I, _P]),
    "mipx_op_gaussblur": (C.c_int, [_U8P, _U8P, _I, _I, _I, _I, C.c_double, C.c_double, _P, C.c_size_t, _P]),
    "mipx_op_watermark": (C.c_int, [_U8P, _U8P, _U8P, _I, _I, _I, _I, _I, _I, _I, _I, _I, C.c_float, _P]),
    "mipx_op_affine": (C.c_int, [_U8P, _U8P, _I, _I, _I, _I, C.c_double, C.c_double, _I, _P]),
    "mipx_op_zoom": (C.c_int, [_U8P, _U8P, _I, _I, _I, _I, _I, _I, _P]),
    "mipx_op_flatten": (C.c_int, [_U8P, _U8P, _I, _I, _I, _I, C.POINTER(_I), _P]),
    "mipx_op_colourspace_bw": (C.c_int, [_U8P, _U8P, _I, _I, _I, _I, _P]),
    "mipx_op_smartcrop_origin": (C.c_int, [_U8P, _P, _I, _I, _I, _I, _I, _I, _P, C.c_size_t, _P]),
    "mipx_op_workspace_bytes": (C.c_size_t, [_I, _I, _I, _I, _I, C.c_double, C.c_double]),
    "mipx_tuning_reload": (C.c_int, []),
    "mipx_set_reduce_sampling": (C.c_int, [C.c_int32]),
    "mipx_reduce_sampling": (C.c_int, []),
    "mipx_set_device": (C.c_int, [C.c_int]),
    "mipx_dev_malloc": (C.c_int, [C.POINTER(C.c_void_p), C.c_size_t]),
    "mipx_dev_free": (C.c_int, [_P]),
    "mipx_memcpy_h2d": (C.c_int, [_P, _P, C.c_size_t]),
    "mipx_memcpy_d2h": (C.c_int, [_P, _P, C.c_size_t]),
    "mipx_memset_dev": (C.c_int, [_P, C.c_int, C.c_size_t]),
    "mipx_stream_sync": (C.c_int, [_P]),
    "mipx_device_sync": (C.c_int, []),
    "mipx_stream_create": (C.c_int, [C.POINTER(C.c_void_p)]),
    "mipx_stream_destroy": (C.c_int, [_P]),
    "mipx_event_create": (C.c_int, [C.POINTER(C.c_void_p)]),
    "mipx_event_destroy": (C.c_int, [_P]),
    "mipx_event_record": (C.c_int, [_P, _P]),
    "mipx_event_elapsed_ms": (C.c_int, [_P, _P, C.POINTER(C.c_float)]),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libmipx.so not found at {LIB_PATH}: build it with "
            "`make -C imaginary_amd` (or __graft_entry__.build()); the engine has no CPU fallback")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIG.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


class MipxError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        detail = lib.mipx_last_error().decode(errors="replace")
        msg = f"{what}: {lib.mipx_strerror(code).decode()} ({code})"
        if detail:
            msg += f" — {detail}"
        super().__init__(msg)


_tuning_seen = None


def sync_tuning() -> None:
    """The library snapshots the MIPX_* kernel-selection knobs on first use; when the
    Python process changed them since (tests, A/B scripts), take a new snapshot.  Call
    between launches only (the library's rule for mipx_tuning_reload)."""
    global _tuning_seen
    cur = tuple(sorted((k, v) for k, v in os.environ.items() if k.startswith("MIPX_")))
    if cur != _tuning_seen:
        lib.mipx_tuning_reload()
        _tuning_seen = cur


def check(code: int, what: str = "mipx") -> int:
    if code != MIPX_OK:
        raise MipxError(code, what)
    return code
