"""Thin Python handle on libmipx.so: device buffers, per-op calls, plan execution.

Everything here calls the HIP library through the C-ABI; there is no CPU
compute path.  Used by the tests, smoke() and bench.py.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from ._abi import (MipxCfg, MipxImg, MipxInput, MipxOpts, MipxPlan, check, lib, MipxError,
                   EXTEND, GRAVITY, TYPES, sync_tuning)

__all__ = ["DeviceBuffer", "make_opts", "make_input", "plan_make", "fit_dimension", "Engine",
           "run_op", "execute", "device_count", "synchronize", "set_reduce_sampling", "reduce_sampling"]

SAMPLING = {"corner": 0, "centre": 1}


def set_reduce_sampling(convention: str) -> None:
    """libvips' Lanczos3 reduce sampling convention, PARITY_ASSUMPTIONS.md row 1:
    "corner" (X = o * shrink) or "centre" (X = (o + 0.5) * shrink - 0.5).  Set it
    while no work is in flight (mipx_set_reduce_sampling)."""
    check(lib.mipx_set_reduce_sampling(SAMPLING[convention]), "mipx_set_reduce_sampling")


def reduce_sampling() -> str:
    return {v: k for k, v in SAMPLING.items()}[lib.mipx_reduce_sampling()]


def device_count() -> int:
    return int(lib.mipx_device_count())


def synchronize():
    check(lib.mipx_device_sync(), "mipx_device_sync")


class DeviceBuffer:
    """Raw device allocation owned by Python (freed on close / GC)."""

    def __init__(self, nbytes: int):
        self.nbytes = int(max(nbytes, 1))
        p = C.c_void_p()
        check(lib.mipx_dev_malloc(C.byref(p), self.nbytes), "mipx_dev_malloc")
        self.ptr = p.value

    @classmethod
    def from_array(cls, a: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(a, dtype=np.uint8)
        b = cls(a.nbytes)
        check(lib.mipx_memcpy_h2d(b.ptr, a.ctypes.data, a.nbytes), "mipx_memcpy_h2d")
        return b

    def download(self, shape, dtype=np.uint8) -> np.ndarray:
        out = np.empty(shape, dtype=dtype)
        check(lib.mipx_memcpy_d2h(out.ctypes.data, self.ptr, out.nbytes), "mipx_memcpy_d2h")
        return out

    def close(self):
        if getattr(self, "ptr", None):
            lib.mipx_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def make_opts(**kw) -> MipxOpts:
    """MipxOpts from bimg-style keyword fields (see include/mipx.h)."""
    o = MipxOpts()
    for k, v in kw.items():
        if k == "background":
            o.background[:] = list(v)[:3]
        elif k == "gravity" and isinstance(v, str):
            o.gravity = GRAVITY[v]
        elif k == "extend" and isinstance(v, str):
            o.extend = EXTEND[v]
        else:
            setattr(o, k, v)
    return o


def make_input(w, h, bands, type="unknown", orientation=0, decoded_w=0, decoded_h=0,
               wm_w=0, wm_h=0, wm_bands=0) -> MipxInput:
    i = MipxInput()
    i.w, i.h, i.bands = w, h, bands
    i.type = TYPES[type] if isinstance(type, str) else int(type)
    i.orientation = orientation
    i.decoded_w, i.decoded_h = decoded_w, decoded_h
    i.wm_w, i.wm_h, i.wm_bands = wm_w, wm_h, wm_bands
    return i


def plan_make(opts: MipxOpts, inp: MipxInput) -> MipxPlan:
    p = MipxPlan()
    check(lib.mipx_plan_make(C.byref(opts), C.byref(inp), C.byref(p)), "mipx_plan_make")
    return p


def plan_chain(stages) -> MipxPlan:
    """mipx_plan_chain: one plan for a /pipeline chain of stage plans."""
    arr = (MipxPlan * len(stages))(*stages)
    p = MipxPlan()
    check(lib.mipx_plan_chain(arr, len(stages), C.byref(p)), "mipx_plan_chain")
    return p


def fit_dimension(iw, ih, fw, fh):
    a, b = C.c_int32(), C.c_int32()
    check(lib.mipx_fit_dimension(iw, ih, fw, fh, C.byref(a), C.byref(b)), "mipx_fit_dimension")
    return a.value, b.value


def _img(a: np.ndarray) -> MipxImg:
    if a.ndim == 2:
        a = a[:, :, None]
    h, w, b = a.shape
    m = MipxImg(a.ctypes.data, w, h, b, a.strides[0])
    return m


class Engine:
    """Request path: pinned staging, per-device queues, batching (mipx_submit/mipx_wait)."""

    def __init__(self, devices: Optional[Sequence[int]] = None, max_batch: int = 64,
                 batch_wait_us: int = 0, queues_per_device: int = 1):
        cfg = MipxCfg()
        cfg.queues_per_device = queues_per_device
        if devices:
            cfg.n_devices = len(devices)
            for i, d in enumerate(devices):
                cfg.device_ids[i] = d
        cfg.max_batch = max_batch
        cfg.batch_wait_us = batch_wait_us
        sync_tuning()
        check(lib.mipx_init(C.byref(cfg)), "mipx_init")

    @classmethod
    def attach(cls) -> "Engine":
        """A handle on the engine already running in this process (started by another
        Engine, with whatever configuration it chose); mipx_init is not called."""
        if lib.mipx_queue_count() <= 0:
            raise MipxError(-7, "Engine.attach: no engine running")
        return cls.__new__(cls)

    def submit(self, plan: MipxPlan, img: np.ndarray, wm: Optional[np.ndarray] = None, device: int = -1,
               out: Optional[np.ndarray] = None):
        """Queue one request; returns (ticket, out).  `out` (optional) receives the
        result: contiguous uint8 of the plan's output shape.  The MIPX_* kernel knobs are
        re-read in Engine(), run_op and execute, not per request: a reload
        must not race the queue workers' launches."""
        if not (img.dtype == np.uint8 and img.ndim == 3 and img.strides[2] == 1
                and img.strides[1] == img.shape[2]):
            img = np.ascontiguousarray(img, dtype=np.uint8)  # rows may keep a wider stride
        shape = (plan.out_h, plan.out_w, plan.out_bands)
        if out is None:
            out = np.empty(shape, np.uint8)
        elif out.shape != shape or out.dtype != np.uint8 or not out.flags.c_contiguous:
            raise ValueError(f"out must be contiguous uint8 {shape}")
        ti = C.c_uint64()
        wmi = C.byref(_img(np.ascontiguousarray(wm, dtype=np.uint8))) if wm is not None else None
        check(lib.mipx_submit(device, C.byref(plan), C.byref(_img(img)), wmi, C.byref(_img(out)),
                              C.byref(ti)), "mipx_submit")
        return ti.value, out

    def wait(self, ticket: int, timeout_ms: int = -1):
        check(lib.mipx_wait(ticket, timeout_ms), "mipx_wait")

    def process(self, plan: MipxPlan, img: np.ndarray, wm: Optional[np.ndarray] = None) -> np.ndarray:
        t, out = self.submit(plan, img, wm)
        self.wait(t)
        return out

    def stats(self, device: int = 0):
        """(batches launched, requests retired) on `device` since mipx_init."""
        b, r = C.c_uint64(), C.c_uint64()
        check(lib.mipx_stats(device, C.byref(b), C.byref(r)), "mipx_stats")
        return b.value, r.value

    def queue_stats(self):
        """[(device, batches, requests, pending_bytes)] for every request queue."""
        out = []
        for q in range(lib.mipx_queue_count()):
            d, b, r, p = C.c_int32(), C.c_uint64(), C.c_uint64(), C.c_int64()
            check(lib.mipx_queue_stats(q, C.byref(d), C.byref(b), C.byref(r), C.byref(p)), "mipx_queue_stats")
            out.append((d.value, b.value, r.value, p.value))
        return out

    def cancel(self, ticket: int):
        check(lib.mipx_cancel(ticket), "mipx_cancel")

    def shutdown(self):
        lib.mipx_shutdown()


def _batch(imgs) -> np.ndarray:
    a = np.ascontiguousarray(imgs, dtype=np.uint8)
    if a.ndim == 3:
        a = a[None]
    return a


def run_op(name: str, imgs: np.ndarray, **p) -> np.ndarray:
    """Run one mipx_op_* kernel on a batch (n, h, w, b) of host images; returns host output."""
    sync_tuning()
    x = _batch(imgs)
    n, h, w, b = x.shape
    din = DeviceBuffer.from_array(x)
    ws = None
    wsb = 0
    if name == "reduce":
        hs, vs = p["hshrink"], p["vshrink"]
        oh, ow, ob = _osz_reduce(h, vs), _osz_reduce(w, hs), b
        wsb = lib.mipx_op_workspace_bytes(4, n, w, h, b, hs, vs)
    elif name == "reducev":
        oh, ow, ob = _osz_reduce(h, p["vshrink"]), w, b
    elif name == "reduceh":
        oh, ow, ob = h, _osz_reduce(w, p["hshrink"]), b
    elif name == "shrink":
        oh, ow, ob = _osz_shrink(h, p["vshrink"]), _osz_shrink(w, p["hshrink"]), b
    elif name == "embed":
        oh, ow, ob = p["height"], p["width"], b
    elif name == "extract":
        oh, ow, ob = p["height"], p["width"], b
    elif name == "rot":
        a = p["angle"] % 360
        oh, ow, ob = (w, h, b) if a in (90, 270) else (h, w, b)
    elif name == "flip":
        oh, ow, ob = h, w, b
    elif name == "gaussblur":
        oh, ow, ob = h, w, b
        wsb = lib.mipx_op_workspace_bytes(8, n, w, h, b, p["sigma"], p.get("min_ampl", 0.2))
    elif name == "watermark":
        oh, ow = h, w
        ob = b if b in (2, 4) else b + 1
    elif name == "affine":
        import math
        ow, oh, ob = int(math.ceil(w * p["xscale"])), int(math.ceil(h * p["yscale"])), b
    elif name == "zoom":
        ow, oh, ob = w * p["xfac"], h * p["yfac"], b
    elif name == "flatten":
        oh, ow, ob = h, w, (b - 1 if b in (2, 4) else b)
    elif name == "bw":
        oh, ow, ob = h, w, (2 if b == 4 else 1 if b == 3 else b)
    else:
        raise ValueError(name)
    dout = DeviceBuffer(n * oh * ow * ob)
    if wsb:
        ws = DeviceBuffer(wsb)
    wsp = ws.ptr if ws else None
    if name == "reduce":
        code = lib.mipx_op_reduce(din.ptr, dout.ptr, n, w, h, b, hs, vs, wsp, wsb, None)
    elif name == "reducev":
        code = lib.mipx_op_reducev(din.ptr, dout.ptr, n, w, h, b, p["vshrink"], None)
    elif name == "reduceh":
        code = lib.mipx_op_reduceh(din.ptr, dout.ptr, n, w, h, b, p["hshrink"], None)
    elif name == "shrink":
        code = lib.mipx_op_shrink(din.ptr, dout.ptr, n, w, h, b, p["hshrink"], p["vshrink"], None)
    elif name == "embed":
        bg = (C.c_int32 * 3)(*p.get("background", (0, 0, 0)))
        code = lib.mipx_op_embed(din.ptr, dout.ptr, n, w, h, b, p["x"], p["y"], p["width"], p["height"],
                                 p["extend"], bg, None)
    elif name == "extract":
        code = lib.mipx_op_extract(din.ptr, dout.ptr, n, w, h, b, p["left"], p["top"], p["width"],
                                   p["height"], None)
    elif name == "rot":
        code = lib.mipx_op_rot(din.ptr, dout.ptr, n, w, h, b, p["angle"], None)
    elif name == "flip":
        code = lib.mipx_op_flip(din.ptr, dout.ptr, n, w, h, b, int(p["vertical"]), None)
    elif name == "gaussblur":
        code = lib.mipx_op_gaussblur(din.ptr, dout.ptr, n, w, h, b, p["sigma"], p.get("min_ampl", 0.2),
                                     wsp, wsb, None)
    elif name == "watermark":
        wm = np.ascontiguousarray(p["wm"], dtype=np.uint8)
        if wm.ndim == 2:
            wm = wm[:, :, None]
        dwm = DeviceBuffer.from_array(wm)
        code = lib.mipx_op_watermark(din.ptr, dwm.ptr, dout.ptr, n, w, h, b, wm.shape[1], wm.shape[0],
                                     wm.shape[2], p["left"], p["top"], p["opacity"], None)
    elif name == "affine":
        code = lib.mipx_op_affine(din.ptr, dout.ptr, n, w, h, b, p["xscale"], p["yscale"], p.get("extend", 1), None)
    elif name == "zoom":
        code = lib.mipx_op_zoom(din.ptr, dout.ptr, n, w, h, b, p["xfac"], p["yfac"], None)
    elif name == "flatten":
        code = lib.mipx_op_flatten(din.ptr, dout.ptr, n, w, h, b, (C.c_int32 * 3)(*p["background"]), None)
    elif name == "bw":
        code = lib.mipx_op_colourspace_bw(din.ptr, dout.ptr, n, w, h, b, None)
    check(code, f"mipx_op_{name}")
    synchronize()
    return dout.download((n, oh, ow, ob))


def smartcrop_origins(imgs: np.ndarray, cw: int, ch: int) -> np.ndarray:
    sync_tuning()
    x = _batch(imgs)
    n, h, w, b = x.shape
    din = DeviceBuffer.from_array(x)
    wsb = lib.mipx_op_workspace_bytes(7, n, w, h, b, cw, ch)
    ws = DeviceBuffer(wsb)
    org = DeviceBuffer(8 * n)
    check(lib.mipx_op_smartcrop_origin(din.ptr, org.ptr, n, w, h, b, cw, ch, ws.ptr, wsb, None),
          "mipx_op_smartcrop_origin")
    synchronize()
    return org.download((n, 2), np.int32)


def execute(plan: MipxPlan, imgs: np.ndarray, wm: Optional[np.ndarray] = None,
            junk: Optional[int] = None) -> np.ndarray:
    """mipx_execute_dev on a batch of host images (uploads, runs the plan, downloads).
    junk: fill the workspace (the ping-pong intermediates) and the output with this byte
    first, so a step that reads outside what the steps before it wrote shows up."""
    sync_tuning()
    x = _batch(imgs)
    n = x.shape[0]
    din = DeviceBuffer.from_array(x)
    dout = DeviceBuffer(n * plan.out_w * plan.out_h * plan.out_bands)
    wsb = lib.mipx_workspace_bytes(C.byref(plan), n)
    ws = DeviceBuffer(wsb) if wsb else None
    if junk is not None:
        check(lib.mipx_memset_dev(dout.ptr, junk, dout.nbytes), "mipx_memset_dev")
        if ws:
            check(lib.mipx_memset_dev(ws.ptr, junk, ws.nbytes), "mipx_memset_dev")
    dwm = DeviceBuffer.from_array(wm) if wm is not None else None
    check(lib.mipx_execute_dev(C.byref(plan), n, din.ptr, dout.ptr, dwm.ptr if dwm else None,
                               ws.ptr if ws else None, wsb, None), "mipx_execute_dev")
    synchronize()
    return dout.download((n, plan.out_h, plan.out_w, plan.out_bands))


def _vips_round(v: float) -> int:
    import math
    return int(math.ceil(v - 0.5)) if v < 0 else int(math.floor(v + 0.5))


def _osz_reduce(n: int, s: float) -> int:
    return _vips_round(n / s)


def _osz_shrink(n: int, s: int) -> int:
    return max(1, _vips_round(n / s))
