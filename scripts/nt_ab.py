#!/usr/bin/env python3
"""Same-process A/B of the row-copy kernels' store / load policy: embed (k_embed_rows one
row at a time / k_embed_rows2 with every row fetched first / + non-temporal stores;
MIPX_EMBED_V=0/1/2) and flip / rot 180 (MIPX_FLIP_NT=0/1) on C5's shapes.  One JSON
line per (op, shape, variant): median ms of 5 groups after a 200 ms warm-up, GB/s
read + written, and whether the output equals the first variant's."""
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from imaginary_amd._abi import check, lib  # noqa: E402


def timed(run, st):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    while True:
        for _ in range(5):
            run()
        e1.record(st)
        torch.cuda.synchronize()
        if e0.elapsed_time(e1) > 200:
            break
    ts = []
    for _ in range(5):
        e0.record(st)
        for _ in range(10):
            run()
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 10)
    return statistics.median(ts)


def main():
    dev = torch.device("cuda", 0)
    check(lib.mipx_set_device(0))
    st = torch.cuda.current_stream(dev)
    sp = C.c_void_p(st.cuda_stream)
    cases = []
    for (w, h, n) in ((3840, 2160, 16), (4000, 3000, 8), (1920, 1080, 32)):
        s = max(w, h)
        for ext in (0, 3):  # black, copy
            cases.append(("embed", w, h, 3, n, dict(ow=s, oh=s, x=(s - w) // 2, y=(s - h) // 2, ext=ext),
                          "MIPX_EMBED_V", ("0", "1", "2")))
        cases.append(("flip", w, h, 3, n, dict(v=0), "MIPX_FLIP_NT", ("0", "1")))
        cases.append(("rot180", w, h, 3, n, {}, "MIPX_FLIP_NT", ("0", "1")))
    for op, w, h, b, n, p, knob, vals in cases:
        x = torch.randint(0, 256, (n * w * h * b,), dtype=torch.uint8, device=dev)
        ow, oh = p.get("ow", w), p.get("oh", h)
        y = torch.empty((n * ow * oh * b,), dtype=torch.uint8, device=dev)
        bg = (C.c_int32 * 3)(9, 8, 7)

        def run():
            if op == "embed":
                check(lib.mipx_op_embed(x.data_ptr(), y.data_ptr(), n, w, h, b, p["x"], p["y"], ow, oh, p["ext"], bg, sp))
            elif op == "flip":
                check(lib.mipx_op_flip(x.data_ptr(), y.data_ptr(), n, w, h, b, p["v"], sp))
            else:
                check(lib.mipx_op_rot(x.data_ptr(), y.data_ptr(), n, w, h, b, 180, sp))
        first = None
        for v in vals:
            os.environ[knob] = v
            lib.mipx_tuning_reload()
            y.zero_()
            run()
            torch.cuda.synchronize()
            ref = y.clone()
            if first is None:
                first = ref
            ms = timed(run, st)
            print(json.dumps({"op": op, "shape": [w, h, b, n], "params": p, knob: v, "ms": round(ms, 4),
                              "GBps": round((x.numel() + y.numel()) / ms / 1e6, 1),
                              "same_as_first": bool(torch.equal(ref, first))}), flush=True)
        os.environ.pop(knob)
        del x, y, first
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
