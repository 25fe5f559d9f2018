#!/usr/bin/env python3
"""Time one libmipx op on a device-resident batch (HIP events on its stream) so
rocprofv3 passes see that kernel alone.

    python scripts/op_bench.py reducev --w 1024 --h 1024 --b 4 --n 512 --s 1.3333333333333333
    ops: reduce reducev reduceh shrink blur embed rot flip extract affine zoom
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from imaginary_amd._abi import check, lib  # noqa: E402


def vips_round(v):
    import math
    return int(math.floor(v + 0.5))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("op")
    ap.add_argument("--w", type=int, default=1024)
    ap.add_argument("--h", type=int, default=1024)
    ap.add_argument("--b", type=int, default=4)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--s", type=float, default=2.0, help="shrink / sigma / angle")
    ap.add_argument("--s2", type=float, default=0.0, help="vertical shrink (reduce/shrink); 0 = same")
    ap.add_argument("--ow", type=int, default=0)
    ap.add_argument("--oh", type=int, default=0)
    ap.add_argument("--extend", type=int, default=1)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ab", default="", help="KNOB=v1,v2,...: same-process A/B of a MIPX_* knob")
    ap.add_argument("--warm-ms", type=float, default=200.0, help="device-time warm-up; 0: none, one group (PMC runs)")
    ap.add_argument("--sampling", choices=["corner", "centre"], default=None,
                    help="reduce sampling convention (mipx_set_reduce_sampling); default: the library's")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    check(lib.mipx_set_device(0))
    if a.sampling:
        check(lib.mipx_set_reduce_sampling({"corner": 0, "centre": 1}[a.sampling]))
    w, h, b, n = a.w, a.h, a.b, a.n
    s2 = a.s2 or a.s
    if a.op in ("reduce", "reducev", "reduceh"):
        ow = vips_round(w / a.s) if a.op != "reducev" else w
        oh = vips_round(h / s2) if a.op != "reduceh" else h
    elif a.op == "shrink":
        ow, oh = max(1, vips_round(w / a.s)), max(1, vips_round(h / s2))
    elif a.op == "affine":
        import math
        ow, oh = math.ceil(w * a.s), math.ceil(h * s2)
    elif a.op == "zoom":
        ow, oh = w * int(a.s), h * int(s2)
    elif a.op == "rot":
        ow, oh = (h, w) if int(a.s) % 180 == 90 else (w, h)
    elif a.op in ("embed", "extract"):
        ow, oh = a.ow or w, a.oh or h
    else:
        ow, oh = w, h
    x = torch.randint(0, 256, (n * w * h * b,), dtype=torch.uint8, device=dev)
    y = torch.empty((n * ow * oh * b,), dtype=torch.uint8, device=dev)
    ws = torch.empty((n * max(w * h, ow * oh) * b + 4096,), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)
    sp = C.c_void_p(st.cuda_stream)
    X, Y, WS, WSB = x.data_ptr(), y.data_ptr(), ws.data_ptr(), ws.numel()
    bg = (C.c_int32 * 3)(10, 20, 30)

    def run():
        if a.op == "reduce":
            return lib.mipx_op_reduce(X, Y, n, w, h, b, a.s, s2, WS, WSB, sp)
        if a.op == "reducev":
            return lib.mipx_op_reducev(X, Y, n, w, h, b, s2, sp)
        if a.op == "reduceh":
            return lib.mipx_op_reduceh(X, Y, n, w, h, b, a.s, sp)
        if a.op == "shrink":
            return lib.mipx_op_shrink(X, Y, n, w, h, b, int(a.s), int(s2), sp)
        if a.op == "blur":
            return lib.mipx_op_gaussblur(X, Y, n, w, h, b, a.s, 0.2, WS, WSB, sp)
        if a.op == "embed":
            return lib.mipx_op_embed(X, Y, n, w, h, b, (ow - w) // 2, (oh - h) // 2, ow, oh, a.extend, bg, sp)
        if a.op == "extract":
            return lib.mipx_op_extract(X, Y, n, w, h, b, (w - ow) // 2, (h - oh) // 2, ow, oh, sp)
        if a.op == "rot":
            return lib.mipx_op_rot(X, Y, n, w, h, b, int(a.s), sp)
        if a.op == "flip":
            return lib.mipx_op_flip(X, Y, n, w, h, b, int(a.s), sp)
        if a.op == "affine":
            return lib.mipx_op_affine(X, Y, n, w, h, b, a.s, s2, a.extend, sp)
        if a.op == "zoom":
            return lib.mipx_op_zoom(X, Y, n, w, h, b, int(a.s), int(s2), sp)
        raise SystemExit(a.op)

    # warm-up of >= 200 ms of device time first: a fresh process's first milliseconds run
    # below the sustained clock (r03: a 20-launch run of a 0.2 ms kernel read 15-20 % slow
    # against the same kernel in a long same-process A/B); then the median of 5 groups
    def measure():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        check(run(), a.op)
        torch.cuda.synchronize()
        warm = 0.0
        while warm < a.warm_ms:
            e0.record(st)
            for _ in range(10):
                check(run(), a.op)
            e1.record(st)
            torch.cuda.synchronize()
            warm += e0.elapsed_time(e1)
        groups = []
        for _ in range(5 if a.warm_ms > 0 else 1):
            e0.record(st)
            for _ in range(a.iters):
                check(run(), a.op)
            e1.record(st)
            torch.cuda.synchronize()
            groups.append(e0.elapsed_time(e1) / a.iters)
        return sorted(groups)[len(groups) // 2]

    alg = n * (w * h * b + ow * oh * b)
    line = {"op": a.op, "w": w, "h": h, "b": b, "n": n, "s": a.s, "s2": s2, "out": [ow, oh],
            "sampling": ["corner", "centre"][lib.mipx_reduce_sampling()]}
    if not a.ab:
        ms = measure()
        print(json.dumps({**line, "ms": round(ms, 4), "alg_GBps": round(alg / ms / 1e6, 1)}))
        return
    # same-process A/B: --ab KNOB=v1,v2,... interleaved over 2 rounds, output checked equal
    knob, vals = a.ab.split("=", 1)
    first = None
    for rnd in range(2):
        for v in vals.split(","):
            os.environ[knob] = v
            lib.mipx_tuning_reload()  # the library snapshots MIPX_* knobs
            ms = measure()
            same = None
            if rnd == 0:
                y.zero_()
                check(run(), a.op)
                torch.cuda.synchronize()
                if first is None:
                    first = y.clone()
                same = bool(torch.equal(y, first))
            print(json.dumps({**line, knob: v, "round": rnd, "ms": round(ms, 4), "alg_GBps": round(alg / ms / 1e6, 1),
                              "same_as_first": same}), flush=True)

if __name__ == "__main__":
    main()
