#!/usr/bin/env python3
"""Same-process A/B of the generic reduce paths on the op_survey shapes: env knobs
are read per launch, so the variants interleave on one box.  One JSON line per
(shape, variant): device ms per launch (HIP events), algorithmic GB/s = in + out."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from imaginary_amd._abi import check, lib  # noqa: E402

SHAPES = [  # w, h, b, n, hs, vs
    (1920, 1080, 3, 64, 1.6, 1.6),
    (1920, 1080, 3, 64, 2.4, 2.4),
    (1024, 1024, 4, 512, 4 / 3, 4 / 3),
    (500, 375, 3, 128, 1.46484375, 1.46484375),
    (364, 273, 3, 128, 1.421875, 1.06640625),
    (480, 270, 3, 256, 1.6, 1.5976331360946747),
    (1920, 1080, 4, 64, 1.6, 1.6),
    (1000, 750, 3, 64, 1.5625, 1.5625),
]
VARIANTS = [dict(MIPX_RSTRIP="1"), dict(MIPX_RSTRIP="0")]


def vr(v):
    import math
    return int(math.floor(v + 0.5))


def main():
    global SHAPES
    args = sys.argv[1:]
    if args and args[0] == "--hshapes":  # horizontal-pass shapes (vshrink 1: reduceh alone)
        args = args[1:]
        SHAPES = [(w, h, b, n, s, 1.0) for (w, h, b, n, s) in (
            (1920, 675, 3, 64, 1.6), (3840, 1350, 3, 16, 1.6), (2000, 1071, 3, 32, 1.4), (800, 462, 3, 128, 1.3),
            (1920, 831, 3, 64, 1.3), (1280, 576, 3, 96, 1.25), (640, 320, 3, 256, 1.5), (500, 256, 3, 256, 1.46484375),
            (1920, 450, 3, 64, 2.4), (1920, 675, 4, 64, 1.6), (1024, 768, 4, 128, 1.3333333333333333),
            (1000, 480, 3, 128, 1.5625), (4000, 1500, 3, 8, 1.9))]
    if os.environ.get("RS_SHAPES"):  # "w,h,b,n,hs,vs;..."
        SHAPES = [tuple(float(t) if "." in t else int(t) for t in sh.split(",")) for sh in os.environ["RS_SHAPES"].split(";")]
    extra = [dict(kv.split("=") for kv in v.split(",")) for v in args]
    variants = extra or VARIANTS
    dev = torch.device("cuda", 0)
    check(lib.mipx_set_device(0))
    if os.environ.get("RS_SAMPLING"):  # corner / centre (mipx_set_reduce_sampling)
        check(lib.mipx_set_reduce_sampling({"corner": 0, "centre": 1}[os.environ["RS_SAMPLING"]]))
    st = torch.cuda.current_stream(dev)
    sp = C.c_void_p(st.cuda_stream)
    for (w, h, b, n, hs, vs) in SHAPES:
        ow, oh = vr(w / hs), vr(h / vs)
        x = torch.randint(0, 256, (n * w * h * b,), dtype=torch.uint8, device=dev)
        y = torch.empty((n * ow * oh * b,), dtype=torch.uint8, device=dev)
        wsb = n * w * oh * b + 4096
        ws = torch.empty((wsb,), dtype=torch.uint8, device=dev)
        outs = {}
        for rep in range(2):
            for v in variants:
                os.environ.update(v)
                lib.mipx_tuning_reload()  # the library snapshots MIPX_* knobs
                def run():
                    check(lib.mipx_op_reduce(x.data_ptr(), y.data_ptr(), n, w, h, b, hs, vs, ws.data_ptr(), wsb, sp))
                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(20):
                    run()
                e1.record(st)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 20
                key = ",".join(f"{k}={val}" for k, val in v.items())
                if rep == 0:
                    outs[key] = y.clone()
                else:
                    alg = n * (w * h * b + ow * oh * b)
                    same = bool(torch.equal(outs[key], outs[list(outs)[0]]))
                    print(json.dumps({"shape": [w, h, b, n, hs, vs], "variant": key, "ms": round(ms, 4),
                                      "alg_GBps": round(alg / ms / 1e6, 1), "same_as_first": same}), flush=True)
        del x, y, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
