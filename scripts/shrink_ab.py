#!/usr/bin/env python3
"""Same-process A/B of the box-shrink kernels on the C5 shapes (env knobs are read
per launch).  One JSON line per (shape, variant): device ms per launch (HIP events),
algorithmic GB/s = in + out, and whether the output equals the first variant's."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from imaginary_amd._abi import check, lib  # noqa: E402

SHAPES = [  # w, h, b, n, s
    (1920, 1080, 3, 64, 2), (3840, 2160, 3, 32, 2), (4000, 3000, 3, 32, 2), (3840, 2160, 3, 32, 3),
    (4000, 3000, 3, 32, 3), (1920, 1080, 3, 64, 4), (3840, 2160, 3, 32, 4), (4000, 3000, 3, 32, 4),
    (2048, 2048, 4, 32, 2), (2048, 2048, 4, 32, 3),
]
if os.environ.get("SHRINK_SHAPES"):  # e.g. "4000x3000x3x32x8;..."
    SHAPES = [tuple(int(v) for v in t.split("x")) for t in os.environ["SHRINK_SHAPES"].split(";")]


def vr(v):
    import math
    return max(1, int(math.floor(v + 0.5)))


def main():
    variants = [dict(kv.split("=") for kv in v.split(",")) for v in sys.argv[1:]] or [
        dict(MIPX_SHRINK_Q="1"), dict(MIPX_SHRINK_Q="0")]
    dev = torch.device("cuda", 0)
    check(lib.mipx_set_device(0))
    st = torch.cuda.current_stream(dev)
    sp = C.c_void_p(st.cuda_stream)
    for (w, h, b, n, s) in SHAPES:
        ow, oh = vr(w / s), vr(h / s)
        x = torch.randint(0, 256, (n * w * h * b,), dtype=torch.uint8, device=dev)
        y = torch.empty((n * ow * oh * b,), dtype=torch.uint8, device=dev)
        outs = {}
        for rep in range(2):
            for v in variants:
                os.environ.update(v)
                lib.mipx_tuning_reload()  # the library snapshots MIPX_* knobs

                def run():
                    check(lib.mipx_op_shrink(x.data_ptr(), y.data_ptr(), n, w, h, b, s, s, sp))
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
                    print(json.dumps({"shape": [w, h, b, n, s], "variant": key, "ms": round(ms, 4),
                                      "alg_GBps": round(alg / ms / 1e6, 1), "same_as_first": same}), flush=True)
        del x, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
