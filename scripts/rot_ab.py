#!/usr/bin/env python3
"""Same-process A/B of rot 90 / 270 on C5's shapes (env knobs read per launch): one
JSON line per (shape, angle, variant) with device ms, algorithmic GB/s (in + out) and
whether the output equals the first variant's."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from imaginary_amd._abi import check, lib  # noqa: E402

SHAPES = [(1920, 1080, 3, 32), (3840, 2160, 3, 16), (4000, 3000, 3, 16), (3840, 2160, 4, 16)]


def main():
    variants = [dict(kv.split("=") for kv in v.split(",")) for v in sys.argv[1:]]
    dev = torch.device("cuda", 0)
    check(lib.mipx_set_device(0))
    st = torch.cuda.current_stream(dev)
    sp = C.c_void_p(st.cuda_stream)
    for (w, h, b, n) in SHAPES:
        x = torch.randint(0, 256, (n * w * h * b,), dtype=torch.uint8, device=dev)
        y = torch.empty((n * w * h * b,), dtype=torch.uint8, device=dev)
        for ang in [int(v) for v in os.environ.get("ANGLES", "90,270").split(",")]:
            outs = {}
            for rep in range(2):
                for v in variants:
                    os.environ.update(v)
                    lib.mipx_tuning_reload()  # the library snapshots MIPX_* knobs

                    def run():
                        check(lib.mipx_op_rot(x.data_ptr(), y.data_ptr(), n, w, h, b, ang, sp))
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
                        alg = n * 2 * w * h * b
                        same = bool(torch.equal(outs[key], outs[list(outs)[0]]))
                        print(json.dumps({"shape": [w, h, b, n], "angle": ang, "variant": key, "ms": round(ms, 4),
                                          "alg_GBps": round(alg / ms / 1e6, 1), "same_as_first": same}), flush=True)
        del x, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
