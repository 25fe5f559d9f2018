#!/usr/bin/env python3
"""Same-process A/B of the embed kernel on C5's shapes (env knobs read per launch):
one JSON line per (shape, extend, variant) with device ms, algorithmic GB/s (in + out)
and whether the output equals the first variant's."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from imaginary_amd._abi import check, lib  # noqa: E402

SHAPES = [(1920, 1080, 16, 1920, 1920), (3840, 2160, 8, 3840, 3840), (4000, 3000, 8, 4000, 4000)]


def main():
    variants = [dict(kv.split("=") for kv in v.split(",")) for v in sys.argv[1:]]
    dev = torch.device("cuda", 0)
    check(lib.mipx_set_device(0))
    st = torch.cuda.current_stream(dev)
    sp = C.c_void_p(st.cuda_stream)
    bg = (C.c_int * 3)(0, 0, 0)
    for (w, h, n, ow, oh) in SHAPES:
        b = 3
        x = torch.randint(0, 256, (n * w * h * b,), dtype=torch.uint8, device=dev)
        y = torch.empty((n * ow * oh * b,), dtype=torch.uint8, device=dev)
        for ext in (0, 1, 2):
            outs = {}
            for rep in range(2):
                for v in variants:
                    os.environ.update(v)
                    lib.mipx_tuning_reload()  # the library snapshots MIPX_* knobs

                    def run():
                        check(lib.mipx_op_embed(x.data_ptr(), y.data_ptr(), n, w, h, b, (ow - w) // 2, (oh - h) // 2,
                                                ow, oh, ext, bg, sp))
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
                        alg = n * (w * h + ow * oh) * b
                        same = bool(torch.equal(outs[key], outs[list(outs)[0]]))
                        print(json.dumps({"shape": [w, h, n, ow, oh], "extend": ext, "variant": key, "ms": round(ms, 4),
                                          "alg_GBps": round(alg / ms / 1e6, 1), "same_as_first": same}), flush=True)
        del x, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
