#!/usr/bin/env python3
"""Same-process A/B of the gaussblur kernels on the op-survey / C3 / C5 shapes (env
knobs are read per launch).  One JSON line per (shape, variant): device ms per
launch, algorithmic GB/s = in + out, and whether the output equals the first variant's."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from imaginary_amd._abi import check, lib  # noqa: E402

SHAPES = [  # w, h, b, n, sigma
    (1920, 1080, 3, 64, 1.0), (1920, 1080, 3, 64, 3.0), (1920, 1080, 3, 64, 5.0), (3840, 2160, 3, 16, 3.0),
    (4000, 3000, 3, 16, 5.0), (768, 512, 4, 512, 5.0),
]


def main():
    variants = [dict(kv.split("=") for kv in v.split(",")) for v in sys.argv[1:]]
    dev = torch.device("cuda", 0)
    check(lib.mipx_set_device(0))
    st = torch.cuda.current_stream(dev)
    sp = C.c_void_p(st.cuda_stream)
    for (w, h, b, n, sg) in SHAPES:
        x = torch.randint(0, 256, (n * w * h * b,), dtype=torch.uint8, device=dev)
        y = torch.empty((n * w * h * b,), dtype=torch.uint8, device=dev)
        wsb = n * w * h * b + 4096
        ws = torch.empty((wsb,), dtype=torch.uint8, device=dev)
        outs = {}
        for rep in range(2):
            for v in variants:
                os.environ.update(v)
                lib.mipx_tuning_reload()  # the library snapshots MIPX_* knobs

                def run():
                    check(lib.mipx_op_gaussblur(x.data_ptr(), y.data_ptr(), n, w, h, b, sg, 0.2, ws.data_ptr(), wsb, sp))
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
                    print(json.dumps({"shape": [w, h, b, n, sg], "variant": key, "ms": round(ms, 4),
                                      "alg_GBps": round(alg / ms / 1e6, 1), "same_as_first": same}), flush=True)
        del x, y, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
