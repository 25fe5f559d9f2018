#!/usr/bin/env python3
"""Same-process A/B of the generic reduce kernels (k_rcol vs the previous default),
interleaved rounds (cdna_hip_programming.md §5.4 rule 24).  Every variant is first
checked bit-exact against the oracle on two images of the shape, then timed with HIP
events on a device-resident batch.  One JSON line per (shape, variant).

    VARIANTS='MIPX_RCOL=1;MIPX_RCOL=0' python scripts/ab_rcol.py
"""
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from imaginary_amd._abi import check, lib  # noqa: E402
from oracle import oracle as o  # noqa: E402

SHAPES = [  # w, h, b, n, hs, vs  (op_survey rows)
    (1920, 1080, 3, 64, 1.6, 1.6),
    (1920, 1080, 3, 64, 2.4, 2.4),
    (500, 375, 3, 128, 1.46484375, 1.46484375),
    (480, 270, 3, 256, 1.6, 1.5976331360946747),
    (1024, 1024, 4, 512, 1.3333333333333333, 1.3333333333333333),
    (1920, 1080, 4, 64, 1.6, 1.6),
    (1000, 750, 3, 64, 1.5625, 1.5625),
    (1333, 1000, 3, 48, 1.6666666666666667, 1.6666666666666667),
]
if os.environ.get("SHAPES"):
    SHAPES = [tuple(float(v) if "." in v else int(v) for v in s.split(",")) for s in os.environ["SHAPES"].split(";")]
variants = [dict(kv.split("=") for kv in v.split(",") if kv) for v in os.environ.get("VARIANTS", "MIPX_RCOL=1;MIPX_RCOL=0").split(";")]
rounds = int(os.environ.get("ROUNDS", "5"))
steps = int(os.environ.get("AB_STEPS", "10"))
dev = torch.device("cuda", 0)
check(lib.mipx_set_device(0))
st = torch.cuda.current_stream(dev)
sp = C.c_void_p(st.cuda_stream)


def vips_round(v):
    import math
    return int(math.floor(v + 0.5))


def setenv(var):
    keys = {k for v in variants for k in v}
    for k in keys:
        os.environ.pop(k, None)
    os.environ.update(var)
    if hasattr(lib, "mipx_tuning_reload"):
        lib.mipx_tuning_reload()


for (w, h, b, n, hs, vs) in SHAPES:
    ow, oh = vips_round(w / hs), vips_round(h / vs)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    x = torch.randint(0, 256, (n * w * h * b,), dtype=torch.uint8, device=dev, generator=g)
    y = torch.empty((n * ow * oh * b,), dtype=torch.uint8, device=dev)
    ws = torch.empty((n * w * h * b + 4096,), dtype=torch.uint8, device=dev)

    def run(nimg):
        check(lib.mipx_op_reduce(x.data_ptr(), y.data_ptr(), nimg, w, h, b, hs, vs, ws.data_ptr(), ws.numel(), sp), "reduce")

    want = [o.reduce(x[i * w * h * b:(i + 1) * w * h * b].cpu().numpy().reshape(h, w, b), hs, vs) for i in range(2)]
    ok = []
    for var in variants:
        setenv(var)
        y.zero_()
        run(2)
        torch.cuda.synchronize()
        got = y[:2 * ow * oh * b].cpu().numpy().reshape(2, oh, ow, b)
        ok.append(all(np.array_equal(got[i], want[i]) for i in range(2)))
    times = [[] for _ in variants]
    for r in range(rounds):
        for k, var in enumerate(variants):
            setenv(var)
            run(n)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(steps):
                run(n)
            e1.record(st)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / steps)
    alg = n * (w * h * b + ow * oh * b)
    for k, var in enumerate(variants):
        med = statistics.median(times[k])
        print(json.dumps({"shape": f"{w}x{h}x{b} n{n} /{hs:.4g},{vs:.4g}", "variant": var, "exact": ok[k],
                          "median_ms": round(med, 4), "GBps": round(alg / med / 1e6, 1),
                          "frac": round(alg / med / 1e6 / 8000, 4)}), flush=True)
