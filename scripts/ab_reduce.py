#!/usr/bin/env python3
"""A/B the fused 2x2 reduce variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Each variant is first checked
bit-exact against the oracle, then timed with HIP events on the C2 batch."""
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import numpy as np  # noqa: E402

import imaginary_amd as ia  # noqa: E402
from imaginary_amd._abi import check, lib  # noqa: E402
from oracle import oracle as o  # noqa: E402

variants = [int(v) for v in os.environ.get("VARIANTS", "0,1,2,3,4,5,6,7").split(",")]
rounds = int(os.environ.get("ROUNDS", "5"))
steps = int(os.environ.get("AB_STEPS", "5"))
bands = int(os.environ.get("BANDS", "3"))
n = int(os.environ.get("BATCH", "256"))
W, H = 3840, 2160
dev = torch.device("cuda", 0)
lib.mipx_set_device(0)
g = torch.Generator(device=dev)
g.manual_seed(1)
x = torch.randint(0, 256, (n, H * W * bands), dtype=torch.uint8, device=dev, generator=g)
y = torch.empty((n, (H // 2) * (W // 2) * bands), dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream(dev)
sp = C.c_void_p(st.cuda_stream)


def run(var, nimg=n):
    os.environ["MIPX_R2_VARIANT"] = str(var)
    lib.mipx_tuning_reload()  # the library snapshots MIPX_* knobs
    check(lib.mipx_op_reduce(x.data_ptr(), y.data_ptr(), nimg, W, H, bands, 2.0, 2.0, None, 0, sp), "reduce")


ok = {}
ref = o.reduce(x[0].cpu().numpy().reshape(H, W, bands), 2.0, 2.0)
for v in variants:
    run(v, 2)
    torch.cuda.synchronize()
    got = y[0].cpu().numpy().reshape(H // 2, W // 2, bands)
    ok[v] = bool(np.array_equal(got, ref))
times = {v: [] for v in variants}
for r in range(rounds):
    for v in variants:
        run(v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(steps):
            run(v)
        e1.record(st)
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) / steps)
alg = n * (H * W * bands + (H // 2) * (W // 2) * bands)
for v in variants:
    med = statistics.median(times[v])
    print(json.dumps({"variant": v, "exact": ok[v], "median_ms": round(med, 4), "min_ms": round(min(times[v]), 4),
                      "GBps": round(alg / med / 1e6, 1), "frac": round(alg / med / 1e6 / 8000, 4)}))
