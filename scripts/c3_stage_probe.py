#!/usr/bin/env python3
"""C3's stages one at a time, same process, device-resident, HIP-event timed (median of 5
groups after a 200 ms warm-up): the blur on its own 768x512 images and on the 768x512
window of 768x768 images (the extract -> blur peephole, as inside C3), the window reduce
(1024^2 -> 768x768, extract 768x512) and the whole chain.  One JSON line per case."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ctypes as C  # noqa: E402

import torch  # noqa: E402

import imaginary_amd as ia  # noqa: E402
from bench_configs import Group, plan_for  # noqa: E402
from imaginary_amd._abi import check, lib  # noqa: E402


def chain(stages, w, h, b):
    plans = []
    for opts in stages:
        plans.append(plan_for(opts, w, h, b))
        w, h = plans[-1].out_w, plans[-1].out_h
    return ia.plan_chain(plans) if len(plans) > 1 else plans[0]


def main():
    n = int(os.environ.get("N", "512"))
    dev = torch.device("cuda", 0)
    check(lib.mipx_set_device(0))
    st = torch.cuda.current_stream(dev)
    sp = C.c_void_p(st.cuda_stream)
    cases = [
        ("blur 768x512", chain([dict(sigma=5.0)], 768, 512, 4)),
        ("crop+blur window of 768x768", chain([dict(width=768, height=512, crop=1), dict(sigma=5.0)], 768, 768, 4)),
        ("reduce 1024->768 + crop", chain([dict(width=768), dict(width=768, height=512, crop=1)], 1024, 1024, 4)),
        ("reduce 1024->768", chain([dict(width=768)], 1024, 1024, 4)),
        ("C3 chain", chain([dict(width=1024, embed=1), dict(width=768, height=512, crop=1), dict(sigma=5.0)], 2048, 2048, 4)),
    ]
    for name, plan in cases:
        g = Group(plan, n, dev, 3)
        run = lambda: g.run(sp)  # noqa: E731
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        k = 0
        while True:
            run()
            k += 1
            if k % 10 == 0:
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
        ms = statistics.median(ts)
        print(json.dumps({"case": name, "n": n, "ms": round(ms, 4), "plan": plan.describe()}), flush=True)
        del g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
