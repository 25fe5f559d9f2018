#!/usr/bin/env python3
"""Debug: where k_rcol (MIPX_RCOL=1) differs from the oracle on a few shapes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
os.environ["MIPX_RCOL"] = "1"
from imaginary_amd import engine as gpu
from oracle import oracle
from test_parity_gpu import rand_img, smooth_img
rng = np.random.default_rng(1)
for (h, w, b, hs, vs) in [(301, 1100, 3, 1.6, 1.6), (64, 256, 3, 1.6, 1.6), (301, 1100, 3, 2.4, 2.4), (200, 640, 4, 1.6, 1.6)]:
    for kind in ("rand", "const", "smooth"):
        if kind == "rand":
            im = rand_img(rng, h, w, b)
        elif kind == "const":
            im = np.full((h, w, b), 100, np.uint8)
        else:
            im = smooth_img(rng, h, w, b)
        imgs = np.stack([im, im])
        got = gpu.run_op("reduce", imgs, hshrink=hs, vshrink=vs)
        for i in range(2):
            want = oracle.reduce(imgs[i], hs, vs)
            d = np.argwhere(got[i] != want)
            print(f"{h}x{w}x{b} /{hs},{vs} {kind} img{i}: {len(d)} diffs", flush=True)
            if len(d):
                rows = sorted(set(d[:, 0].tolist()))
                cols = sorted(set(d[:, 1].tolist()))
                print("  rows", rows[:40], "cols", cols[:40])
                for q in d[:6]:
                    print("   ", q.tolist(), "got", got[i][tuple(q)], "want", want[tuple(q)])
