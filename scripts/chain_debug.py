#!/usr/bin/env python3
"""Diagnostics for k_rchain mismatches: per case, where the chained output differs from
the two-kernel path (rows / columns / channels of the first differences)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import imaginary_amd as ia  # noqa: E402

CASES = [(512, 512, 3, dict(width=192, height=128, crop=1)), (512, 512, 4, dict(width=192, height=128, crop=1)),
         (600, 400, 3, dict(width=225, height=150, embed=1)), (132, 90, 3, dict(width=40, height=28, embed=1))]
for w, h, b, o2 in CASES:
    p1 = ia.plan_make(ia.make_opts(width=w // 2, embed=1), ia.make_input(w, h, b, "png"))
    p2 = ia.plan_make(ia.make_opts(**o2), ia.make_input(p1.out_w, p1.out_h, b, "png"))
    plan = ia.plan_chain([p1, p2])
    px = np.random.default_rng(1).integers(0, 256, (1, h, w, b), dtype=np.uint8)
    os.environ["MIPX_CHAIN"] = "0"
    ref = ia.execute(plan, px)[0].astype(int)
    os.environ["MIPX_CHAIN"] = "2"
    os.environ["MIPX_CHAIN_DBG"] = sys.argv[1] if len(sys.argv) > 1 else "0"
    got = ia.execute(plan, px)[0].astype(int)
    os.environ["MIPX_CHAIN_DBG"] = "0"
    d = np.argwhere(got != ref)
    print(f"{w}x{h}x{b} {o2}: out {ref.shape}, {len(d)} differ")
    if len(d):
        rows = np.unique(d[:, 0]); cols = np.unique(d[:, 1])
        print("  rows", rows[:10], "...", rows[-5:], " cols", cols[:10], "...", cols[-5:])
        print("  chans", np.unique(d[:, 2]))
        y, x = d[0][:2]
        print("  ref row", y, ref[y, x:x + 6].tolist(), "got", got[y, x:x + 6].tolist())
        # shifted copies?
        for dy in range(-3, 4):
            for dx in range(-3, 4):
                a = got[8:-8, 8:-8]; r = ref[8 + dy:ref.shape[0] - 8 + dy, 8 + dx:ref.shape[1] - 8 + dx]
                if a.shape == r.shape and np.mean(a == r) > 0.9:
                    print("  got ~ ref shifted by", dy, dx, np.mean(a == r))
        for c in range(b):
            for c2 in range(b):
                if c != c2 and np.mean(got[..., c] == ref[..., c2]) > 0.9:
                    print("  channel", c, "~ ref channel", c2)
