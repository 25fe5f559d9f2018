"""CPU check of k_enlarge2's index arithmetic (k_affine.hip): a numpy replica of the
kernel's lane windows (staged bytes 2 l B .. of a 134-column strip row), its fixed
phase-96 / phase-32 taps, the 4-row H ring and the emission of output rows 2r-2 / 2r-3
per input row r, bands of 32 input rows and strips of 256 output pixels, against the
oracle's vips_affine at 2 x 2 on small images (every extend mode, 1-4 bands, several
strips and bands).  The GPU kernel itself is tested in test_affine_gpu.py."""
import numpy as np
import pytest

from oracle import oracle as o


def _taps():
    """oracle/vips_ref.c ref_bicubic_table: Catmull-Rom x 4096, truncated, 129 phases"""
    t = []
    for x in range(129):
        xx = float(np.float32(x / 128.0))
        cr1 = 1.0 - xx
        cr2 = -0.5 * xx
        cr3 = cr1 * cr2
        cone = cr1 * cr3
        cfou = xx * cr3
        cr4 = cfou - cone
        ctwo = cr1 - cr4 + cfou
        cthr = xx - cfou + cr4
        t += [int(cone * 4096), int(ctwo * 4096), int(cthr * 4096), int(cfou * 4096)]
    return t


def ext(v, n, e):
    if 0 <= v < n: return v
    if e == 1: return min(max(v, 0), n - 1)      # COPY
    if e == 2: return v % n                       # REPEAT
    if e == 3:
        u = v % (2 * n); return u if u < n else 2 * n - 1 - u   # MIRROR
    return -1
def run(img, extend, T):
    h, w, B = img.shape
    ow, oh = 2 * w, 2 * h
    fill = 255 if extend == 4 else 0
    out = np.zeros((oh, ow, B), np.uint8)
    e = T[96 * 4: 96 * 4 + 4]; od = T[32 * 4: 32 * 4 + 4]
    strips = (ow + 255) // 256; RB = 32; bands = (h + RB - 1) // RB
    for strip in range(strips):
        x0 = 256 * strip; c0 = x0 // 2 - 2
        for band in range(bands):
            ma = RB * band; mb = min(ma + RB, h); rfirst = ma - 2; rlast = mb + 1
            def staged(r):
                sr = ext(r, h, extend)
                row = np.zeros(134 * B + 64, np.int64)
                for t in range(134 * B):
                    col = c0 + t // B; ch = t % B
                    if sr < 0: row[t] = fill; continue
                    sc = ext(col, w, extend)
                    row[t] = fill if sc < 0 else img[sr, sc, ch]
                return row
            ring = {}
            for r in range(rfirst, rlast + 1):
                row = staged(r)
                H = np.zeros((64, 4 * B), np.int64)
                for lane in range(64):
                    wb = 2 * lane * B
                    win = row[wb: wb + 6 * B]
                    for px in range(4):
                        s = [0, 1, 1, 2][px]; taps = od if px & 1 else e
                        for c in range(B):
                            acc = 2048 + sum(taps[i] * win[(s + i) * B + c] for i in range(4))
                            H[lane, px * B + c] = acc >> 12
                ring[r] = H
                for (y, taps, ok) in ((2 * r - 2, e, ma <= r - 1 < mb), (2 * r - 3, od, ma <= r - 2 < mb)):
                    if not ok or y >= oh: continue
                    acc = 2048 + sum(taps[i] * ring[r - 3 + i] for i in range(4))
                    v = np.clip(acc >> 12, 0, 255)
                    for lane in range(64):
                        xl = x0 + 4 * lane
                        for px in range(4):
                            if xl + px < ow:
                                out[y, xl + px, :] = v[lane, px * B:(px + 1) * B]
    return out


@pytest.mark.parametrize("h,w,b,extend", [(9, 7, 3, 1), (5, 300, 4, 0), (40, 9, 1, 3), (3, 2, 2, 2), (1, 1, 4, 1),
                                          (6, 10, 3, 4), (4, 5, 3, 5)])
def test_enlarge2_replica_matches_oracle(h, w, b, extend):
    rng = np.random.default_rng(h * 1000 + w * 10 + b)
    img = rng.integers(0, 256, (h, w, b), dtype=np.uint8)
    got = run(img, extend, _taps())
    want = o.affine(img, 2.0, 2.0, extend).reshape(got.shape)
    assert np.array_equal(got, want), int((got != want).sum())
