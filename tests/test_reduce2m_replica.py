"""CPU check of k_reduce2m's index arithmetic (k_reduce2m.hip): a numpy replica of its
two banded products at the centre sampling convention -- the vertical one over K = 64
staged rows (lane group kg, element e <-> row 8 kg + e / 32 + 8 kg + e - 8, tap row - 2 n),
the horizontal one over a 64-byte window starting 8-byte aligned (output byte j takes tap
i at window byte SH + B (2 (j / B) + i) + j % B), both with taps split 64 hi + lo, pixels
- 128 and the seed 128 sum(T) + 2048 -- plus the staging (16-byte-aligned strip origin,
zeros left of the image, rows clamped) and the COPY-edge fix-up of the intermediate,
against the oracle's reduce 2 x 2 on small images.  The GPU kernel itself is tested in
test_parity_gpu.py::test_reduce2x2_variants_exact."""
import numpy as np
import pytest

from oracle import oracle as o

T = [15, 61, -139, -272, 555, 1828, 1828, 555, -272, -139, 61, 15]  # phase 64 of shrink 2


def _split(t):
    hi = t >> 6
    return hi, t - 64 * hi


def _replica(img):
    h, w, B = img.shape
    ow, oh = (w + 1) // 2, (h + 1) // 2  # out_size_reduce(w, 2) for these sizes
    OFF = 1 if B == 3 else 12
    ISH = 0 if B == 3 else 4
    seed = 128 * sum(T) + 2048
    out = np.zeros((oh, ow, B), np.int64)
    for strip in range((ow + 63) // 64):
        x0 = 64 * strip
        px0 = 2 * x0 - 5
        org = (B * px0) & ~15
        assert (B * px0) - org == OFF
        for k in range((oh + 15) // 16):
            bk = 32 * k - 5
            # staged rows bk .. bk + 63 (only 42 carry taps), bytes org .. org + 16 CPR
            nbytes = OFF + B * (2 * 64 + 10) + 15 & ~15
            ring = np.zeros((64, nbytes + 64), np.int64)
            for rr in range(64):
                r = min(max(bk + rr, 0), h - 1)
                row = img[r].reshape(-1).astype(np.int64)
                for c in range(nbytes):
                    ib = org + c
                    ring[rr, c] = row[ib] if 0 <= ib < w * B else 0
            # vertical: output row n of the step, byte column c (all staged bytes)
            inter = np.zeros((16, nbytes + 64), np.int64)
            for n in range(16):
                acc = np.full(nbytes, seed, np.int64)
                for kg in range(4):
                    for e in range(16):
                        row = 8 * kg + e if e < 8 else 32 + 8 * kg + e - 8
                        i = row - 2 * n
                        if 0 <= i < 12:
                            hi, lo = _split(T[i])
                            acc += (64 * hi + lo) * (ring[row, :nbytes] - 128)
                inter[n, ISH: ISH + nbytes] = np.clip(acc >> 12, 0, 255)
            # COPY edge: strip pixels outside the image copy the edge pixel
            ib0 = OFF + ISH
            for p in range(2 * 64 + 10):
                ip = px0 + p
                if ip < 0 or ip >= w:
                    src = -px0 if ip < 0 else w - 1 - px0
                    inter[:, ib0 + B * p: ib0 + B * p + B] = inter[:, ib0 + B * src: ib0 + B * src + B]
            # horizontal: groups of GP output pixels, window from (ib0 & ~7) + 2 B GP g
            GP = 4 if B == 3 else 2
            SH = ib0 & 7
            for g in range(64 // GP):
                ws = (ib0 & ~7) + 2 * B * GP * g
                win = inter[:, ws: ws + 64] - 128
                for j in range(B * GP):
                    acc = np.full(16, seed, np.int64)
                    for kk in range(64):
                        r = kk - SH - j % B
                        if r >= 0 and r % B == 0:
                            i = r // B - 2 * (j // B)
                            if 0 <= i < 12:
                                hi, lo = _split(T[i])
                                acc += (64 * hi + lo) * win[:, kk]
                    x = x0 + GP * g + j // B
                    for n in range(16):
                        y = 16 * k + n
                        if x < ow and y < oh:
                            out[y, x, j % B] = np.clip(acc[n] >> 12, 0, 255)
    return out.astype(np.uint8)


@pytest.mark.parametrize("h,w,b", [(9, 12, 3), (40, 20, 4), (33, 140, 3), (17, 131, 4)])
def test_reduce2m_replica_matches_oracle(h, w, b):
    rng = np.random.default_rng(h * 100 + w + b)
    img = rng.integers(0, 256, (h, w, b), dtype=np.uint8)
    prev = o.get_switch("reduce_centre")
    o.set_switch("reduce_centre", 1)
    try:
        want = o.reduce(img, 2.0, 2.0)
    finally:
        o.set_switch("reduce_centre", prev)
    got = _replica(img)
    assert got.shape == want.shape
    assert np.array_equal(got, want), int((got != want).sum())
