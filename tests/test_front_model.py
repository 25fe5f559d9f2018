"""CPU model of the 2 x 2 front's operand tables (imaginary_amd/csrc/r2front.h rch_operands,
restated) under the v_mfma_i32_16x16x64_i8 lane layout (A lane l: M = l & 15, K = 16 (l >> 4)
+ e; B lane l: K = 16 (l >> 4) + e, N = l & 15; D lane l: M = 4 (l >> 4) + j, N = l & 15):
the vertical operand on dword columns of 16-row blocks and the horizontal operand on 64-byte
windows reproduce libvips' 2 x 2 Lanczos3 sums at both sampling conventions.  This is the
index check run before the kernels' first GPU run (the kernels themselves are checked on the
GPU by tests/test_chain_gpu.py)."""
import numpy as np
import pytest

CORNER = np.array([49, 0, -277, 0, 1248, 2053, 1248, 0, -277, 0, 49, 0])
CENTRE = np.array([15, 61, -139, -272, 555, 1828, 1828, 555, -272, -139, 61, 15])


def rch_operands(tap, B):
    GP = 4 if B == 3 else 3
    SH = 1 if B == 3 else 0
    v = np.zeros((64, 4, 16), np.int64)  # lane, [vh, vl, wh, wl], byte e
    for lane in range(64):
        m, kg = lane & 15, lane >> 4
        for e in range(16):
            r, cm = m >> 2, m & 3
            i = 4 * kg + (e >> 2) - 2 * r
            tv = tap[i] if (r < 3 and (e & 3) == cm and 0 <= i < 12) else 0
            k = 16 * kg + e - SH - m % B
            ih = k // B - 2 * (m // B) if (k >= 0 and k % B == 0) else -1
            th = tap[ih] if (m < B * GP and 0 <= ih < 12) else 0
            for o, val in enumerate([tv >> 6, tv - 64 * (tv >> 6), th >> 6, th - 64 * (th >> 6)]):
                v[lane, o, e] = val
    return v


def mfma(A, Bm):
    Am = np.zeros((16, 64), np.int64)
    Bk = np.zeros((64, 16), np.int64)
    for l in range(64):
        Am[l & 15, 16 * (l >> 4):16 * (l >> 4) + 16] = A[l]
        Bk[16 * (l >> 4):16 * (l >> 4) + 16, l & 15] = Bm[l]
    D = Am @ Bk
    out = np.zeros((64, 4), np.int64)
    for l in range(64):
        out[l] = D[4 * (l >> 4):4 * (l >> 4) + 4, l & 15]
    return out


def u8_minus_128(x):
    return np.clip(x >> 12, -128, 127)


@pytest.mark.parametrize("tap", [CORNER, CENTRE], ids=["corner", "centre"])
@pytest.mark.parametrize("B", [3, 4])
def test_front_operands_reproduce_the_2x2_sums(tap, B):
    rng = np.random.default_rng(1)
    ops = rch_operands(tap, B)
    seed = 128 * int(tap.sum()) + 2048 - (128 << 12)
    H = 80
    img = rng.integers(0, 256, (H, 64), dtype=np.int64)  # 16 dword columns
    P = 7
    for g in range(5):  # vertical: 3-row groups of a 15-row step
        Bop = np.zeros((64, 16), np.int64)
        for l in range(64):
            n, kg = l & 15, l >> 4
            for j in range(4):
                r = min(max(2 * (P + 3 * g) - 5 + 4 * kg + j, 0), H - 1)
                for by in range(4):
                    Bop[l, 4 * j + by] = img[r, 4 * n + by] - 128
        val = u8_minus_128((mfma(ops[:, 0], Bop) << 6) + mfma(ops[:, 1], Bop) + seed)
        for l in range(64):
            n, kg = l & 15, l >> 4
            if kg >= 3:
                continue
            R = P + 3 * g + kg
            for c in range(4):
                want = sum(int(tap[i]) * int(img[min(max(2 * R - 5 + i, 0), H - 1), 4 * n + c]) for i in range(12))
                assert val[l, c] == min(max((want + 2048) >> 12, 0), 255) - 128
    GP = 4 if B == 3 else 3
    SH = 1 if B == 3 else 0
    inter = rng.integers(-128, 128, (16, 256), dtype=np.int64)
    for ish in (SH, SH + 8, SH + 40):  # horizontal: groups of GP pixels from a 64-byte window
        for q in range(3):
            base = (ish & ~7) + 2 * B * GP * q
            Bop = np.stack([inter[l & 15, base + 16 * (l >> 4): base + 16 * (l >> 4) + 16] for l in range(64)])
            val = u8_minus_128((mfma(ops[:, 2], Bop) << 6) + mfma(ops[:, 3], Bop) + seed)
            for l in range(64):
                n, kg = l & 15, l >> 4
                for jj in range(4):
                    j = 4 * kg + jj
                    if j >= B * GP:
                        continue
                    x, c = GP * q + j // B, j % B
                    want = sum(int(tap[i]) * (int(inter[n, ish + B * (2 * x + i) + c]) + 128) for i in range(12))
                    assert val[l, jj] == min(max((want + 2048) >> 12, 0), 255) - 128
