// r2front.h — the 2 x 2 reduce "front" shared by k_rchain (k_rcol.hip) and k_reduce2d
// (k_reduce2m.hip): its geometry constants and the host-built per-lane MFMA operands.
//
// The vertical pass runs straight from HBM into v_mfma_i32_16x16x64_i8: a lane (n, kg)
// loads dword column n of input rows 4 kg .. 4 kg + 3 of a 16-row block (the B operand,
// K = (row, byte)); the A operand holds the taps at M = (output row r < 3, byte c), so D
// lane (n, kg) is output row kg's dword n (3 output rows per 16-row block: 2 r + 12 taps
// <= 16).  The horizontal pass is k_reduce2m's banded product: GP output pixels from a
// 64-byte window of each of 16 vertical-result rows.  Both conventions: the 12 taps from
// 2x - 5 of the phase the convention gives (reduce2_front_taps).
#pragma once
#include <cstdint>
#include <vector>

namespace mipx {

template <int B>
struct RCH {
    static constexpr int GP = B == 3 ? 4 : 3;    // output pixels per horizontal group (<= 64-byte window)
    static constexpr int LOFF = B == 3 ? 0 : 4;  // LDS byte of the vertical result's 64-byte tile origin
    // (B (2 x0 - 5) - 64-byte aligned base + LOFF) mod 8 for every strip origin x0 on 4 pixels:
    // the 12-tap window of GP pixels then fits 64 bytes (RGBA: 0 + 4 x 15 + 4; RGB: 1 + 3 x 17 + 3)
    static constexpr int SH = B == 3 ? 1 : 0;
};

// The front's per-lane MFMA operands, [lane][vh, vl, wh, wl] x 16 bytes (taps = the 12
// taps from 2x - 5 of the 2 x 2 reduce at the sampling convention's phase):
//   vertical A, lane (m, kg): M = (row r = m / 4 < 3, byte c = m % 4), K = 16 kg + e =
//     (block row 4 kg + e / 4, byte e % 4): tap (block row - 2 r) where the bytes match;
//   horizontal A (k_reduce2m's W): output byte j = m < B GP takes tap i at window byte
//     SH + B (2 (j / B) + i) + j % B.
// Every tap T = 64 hi + lo (lo in [0, 63]).
template <int B>
inline std::vector<uint32_t> rch_operands(const int *tap) {
    using G = RCH<B>;
    std::vector<uint32_t> v(64 * 16, 0);
    for (int lane = 0; lane < 64; ++lane) {
        const int m = lane & 15, kg = lane >> 4;
        for (int e = 0; e < 16; ++e) {
            const int r = m >> 2, cm = m & 3;
            const int i = 4 * kg + (e >> 2) - 2 * r;
            const int tv = (r < 3 && (e & 3) == cm && i >= 0 && i < 12) ? tap[i] : 0;
            const int k = 16 * kg + e - G::SH - m % B;
            const int ih = k >= 0 && k % B == 0 ? k / B - 2 * (m / B) : -1;
            const int th = (m < B * G::GP && ih >= 0 && ih < 12) ? tap[ih] : 0;
            const int t4[4] = {tv >> 6, tv - 64 * (tv >> 6), th >> 6, th - 64 * (th >> 6)};
            for (int o = 0; o < 4; ++o)
                v[16 * lane + 4 * o + e / 4] |= (static_cast<uint32_t>(t4[o]) & 0xffu) << (8 * (e % 4));
        }
    }
    return v;
}


}  // namespace mipx
