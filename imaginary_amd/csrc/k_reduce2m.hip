// k_reduce2m.hip — the fused 2 x 2 Lanczos3 reduce under libvips' centre sampling
// convention (PARITY_ASSUMPTIONS.md row 1: X = (o + 0.5) * 2 - 0.5), with the vertical
// products on the i8 matrix cores.
//
// Every output of either pass is o = sum_{i=0..11} T_i p[2o - 5 + i] (phase 64; tap 12
// is zero).  k_reduce2c (k_reduce.hip) does both passes as f32 multiply-adds and is
// bound by that arithmetic.  Here the vertical pass, 12 of every 24
// multiply-adds per output byte and the more expensive half (its pixels also need
// converting), runs as a banded matrix product:
//   D[byte column][output row] = A[byte column][input row] x B[input row][output row]
// on v_mfma_i32_16x16x64_i8: 16 output rows need 42 input rows (K = 64, the rest carry
// zero taps), A is the staged pixels - 128 (two ds_read_b64_tr_b8 per 16-byte column
// tile), B the taps at row 2n + i of output row n, split T = 64 hi + lo (both i8) into
// two products rejoined as 64 D_hi + D_lo, with 128 sum(T) + 2048 seeded into D_lo, so
// (64 D_hi + D_lo) >> 12 clamped is libvips' rounded uchar intermediate exactly.  The
// horizontal pass stays k_reduce2c's f32 push form (12 v_fma_f32 per output byte).
//
// A block (4 waves) owns a strip of 64 output pixels of one image and walks a band of
// 16-row steps.  The strip's input rows (138 pixels, from the 16-byte-aligned-down start)
// live in an LDS ring of 64 rows; a step adds 32 rows (2 per output row), loaded one step
// ahead into registers as 16-byte chunks dealt over the 256 lanes, written to the ring
// XOR 0x80 once the previous step's vertical pass has read its rows.  Per step: barrier
// -> vertical (ring -> LDS intermediate, 16 rows) -> barrier -> next rows to the ring,
// next loads issued -> COPY-edge fix-up of the intermediate at the image edges ->
// horizontal (intermediate -> 12 / 8-byte stores).  Rows clamp at the load (COPY edge);
// input bytes left of the image are staged as zeros and replaced in the intermediate.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "device_common.h"
#include "lds_ops.h"

namespace mipx {
namespace {

using namespace dev;

constexpr int kMTW = 64;    // output pixels per strip
constexpr int kMN = 16;     // output rows per step (the MFMA N)
constexpr int kMNT = 256;

template <int B>
struct R2M {
    static constexpr int K = B == 3 ? 4 : 2;                 // output pixels per horizontal item
    static constexpr int OFF = B == 3 ? 1 : 12;              // (B px0) mod 16 for every strip
    static constexpr int ISH = B == 3 ? 0 : 4;               // intermediate byte shift: windows aligned
    static constexpr int CPR = (OFF + B * (2 * kMTW + 10) + 15) / 16;  // 16-byte chunks per staged row
    static constexpr int RS = B == 3 ? 432 : 592;            // row stride: (RS / 4 mod 64) / 4 odd
    static constexpr int KM = (32 * CPR + kMNT - 1) / kMNT;  // chunks per lane per step (32 rows)
    static constexpr int OS = B == 3 ? 208 : 272;            // HM output tile row stride (conflict-free)
    static_assert(RS >= 16 * CPR + ISH, "row stride");
    static_assert(((RS / 4) % 64 / 4) % 2 == 1, "conflict-free transposed reads");
};

struct R2mArgs {
    const u8 *in;
    u8 *out;
    int w, h, ow, oh;
    int x_end, y_end;       // computed region ends (exclusive); rows / strips start at k_base / s_base
    int s_base, k_base;
    int n_strips, n_bands, band_steps;
    long long in_img, out_img;
    int seed;               // 128 sum(T) + 2048
    const rc_u4 *ops;       // [64 lanes][bh, bl, wh, wl]: the MFMA tap operands (r2m_operands)
    float tf[6];            // T_0..T_5 / 4096 for the horizontal pass (T_11-i = T_i)
    float bias;             // 2^-13
};

// RG: staged input rows in the ring (slot = row mod RG; a step reads 42 rows and stages
// the next 32 once they are read, so any RG >= 42 holds them; smaller rings let more
// workgroups share a CU)
template <int B, bool HM, int RG>
__global__ void __launch_bounds__(kMNT) k_reduce2m(R2mArgs a) {
    using G = R2M<B>;
    constexpr int K = G::K, RS = G::RS, CPR = G::CPR, KM = G::KM;
    static_assert(RG >= 42, "ring holds a step's rows");
    __shared__ __attribute__((aligned(16))) u8 smem[(RG + kMN) * RS + (HM ? kMN * G::OS : 0)];
    const uint32_t ring_l = rc_lds(smem), inter_l = ring_l + RG * RS;
    u8 *inter = smem + RG * RS;
    const uint32_t otile_l = inter_l + kMN * RS;  // HM: [16 rows][OS]; wave w owns bytes 4 (16 w) B ..
    auto slot = [](int r) { return static_cast<uint32_t>(r + 2 * RG) % static_cast<uint32_t>(RG); };  // r >= -5

    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int strip = static_cast<int>(t % static_cast<uint32_t>(a.n_strips)) + a.s_base;
    const int rest = static_cast<int>(t / static_cast<uint32_t>(a.n_strips));
    const int band = rest % a.n_bands;
    const int img = __builtin_amdgcn_readfirstlane(rest / a.n_bands);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n = lane & 15, kg = lane >> 4;

    const int x0 = strip * kMTW;
    const int px0 = 2 * x0 - 5;
    const int org = (B * px0) & ~15;  // staged byte 0 (16-byte aligned: no chunk straddles the image start)
    const int pitch = a.w * B;
    const int ka = a.k_base + band * a.band_steps;
    const int kb = min(ka + a.band_steps, (a.y_end + kMN - 1) / kMN);
    const __amdgpu_buffer_rsrc_t src = image_rsrc(a.in + img * a.in_img, a.in_img);
    u8 *dst = a.out + img * a.out_img;

    // ---- staging: chunk c = tid + 256 j of a 32-row batch is (row rr, 16-byte column col) ----
    int rr[KM], cof[KM];
    uint32_t lof[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        const int c = tid + kMNT * j;
        rr[j] = c < 32 * CPR ? c / CPR : 64;  // 64: idle
        const int col = c - (c / CPR) * CPR;
        cof[j] = org + 16 * col;
        lof[j] = static_cast<uint32_t>(16 * col);
    }
    // a chunk left of the image (negative offset) reads zeros whole: the edge fix-up
    // replaces those pixels; rows clamp to the image (COPY edge)
    auto load = [&](rc_u4 *v, int r0, int nrows) {
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            const int r = clampi(r0 + rr[j], 0, a.h - 1);
            const int off = rr[j] < nrows && cof[j] + 16 > 0 ? r * pitch + cof[j] : 0x7ffffff0;
            v[j] = __builtin_bit_cast(rc_u4, __builtin_amdgcn_raw_buffer_load_b128(src, off, 0, 0));
        }
    };
    auto store_ring = [&](const rc_u4 *v, int r0, int nrows) {
#pragma unroll
        for (int j = 0; j < KM; ++j)
            if (rr[j] < nrows)
                lds_wr128(ring_l + slot(r0 + rr[j]) * RS + lof[j],
                          v[j] ^ 0x80808080u);
    };

    // ---- the tap operands of both products (host-built, r2m_operands) ----
    const rc_u4 *op = a.ops + 4 * lane;
    const rc_v4i bh = __builtin_bit_cast(rc_v4i, op[0]), bl = __builtin_bit_cast(rc_v4i, op[1]);
    rc_v4i wh{0, 0, 0, 0}, wl{0, 0, 0, 0};
    if (HM) {
        wh = __builtin_bit_cast(rc_v4i, op[2]);
        wl = __builtin_bit_cast(rc_v4i, op[3]);
    }
    const int sd = a.seed;
    const bool row_al16 = ((a.ow * B) & 15) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15u) == 0;

    // ---- prime: the first step's 42 rows, then the next step's 32 into registers ----
    {
        const int bk = 32 * ka - 5;
        rc_u4 v[KM];
        load(v, bk, 32);
        store_ring(v, bk, 32);
        load(v, bk + 32, 10);
        store_ring(v, bk + 32, 10);
    }
    rc_u4 pf[KM];
    load(pf, 32 * ka + 37, 32);  // rows 2 (16 (ka + 1)) + 6 .. : step ka + 1's new rows

    // horizontal taps and edge geometry
    const float t0 = a.tf[0], t1 = a.tf[1], t2 = a.tf[2], t3 = a.tf[3], t4 = a.tf[4], t5 = a.tf[5], bias = a.bias;
    auto tap = [&](int k) -> float {
        const int m = k < 6 ? k : 11 - k;
        return m == 0 ? t0 : m == 1 ? t1 : m == 2 ? t2 : m == 3 ? t3 : m == 4 ? t4 : t5;
    };
    const int x_last = min(x0 + kMTW, a.ow) - 1;
    const int nl = px0 < 0 ? -px0 : 0;                       // intermediate pixels left of the image
    const int fr = a.w - px0;                                // strip pixel index of image pixel w
    const int fr_end = min(2 * x_last + 6 - px0, 2 * kMTW + 9);
    const int nr = fr_end >= fr ? fr_end - fr + 1 : 0;
    const bool edge = nl > 0 || nr > 0;
    const int ib0 = G::OFF + G::ISH;                         // intermediate byte of strip pixel 0

    for (int k = ka; k < kb; ++k) {
        const int bk = 32 * k - 5;
        rc_barrier();  // ring rows of step k staged; the intermediate free
        // ---- vertical: 16-byte column tiles dealt to the waves ----
        {
            const int r1 = bk + 8 * kg + (n >> 1);
            const uint32_t a1 = ring_l + slot(r1) * RS + 8 * (n & 1);
            const uint32_t a2 = ring_l + slot(r1 + 32) * RS + 8 * (n & 1);
            const uint32_t iq = inter_l + static_cast<uint32_t>(n * RS + 4 * kg + G::ISH);
            auto tile = [&](int c, rc_v2i u1, rc_v2i u2) {
                const rc_v4i av = rc_v4i{u1.x, u1.y, u2.x, u2.y};
                rc_v4i dh = rc_v4i{0, 0, 0, 0}, dl = rc_v4i{sd, sd, sd, sd};
                dh = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bh, dh, 0, 0, 0);
                dl = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bl, dl, 0, 0, 0);
                uint32_t lo, hi;
                const int s0 = (dh[0] << 6) + dl[0], s1 = (dh[1] << 6) + dl[1];
                const int s2 = (dh[2] << 6) + dl[2], s3 = (dh[3] << 6) + dl[3];
                asm("v_ashr_pk_u8_i32 %0, %1, %2, 12" : "=v"(lo) : "v"(s0), "v"(s1));
                asm("v_ashr_pk_u8_i32 %0, %1, %2, 12" : "=v"(hi) : "v"(s2), "v"(s3));
                // HM: the intermediate is kept as byte - 128 (the horizontal MFMA's B operand)
                lds_wr32(iq + 16 * c, __builtin_amdgcn_perm(hi, lo, 0x05040100u) ^ (HM ? 0x80808080u : 0u));
            };
            // four tiles per batch: their reads under one wait, their products interleaved
            for (int c0 = wave; c0 < CPR; c0 += 16) {
                rc_v2i p[4][2];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int ct = c0 + 4 * i;
                    if (ct < CPR) {
                        p[i][0] = lds_tr8(a1 + 16 * ct);
                        p[i][1] = lds_tr8(a2 + 16 * ct);
                    } else {
                        p[i][0] = p[i][1] = rc_v2i{0, 0};
                    }
                }
                lgkm_wait_for<0>(p[0][0], p[0][1], p[1][0], p[1][1], p[2][0], p[2][1], p[3][0], p[3][1]);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (c0 + 4 * i < CPR) tile(c0 + 4 * i, p[i][0], p[i][1]);
            }
        }
        rc_barrier();  // the intermediate complete; the ring's rows of step k read
        if (k + 1 < kb) {
            store_ring(pf, 32 * k + 37, 32);
            if (k + 2 < kb) load(pf, 32 * k + 69, 32);
        }
        if (edge) {  // EXTEND_COPY: strip pixels outside the image copy the edge pixel
            const int nfill = nl + nr;
            for (int i = tid; i < kMN * nfill * B; i += kMNT) {
                const int u = i / (nfill * B);
                const int rem = i - u * nfill * B;
                const int f = rem / B, c = rem - f * B;
                const int d = f < nl ? f : fr + (f - nl);
                const int sp = f < nl ? nl : fr - 1;
                inter[u * RS + ib0 + B * d + c] = inter[u * RS + ib0 + B * sp + c];
            }
            rc_barrier();
        }
        if (HM) {
            // ---- horizontal on the matrix cores: D[out byte j][row u] = W[j][window byte] x
            // inter[window byte][u]; a group = GP output pixels of all 16 rows ----
            constexpr int GP = B == 3 ? 4 : 2, NG = kMTW / GP;
            // wave w: groups GPW w .. (16 px); D dwords -> the wave's part of the output tile,
            // then 16-byte row pieces to HBM
            constexpr int GPW = NG / 4;
            if (x0 + 16 * wave >= a.ow) continue;
#pragma unroll
            for (int gb = 0; gb < GPW; gb += 4) {
                rc_v4i bv[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t ws = static_cast<uint32_t>((ib0 & ~7) + 2 * B * GP * (GPW * wave + gb + i));
                    bv[i] = __builtin_bit_cast(rc_v4i, lds_rd2x64(inter_l + static_cast<uint32_t>(n * RS) + ws + 16 * kg));
                }
                lgkm_wait_for<0>(bv[0], bv[1], bv[2], bv[3]);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    rc_v4i dh = rc_v4i{0, 0, 0, 0}, dl = rc_v4i{sd, sd, sd, sd};
                    dh = __builtin_amdgcn_mfma_i32_16x16x64_i8(wh, bv[i], dh, 0, 0, 0);
                    dl = __builtin_amdgcn_mfma_i32_16x16x64_i8(wl, bv[i], dl, 0, 0, 0);
                    uint32_t lo, hi;
                    const int s0 = (dh[0] << 6) + dl[0], s1 = (dh[1] << 6) + dl[1];
                    const int s2 = (dh[2] << 6) + dl[2], s3 = (dh[3] << 6) + dl[3];
                    asm("v_ashr_pk_u8_i32 %0, %1, %2, 12" : "=v"(lo) : "v"(s0), "v"(s1));
                    asm("v_ashr_pk_u8_i32 %0, %1, %2, 12" : "=v"(hi) : "v"(s2), "v"(s3));
                    if (4 * kg < B * GP)
                        lds_wr32(otile_l + static_cast<uint32_t>(n * G::OS + 16 * B * wave + B * GP * (gb + i) + 4 * kg),
                                 __builtin_amdgcn_perm(hi, lo, 0x05040100u));
                }
            }
            {
                constexpr int LPR = B;  // 16-byte pieces per tile row of a wave (16 px x B bytes)
                const int u = lane / LPR, c = lane - u * LPR;
                lgkm_wait();
                if (u < kMN) {
                    const rc_u4 v = lds_rd128(otile_l + static_cast<uint32_t>(u * G::OS + 16 * B * wave + 16 * c));
                    lgkm_wait();
                    const int y = kMN * k + u;
                    const int xb = (x0 + 16 * wave) * B + 16 * c;
                    const int rowb = a.ow * B;
                    if (y < a.oh && xb < rowb) {
                        u8 *q = dst + static_cast<size_t>(y) * rowb + xb;
                        if (row_al16 && xb + 16 <= rowb) {
                            *reinterpret_cast<rc_u4 *>(q) = v;
                        } else {
                            const int nb = min(16, rowb - xb);
                            for (int e = 0; e < nb; ++e) q[e] = static_cast<u8>(v[e >> 2] >> (8 * (e & 3)));
                        }
                    }
                }
            }
            continue;
        }
        // ---- horizontal: items of K output pixels, 14 window dwords each ----
        constexpr int ipr = kMTW / K;
        for (int it = tid; it < kMN * ipr; it += kMNT) {
            const int u = it / ipr, j = it - u * ipr;
            const int x = x0 + K * j, y = kMN * k + u;
            if (y >= a.oh || x >= a.ow) continue;
            const u8 *row = inter + u * RS;
            uint32_t win[14];
            if (B == 3) {  // window bytes from 1 + 24 j: dwords 6 j .. 6 j + 13
                const uint2 *r2 = reinterpret_cast<const uint2 *>(row + 24 * j);
#pragma unroll
                for (int q = 0; q < 7; ++q) {
                    const uint2 dd = r2[q];
                    win[2 * q] = dd.x;
                    win[2 * q + 1] = dd.y;
                }
            } else {       // from 16 + 16 j
                const uint4 *r4 = reinterpret_cast<const uint4 *>(row + 16 + 16 * j);
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const uint4 dd = r4[q];
                    win[4 * q] = dd.x, win[4 * q + 1] = dd.y, win[4 * q + 2] = dd.z, win[4 * q + 3] = dd.w;
                }
                const uint2 dd = *reinterpret_cast<const uint2 *>(row + 16 + 16 * j + 48);
                win[12] = dd.x;
                win[13] = dd.y;
            }
            constexpr int OFF0 = B == 3 ? 1 : 0;
            float o[K][B];
#pragma unroll
            for (int kk = 0; kk < K; ++kk)
#pragma unroll
                for (int c = 0; c < B; ++c) o[kk][c] = bias;
#pragma unroll
            for (int tt = 0; tt < 2 * K + 10; ++tt) {
                float v[B];
#pragma unroll
                for (int c = 0; c < B; ++c) {
                    const int lb = B * tt + c + OFF0;
                    const uint32_t dd = win[lb >> 2];
                    switch (lb & 3) {
                        case 0: v[c] = ubyte_once<0>(dd); break;
                        case 1: v[c] = ubyte_once<1>(dd); break;
                        case 2: v[c] = ubyte_once<2>(dd); break;
                        default: v[c] = ubyte_once<3>(dd); break;
                    }
                }
#pragma unroll
                for (int kk = 0; kk < K; ++kk) {
                    const int ti = tt - 2 * kk;
                    if (ti < 0 || ti > 11) continue;
                    const float tk = tap(ti);
#pragma unroll
                    for (int c = 0; c < B; ++c) o[kk][c] = __builtin_fmaf(tk, v[c], o[kk][c]);
                }
            }
            u8 *q = dst + (static_cast<size_t>(y) * a.ow + x) * B;
            const bool full = x + K <= a.ow;
            auto pk = [](float p, float q1, float r, float s) {
                uint32_t v = __builtin_amdgcn_cvt_pk_u8_f32(p, 0, 0u);
                v = __builtin_amdgcn_cvt_pk_u8_f32(q1, 1, v);
                v = __builtin_amdgcn_cvt_pk_u8_f32(r, 2, v);
                return __builtin_amdgcn_cvt_pk_u8_f32(s, 3, v);
            };
            if (B == 3) {
                const uint32_t d0 = pk(o[0][0], o[0][1], o[0][2], o[1][0]);
                const uint32_t d1 = pk(o[1][1], o[1][2], o[2][0], o[2][1]);
                const uint32_t d2 = pk(o[2][2], o[3][0], o[3][1], o[3][2]);
                if (full && (reinterpret_cast<uintptr_t>(q) & 3u) == 0) {
                    *reinterpret_cast<uint3 *>(q) = uint3{d0, d1, d2};
                } else {
                    const uint32_t dd[3] = {d0, d1, d2};
                    const int nb = (full ? K : a.ow - x) * B;
                    for (int i = 0; i < nb; ++i) q[i] = static_cast<u8>(dd[i >> 2] >> (8 * (i & 3)));
                }
            } else {
                const uint32_t d0 = pk(o[0][0], o[0][1], o[0][2], o[0][3]);
                const uint32_t d1 = pk(o[1][0], o[1][1], o[1][2], o[1][3]);
                uint32_t *q32 = reinterpret_cast<uint32_t *>(q);
                if (full && (reinterpret_cast<uintptr_t>(q) & 7u) == 0) {
                    *reinterpret_cast<uint2 *>(q) = uint2{d0, d1};
                } else {
                    q32[0] = d0;
                    if (full) q32[1] = d1;
                }
            }
        }
    }
}

// The per-lane tap operands, [lane][bh, bl, wh, wl] x 16 bytes.  Lane (n = lane & 15,
// kg = lane >> 4) holds K = 16 kg + e, e = 0..15 (the same labelling on both operands
// of a product, so the contraction order is free):
//   vertical B, output row n: K <-> staged row 8 kg + e (e < 8) or 32 + 8 kg + e - 8
//     (the two ds_read_b64_tr_b8 of a column tile), tap i = row - 2 n;
//   horizontal A, output byte j = n of a group (pixel j / B, channel j % B; j < B GP):
//     K = window byte = SH + B (2 (j / B) + i) + j % B, SH = ib0 mod 8 (the window starts
//     8-byte aligned).
// Every tap T = 64 hi + lo (floor split: lo in [0, 63]), hi in bh / wh, lo in bl / wl.
template <int B>
std::vector<uint32_t> r2m_operands(const int *tap) {
    using G = R2M<B>;
    constexpr int GPB = B == 3 ? 12 : 8, SH = (G::OFF + G::ISH) & 7;
    std::vector<uint32_t> v(64 * 16, 0);
    for (int lane = 0; lane < 64; ++lane) {
        const int n = lane & 15, kg = lane >> 4;
        for (int e = 0; e < 16; ++e) {
            const int row = e < 8 ? 8 * kg + e : 32 + 8 * kg + e - 8;
            const int iv = row - 2 * n;
            const int tv = (iv >= 0 && iv < 12) ? tap[iv] : 0;
            const int r = 16 * kg + e - SH - n % B;
            const int ih = r >= 0 && r % B == 0 ? r / B - 2 * (n / B) : -1;
            const int th = (n < GPB && ih >= 0 && ih < 12) ? tap[ih] : 0;
            const int t4[4] = {tv >> 6, tv - 64 * (tv >> 6), th >> 6, th - 64 * (th >> 6)};
            for (int o = 0; o < 4; ++o)
                v[16 * lane + 4 * o + e / 4] |= (static_cast<uint32_t>(t4[o]) & 0xffu) << (8 * (e % 4));
        }
    }
    return v;
}

}  // namespace

// k_reduce2m over the output region [x0, x1) x [y0, y1) of a 2 x 2 reduce at the centre
// convention; taps = matrixi[64][0..11] (symmetric, host-checked by reduce2c_taps).
// Rows and columns of whole strips / steps around the region are computed too (they
// are the same values), never past the output image.
int reduce2m_window_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int x0, int y0, int x1, int y1,
                           const int *taps12, hipStream_t st) {
    if (b != 3 && b != 4) return MIPX_EUNSUPPORTED;
    R2mArgs a{};
    a.in = in;
    a.out = out;
    a.w = w;
    a.h = h;
    a.ow = out_size_reduce(w, 2.0);
    a.oh = out_size_reduce(h, 2.0);
    if (x0 < 0 || y0 < 0 || x1 > a.ow || y1 > a.oh || x0 >= x1 || y0 >= y1) return MIPX_EINVAL;
    a.in_img = img_bytes(w, h, b);
    a.out_img = img_bytes(a.ow, a.oh, b);
    if (a.in_img >= 0x7fffffffLL - 64) return MIPX_EUNSUPPORTED;
    int sum = 0;
    for (int i = 0; i < 12; ++i) {
        sum += taps12[i];
        if (taps12[i] < -128 * 64 || taps12[i] > 127 * 64 + 63) return MIPX_EUNSUPPORTED;  // i8 hi / lo split
    }
    const std::vector<uint32_t> ops = b == 3 ? r2m_operands<3>(taps12) : r2m_operands<4>(taps12);
    a.ops = static_cast<const rc_u4 *>(device_blob(ops.data(), ops.size() * sizeof(uint32_t)));
    if (!a.ops) return MIPX_EDEVICE;
    for (int i = 0; i < 6; ++i) a.tf[i] = static_cast<float>(taps12[i]) / 4096.0f;
    a.bias = 1.0f / 8192.0f;
    a.seed = 128 * sum + 2048;
    a.x_end = x1;
    a.y_end = y1;
    a.s_base = x0 / kMTW;
    a.k_base = y0 / kMN;
    a.n_strips = (x1 + kMTW - 1) / kMTW - a.s_base;
    const int steps = (y1 + kMN - 1) / kMN - a.k_base;
    const char *eb = tune_env("MIPX_R2M_BAND");  // 16-row steps per band (A/B)
    a.band_steps = std::max(1, std::min(steps, (eb && *eb) ? std::atoi(eb) : 4));
    a.n_bands = (steps + a.band_steps - 1) / a.band_steps;
    const long long blocks = static_cast<long long>(a.n_strips) * a.n_bands * n;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    const dim3 grid(static_cast<unsigned>(blocks)), blk(kMNT);
    const char *eh = tune_env("MIPX_R2M_H");  // 0: horizontal pass on the VALU (A/B)
    const bool hm = !(eh && *eh == '0');
    const char *eg = tune_env("MIPX_R2M_RING");  // staged rows in the ring: 42 / 48 / 64 (A/B)
    const int rg = (eg && *eg) ? std::atoi(eg) : 48;
#define MIPX_R2M_GO(B_)                                                                          \
    if (rg == 42) {                                                                              \
        if (hm) hipLaunchKernelGGL((k_reduce2m<B_, true, 42>), grid, blk, 0, st, a);            \
        else hipLaunchKernelGGL((k_reduce2m<B_, false, 42>), grid, blk, 0, st, a);              \
    } else if (rg == 64) {                                                                       \
        if (hm) hipLaunchKernelGGL((k_reduce2m<B_, true, 64>), grid, blk, 0, st, a);            \
        else hipLaunchKernelGGL((k_reduce2m<B_, false, 64>), grid, blk, 0, st, a);              \
    } else {                                                                                     \
        if (hm) hipLaunchKernelGGL((k_reduce2m<B_, true, 48>), grid, blk, 0, st, a);            \
        else hipLaunchKernelGGL((k_reduce2m<B_, false, 48>), grid, blk, 0, st, a);              \
    }
    if (b == 3) {
        MIPX_R2M_GO(3)
    } else {
        MIPX_R2M_GO(4)
    }
#undef MIPX_R2M_GO
    return launch_check("k_reduce2m");
}

}  // namespace mipx
