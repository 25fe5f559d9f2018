// k_reduce2m.hip — the fused 2 x 2 Lanczos3 reduce under libvips' centre sampling
// convention (PARITY_ASSUMPTIONS.md row 1: X = (o + 0.5) * 2 - 0.5), both passes on the
// i8 matrix cores.
//
// Every output of either pass is o = sum_{i=0..11} T_i p[2o - 5 + i] (phase 64; tap 12
// is zero): twelve multiply-adds per byte and pass against the corner convention's seven.
// As f32 VALU work (r04's k_reduce2c, profiles/r04/reduce2c/) that arithmetic, not HBM,
// bounded the kernel, so both passes are banded matrix products on
// v_mfma_i32_16x16x64_i8, each tap split T = 64 hi + lo (both i8) into two products
// rejoined as 64 D_hi + D_lo, with 128 sum(T) + 2048 seeded into D_lo (the operands are
// pixel - 128), so (64 D_hi + D_lo) >> 12 clamped (v_ashr_pk_u8_i32) is libvips' rounded
// uchar exactly:
//  * vertical: D[byte column][output row] = A[byte column][input row] x B[input row][row];
//    16 output rows need 42 input rows (K = 64, the rest carry zero taps); A = two
//    ds_read_b64_tr_b8 per 16-byte column tile of the staged rows, B the taps at row
//    2n + i of output row n.  The result (byte - 128) goes to an LDS intermediate.
//  * horizontal: D[output byte][row] = W[output byte][window byte] x inter[window][row];
//    a group of 4 (RGB) / 2 (RGBA) output pixels of all 16 rows reads a 64-byte window
//    (8-byte aligned) of each intermediate row as its B operand (two ds_read_b64);
//    W, the taps at byte SH + B (2 (j / B) + i) + j % B of output byte j, is constant.
//    D dwords go to an output tile in intermediate bytes only the wave's own windows
//    cover (no LDS of its own: RGBA -1.4 %), then out as 16-byte row pieces.
// The tap operands are built on the host (r2m_operands) and read once per block.
//
// A block (4 waves) owns a strip of 64 output pixels of one image and walks a band of
// 16-row steps.  The strip's input rows (138 pixels, from the 16-byte-aligned-down start)
// live in an LDS ring of 42 rows; a step adds 32 rows (2 per output row), loaded one step
// ahead into registers as 16-byte chunks dealt over the 256 lanes, written to the ring
// XOR 0x80 once the previous step's vertical pass has read its rows.  Per step: barrier
// -> vertical (ring -> LDS intermediate, 16 rows) -> barrier -> next rows to the ring,
// next loads issued -> COPY-edge fix-up of the intermediate at the image edges ->
// horizontal (intermediate -> output tile -> HBM).  Rows clamp at the load (COPY edge);
// input bytes left of the image are staged as zeros and replaced in the intermediate.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "device_common.h"
#include "lds_ops.h"

namespace mipx {
namespace {

using namespace dev;

constexpr int kMaxDevices = 64;  // operand-table cache slots (HIP device ordinals)
constexpr int kMTW = 64;    // output pixels per strip
constexpr int kMN = 16;     // output rows per step (the MFMA N)
constexpr int kMNT = 256;
constexpr int kMRing = 42;  // staged rows (slot = row mod 42): a step reads 42 rows, then stages
                            // the next 32 over the 32 it no longer needs (48 / 64: same speed,
                            // fewer workgroups per CU for RGBA, profiles/r04/reduce2m/)

template <int B>
struct R2M {
    static constexpr int OFF = B == 3 ? 1 : 12;              // (B px0) mod 16 for every strip
    static constexpr int ISH = B == 3 ? 0 : 4;               // intermediate byte shift: windows aligned
    static constexpr int CPR = (OFF + B * (2 * kMTW + 10) + 15) / 16;  // 16-byte chunks per staged row
    static constexpr int RS = B == 3 ? 432 : 592;            // row stride: (RS / 4 mod 64) / 4 odd
    static constexpr int KM = (32 * CPR + kMNT - 1) / kMNT;  // chunks per lane per step (32 rows)
    // intermediate rows IS at (dwords mod 32) = 2 x odd, so the 16 rows x 2 dwords of a
    // half-wave's ds_write_b32 hit 32 distinct banks (writes map banks mod 32), read back
    // with ds_read_b64 pairs (ds_read2_b64 costs 16 LDS cycles, two ds_read_b64 4):
    // bank-conflict cycles halved against IS = RS, C2 -0.4 %, RGBA -1.5 %
    // (profiles/r04/reduce2m/f_lds_layout_ab.jsonl, f_pmc_layout.txt)
    static constexpr int IS = B == 3 ? 424 : 584;
    // the horizontal pass: groups of GP output pixels (a 64-byte window from byte WB + 2 B GP g
    // of each intermediate row), GPW groups per wave; wave w's windows alone cover the bytes
    // EXS + EXW w .. + EXN, where its output tile (16 B bytes per row) goes
    static constexpr int GP = B == 3 ? 4 : 2, GPW = kMTW / GP / 4, WB = (OFF + ISH) & ~7;
    static constexpr int EXW = 2 * B * GP * GPW, EXS = WB + 64 - 2 * B * GP, EXN = EXW - EXS + WB;
    static_assert(EXN >= 16 * B && EXS % 8 == 0 && EXS + 3 * EXW + 16 * B <= IS, "output tile in the intermediate");
    static_assert((IS / 4) % 32 % 4 == 2 && IS % 8 == 0, "write banks");
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
    int alt;                // odd bands walk up (their edge rows meet the neighbours' in L2)
    int pp;                 // prime: both row batches in flight together
    int dbg;                // PROBES builds only: 8 = per-step phase stamps (MIPX_R2M_DBG)
    unsigned long long *stamps;  // PROBES, dbg 8: [block][2 + 10 band_steps]
};
#ifdef MIPX_PROBES
__device__ __forceinline__ int r2m_dbg(const R2mArgs &a) { return a.dbg; }
#else
__device__ __forceinline__ int r2m_dbg(const R2mArgs &) { return 0; }
#endif

template <int B>
__global__ void __launch_bounds__(kMNT) k_reduce2m(R2mArgs a) {
    using G = R2M<B>;
    constexpr int RS = G::RS, CPR = G::CPR, KM = G::KM, RG = kMRing, IS = G::IS;
    __shared__ __attribute__((aligned(16))) u8 smem[RG * RS + kMN * IS];
    const uint32_t ring_l = rc_lds(smem), inter_l = ring_l + RG * RS;
    u8 *inter = smem + RG * RS;
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
    // a band's first step stages 10 rows its neighbour above also reads; walking odd bands
    // bottom-up puts both reads of every shared row at about the same time (the bands of a
    // strip are co-resident on one XCD), so the second comes from L2
    const bool rev = a.alt && (band & 1);
    const int kf = rev ? kb - 1 : ka, dk = rev ? -1 : 1, nst = kb - ka;
    auto new_rows = [&](int k) { return rev ? 32 * k - 37 : 32 * k + 37; };  // first row step k + dk adds
    const __amdgpu_buffer_rsrc_t src = image_rsrc(a.in + img * a.in_img, a.in_img);
    u8 *dst = a.out + img * a.out_img;
    // PROBES, dbg 8: wave 0 lane 0 stamps the block's start / end and each step's phases
    unsigned long long *stp = nullptr;
    if (r2m_dbg(a) == 8 && tid == 0) stp = a.stamps + static_cast<size_t>(blockIdx.x) * (2 + 10 * a.band_steps);
    auto stamp = [&](int sl) {
        if (r2m_dbg(a) == 8 && stp) stp[sl] = __builtin_amdgcn_s_memtime();
    };
    stamp(0);

    // ---- staging: chunk c = tid + 256 j of a 32-row batch is (row rr, 16-byte column col) ----
    // packed (row rr << 16 | 16 col), one register per chunk
    uint32_t sg[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        const int c = tid + kMNT * j;
        const int r = c < 32 * CPR ? c / CPR : 64;  // 64: idle
        sg[j] = static_cast<uint32_t>(r << 16 | 16 * (c - (c / CPR) * CPR));
    }
    // a chunk left of the image (negative offset) reads zeros whole: the edge fix-up
    // replaces those pixels; rows clamp to the image (COPY edge)
    auto load = [&](rc_u4 *v, int r0, int nrows) {
#pragma unroll
        for (int j = 0; j < KM; ++j) {
            const int rj = static_cast<int>(sg[j] >> 16), cof = org + static_cast<int>(sg[j] & 0xffffu);
            const int r = clampi(r0 + rj, 0, a.h - 1);
            const int off = rj < nrows && cof + 16 > 0 ? r * pitch + cof : 0x7ffffff0;
            v[j] = __builtin_bit_cast(rc_u4, __builtin_amdgcn_raw_buffer_load_b128(src, off, 0, 0));
        }
    };
    auto store_ring = [&](const rc_u4 *v, int r0, int nrows) {
#pragma unroll
        for (int j = 0; j < KM; ++j)
            if (static_cast<int>(sg[j] >> 16) < nrows)
                lds_wr128(ring_l + slot(r0 + static_cast<int>(sg[j] >> 16)) * RS + (sg[j] & 0xffffu),
                          v[j] ^ 0x80808080u);
    };

    // ---- the tap operands of both products (host-built, r2m_operands) ----
    const rc_u4 *op = a.ops + 4 * lane;
    const rc_v4i bh = __builtin_bit_cast(rc_v4i, op[0]), bl = __builtin_bit_cast(rc_v4i, op[1]);
    const rc_v4i wh = __builtin_bit_cast(rc_v4i, op[2]), wl = __builtin_bit_cast(rc_v4i, op[3]);
    const int sd = a.seed;
    const bool row_al16 = ((a.ow * B) & 15) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15u) == 0;

    // ---- prime: the first step's 42 rows, then the next step's 32 into registers ----
    rc_u4 pf[KM];
    {
        const int bk = 32 * kf - 5;
        rc_u4 v[KM];
        load(v, bk, 32);
        if (a.pp) {  // the 10 rows in the prefetch registers, in flight with the 32
            load(pf, bk + 32, 10);
            store_ring(v, bk, 32);
            store_ring(pf, bk + 32, 10);
        } else {
            store_ring(v, bk, 32);
            load(v, bk + 32, 10);
            store_ring(v, bk + 32, 10);
        }
    }
    load(pf, new_rows(kf), 32);  // step kf + dk's new rows

    // edge geometry
    const int x_last = min(x0 + kMTW, a.ow) - 1;
    const int nl = px0 < 0 ? -px0 : 0;                       // intermediate pixels left of the image
    const int fr = a.w - px0;                                // strip pixel index of image pixel w
    const int fr_end = min(2 * x_last + 6 - px0, 2 * kMTW + 9);
    const int nr = fr_end >= fr ? fr_end - fr + 1 : 0;
    const bool edge = nl > 0 || nr > 0;
    const int ib0 = G::OFF + G::ISH;                         // intermediate byte of strip pixel 0

    for (int s = 0; s < nst; ++s) {
        const int k = kf + dk * s;
        const int bk = 32 * k - 5;
        const int sb = 2 + 10 * s;  // stamp slots (dbg 8)
        stamp(sb);
        rc_barrier();  // ring rows of step k staged; the intermediate free
        stamp(sb + 1);
        // ---- vertical: 16-byte column tiles dealt to the waves ----
        {
            const int r1 = bk + 8 * kg + (n >> 1);
            const uint32_t a1 = ring_l + slot(r1) * RS + 8 * (n & 1);
            const uint32_t a2 = ring_l + slot(r1 + 32) * RS + 8 * (n & 1);
            const uint32_t iq = inter_l + static_cast<uint32_t>(n * IS + 4 * kg + G::ISH);
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
                // the intermediate is kept as byte - 128 (the horizontal product's B operand)
                lds_wr32(iq + 16 * c, __builtin_amdgcn_perm(hi, lo, 0x05040100u) ^ 0x80808080u);
            };
            // VB tiles per batch: their reads under one wait, their products interleaved (6
            // waves per SIMD at 80 VGPRs needs VB = HB = 1 for RGB: -1.4 % from the occupancy,
            // +2 % from the serialised reads, profiles/r04/reduce2m/h_otile_occupancy_ab.jsonl)
            constexpr int VB = 4;
            for (int c0 = wave; c0 < CPR; c0 += 4 * VB) {
                rc_v2i p[VB][2];
#pragma unroll
                for (int i = 0; i < VB; ++i) {
                    const int ct = c0 + 4 * i;
                    if (ct < CPR) {
                        p[i][0] = lds_tr8(a1 + 16 * ct);
                        p[i][1] = lds_tr8(a2 + 16 * ct);
                    } else {
                        p[i][0] = p[i][1] = rc_v2i{0, 0};
                    }
                }
                if constexpr (VB == 4) lgkm_wait_for<0>(p[0][0], p[0][1], p[1][0], p[1][1], p[2][0], p[2][1], p[3][0], p[3][1]);
                else if constexpr (VB == 2) lgkm_wait_for<0>(p[0][0], p[0][1], p[1][0], p[1][1]);
                else lgkm_wait_for<0>(p[0][0], p[0][1]);
#pragma unroll
                for (int i = 0; i < VB; ++i)
                    if (c0 + 4 * i < CPR) tile(c0 + 4 * i, p[i][0], p[i][1]);
            }
        }
        stamp(sb + 2);
        rc_barrier();  // the intermediate complete; the ring's rows of step k read
        stamp(sb + 3);
        if (s + 1 < nst) {
            store_ring(pf, new_rows(k), 32);
            stamp(sb + 4);
            if (s + 2 < nst) load(pf, new_rows(k + dk), 32);
        } else {
            stamp(sb + 4);
        }
        stamp(sb + 5);
        if (edge) {  // EXTEND_COPY: strip pixels outside the image copy the edge pixel
            const int nfill = nl + nr;
            for (int i = tid; i < kMN * nfill * B; i += kMNT) {
                const int u = i / (nfill * B);
                const int rem = i - u * nfill * B;
                const int f = rem / B, c = rem - f * B;
                const int d = f < nl ? f : fr + (f - nl);
                const int sp = f < nl ? nl : fr - 1;
                inter[u * IS + ib0 + B * d + c] = inter[u * IS + ib0 + B * sp + c];
            }
            rc_barrier();
        }
        stamp(sb + 6);
        // ---- horizontal on the matrix cores: D[out byte j][row u] = W[j][window byte] x
        // inter[window byte][u]; a group = GP output pixels of all 16 rows ----
        constexpr int GP = G::GP, GPW = G::GPW, HB = 4;
        // wave w: groups GPW w .. (16 px); D dwords -> the wave's output tile, then 16-byte
        // row pieces to HBM
        if (x0 + 16 * wave >= a.ow) continue;  // (the next step starts with a barrier)
        uint32_t pk[GPW];  // the packed D dwords of the wave's groups (after all its window reads)
#pragma unroll
        for (int gb = 0; gb < GPW; gb += HB) {
            rc_u2x2 bq[HB];
#pragma unroll
            for (int i = 0; i < HB; ++i) {
                const uint32_t ws = static_cast<uint32_t>((ib0 & ~7) + 2 * B * GP * (GPW * wave + gb + i));
                const uint32_t ad = inter_l + static_cast<uint32_t>(n * IS) + ws + 16 * kg;
                bq[i] = lds_rd64x2(ad);
            }
            if constexpr (HB == 4) lgkm_wait_for<0>(bq[0], bq[1], bq[2], bq[3]);
            else if constexpr (HB == 2) lgkm_wait_for<0>(bq[0], bq[1]);
            else lgkm_wait_for<0>(bq[0]);
            rc_v4i bv[HB];
#pragma unroll
            for (int i = 0; i < HB; ++i) bv[i] = __builtin_bit_cast(rc_v4i, rc_join(bq[i]));
#pragma unroll
            for (int i = 0; i < HB; ++i) {
                rc_v4i dh = rc_v4i{0, 0, 0, 0}, dl = rc_v4i{sd, sd, sd, sd};
                dh = __builtin_amdgcn_mfma_i32_16x16x64_i8(wh, bv[i], dh, 0, 0, 0);
                dl = __builtin_amdgcn_mfma_i32_16x16x64_i8(wl, bv[i], dl, 0, 0, 0);
                uint32_t lo, hi;
                const int s0 = (dh[0] << 6) + dl[0], s1 = (dh[1] << 6) + dl[1];
                const int s2 = (dh[2] << 6) + dl[2], s3 = (dh[3] << 6) + dl[3];
                asm("v_ashr_pk_u8_i32 %0, %1, %2, 12" : "=v"(lo) : "v"(s0), "v"(s1));
                asm("v_ashr_pk_u8_i32 %0, %1, %2, 12" : "=v"(hi) : "v"(s2), "v"(s3));
                pk[gb + i] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
            }
        }
        // the output tile: 16 rows x 16 B bytes in the intermediate bytes only this wave's
        // windows cover (EXS on), written once the wave has read all its windows (a wave's
        // LDS operations complete in order); the next step's vertical pass overwrites them
        // only after its barrier
        stamp(sb + 7);
        const uint32_t otile_w = inter_l + static_cast<uint32_t>(G::EXS + G::EXW * wave);
#pragma unroll
        for (int g = 0; g < GPW; ++g)
            if (4 * kg < B * GP) lds_wr32(otile_w + static_cast<uint32_t>(n * IS + B * GP * g + 4 * kg), pk[g]);
        {
            constexpr int LPR = B;  // 16-byte pieces per tile row of a wave (16 px x B bytes)
            const int u = lane / LPR, c = lane - u * LPR;
            lgkm_wait();
            if (u < kMN) {
                const uint32_t ad = otile_w + static_cast<uint32_t>(u * IS + 16 * c);
                rc_u2x2 vq = lds_rd64x2(ad);
                lgkm_wait_for<0>(vq);
                const rc_u4 v = rc_join(vq);
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
        stamp(sb + 8);
    }
    stamp(1);
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
    // the operand table depends on (device, bands) only (taps12 is always the phase-64 row
    // of the shrink-2 table): cached lock-free after the first launch (it was
    // rebuilt and looked up by contents under the table mutex on every launch)
    struct Cached {
        const rc_u4 *ops;
        unsigned gen;
    };
    static std::mutex mu;
    static Cached cache[kMaxDevices][2];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return MIPX_EDEVICE;
    const unsigned gen = device_tables_generation();
    {
        std::lock_guard<std::mutex> lk(mu);
        Cached *slot = dev < kMaxDevices ? &cache[dev][b - 3] : nullptr;
        a.ops = slot && slot->gen == gen ? slot->ops : nullptr;
        if (!a.ops) {
            const std::vector<uint32_t> ops = b == 3 ? r2m_operands<3>(taps12) : r2m_operands<4>(taps12);
            a.ops = static_cast<const rc_u4 *>(device_blob(ops.data(), ops.size() * sizeof(uint32_t)));
            if (!a.ops) return MIPX_EDEVICE;
            if (slot) *slot = Cached{a.ops, gen};
        }
    }
    a.seed = 128 * sum + 2048;
    a.x_end = x1;
    a.y_end = y1;
    a.s_base = x0 / kMTW;
    a.k_base = y0 / kMN;
    a.n_strips = (x1 + kMTW - 1) / kMTW - a.s_base;
    const int steps = (y1 + kMN - 1) / kMN - a.k_base;
    // 16-row steps per band: 7 (RGB) / 16 (RGBA), measured best (profiles/r04/reduce2m/d_band_sweep.jsonl;
    // with the alternating walk RGB 7 beats 8 by 0.7 %, profiles/r05/reduce2m/band_fine_ab.jsonl);
    // MIPX_R2M_BAND overrides (A/B)
    const char *eb = tune_env("MIPX_R2M_BAND");
    a.band_steps = std::max(1, std::min(steps, (eb && *eb) ? std::atoi(eb) : (b == 3 ? 7 : 16)));
    const char *ea = tune_env("MIPX_R2M_ALT");  // A/B: 0 = every band walks down
    a.alt = !(ea && *ea == '0');
    const char *epp = tune_env("MIPX_R2M_PP");  // A/B: 0 = the prime's two row batches one after the other
    a.pp = !(epp && *epp == '0');
    a.n_bands = (steps + a.band_steps - 1) / a.band_steps;
    const long long blocks = static_cast<long long>(a.n_strips) * a.n_bands * n;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    const dim3 grid(static_cast<unsigned>(blocks)), blk(kMNT);
#ifdef MIPX_PROBES
    const char *edb = tune_env("MIPX_R2M_DBG");
    a.dbg = edb && *edb ? std::atoi(edb) : 0;
    static int calls = 0;
    std::vector<unsigned long long> hs;
    const size_t per = 2 + 10 * static_cast<size_t>(a.band_steps), cnt = per * static_cast<size_t>(blocks);
    if (a.dbg == 8) {
        if (hipMalloc(&a.stamps, cnt * 8) != hipSuccess) return MIPX_EDEVICE;
        (void)hipMemsetAsync(a.stamps, 0, cnt * 8, st);
    }
#endif
    if (b == 3) hipLaunchKernelGGL(k_reduce2m<3>, grid, blk, 0, st, a);
    else hipLaunchKernelGGL(k_reduce2m<4>, grid, blk, 0, st, a);
#ifdef MIPX_PROBES
    if (a.dbg == 8) {  // one JSON line on the third launch: each phase's mean cycles per step
        int e = launch_check("k_reduce2m");
        hs.resize(cnt);
        if (!e && hipStreamSynchronize(st) == hipSuccess &&
            hipMemcpy(hs.data(), a.stamps, cnt * 8, hipMemcpyDeviceToHost) == hipSuccess && ++calls == 3) {
            double ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, dur = 0;
            long long nst = 0, nb = 0;
            for (long long q = 0; q < blocks; ++q) {
                const unsigned long long *p = hs.data() + q * per;
                if (!p[0] || !p[1]) continue;
                dur += static_cast<double>(p[1] - p[0]);
                ++nb;
                for (int s2 = 0; s2 < a.band_steps; ++s2) {
                    const unsigned long long *r = p + 2 + 10 * s2;
                    if (!r[0] || !r[8]) continue;
                    for (int i = 0; i < 8; ++i) ph[i] += static_cast<double>(r[i + 1] - r[i]);
                    ++nst;
                }
            }
            const double d = static_cast<double>(std::max(1LL, nst));
            fprintf(stderr,
                    "{\"r2m_stamps\": 1, \"w\": %d, \"h\": %d, \"b\": %d, \"n\": %d, \"blocks\": %lld, \"band_steps\": %d, "
                    "\"block_mean\": %.0f, \"steps\": %lld, \"barrier1\": %.1f, \"vertical\": %.1f, \"barrier2\": %.1f, "
                    "\"ring_store\": %.1f, \"loads\": %.1f, \"edge\": %.1f, \"horizontal\": %.1f, \"store\": %.1f}\n",
                    w, h, b, n, blocks, a.band_steps, dur / std::max(1.0, static_cast<double>(nb)), nst, ph[0] / d,
                    ph[1] / d, ph[2] / d, ph[3] / d, ph[4] / d, ph[5] / d, ph[6] / d, ph[7] / d);
        }
        (void)hipFree(a.stamps);
        return e;
    }
#endif
    return launch_check("k_reduce2m");
}

}  // namespace mipx
