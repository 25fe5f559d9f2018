// k_sep.hip — the generic separable passes behind libvips vips_reduce
// (reducev -> reduceh, Lanczos3, any shrink) and vips_gaussblur (convsep:
// horizontal 1 x n mask, then vertical), on gfx950.
//
// Both libvips ops are "one 1-D integer mask per output position, uchar result":
//   reduce (reducev.cpp / reduceh.cpp): position o samples X = o * shrink, taps
//     start at floor(X) - (n/2 - 1), phase ((int(X*256) & 255) + 1) >> 1 of the
//     129-phase 12-bit table, result (sum + 2048) >> 12 clipped;
//   conv (convi.c via convsep): position o starts at o - n/2, one mask, result
//     (sum + (scale+1)/2) / scale clipped;
// both with EXTEND_COPY edges (restated in oracle/vips_ref.c).  Sums are
// integers below 2^24, so fp32 FMAs reproduce them exactly in any order.
//
//  * k_vpass<MODE, DMA>: a block = one 1 KiB column block x kr output rows.
//    The input rows those outputs need are staged in LDS once with direct-to-
//    LDS buffer loads (no VGPR staging, all in flight together); lanes own
//    4-byte columns (channel agnostic) and read their taps from LDS.
//  * k_hpass<B, RB, MODE, DW, TREG>: a block = 256 output pixels x RB
//    rows; the input spans are DMA'd to LDS and repacked to one u32 per pixel
//    with the COPY edge; each lane reads its taps from LDS (reduce taps of
//    <= 16 held per lane in registers).
// Both take a window (row / column offset and clamp range), so an extract that
// follows a reduce or precedes a blur folds into the pass (mipx_runtime.cpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "device_common.h"

namespace mipx {
namespace {

using namespace dev;

struct SepTaps {
    const float *tab;        // phased: (kTransformScale + 1) x taps, else 1 x taps
    int taps, pad, phased;
    double shrink;
    float rounding, inv_scale;  // conv rounding
    int dot;                 // integer dot paths (MIPX_SEP_DOT=0 selects the float path)
    int tq;                  // conv vpass: rows transposed once per 4-row quad (MIPX_SEP_TQ=0: per output row)
    int centre;              // reduce: centre sampling convention (mipx_set_reduce_sampling)
};

constexpr int kVpPairs = 8;     // tap pairs of the unrolled vertical reduce (taps <= 16: shrink < 2.75)

// Reduce masks are 12-bit signed integers (x 4096), so tap pairs fit packed
// int16 and v_dot2_i32_i16 sums byte pairs zero-extended to int16 exactly:
// 4 v_perm_b32 + 4 dot2 per 2 taps x 4 bytes instead of 8 conversions + 8
// FMAs, and libvips' (sum + 2048) >> 12 becomes an integer shift.
typedef short short2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int dot2_byte(uint32_t lo_row, uint32_t hi_row, int z, uint32_t cw, int acc) {
    const uint32_t sel = 0x0C040C00u + 0x00010001u * static_cast<uint32_t>(z);  // [lo.z, 0, hi.z, 0]
    const uint32_t pr = __builtin_amdgcn_perm(hi_row, lo_row, sel);
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, pr), __builtin_bit_cast(short2v, cw), acc, false);
}
// The asm barrier keeps the backend from fusing shift + clamp + byte packing of
// two channels into gfx950's v_ashr_pk_u8_i32: that instruction writes only the
// low 16 bits of its destination, yet the fused code ORs the next channels into
// bits 16-31 as if they were zero (seen as a channel-2 error on 4-band rows).
__device__ __forceinline__ uint32_t fixed_round_i(int sum) {
    int v = clampi((sum + 2048) >> 12, 0, 255);
    asm("" : "+v"(v));
    return static_cast<uint32_t>(v);
}
// (acc0..3 + 2048) >> 12 clamped to 0..255, packed: gfx950's v_ashr_pk_u8_i32
// does shift + saturate + pack for two channels (it writes only the low 16 bits
// of its destination, so the halves are joined with a v_perm, never ORed).
// The accumulators start at 2048, so the rounding add is free.
__device__ __forceinline__ uint32_t round_pack4(int a0, int a1, int a2, int a3) {
    uint32_t lo, hi;
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 12" : "=v"(lo) : "v"(a0), "v"(a1));
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 12" : "=v"(hi) : "v"(a2), "v"(a3));
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}
__device__ __forceinline__ uint32_t pack_pair(float c0, float c1) {
    return (static_cast<uint32_t>(static_cast<int>(c0)) & 0xffffu) | (static_cast<uint32_t>(static_cast<int>(c1)) << 16);
}

// taps 4q .. 4q+3 of a 1-phase table as packed u8 (0 past the last tap)
__device__ __forceinline__ uint32_t pack_taps(const float *c, int taps, int q) {
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (4 * q + j < taps) w |= static_cast<uint32_t>(c[4 * q + j]) << (8 * j);
    return w;
}

__device__ __forceinline__ void sep_position(const SepTaps &t, int o, int *start, int *phase) {
    if (t.phased) {
        const double X = reduce_x(o, t.shrink, t.centre);
        *start = static_cast<int>(X) - t.pad;
        *phase = ((static_cast<int>(X * 256.0) & 255) + 1) >> 1;
    } else {
        *start = o - t.pad;
        *phase = 0;
    }
}

template <int MODE>
__device__ __forceinline__ uint32_t sep_round(float acc, const SepTaps &t) {
    if (MODE == kSepReduce) return fixed_round_u(acc);
    return min(div_floor(acc + t.rounding, t.inv_scale), 255u);
}

// ===========================================================================
// vertical pass
// ===========================================================================
struct VPassArgs {
    const u8 *in;
    u8 *out;
    int row_bytes;        // bytes per output row == bytes the pass covers per input row
    int in_pitch;         // bytes between input rows
    long long in_base;    // byte offset of local input (row 0, first column) in an image
    long long in_img, out_img;
    int hl;               // local input rows (COPY clamp range)
    int oy0, oh;          // output rows [oy0, oy0 + oh) in op-output coordinates
    int col_blocks, kr_blocks;
    int kr;               // output rows per block
    int lrows;            // LDS input-row capacity (>= (kr - 1) * shrink + taps + 1)
    SepTaps tp;
};

constexpr int kVStride = 260;  // LDS dwords per staged row: 256 + 1 (skewed rows) + pad

typedef __attribute__((address_space(3))) void lds_void;
__device__ __forceinline__ lds_void *to_lds(void *p) { return (lds_void *)p; }  // generic -> LDS addrspacecast

// Stage input rows r_lo .. r_lo + L - 1 (COPY-clamped) of 1 KiB column block cb
// into LDS rows of kVStride dwords with direct-to-LDS buffer loads (DMA bytes per
// lane; DMA 0: dword loads from each row's aligned-down start plus one dword).
template <int DMA>
__device__ __forceinline__ void vstage_rows(const VPassArgs &a, uint32_t *rows, int img, int cb, int r_lo, int L,
                                            int wave, int lane, int *delta) {
    const u8 *src = a.in + img * a.in_img;
    const long long col0 = a.in_base + static_cast<long long>(cb) * 1024;
    if (DMA == 16) {
        const __amdgpu_buffer_rsrc_t rs = image_rsrc(src, a.in_img);
        for (int l = wave; l < L; l += 4) {
            const int r = clampi(r_lo + l, 0, a.hl - 1);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, to_lds(rows + l * kVStride), 16,
                                                     static_cast<int>(col0 + static_cast<long long>(r) * a.in_pitch) + lane * 16,
                                                     0, 0, 0);
        }
    } else if (DMA == 4) {
        const __amdgpu_buffer_rsrc_t rs = image_rsrc(src, a.in_img);
        for (int l = 0; l < L; ++l) {
            const int r = clampi(r_lo + l, 0, a.hl - 1);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, to_lds(rows + l * kVStride + wave * 64), 4,
                                                     static_cast<int>(col0 + static_cast<long long>(r) * a.in_pitch) +
                                                         wave * 256 + lane * 4,
                                                     0, 0, 0);
        }
    } else {
        const __amdgpu_buffer_rsrc_t rs = image_rsrc_aligned(src, a.in_img, delta);
        for (int l = 0; l < L; ++l) {
            const int r = clampi(r_lo + l, 0, a.hl - 1);
            const int a4 = static_cast<int>(*delta + col0 + static_cast<long long>(r) * a.in_pitch) & ~3;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, to_lds(rows + l * kVStride + wave * 64), 4,
                                                     a4 + wave * 256 + lane * 4, 0, 0, 0);
            if (wave == 0 && lane == 0)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, to_lds(rows + l * kVStride + 256), 4, a4 + 1024, 0, 0, 0);
        }
    }
}

// Vertical reduce with TP2 tap pairs known at compile time (16 / 4-byte aligned
// rows, 4-byte output rows): per output row and lane 2 TP2 LDS reads issued
// together, 4 v_perm + 4 v_dot2 per pair, the rounding folded into the
// accumulator seed and v_ashr_pk_u8_i32, one buffer store with the row offset in
// an SGPR.  k_vpass's generic loop spent ~2x the VALU on loop, rounding and
// address work (profiles/r02 pmc: 97.6M VALU for 1080p RGB /1.6 x 64).
template <int TP2, int DMA>
__global__ void __launch_bounds__(256) k_vreduce(VPassArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t vsm[];
    uint32_t *rows = vsm;                              // lrows x kVStride dwords
    uint32_t *cpk = vsm + a.lrows * kVStride;          // kr x kVpPairs int16 tap pairs (16-byte aligned)
    int *soff = reinterpret_cast<int *>(cpk + a.kr * kVpPairs);
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int cb = t % a.col_blocks;
    const int rest = t / a.col_blocks;
    const int kb = rest % a.kr_blocks;
    const int img = rest / a.kr_blocks;
    const int taps = a.tp.taps;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int y0 = kb * a.kr;
    const int nk = min(a.kr, a.oh - y0);
    int r_lo, r_last, ph;
    sep_position(a.tp, a.oy0 + y0, &r_lo, &ph);
    sep_position(a.tp, a.oy0 + y0 + nk - 1, &r_last, &ph);
    int delta = 0;
    vstage_rows<DMA>(a, rows, img, cb, r_lo, r_last + taps - r_lo, wave, lane, &delta);
    for (int i = tid; i < nk * kVpPairs; i += 256) {
        const int k = i / kVpPairs, m = i - k * kVpPairs;
        int st;
        sep_position(a.tp, a.oy0 + y0 + k, &st, &ph);
        const float *c = a.tp.tab + ph * taps;
        cpk[i] = m < TP2 ? pack_pair(2 * m < taps ? c[2 * m] : 0.f, 2 * m + 1 < taps ? c[2 * m + 1] : 0.f) : 0u;
        if (m == 0) soff[k] = st - r_lo;
    }
    __syncthreads();
    const int j = cb * 1024 + tid * 4;
    if (j >= a.row_bytes) return;
    const __amdgpu_buffer_rsrc_t os =
        __builtin_amdgcn_make_buffer_rsrc(a.out + img * a.out_img, 0, static_cast<int>(a.out_img), 0x00020000);
    for (int k = 0; k < nk; ++k) {
        const uint32_t *rp = rows + __builtin_amdgcn_readfirstlane(soff[k]) * kVStride + tid;
        uint32_t v[2 * TP2];
#pragma unroll
        for (int i = 0; i < 2 * TP2; ++i) v[i] = rp[i * kVStride];
        const uint4 c0 = reinterpret_cast<const uint4 *>(cpk + k * kVpPairs)[0];
        const uint4 c1 = reinterpret_cast<const uint4 *>(cpk + k * kVpPairs)[1];
        const uint32_t cw[kVpPairs] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        int acc[4] = {2048, 2048, 2048, 2048};
#pragma unroll
        for (int m = 0; m < TP2; ++m)
#pragma unroll
            for (int z = 0; z < 4; ++z) acc[z] = dot2_byte(v[2 * m], v[2 * m + 1], z, cw[m], acc[z]);
        __builtin_amdgcn_raw_buffer_store_b32(round_pack4(acc[0], acc[1], acc[2], acc[3]), os, j,
                                              (y0 + k) * a.row_bytes, 0);
    }
}

// DMA: 16 / 4 = bytes per lane of the direct-to-LDS buffer loads when rows are
// 16 / 4 byte aligned; 0 = any alignment (dword DMA from each row's aligned-down
// start, bytes shifted into place with v_alignbyte).
template <int MODE, int DMA>
__global__ void __launch_bounds__(256) k_vpass(VPassArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t vsm[];
    uint32_t *rows = vsm;                                                // lrows x kVStride dwords
    float *vcoef = reinterpret_cast<float *>(vsm + a.lrows * kVStride);  // kr x taps
    int *soff = reinterpret_cast<int *>(vcoef + a.kr * a.tp.taps);  // kr start rows
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int cb = t % a.col_blocks;
    const int rest = t / a.col_blocks;
    const int kb = rest % a.kr_blocks;
    const int img = rest / a.kr_blocks;
    const int taps = a.tp.taps;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: no waterfall around the DMA
    const int y0 = kb * a.kr;
    const int nk = min(a.kr, a.oh - y0);
    int r_lo, r_last, ph;
    sep_position(a.tp, a.oy0 + y0, &r_lo, &ph);
    sep_position(a.tp, a.oy0 + y0 + nk - 1, &r_last, &ph);
    const int L = r_last + taps - r_lo;
    // ---- stage the L input rows of this 1 KiB column block in LDS ----
    int delta = 0;
    vstage_rows<DMA>(a, rows, img, cb, r_lo, L, wave, lane, &delta);
    const long long col0 = a.in_base + static_cast<long long>(cb) * 1024;
    if (!a.tp.dot) {
        for (int i = tid; i < nk * taps; i += 256) {
            const int k = i / taps;
            int s;
            sep_position(a.tp, a.oy0 + y0 + k, &s, &ph);
            vcoef[i] = a.tp.tab[ph * taps + (i - k * taps)];
        }
    }
    if (tid < nk) {
        int s;
        sep_position(a.tp, a.oy0 + y0 + tid, &s, &ph);
        soff[tid] = s - r_lo;
    }
    // conv: packed u8 taps; reduce: int16 pairs per row (16-byte aligned for b128 reads)
    uint32_t *cpk = vsm + ((a.lrows * kVStride + a.kr * (taps + 1) + 3) & ~3);
    const int tq = (taps + 3) >> 2, tp2 = (taps + 1) >> 1;
    if (MODE == kSepConv && tid < tq) cpk[tid] = pack_taps(a.tp.tab, taps, tid);
    // conv, quad-transposed rows: coefficient set p (output row k with k % 4 == p) for
    // quad j holds taps 4j + b - p, b = 0..3 (0 outside the mask)
    const int tqp = (taps + 6) >> 2;
    if (MODE == kSepConv && tid < 4 * tqp) {
        const int p = tid / tqp, j = tid - p * tqp;
        uint32_t w = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int t = 4 * j + b - p;
            if (t >= 0 && t < taps) w |= static_cast<uint32_t>(a.tp.tab[t]) << (8 * b);
        }
        cpk[tq + tid] = w;
    }
    if (MODE == kSepReduce && a.tp.dot) {
        for (int i = tid; i < nk * tp2; i += 256) {
            const int k = i / tp2, m = i - k * tp2;
            int st;
            sep_position(a.tp, a.oy0 + y0 + k, &st, &ph);
            const float *c = a.tp.tab + ph * taps;
            cpk[i] = pack_pair(c[2 * m], 2 * m + 1 < taps ? c[2 * m + 1] : 0.f);
        }
    }
    __syncthreads();
    // ---- KR output rows from LDS ----
    const int j = cb * 1024 + tid * 4;
    if (j >= a.row_bytes) return;
    const int nb = min(4, a.row_bytes - j);
    u8 *dst = a.out + img * a.out_img + static_cast<long long>(y0) * a.row_bytes + j;
    const long long skew0 = delta + col0;
    if (MODE == kSepConv && a.tp.dot && DMA != 0 && a.tp.tq) {
        // each lane transposes its own column's staged rows in place, 4-row quads at a time
        // (no other lane touches them), so an output row costs 4 LDS reads + 4 v_dot4 per
        // quad instead of 4 reads + 8 v_perm + 4 v_dot4 (conv: soff[k] == k)
        const int nq = (nk + taps + 2) >> 2;
        for (int m = 0; m < nq; ++m) {
            uint32_t *rq = rows + 4 * m * kVStride + tid;
            uint32_t t[4];
            transpose4x4(rq[0], rq[kVStride], rq[2 * kVStride], rq[3 * kVStride], t);
#pragma unroll
            for (int z = 0; z < 4; ++z) rq[z * kVStride] = t[z];
        }
        const uint32_t *cph = cpk + tq;
        for (int k = 0; k < nk; ++k) {
            const int p = k & 3, nqk = (p + taps + 3) >> 2;
            const uint32_t *rq = rows + 4 * (k >> 2) * kVStride + tid;
            const uint32_t *cw = cph + p * tqp;
            uint32_t acc[4] = {0u, 0u, 0u, 0u};
            for (int j = 0; j < nqk; ++j) {
                const uint32_t c = cw[j];
#pragma unroll
                for (int z = 0; z < 4; ++z) acc[z] = __builtin_amdgcn_udot4(rq[(4 * j + z) * kVStride], c, acc[z], false);
            }
            uint32_t o = 0;
#pragma unroll
            for (int z = 0; z < 4; ++z) o |= sep_round<MODE>(static_cast<float>(acc[z]), a.tp) << (8 * z);
            u8 *q = dst + static_cast<long long>(k) * a.row_bytes;
            if (nb == 4 && (reinterpret_cast<uintptr_t>(q) & 3u) == 0) {
                *reinterpret_cast<uint32_t *>(q) = o;
            } else {
                for (int z = 0; z < nb; ++z) q[z] = static_cast<u8>(o >> (8 * z));
            }
        }
        return;
    }
    if (MODE == kSepConv && a.tp.dot) {
        for (int k = 0; k < nk; ++k) {
            const uint32_t *rp = rows + soff[k] * kVStride + tid;
            uint32_t acc[4] = {0u, 0u, 0u, 0u};
            for (int q = 0; q < tq; ++q) {
                uint32_t v[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    v[i] = rp[(4 * q + i) * kVStride];
                    if (DMA == 0) {
                        const int r = clampi(r_lo + soff[k] + 4 * q + i, 0, a.hl - 1);
                        const int sh = static_cast<int>(skew0 + static_cast<long long>(r) * a.in_pitch) & 3;
                        v[i] = __builtin_amdgcn_alignbyte(rp[(4 * q + i) * kVStride + 1], v[i], sh);
                    }
                }
                uint32_t t[4];
                transpose4x4(v[0], v[1], v[2], v[3], t);
                const uint32_t cw = cpk[q];
#pragma unroll
                for (int z = 0; z < 4; ++z) acc[z] = __builtin_amdgcn_udot4(t[z], cw, acc[z], false);
            }
            uint32_t o = 0;
#pragma unroll
            for (int z = 0; z < 4; ++z) o |= sep_round<MODE>(static_cast<float>(acc[z]), a.tp) << (8 * z);
            u8 *q = dst + static_cast<long long>(k) * a.row_bytes;
            if (nb == 4 && (reinterpret_cast<uintptr_t>(q) & 3u) == 0) {
                *reinterpret_cast<uint32_t *>(q) = o;
            } else {
                for (int z = 0; z < nb; ++z) q[z] = static_cast<u8>(o >> (8 * z));
            }
        }
        return;
    }
    if (MODE == kSepReduce && a.tp.dot) {
        for (int k = 0; k < nk; ++k) {
            const uint32_t *rp = rows + soff[k] * kVStride + tid;
            const uint32_t *ck = cpk + k * tp2;
            int acc[4] = {0, 0, 0, 0};
            for (int m = 0; m < tp2; ++m) {
                uint32_t v[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    v[i] = rp[(2 * m + i) * kVStride];
                    if (DMA == 0) {
                        const int r = clampi(r_lo + soff[k] + 2 * m + i, 0, a.hl - 1);
                        const int sh = static_cast<int>(skew0 + static_cast<long long>(r) * a.in_pitch) & 3;
                        v[i] = __builtin_amdgcn_alignbyte(rp[(2 * m + i) * kVStride + 1], v[i], sh);
                    }
                }
                const uint32_t cw = ck[m];
#pragma unroll
                for (int z = 0; z < 4; ++z) acc[z] = dot2_byte(v[0], v[1], z, cw, acc[z]);
            }
            uint32_t o = 0;
#pragma unroll
            for (int z = 0; z < 4; ++z) o |= fixed_round_i(acc[z]) << (8 * z);
            u8 *q = dst + static_cast<long long>(k) * a.row_bytes;
            if (nb == 4 && (reinterpret_cast<uintptr_t>(q) & 3u) == 0) {
                *reinterpret_cast<uint32_t *>(q) = o;
            } else {
                for (int z = 0; z < nb; ++z) q[z] = static_cast<u8>(o >> (8 * z));
            }
        }
        return;
    }
    for (int k = 0; k < nk; ++k) {
        const uint32_t *rp = rows + soff[k] * kVStride + tid;
        const float *ck = vcoef + k * taps;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll 4
        for (int i = 0; i < taps; ++i) {
            uint32_t v = rp[i * kVStride];
            if (DMA == 0) {  // shift the row's bytes into place (row start skew is uniform)
                const int r = clampi(r_lo + soff[k] + i, 0, a.hl - 1);
                const int sh = static_cast<int>(skew0 + static_cast<long long>(r) * a.in_pitch) & 3;
                v = __builtin_amdgcn_alignbyte(rp[i * kVStride + 1], v, sh);
            }
            const float c = ck[i];
            a0 = __builtin_fmaf(c, ubyte_f<0>(v), a0);
            a1 = __builtin_fmaf(c, ubyte_f<1>(v), a1);
            a2 = __builtin_fmaf(c, ubyte_f<2>(v), a2);
            a3 = __builtin_fmaf(c, ubyte_f<3>(v), a3);
        }
        const uint32_t o = sep_round<MODE>(a0, a.tp) | (sep_round<MODE>(a1, a.tp) << 8) |
                           (sep_round<MODE>(a2, a.tp) << 16) | (sep_round<MODE>(a3, a.tp) << 24);
        u8 *q = dst + static_cast<long long>(k) * a.row_bytes;
        if (nb == 4 && (reinterpret_cast<uintptr_t>(q) & 3u) == 0) {
            *reinterpret_cast<uint32_t *>(q) = o;
        } else {
            for (int z = 0; z < nb; ++z) q[z] = static_cast<u8>(o >> (8 * z));
        }
    }
}

// vertical pass for masks too tall for LDS staging: taps gathered through L1
template <int MODE>
__global__ void __launch_bounds__(256) k_vpass_gather(VPassArgs a) {
    const int j = (blockIdx.x * 256 + threadIdx.x) * 4;
    const int y = blockIdx.y;
    const int img = blockIdx.z;
    if (j >= a.row_bytes) return;
    const int nb = min(4, a.row_bytes - j);
    int s, ph;
    sep_position(a.tp, a.oy0 + y, &s, &ph);
    const float *c = a.tp.tab + ph * a.tp.taps;
    const u8 *src = a.in + img * a.in_img + a.in_base + j;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int i = 0; i < a.tp.taps; ++i) {
        const u8 *p = src + static_cast<long long>(clampi(s + i, 0, a.hl - 1)) * a.in_pitch;
        const float ci = c[i];
        for (int z = 0; z < nb; ++z) acc[z] = __builtin_fmaf(ci, static_cast<float>(p[z]), acc[z]);
    }
    u8 *q = a.out + img * a.out_img + static_cast<long long>(y) * a.row_bytes + j;
    for (int z = 0; z < nb; ++z) q[z] = static_cast<u8>(sep_round<MODE>(acc[z], a.tp));
}

// ===========================================================================
// horizontal pass
// ===========================================================================
struct HPassArgs {
    const u8 *in;
    u8 *out;
    int in_pitch;         // bytes between input rows
    long long in_base;    // byte offset of local input (row 0, column 0) in an image
    long long in_img, out_img;
    int wl;               // local input width, pixels (COPY clamp range)
    int rows;             // rows processed == output rows
    int ox0, ow;          // output columns [ox0, ox0 + ow) in op-output coordinates
    int x_blocks, rb_blocks;
    int span_max;         // LDS pixels per staged row (incl. 64 of DMA overrun)
    int raw_max;          // LDS dwords per staged raw row (B < 4; incl. 64 of overrun)
    int ntab;             // floats of the tap table staged in LDS (0: taps in registers)
    int repack4;          // raw path: 4-pixel vector repack (MIPX_HP_REPACK=0: one pixel per item)
    int pack3;            // B = 3: 4 lanes' pixels stored as 3 dwords (MIPX_HP_PACK3=1/0 forces; default: reduce, shrink >= 2)
    SepTaps tp;
    const uint32_t *pairs;  // k_hreduce: int16 tap pairs [129][2][tpa] (device_reduce_pairs)
    int tpa;
    int rbn;                // k_hreduce: rows per block (runtime; k_hpass uses its RB)
};

template <int B>
__device__ __forceinline__ uint32_t load_px_g(const u8 *p) {
    uint32_t v = p[0];
    if (B > 1) v |= static_cast<uint32_t>(p[1]) << 8;
    if (B > 2) v |= static_cast<uint32_t>(p[2]) << 16;
    if (B > 3) v |= static_cast<uint32_t>(p[3]) << 24;
    return v;
}

// One 3-band output pixel per lane (o: 24 bits). pack3: the 4 lanes of an
// aligned 4-pixel group exchange neighbours (one ds_bpermute) and store the
// group's 12 bytes as 3 dwords instead of 12 byte stores; groups that are
// partial (row end) or not dword aligned fall back to bytes.  j = x & 3 is the
// lane's slot in its group (x0 is a multiple of 256, so lanes of a group are
// adjacent lanes of one wave).  Every lane of the wave must call it.
__device__ __forceinline__ void store_rgb_px(u8 *q, uint32_t o, int j, bool full, bool pack3) {
    const uint32_t nx = __shfl_down(o, 1, 64);
    u8 *qg = q - 3 * j;
    if (pack3 && full && (reinterpret_cast<uintptr_t>(qg) & 3u) == 0) {
        if (j < 3) {
            const uint32_t w = j == 0 ? (o | (nx << 24)) : j == 1 ? ((o >> 8) | (nx << 16)) : ((o >> 16) | (nx << 8));
            *reinterpret_cast<uint32_t *>(qg + 4 * j) = w;
        }
    } else {
        q[0] = static_cast<u8>(o);
        q[1] = static_cast<u8>(o >> 8);
        q[2] = static_cast<u8>(o >> 16);
    }
}

// Horizontal staging, shared by k_hpass and k_hreduce: rows y_first .. y_first +
// nr - 1 of the input span feeding output columns [x0, x_last] of block xb,
// DMA'd to LDS (hstage_issue), then edge-filled or repacked to one u32 per pixel
// (hstage_finish: both barriers included; htq: conv's in-place 4x4 transposes).
struct HStage {
    int x0, x_last, lo, hi, span, y_first, nr, cl, ch, org, delta;
    long long row0;
};

template <int B, int DW>
__device__ __forceinline__ void hstage_issue(const HPassArgs &a, uint32_t *spx, uint32_t *raw, int xb, int rb,
                                             int rbn, int img, int wave, int lane, HStage &g) {
    const int taps = a.tp.taps;
    const int x0 = xb * 256;
    const int x_last = min(x0 + 255, a.ow - 1);
    int lo, hi, ph;
    sep_position(a.tp, a.ox0 + x0, &lo, &ph);
    sep_position(a.tp, a.ox0 + x_last, &hi, &ph);
    hi += taps - 1;
    const int span = hi - lo + 1;
    const int y_first = rb * rbn;
    const int nr = min(rbn, a.rows - y_first);
    const int cl = max(lo, 0), ch = min(hi, a.wl - 1);  // pixels actually inside the row
    const int org = DW == 16 ? (lo & ~3) : lo;           // pixel of LDS slot 0 (floor for lo < 0)
    const u8 *img_base = a.in + img * a.in_img;
    const long long row0 = a.in_base + static_cast<long long>(y_first) * a.in_pitch;
    int delta = 0;
    // (row, chunk) pairs dealt to the 4 waves round robin, walked without divisions
    auto for_chunks = [&](int chunks, auto &&issue) {
        int rr = 0, q = wave;
        while (q >= chunks) q -= chunks, ++rr;
        while (rr < nr) {
            issue(rr, q);
            q += 4;
            while (q >= chunks) q -= chunks, ++rr;
        }
    };
    if (DW == 16) {  // B = 4, rows 16-byte aligned: 4 pixels per lane straight into their slots
        const __amdgpu_buffer_rsrc_t rs = image_rsrc(img_base, a.in_img);
        const int cl4 = cl & ~3;
        const int chunks = (((ch - cl4 + 4) >> 2) + 63) >> 6;
        for_chunks(chunks, [&](int rr, int q) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, to_lds(spx + rr * a.span_max + (cl4 - org) + q * 256), 16,
                static_cast<int>(row0 + static_cast<long long>(rr) * a.in_pitch) + 4 * cl4 + 16 * (q * 64 + lane), 0, 0, 0);
        });
    } else if (DW == 4) {  // B = 4, rows dword aligned
        const __amdgpu_buffer_rsrc_t rs = image_rsrc(img_base, a.in_img);
        const int chunks = (ch - cl + 1 + 63) >> 6;
        for_chunks(chunks, [&](int rr, int q) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, to_lds(spx + rr * a.span_max + (cl - org) + q * 64), 4,
                static_cast<int>(row0 + static_cast<long long>(rr) * a.in_pitch) + 4 * (cl + q * 64 + lane), 0, 0, 0);
        });
    } else {  // any alignment: each row's raw bytes from its dword-aligned-down start
        const __amdgpu_buffer_rsrc_t rs = image_rsrc_aligned(img_base, a.in_img, &delta);
        const int nd = (B * (ch - cl + 1) + 3 + 3) >> 2;
        const int chunks = (nd + 63) >> 6;
        for_chunks(chunks, [&](int rr, int q) {
            const int a4 = static_cast<int>(delta + row0 + static_cast<long long>(rr) * a.in_pitch + B * cl) & ~3;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, to_lds(raw + rr * a.raw_max + q * 64), 4,
                                                     a4 + 4 * (q * 64 + lane), 0, 0, 0);
        });
    }
    g = HStage{x0, x_last, lo, hi, span, y_first, nr, cl, ch, org, delta, row0};
}

template <int B, int DW>
__device__ __forceinline__ void hstage_finish(const HPassArgs &a, uint32_t *spx, uint32_t *raw, const HStage &g,
                                              int tid, bool htq) {
    constexpr bool DIRECT = DW != 0;
    const int lo = g.lo, hi = g.hi, span = g.span, nr = g.nr, cl = g.cl, ch = g.ch, org = g.org, delta = g.delta;
    const long long row0 = g.row0;
    __syncthreads();
    {  // COPY edges (direct) or the repack of the raw bytes with each row's skew
        if (DIRECT) {
            const int nl = cl - lo, nrt = hi - ch;
            for (int i = tid; i < nr * (nl + nrt); i += 256) {
                const int rr = i / (nl + nrt), f = i - rr * (nl + nrt);
                uint32_t *row = spx + rr * a.span_max - org;  // indexed by pixel
                if (f < nl) row[lo + f] = row[cl];
                else row[ch + 1 + (f - nl)] = row[ch];
            }
        } else {
            const u8 *rb8 = reinterpret_cast<const u8 *>(raw);
            auto px1 = [&](int rr, int p) -> uint32_t {  // one pixel, COPY edge by clamping
                const int c = clampi(lo + p, 0, a.wl - 1);
                const int skew = static_cast<int>(delta + row0 + static_cast<long long>(rr) * a.in_pitch + B * cl) & 3;
                const u8 *q = rb8 + rr * a.raw_max * 4 + (c - cl) * B + skew;
                uint32_t v = q[0];
                if (B > 1) v |= static_cast<uint32_t>(q[1]) << 8;
                if (B > 2) v |= static_cast<uint32_t>(q[2]) << 16;
                if (B > 3) v |= static_cast<uint32_t>(q[3]) << 24;
                return v;
            };
            auto repack1 = [&](int rr, int p) { spx[rr * a.span_max + p] = px1(rr, p); };
            if (a.repack4) {
                // 4 pixels per item: 4 B bytes from the raw row as 4 dword reads + v_alignbyte,
                // split into one u32 per pixel with v_perm_b32, one 16-byte LDS write
                const int groups = (span + 3) >> 2;
                const int dy = 256 / groups, dq = 256 - dy * groups;
                int rr = tid / groups, g = tid - rr * groups;
                for (; rr < nr; rr += dy, g += dq, rr += g >= groups ? 1 : 0, g -= g >= groups ? groups : 0) {
                    const int p0 = 4 * g, c0 = lo + p0;
                    if (c0 < 0 || c0 + 3 > a.wl - 1 || p0 + 3 >= span) {
                        if (htq) {  // whole group (clamped past the span) so it can be transposed
                            uint32_t t[4];
                            transpose4x4(px1(rr, p0), px1(rr, p0 + 1), px1(rr, p0 + 2), px1(rr, p0 + 3), t);
                            *reinterpret_cast<uint4 *>(spx + rr * a.span_max + p0) = uint4{t[0], t[1], t[2], t[3]};
                        } else {
                            for (int k = 0; k < 4 && p0 + k < span; ++k) repack1(rr, p0 + k);
                        }
                        continue;
                    }
                    const int skew = static_cast<int>(delta + row0 + static_cast<long long>(rr) * a.in_pitch + B * cl) & 3;
                    const int o = (c0 - cl) * B + skew;
                    const uint32_t *rw = raw + rr * a.raw_max + (o >> 2);
                    const int sh = o & 3;
                    uint32_t d[B];
#pragma unroll
                    for (int k = 0; k < B; ++k) d[k] = __builtin_amdgcn_alignbyte(rw[k + 1], rw[k], sh);
                    uint4 px4;
                    if (B == 1) {
                        px4 = uint4{d[0] & 0xffu, (d[0] >> 8) & 0xffu, (d[0] >> 16) & 0xffu, d[0] >> 24};
                    } else if (B == 2) {
                        px4 = uint4{d[0] & 0xffffu, d[0] >> 16, d[B - 1] & 0xffffu, d[B - 1] >> 16};
                    } else if (B == 3) {
                        px4 = uint4{__builtin_amdgcn_perm(d[1], d[0], 0x0C020100u),
                                    __builtin_amdgcn_perm(d[1], d[0], 0x0C050403u),
                                    __builtin_amdgcn_perm(d[B - 1], d[1], 0x0C040302u),
                                    __builtin_amdgcn_perm(d[B - 1], d[B - 1], 0x0C030201u)};
                    } else {
                        px4 = uint4{d[0], d[1 % B], d[2 % B], d[3 % B]};
                    }
                    if (htq) {
                        uint32_t t[4];
                        transpose4x4(px4.x, px4.y, px4.z, px4.w, t);
                        px4 = uint4{t[0], t[1], t[2], t[3]};
                    }
                    *reinterpret_cast<uint4 *>(spx + rr * a.span_max + p0) = px4;
                }
            } else {
                for (int i = tid; i < nr * span; i += 256) {
                    const int rr = i / span;
                    repack1(rr, i - rr * span);
                }
            }
        }
        __syncthreads();
        if (DIRECT && htq) {  // transpose the DMA'd (and edge-filled) slots in place, 4 at a time
            const int groups = (hi - org + 4) >> 2;
            const int dy = 256 / groups, dq = 256 - dy * groups;
            int rr = tid / groups, g = tid - rr * groups;
            for (; rr < nr; rr += dy, g += dq, rr += g >= groups ? 1 : 0, g -= g >= groups ? groups : 0) {
                uint4 *q4 = reinterpret_cast<uint4 *>(spx + rr * a.span_max + 4 * g);
                const uint4 v = *q4;
                uint32_t t[4];
                transpose4x4(v.x, v.y, v.z, v.w, t);
                *q4 = uint4{t[0], t[1], t[2], t[3]};
            }
            __syncthreads();
        }
    }
}

// DW = 16 / 4 (B = 4, rows 16 / 4 byte aligned): direct-to-LDS dwordx4 / dword
// DMA of the span into the pixel slots (DW 16 stages from the 4-pixel-aligned
// start, so each row's LDS origin is lo rounded down to 4 pixels); DW = 0: DMA
// of each row's raw bytes from its aligned-down start, repacked to one u32 per
// pixel in LDS (any alignment, any band count).
// TREG > 0: each lane holds its (<= TREG) taps in registers (reduce); 0: taps
// from the LDS table.
template <int B, int RB, int MODE, int DW, int TREG>
__global__ void __launch_bounds__(256) k_hpass(HPassArgs a) {
    constexpr bool DIRECT = DW != 0;
    extern __shared__ __attribute__((aligned(16))) uint32_t hsm[];
    float *ctab = reinterpret_cast<float *>(hsm);
    uint32_t *spx = hsm + a.ntab;
    uint32_t *raw = spx + RB * a.span_max;
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int xb = t % a.x_blocks;
    const int rest = t / a.x_blocks;
    const int rb = rest % a.rb_blocks;
    const int img = rest / a.rb_blocks;
    const int taps = a.tp.taps;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: no waterfall around the DMA
    HStage g;
    hstage_issue<B, DW>(a, spx, raw, xb, rb, RB, img, wave, lane, g);
    const int x0 = g.x0, x_last = g.x_last, org = g.org;
    const int y_first = g.y_first, nr = g.nr;
    // this lane's taps
    const int x = x0 + tid;
    int s = 0, xph = 0;
    sep_position(a.tp, a.ox0 + min(x, x_last), &s, &xph);
    float cr[TREG > 0 ? TREG : 1];
    if (TREG > 0) {
        const float *c = a.tp.tab + xph * taps;
#pragma unroll
        for (int i = 0; i < TREG; ++i) cr[i] = i < taps ? c[i] : 0.f;
    } else {
        const int nt = (a.tp.phased ? kTransformScale + 1 : 1) * taps;
        const int nfl = MODE == kSepConv ? ((taps + 3) & ~3) : a.ntab;  // conv: packed phase sets follow
        for (int i = tid; i < nfl; i += 256) ctab[i] = i < nt ? a.tp.tab[i] : 0.f;
        if (MODE == kSepConv) {
            const int tqp = (taps + 6) >> 2;
            for (int i = tid; i < 4 * tqp; i += 256) {
                const int p = i / tqp, j = i - p * tqp;
                uint32_t w = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int t = 4 * j + b - p;
                    if (t >= 0 && t < taps) w |= static_cast<uint32_t>(a.tp.tab[t]) << (8 * b);
                }
                reinterpret_cast<uint32_t *>(ctab)[nfl + i] = w;
            }
        }
    }
    // conv: staged pixels transposed per 4-slot group (channel-major dwords), so an
    // output pixel costs B LDS reads + B v_dot4 per group, no per-pixel v_perm
    const bool htq = MODE == kSepConv && a.tp.dot && a.tp.tq && (DIRECT || a.repack4);
    hstage_finish<B, DW>(a, spx, raw, g, tid, htq);
    if (x > x_last) return;
    const uint32_t *sp = spx + (s - org);
    float acc[RB][B];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int z = 0; z < B; ++z) acc[r][z] = 0.f;
    auto tap = [&](int i, float ci) {
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            if (r < nr) {
                const uint32_t v = sp[r * a.span_max + i];
#pragma unroll
                for (int z = 0; z < B; ++z) {
                    const float pz = z == 0 ? ubyte_f<0>(v) : z == 1 ? ubyte_f<1>(v) : z == 2 ? ubyte_f<2>(v) : ubyte_f<3>(v);
                    acc[r][z] = __builtin_fmaf(ci, pz, acc[r][z]);
                }
            }
        }
    };
    if (MODE == kSepReduce && TREG > 0 && a.tp.dot) {  // reduce: this lane's taps as int16 pairs
        uint32_t cp[TREG > 0 ? TREG / 2 : 1];
#pragma unroll
        for (int m = 0; m < TREG / 2; ++m) cp[m] = pack_pair(cr[2 * m], cr[2 * m + 1]);
        int iacc[RB][B];
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int z = 0; z < B; ++z) iacc[r][z] = 0;
#pragma unroll
        for (int m = 0; m < TREG / 2; ++m) {
            if (2 * m < taps) {
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    if (r < nr) {
                        const uint32_t *pr = sp + r * a.span_max + 2 * m;
                        const uint32_t v0 = pr[0], v1 = pr[1];
#pragma unroll
                        for (int z = 0; z < B; ++z) iacc[r][z] = dot2_byte(v0, v1, z, cp[m], iacc[r][z]);
                    }
                }
            }
        }
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            if (r >= nr) continue;
            u8 *q = a.out + img * a.out_img + (static_cast<long long>(y_first + r) * a.ow + x) * B;
            if (B == 4) {
                uint32_t o = 0;
#pragma unroll
                for (int z = 0; z < B; ++z) o |= fixed_round_i(iacc[r][z]) << (8 * z);
                *reinterpret_cast<uint32_t *>(q) = o;
            } else if (B == 3) {
                store_rgb_px(q, fixed_round_i(iacc[r][0]) | (fixed_round_i(iacc[r][1 % B]) << 8) |
                                    (fixed_round_i(iacc[r][2 % B]) << 16),
                             tid & 3, (x | 3) <= x_last, a.pack3 != 0);
            } else {
#pragma unroll
                for (int z = 0; z < B; ++z) q[z] = static_cast<u8>(fixed_round_i(iacc[r][z]));
            }
        }
        return;
    }
    if (MODE == kSepConv && htq) {  // conv on transposed groups: phase set by this lane's slot
        const int base = s - org, p = base & 3, nqk = (p + taps + 3) >> 2;
        const uint32_t *cph = reinterpret_cast<const uint32_t *>(ctab) + ((taps + 3) & ~3) + p * ((taps + 6) >> 2);
        uint32_t iacc[RB][4];
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int z = 0; z < 4; ++z) iacc[r][z] = 0u;
        for (int j = 0; j < nqk; ++j) {
            const uint32_t c = cph[j];
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                if (r < nr) {
                    const uint32_t *qd = spx + r * a.span_max + 4 * ((base >> 2) + j);
#pragma unroll
                    for (int z = 0; z < B; ++z) iacc[r][z] = __builtin_amdgcn_udot4(qd[z], c, iacc[r][z], false);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int z = 0; z < B; ++z) acc[r][z] = static_cast<float>(iacc[r][z]);
    } else if (MODE == kSepConv && a.tp.dot) {  // conv: one phase, taps packed u8 (uniform)
        uint32_t iacc[RB][4];
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int z = 0; z < 4; ++z) iacc[r][z] = 0u;
        const int tq = (taps + 3) >> 2;
        for (int q = 0; q < tq; ++q) {
            const uint32_t cw = pack_taps(ctab, taps, q);
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                if (r < nr) {
                    const uint32_t *pr = sp + r * a.span_max + 4 * q;
                    uint32_t t[4];
                    transpose4x4(pr[0], pr[1], pr[2], pr[3], t);
#pragma unroll
                    for (int z = 0; z < B; ++z) iacc[r][z] = __builtin_amdgcn_udot4(t[z], cw, iacc[r][z], false);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int z = 0; z < B; ++z) acc[r][z] = static_cast<float>(iacc[r][z]);
    } else if (TREG > 0) {
#pragma unroll
        for (int i = 0; i < TREG; ++i)
            if (i < taps) tap(i, cr[i]);
    } else {
        const float *c = ctab + xph * taps;
        for (int i = 0; i < taps; ++i) tap(i, c[i]);
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        if (r >= nr) continue;
        u8 *q = a.out + img * a.out_img + (static_cast<long long>(y_first + r) * a.ow + x) * B;
        if (B == 4) {
            uint32_t o = 0;
#pragma unroll
            for (int z = 0; z < B; ++z) o |= sep_round<MODE>(acc[r][z], a.tp) << (8 * z);
            *reinterpret_cast<uint32_t *>(q) = o;
        } else if (B == 3) {
            store_rgb_px(q, sep_round<MODE>(acc[r][0], a.tp) | (sep_round<MODE>(acc[r][1 % B], a.tp) << 8) |
                                (sep_round<MODE>(acc[r][2 % B], a.tp) << 16),
                         tid & 3, (x | 3) <= x_last, a.pack3 != 0);
        } else {
#pragma unroll
            for (int z = 0; z < B; ++z) q[z] = static_cast<u8>(sep_round<MODE>(acc[r][z], a.tp));
        }
    }
}

// horizontal reduce without LDS staging, for shrinks whose span exceeds the
// LDS budget: taps gathered through L1
// Horizontal reduce with TP2 tap pairs known at compile time (B = 3 / 4): the
// lane's tap pairs are TP2 dword loads from the int16 pair table (no float
// conversion), rows are walked outermost with the pairs in registers, each row's
// 2 TP2 pixel slots read together, rounding folded into the accumulator seed and
// v_ashr_pk_u8_i32.  k_hpass's TREG path guarded every (pair, row) step with a
// uniform branch and re-derived addresses (97M VALU + 70M SALU for 1080p RGB /1.6 x 64).
template <int B, int DW, int TP2>
__global__ void __launch_bounds__(256) k_hreduce(HPassArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hsm[];
    uint32_t *spx = hsm;
    uint32_t *raw = spx + a.rbn * a.span_max;
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int xb = t % a.x_blocks;
    const int rest = t / a.x_blocks;
    const int rb = rest % a.rb_blocks;
    const int img = rest / a.rb_blocks;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    HStage g;
    hstage_issue<B, DW>(a, spx, raw, xb, rb, a.rbn, img, wave, lane, g);
    const int x = g.x0 + tid;
    int s = 0, xph = 0;
    sep_position(a.tp, a.ox0 + min(x, g.x_last), &s, &xph);
    const uint32_t *pt = a.pairs + xph * 2 * a.tpa;  // alignment 0: (c[2m], c[2m + 1])
    uint32_t cp[TP2];
#pragma unroll
    for (int m = 0; m < TP2; ++m) cp[m] = pt[m];
    hstage_finish<B, DW>(a, spx, raw, g, tid, false);
    if (x > g.x_last) return;
    const uint32_t *sp = spx + (s - g.org);
    u8 *ob = a.out + img * a.out_img;
    const __amdgpu_buffer_rsrc_t os = __builtin_amdgcn_make_buffer_rsrc(ob, 0, static_cast<int>(a.out_img), 0x00020000);
    for (int r = 0; r < g.nr; ++r) {
        const uint32_t *pr = sp + r * a.span_max;
        uint32_t v[2 * TP2];
#pragma unroll
        for (int i = 0; i < 2 * TP2; ++i) v[i] = pr[i];
        int acc[4] = {2048, 2048, 2048, 2048};
#pragma unroll
        for (int m = 0; m < TP2; ++m)
#pragma unroll
            for (int z = 0; z < B; ++z) acc[z] = dot2_byte(v[2 * m], v[2 * m + 1], z, cp[m], acc[z]);
        const uint32_t o = round_pack4(acc[0], acc[1], acc[2], acc[3]);
        const long long row = static_cast<long long>(g.y_first + r) * a.ow;
        if (B == 4) {
            __builtin_amdgcn_raw_buffer_store_b32(o, os, x * 4, static_cast<int>(row * 4), 0);
        } else {  // 3 bytes per lane: short + byte, or the 4-lane group's 12 bytes as 3 dwords
            const int ro = static_cast<int>(row * 3);
            const uint32_t nx = __shfl_down(o, 1, 64);
            const int j = tid & 3;
            const bool p3 = a.pack3 && ((reinterpret_cast<uintptr_t>(ob) + ro) & 3u) == 0;  // uniform
            if (p3 && (x | 3) <= g.x_last) {
                if (j < 3) {
                    const uint32_t w = j == 0 ? (o | (nx << 24)) : j == 1 ? ((o >> 8) | (nx << 16)) : ((o >> 16) | (nx << 8));
                    __builtin_amdgcn_raw_buffer_store_b32(w, os, 3 * x + j, ro, 0);
                }
            } else {
                __builtin_amdgcn_raw_buffer_store_b16(static_cast<unsigned short>(o), os, 3 * x, ro, 0);
                __builtin_amdgcn_raw_buffer_store_b8(static_cast<unsigned char>(o >> 16), os, 3 * x + 2, ro, 0);
            }
        }
    }
}

// ===========================================================================
// banded products on the i8 matrix cores (k_rmf2's horizontal pass)
// ===========================================================================
// A 16-pixel output group of 16 image rows is a banded product: out[px][row] =
// sum_k C[px][k] * in[row][base + k], k over the 64-pixel K steps covering the
// group's taps.  v_mfma_i32_16x16x64_i8 takes it exactly in integers:
//  - pixels are staged channel-planar in LDS as p - 128 (XOR 0x80: signed i8);
//  - the 12-bit taps split c = 64 hi + lo (hi = c >> 6, lo = c & 63, both i8),
//    one MFMA each, the sums rejoined as (D_hi << 6) + D_lo;
//  - the offset comes back as a bias 128 * sum(c) + 2048 seeded into D_lo.
// Operand maps (checked by scripts/probe/mfma_i8_probe.hip): lane l holds
// A[l & 15][16 (l >> 4) + j], B[16 (l >> 4) + j][l & 15] (byte j) and
// D[4 (l >> 4) + i][l & 15] (register i).  A = taps of output pixel l & 15 from
// the i8 table (row ph, bytes from kHmTabPad + k - start), B = 16 staged bytes
// of image row l & 15, so each lane ends with 4 consecutive output pixels of one
// row per channel: 12 / 16 contiguous bytes to store.
typedef int hm_v4i __attribute__((ext_vector_type(4)));

// The 16-byte fragment of an i8 tap row at window offset o (tap o + j in byte j,
// 0 outside the taps): rows hold taps <= 16 after kHmTabPad zeros, so windows
// further out than 16 bytes are all zero and o clamps to [-16, 16].
__device__ __forceinline__ hm_v4i load_taps16(const signed char *row, int o) {
    o = clampi(o - kHmTabPad, -16, 16) + kHmTabPad;
    const uint32_t *p = reinterpret_cast<const uint32_t *>(row + (o & ~3));
    const int sh = o & 3;
    const uint4 d = *reinterpret_cast<const uint4 *>(p);
    const uint32_t e = p[4];
    hm_v4i r;
    r[0] = static_cast<int>(__builtin_amdgcn_alignbyte(d.y, d.x, sh));
    r[1] = static_cast<int>(__builtin_amdgcn_alignbyte(d.z, d.y, sh));
    r[2] = static_cast<int>(__builtin_amdgcn_alignbyte(d.w, d.z, sh));
    r[3] = static_cast<int>(__builtin_amdgcn_alignbyte(e, d.w, sh));
    return r;
}

// ===========================================================================
// fused reduce on the matrix cores (k_rmf2): both passes on v_mfma_i32_16x16x64_i8
// ===========================================================================
constexpr int kRmRows = 16;
constexpr int kRmMaxCt = 16;  // k_rmf2: 16-byte column tiles per wave (staged span <= 1024 bytes)

struct RmArgs {
    const u8 *in;
    u8 *out;
    int w, h, ox0, oy0, ow, oh;
    long long in_img, out_img;
    int x_blocks, y_blocks;
    int lrows;    // staged input rows per block (>= 15 vs + vtaps)
    int plane_w;  // bytes per channel plane row (multiple of 16)
    int row_w;    // bytes per intermediate row (B planes; / 16 odd)
    int nks;      // 64-pixel K steps per horizontal group
    const signed char *tab;   // device_reduce_i8(hs)
    const int *tsum;
    const signed char *tabv;  // device_reduce_i8(vs)
    const int *tsumv;
    int iw;                   // bytes per row-major intermediate row (16 x column tiles)
    int direct;               // output rows and images dword aligned (12-byte stores, no tile)
    int rsd;                  // staged row stride in dwords, (rsd mod 64) / 4 odd
    SepTaps tv, th;
};

// k_rmf2: reducev -> reduceh in one launch, the products of both passes on the i8
// matrix cores (the generic reduce for unaligned rows and shapes k_rcol declines).
// Per 16-byte column tile of the staged rows: D[byte column][output row] =
// A[byte column][staged row] x B[staged row][output row] on v_mfma_i32_16x16x64_i8,
// where A (the pixels, K = 64 staged rows) comes from two ds_read_b64_tr_b8 (the
// transposing LDS read: a 16-lane group's lanes name 8 rows x 2 half-rows, each
// lane receives one byte column of those 8 rows; scripts/probe/ds_tr8_probe.hip)
// and B is each output row's taps from the i8 table.  The lane then holds 4
// consecutive intermediate bytes of one output row: one dword write into a
// row-major intermediate, deinterleaved to channel planes for the horizontal MFMA.
// Needs 15 vs + vtaps <= 64 staged rows.
template <int B, int XW, int HT>
__global__ void __launch_bounds__(256) k_rmf2(RmArgs a) {
    constexpr int GPW = XW / 64;
    const int RS = a.rsd;
    extern __shared__ __attribute__((aligned(16))) uint32_t rsm[];
    int *ps = reinterpret_cast<int *>(rsm);  // [XW] horizontal: first tap pixel
    int *pph = ps + XW;                      // [XW] phase
    int *pbias = pph + XW;                   // [XW] 128 * tap sum + 2048
    int *vso = pbias + XW;                   // [kRmRows] vertical: first staged row of each output row
    int *vph = vso + kRmRows;                // [kRmRows] phase
    int *vbias = vph + kRmRows;              // [kRmRows] 128 * tap sum + 2048
    // one region for the staged rows, then (aliased, barrier-separated) the row-major
    // intermediate and the channel planes, then the output tile over the intermediate:
    // 31 KB at / 1.6, so 5 workgroups share a CU
    uint32_t *raw = reinterpret_cast<uint32_t *>(vbias + kRmRows);  // [lrows][RS]
    u8 *inter = reinterpret_cast<u8 *>(raw);                         // [kRmRows][iw] (pixel - 128)
    u8 *planes = inter + kRmRows * a.iw + 64;                        // [kRmRows][row_w] channel planes
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int xb = t % a.x_blocks;
    const int rest = t / a.x_blocks;
    const int yb = rest % a.y_blocks;
    const int img = rest / a.y_blocks;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int x0 = xb * XW, x_last = min(x0 + XW - 1, a.ow - 1);
    const int y0 = yb * kRmRows, nr = min(kRmRows, a.oh - y0);
    int lo, hi, ph0, r_lo, r_last;
    sep_position(a.th, a.ox0 + x0, &lo, &ph0);
    sep_position(a.th, a.ox0 + x_last, &hi, &ph0);
    hi += a.th.taps - 1;
    sep_position(a.tv, a.oy0 + y0, &r_lo, &ph0);
    sep_position(a.tv, a.oy0 + y0 + nr - 1, &r_last, &ph0);
    const int org = lo & ~3;  // first staged pixel: floor to 4 pixels (B org stays dword aligned)
    const int nqv = ((hi - org) >> 2) + 1;
    const int L = r_last + a.tv.taps - r_lo;
    {
        const __amdgpu_buffer_rsrc_t rs = image_rsrc(a.in + img * a.in_img, a.in_img);
        const int pitch = a.w * B;
        const int chunks = (B * nqv + 63) >> 6;
        for (int l = wave; l < L; l += 4) {
            const int r = clampi(r_lo + l, 0, a.h - 1);
            for (int c = 0; c < chunks; ++c)
                if (c * 64 + lane < RS) {  // the last chunk stops at the row stride
                    // rows of any alignment: a dword that starts in the image's last 3 bytes
                    // would be dropped whole by the range check, so it is loaded ending at
                    // the image's last byte and shifted into place below (tail fix-up)
                    int vo = B * org + 4 * (c * 64 + lane);
                    const int over = r * pitch + vo + 4 - static_cast<int>(a.in_img);
                    if (over > 0 && over < 4) vo -= over;
                    // the row offset rides in the VGPR offset: the buffer range check covers the
                    // VGPR offset only (not the SGPR one), so bytes past the image read 0 instead
                    // of the next image (or past the allocation), and a shifted dword stays >= 0
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, to_lds(raw + l * RS + c * 64), 4, r * pitch + vo, 0, 0, 0);
                }
        }
    }
    // HT: the lane's tap fragments (vertical: its output row; horizontal: its pixel of
    // each group, first K step) are loaded here, while the staged rows are in flight,
    // instead of after the barriers that precede the two products
    hm_v4i hbh = hm_v4i{0, 0, 0, 0}, hbl = hbh, hah[GPW], hal[GPW];
    if constexpr (HT != 0) {
        const int n = lane & 15, kg = lane >> 4;
        int sv, ph;
        sep_position(a.tv, a.oy0 + y0 + min(n, nr - 1), &sv, &ph);
        const signed char *tv = a.tabv + static_cast<size_t>(ph) * 2 * kHmTabW;
        const int ov = 16 * kg - (sv - r_lo) + kHmTabPad;
        hbh = load_taps16(tv, ov);
        hbl = load_taps16(tv + kHmTabW, ov);
#pragma unroll
        for (int gi = 0; gi < GPW; ++gi) {
            const int g = wave * GPW + gi;
            hah[gi] = hal[gi] = hm_v4i{0, 0, 0, 0};
            if (x0 + 16 * g > x_last) continue;
            int s0, sp, pp;
            sep_position(a.th, a.ox0 + x0 + 16 * g, &s0, &pp);
            const int p = min(16 * g + n, x_last - x0);
            sep_position(a.th, a.ox0 + x0 + p, &sp, &pp);
            const int o0 = ((s0 - org) & ~15) + 16 * kg - (sp - org) + kHmTabPad;
            const signed char *thr = a.tab + static_cast<size_t>(pp) * 2 * kHmTabW;
            hah[gi] = load_taps16(thr, o0);
            hal[gi] = load_taps16(thr + kHmTabW, o0);
        }
    }
    if (tid < XW) {
        int sp, ph;
        sep_position(a.th, a.ox0 + min(x0 + tid, x_last), &sp, &ph);
        ps[tid] = sp;
        pph[tid] = ph;
        pbias[tid] = 128 * a.tsum[ph] + 2048;
    } else if (tid < XW + kRmRows) {
        const int k = tid - XW;
        int sv, ph;
        sep_position(a.tv, a.oy0 + y0 + min(k, nr - 1), &sv, &ph);
        vso[k] = sv - r_lo;
        vph[k] = ph;
        vbias[k] = 128 * a.tsumv[ph] + 2048;
    }
    __syncthreads();
    // ---- tail fix-up: blocks that stage the image's last row with a row end off the dword grid ----
    if ((a.w * B) % 4 != 0 && r_lo + L > a.h - 1) {  // uniform
        const int pitch = a.w * B;
        const int chunks = (B * nqv + 63) >> 6;
        for (int l = wave; l < L; l += 4) {
            if (clampi(r_lo + l, 0, a.h - 1) != a.h - 1) continue;
            for (int c = 0; c < chunks; ++c) {
                const int over = (a.h - 1) * pitch + B * org + 4 * (c * 64 + lane) + 4 - static_cast<int>(a.in_img);
                if (c * 64 + lane < RS && over > 0 && over < 4) {
                    uint32_t *q = raw + l * RS + c * 64 + lane;
                    *q = *q >> (8 * over);
                }
            }
        }
        __syncthreads();
    }
    // ---- vertical pass on the matrix cores, 16-byte column tiles dealt to the waves ----
    {
        const int n = lane & 15, kg = lane >> 4;
        hm_v4i bh = hbh, bl = hbl;
        if constexpr (HT == 0) {
            const signed char *tv = a.tabv + static_cast<size_t>(vph[n]) * 2 * kHmTabW;
            const int ov = 16 * kg - vso[n] + kHmTabPad;
            bh = load_taps16(tv, ov);
            bl = load_taps16(tv + kHmTabW, ov);
        }
        const int vb = vbias[n];
        const int nt = (B * (hi - org + 1) + 15) >> 4;
        const u8 *rawb = reinterpret_cast<const u8 *>(raw);
        const int r1 = min(16 * kg + (n >> 1), L - 1), r2 = min(16 * kg + 8 + (n >> 1), L - 1);
        uint32_t res[kRmMaxCt];  // this wave's tiles, written after every wave has read the staged rows
        typedef int v2i_t __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int i = 0; i < kRmMaxCt; ++i) {
            const int ct = wave + 4 * i;
            if (ct >= nt) continue;  // uniform; no break: results of skipped tiles stay undefined, no copies
            const int cb = 16 * ct + 8 * (n & 1);  // the tile's 16 staged rows of this lane's byte column
            const v2i_t t1 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
                (__attribute__((address_space(3))) v2i_t *)(to_lds(const_cast<u8 *>(rawb + r1 * RS * 4 + cb))));
            const v2i_t t2 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
                (__attribute__((address_space(3))) v2i_t *)(to_lds(const_cast<u8 *>(rawb + r2 * RS * 4 + cb))));
            const hm_v4i av = hm_v4i{t1.x ^ static_cast<int>(0x80808080u), t1.y ^ static_cast<int>(0x80808080u),
                                     t2.x ^ static_cast<int>(0x80808080u), t2.y ^ static_cast<int>(0x80808080u)};
            hm_v4i dh = hm_v4i{0, 0, 0, 0}, dl = hm_v4i{vb, vb, vb, vb};
            dh = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bh, dh, 0, 0, 0);
            dl = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bl, dl, 0, 0, 0);
            const uint32_t w = round_pack4((dh[0] << 6) + dl[0], (dh[1] << 6) + dl[1], (dh[2] << 6) + dl[2],
                                           (dh[3] << 6) + dl[3]);
            res[i] = w ^ 0x80808080u;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kRmMaxCt; ++i) {
            const int ct = wave + 4 * i;
            if (ct >= nt) continue;
            *reinterpret_cast<uint32_t *>(inter + n * a.iw + 16 * ct + 4 * kg) = res[i];
        }
    }
    __syncthreads();
    // ---- row-major intermediate -> channel planes, 4 pixels per item ----
    for (int k = wave; k < nr; k += 4) {
        const uint32_t *ir = reinterpret_cast<const uint32_t *>(inter + k * a.iw);
        u8 *pl = planes + k * a.row_w;
        for (int q = lane; q < nqv; q += 64) {
            uint32_t xw[4], pw[4];
#pragma unroll
            for (int d = 0; d < B; ++d) xw[d] = ir[B * q + d];
            if (B == 3) {
                pw[0] = __builtin_amdgcn_perm(xw[2], __builtin_amdgcn_perm(xw[1], xw[0], 0x0c060300u), 0x05020100u);
                pw[1] = __builtin_amdgcn_perm(xw[2], __builtin_amdgcn_perm(xw[1], xw[0], 0x0c070401u), 0x06020100u);
                pw[2] = __builtin_amdgcn_perm(xw[2], __builtin_amdgcn_perm(xw[1], xw[0], 0x0c0c0502u), 0x07040100u);
            } else {
                transpose4x4(xw[0], xw[1], xw[2], xw[3], pw);
            }
#pragma unroll
            for (int z = 0; z < B; ++z) reinterpret_cast<uint32_t *>(pl + z * a.plane_w)[q] = pw[z];
        }
    }
    __syncthreads();
    // ---- COPY edge of the horizontal pass: pixels outside the image repeat its edge ----
    if (lo < 0 || hi >= a.w) {
        for (int i = tid; i < nr * (hi - org + 1); i += 256) {
            const int k = i / (hi - org + 1), pq = i - k * (hi - org + 1);
            const int p = org + pq;
            if (p >= 0 && p < a.w) continue;
            const int src = clampi(p, 0, a.w - 1) - org;
#pragma unroll
            for (int z = 0; z < B; ++z) planes[k * a.row_w + z * a.plane_w + pq] = planes[k * a.row_w + z * a.plane_w + src];
        }
        __syncthreads();
    }
    // ---- horizontal pass on the matrix cores (k_hmfma's group loop) ----
    const int n = lane & 15, kg = lane >> 4;
    u8 *ob = a.out + img * a.out_img;
    u8 *tile = inter;  // output tile [kRmRows][XW * 3 + 4] over the intermediate (dead after the deinterleave)
    const __amdgpu_buffer_rsrc_t os = __builtin_amdgcn_make_buffer_rsrc(ob, 0, static_cast<int>(a.out_img), 0x00020000);
    __syncthreads();
#pragma unroll
    for (int gi = 0; gi < GPW; ++gi) {
        const int g = wave * GPW + gi;
        if (x0 + 16 * g > x_last) break;
        const int qb = (__builtin_amdgcn_readfirstlane(ps[16 * g]) - org) & ~15;  // plane offset of the group's window
        const int p = min(16 * g + n, x_last - x0);
        const int o0 = qb + 16 * kg - (ps[p] - org) + kHmTabPad;
        const signed char *thr = a.tab + static_cast<size_t>(pph[p]) * 2 * kHmTabW;
        const int4 bias = *reinterpret_cast<const int4 *>(pbias + 16 * g + 4 * kg);
        hm_v4i acc_h[B], acc_l[B];
#pragma unroll
        for (int z = 0; z < B; ++z) {
            acc_h[z] = hm_v4i{0, 0, 0, 0};
            acc_l[z] = hm_v4i{bias.x, bias.y, bias.z, bias.w};
        }
        for (int ks = 0; ks < a.nks; ++ks) {
            hm_v4i ah, al;
            if (HT != 0 && ks == 0) {
                ah = hah[gi];
                al = hal[gi];
            } else {
                ah = load_taps16(thr, o0 + 64 * ks);
                al = load_taps16(thr + kHmTabW, o0 + 64 * ks);
            }
#pragma unroll
            for (int z = 0; z < B; ++z) {
                const hm_v4i bz =
                    *reinterpret_cast<const hm_v4i *>(planes + n * a.row_w + z * a.plane_w + qb + 64 * ks + 16 * kg);
                acc_h[z] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, bz, acc_h[z], 0, 0, 0);
                acc_l[z] = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, bz, acc_l[z], 0, 0, 0);
            }
        }
        uint32_t wz[4];
#pragma unroll
        for (int z = 0; z < B; ++z)
            wz[z] = round_pack4((acc_h[z][0] << 6) + acc_l[z][0], (acc_h[z][1] << 6) + acc_l[z][1],
                                (acc_h[z][2] << 6) + acc_l[z][2], (acc_h[z][3] << 6) + acc_l[z][3]);
        const int x = x0 + 16 * g + 4 * kg;
        if (n >= nr || x > x_last) continue;
        uint32_t wo[4];  // the 4 pixels interleaved: B dwords
        if (B == 3) {
            wo[0] = __builtin_amdgcn_perm(wz[2], __builtin_amdgcn_perm(wz[1], wz[0], 0x010c0400u), 0x03040100u);
            wo[1] = __builtin_amdgcn_perm(wz[2], __builtin_amdgcn_perm(wz[1], wz[0], 0x06020c05u), 0x03020500u);
            wo[2] = __builtin_amdgcn_perm(wz[2], __builtin_amdgcn_perm(wz[1], wz[0], 0x0c07030cu), 0x07020106u);
        } else {
            transpose4x4(wz[0], wz[1], wz[2], wz[3], wo);
        }
        if (a.direct && x + 3 <= x_last) {  // dword-aligned output rows: the lane's 4 pixels in one store
            const int qo = ((y0 + n) * a.ow + x) * B;
            if (B == 3) {
                typedef int v3i_t __attribute__((ext_vector_type(3)));
                __builtin_amdgcn_raw_buffer_store_b96(
                    v3i_t{static_cast<int>(wo[0]), static_cast<int>(wo[1]), static_cast<int>(wo[2])}, os, qo, 0, 0);
            } else {
                __builtin_amdgcn_raw_buffer_store_b128(hm_v4i{static_cast<int>(wo[0]), static_cast<int>(wo[1]),
                                                              static_cast<int>(wo[2]), static_cast<int>(wo[3])},
                                                       os, qo, 0, 0);
            }
            continue;
        }
        uint32_t *tq = reinterpret_cast<uint32_t *>(tile + n * (XW * B + 4) + (x - x0) * B);
#pragma unroll
        for (int d = 0; d < B; ++d) tq[d] = wo[d];
    }
    __syncthreads();
    // ---- each tile row to its output row as whole dwords at the row's own alignment ----
    // (direct mode: only the partial last group of the row's last block went through the tile)
    const int nb = (x_last - x0 + 1) * B;
    const int tb = a.direct ? ((x_last - x0 + 1) & ~3) * B : 0;  // tile bytes already stored
    for (int r = wave; r < nr && tb < nb; r += 4) {
        const u8 *tr = tile + r * (XW * B + 4);
        const uint32_t *tw = reinterpret_cast<const uint32_t *>(tr);
        const int qo0 = ((y0 + r) * a.ow + x0) * B + static_cast<int>(reinterpret_cast<uintptr_t>(ob) & 3u);
        const int d0 = qo0 >> 2, nd = ((qo0 + nb + 3) >> 2) - d0;
        const int sh = (4 - (qo0 & 3)) & 3;
        const int bias0 = static_cast<int>(reinterpret_cast<uintptr_t>(ob) & 3u);
        for (int i = lane; i < nd; i += 64) {
            const int e = 4 * (d0 + i) - qo0;
            if (e + 4 <= tb) continue;
            if (e >= tb && e + 4 <= nb) {
                const uint32_t w = sh ? __builtin_amdgcn_alignbyte(tw[(e >> 2) + 1], tw[e >> 2], e & 3) : tw[e >> 2];
                __builtin_amdgcn_raw_buffer_store_b32(w, os, 4 * (d0 + i) - bias0, 0, 0);
            } else {
                for (int k = 0; k < 4; ++k)
                    if (e + k >= tb && e + k < nb)
                        __builtin_amdgcn_raw_buffer_store_b8(tr[e + k], os, 4 * (d0 + i) + k - bias0, 0, 0);
            }
        }
    }
}

template <int B>
__global__ void __launch_bounds__(256) k_hpass_gather(HPassArgs a) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int img = blockIdx.z;
    if (x >= a.ow) return;
    int s, ph;
    sep_position(a.tp, a.ox0 + x, &s, &ph);
    const float *c = a.tp.tab + ph * a.tp.taps;
    const u8 *row = a.in + img * a.in_img + a.in_base + static_cast<long long>(y) * a.in_pitch;
    float acc[B];
#pragma unroll
    for (int z = 0; z < B; ++z) acc[z] = 0.f;
    for (int i = 0; i < a.tp.taps; ++i) {
        const u8 *p = row + clampi(s + i, 0, a.wl - 1) * B;
        const float ci = c[i];
#pragma unroll
        for (int z = 0; z < B; ++z) acc[z] = __builtin_fmaf(ci, static_cast<float>(p[z]), acc[z]);
    }
    u8 *q = a.out + img * a.out_img + (static_cast<long long>(y) * a.ow + x) * B;
#pragma unroll
    for (int z = 0; z < B; ++z) q[z] = static_cast<u8>(fixed_round_u(acc[z]));
}

// ===========================================================================
// fused reduce: reducev -> reduceh for any shrink pair in one launch, the
// rounded uchar intermediate kept in LDS (libvips materialises it; every value
// is the same, it just never reaches HBM).
//
// A block = kFW output columns x th output rows of one image.  The input rows
// [r_lo, r_lo + L) x columns [cl, ch] it needs are DMA'd to LDS (raw bytes from
// each row's dword-aligned-down start, any alignment); the vertical pass turns
// them into th intermediate rows (dword lanes, channel agnostic, byte skew
// fixed with v_alignbyte); the rows are repacked to one u32 per pixel; the
// horizontal pass (taps <= 16 per lane in registers) writes the outputs.
// ===========================================================================
constexpr int kFW = 64;          // output columns per block
constexpr int kFMaxTaps = 16;

struct FusedArgs {
    const u8 *in;
    u8 *out;
    int w, h, in_pitch;
    long long in_img, out_img;
    int ox0, oy0, ow, oh;        // output window (op-output coordinates) and its size
    int th;                      // output rows per block
    int x_blocks, y_blocks;
    int raw_stride;              // LDS dwords per staged input row
    int lrows;                   // staged input rows capacity
    int span_max;                // intermediate pixels per row capacity
    SepTaps tv, thz;             // vertical / horizontal taps
};

template <int B>
__global__ void __launch_bounds__(256) k_reduce_fused(FusedArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t fsm[];
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int xb = t % a.x_blocks;
    const int rest = t / a.x_blocks;
    const int yb = rest % a.y_blocks;
    const int img = rest / a.y_blocks;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tv = a.tv.taps, thz = a.thz.taps;
    // ---- geometry of this tile ----
    const int x0 = xb * kFW, y0 = yb * a.th;
    const int nx = min(kFW, a.ow - x0), ny = min(a.th, a.oh - y0);
    int lo, hi, r_lo, r_last, ph;
    sep_position(a.thz, a.ox0 + x0, &lo, &ph);
    sep_position(a.thz, a.ox0 + x0 + nx - 1, &hi, &ph);
    hi += thz - 1;
    sep_position(a.tv, a.oy0 + y0, &r_lo, &ph);
    sep_position(a.tv, a.oy0 + y0 + ny - 1, &r_last, &ph);
    const int L = r_last + tv - r_lo;
    const int cl = max(lo, 0), ch = min(hi, a.w - 1);   // intermediate columns actually computed
    const int ncol = ch - cl + 1;
    const int nd = (B * ncol + 3) >> 2;                 // intermediate dwords per row
    uint32_t *raw = fsm;                                 // lrows x raw_stride
    uint32_t *mid = raw + a.lrows * a.raw_stride;        // th x span_max (u32 per pixel)
    float *vco = reinterpret_cast<float *>(mid + a.th * a.span_max);  // th x tv
    int *vso = reinterpret_cast<int *>(vco + a.th * tv);               // th row starts
    // ---- DMA the input rows ----
    int delta = 0;
    const u8 *src = a.in + img * a.in_img;
    const __amdgpu_buffer_rsrc_t rs = image_rsrc_aligned(src, a.in_img, &delta);
    const int ndl = (B * ncol + 3 + 3) >> 2;            // dwords to cover any skew
    const int chunks = (ndl + 63) >> 6;
    for (int idx = wave; idx < L * chunks; idx += 4) {
        const int l = idx / chunks, q = idx - l * chunks;
        const int r = clampi(r_lo + l, 0, a.h - 1);
        const int a4 = static_cast<int>(delta + static_cast<long long>(r) * a.in_pitch + B * cl) & ~3;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, to_lds(raw + l * a.raw_stride + q * 64), 4,
                                                 4 * (q * 64 + lane), a4, 0, 0);
    }
    for (int i = tid; i < ny * tv; i += 256) {
        const int k = i / tv;
        int s2;
        sep_position(a.tv, a.oy0 + y0 + k, &s2, &ph);
        vco[i] = a.tv.tab[ph * tv + (i - k * tv)];
    }
    if (tid < ny) {
        int s2;
        sep_position(a.tv, a.oy0 + y0 + tid, &s2, &ph);
        vso[tid] = s2 - r_lo;
    }
    // this lane's horizontal taps (lane -> output column x0 + (tid & 63))
    const int xi = tid & 63, rgrp = tid >> 6;
    int xs = 0, xph = 0;
    sep_position(a.thz, a.ox0 + x0 + min(xi, nx - 1), &xs, &xph);
    float cr[kFMaxTaps];
    {
        const float *c = a.thz.tab + xph * thz;
#pragma unroll
        for (int i = 0; i < kFMaxTaps; ++i) cr[i] = i < thz ? c[i] : 0.f;
    }
    __syncthreads();
    // ---- vertical pass: ny intermediate rows x nd dwords ----
    u8 *mid8 = reinterpret_cast<u8 *>(mid);
    for (int it = tid; it < ny * nd; it += 256) {
        const int k = it / nd, d = it - k * nd;
        const int s0 = vso[k];
        const float *ck = vco + k * tv;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        for (int i = 0; i < tv; ++i) {
            const int l = s0 + i;
            const int r = clampi(r_lo + l, 0, a.h - 1);
            const int sh = static_cast<int>(delta + static_cast<long long>(r) * a.in_pitch + B * cl) & 3;
            const uint32_t *rp = raw + l * a.raw_stride + d;
            const uint32_t v = __builtin_amdgcn_alignbyte(rp[1], rp[0], sh);
            const float c = ck[i];
            a0 = __builtin_fmaf(c, ubyte_f<0>(v), a0);
            a1 = __builtin_fmaf(c, ubyte_f<1>(v), a1);
            a2 = __builtin_fmaf(c, ubyte_f<2>(v), a2);
            a3 = __builtin_fmaf(c, ubyte_f<3>(v), a3);
        }
        const uint32_t o = fixed_round_u(a0) | (fixed_round_u(a1) << 8) | (fixed_round_u(a2) << 16) |
                           (fixed_round_u(a3) << 24);
        if (B == 4) {
            mid[k * a.span_max + (cl - lo) + d] = o;  // one pixel per dword already
        } else {  // scatter the 4 bytes to their pixel slots (u32 per pixel)
#pragma unroll
            for (int z = 0; z < 4; ++z) {
                const int byte = 4 * d + z;
                if (byte < B * ncol) {
                    const int px = byte / B, c = byte - px * B;
                    mid8[(k * a.span_max + (cl - lo) + px) * 4 + c] = static_cast<u8>(o >> (8 * z));
                }
            }
        }
    }
    __syncthreads();
    // COPY edge of the intermediate rows: slots outside [cl, ch]
    {
        const int nl = cl - lo, nr = hi - ch;
        for (int i = tid; i < ny * (nl + nr); i += 256) {
            const int k = i / (nl + nr), f = i - k * (nl + nr);
            uint32_t *row = mid + k * a.span_max;
            if (f < nl) row[f] = row[nl];
            else row[ch - lo + 1 + (f - nl)] = row[ch - lo];
        }
    }
    __syncthreads();
    // ---- horizontal pass: lane = column xi, rows rgrp, rgrp + 4, ... ----
    if (xi >= nx) return;
    const uint32_t *sp = mid + (xs - lo);
    for (int k = rgrp; k < ny; k += 4) {
        const uint32_t *rowp = sp + k * a.span_max;
        float acc[B];
#pragma unroll
        for (int z = 0; z < B; ++z) acc[z] = 0.f;
#pragma unroll
        for (int i = 0; i < kFMaxTaps; ++i) {
            if (i < thz) {
                const uint32_t v = rowp[i];
#pragma unroll
                for (int z = 0; z < B; ++z) {
                    const float pz = z == 0 ? ubyte_f<0>(v) : z == 1 ? ubyte_f<1>(v) : z == 2 ? ubyte_f<2>(v) : ubyte_f<3>(v);
                    acc[z] = __builtin_fmaf(cr[i], pz, acc[z]);
                }
            }
        }
        u8 *q = a.out + img * a.out_img + (static_cast<long long>(y0 + k) * a.ow + x0 + xi) * B;
        if (B == 4 && (reinterpret_cast<uintptr_t>(q) & 3u) == 0) {
            uint32_t o = 0;
#pragma unroll
            for (int z = 0; z < B; ++z) o |= fixed_round_u(acc[z]) << (8 * z);
            *reinterpret_cast<uint32_t *>(q) = o;
        } else {
#pragma unroll
            for (int z = 0; z < B; ++z) q[z] = static_cast<u8>(fixed_round_u(acc[z]));
        }
    }
}

bool aligned4(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 3u) == 0; }

SepTaps make_taps(const SepSpec &s) {
    SepTaps t{};
    t.tab = s.tab;
    t.taps = s.taps;
    t.phased = s.mode == kSepReduce;
    t.pad = t.phased ? s.taps / 2 - 1 : s.taps / 2;
    t.shrink = s.shrink;
    t.rounding = static_cast<float>((s.scale + 1) / 2);
    t.inv_scale = s.scale > 0 ? 1.0f / s.scale : 1.0f;
    const char *e = tune_env("MIPX_SEP_DOT");
    t.dot = !(e && *e == '0');
    const char *eq = tune_env("MIPX_SEP_TQ");
    t.tq = !(eq && *eq == '0') && s.taps >= 7;
    t.centre = t.phased && reduce_centre();  // 3-tap masks lose to the transpose (v14/ab_conv_quad_transpose.log)
    return t;
}

}  // namespace

bool sep_spec_reduce(double shrink, SepSpec *s) {
    int taps = 0;
    s->tab = device_reduce_table(shrink, &taps);
    if (!s->tab) return false;
    s->taps = taps;
    s->mode = kSepReduce;
    s->shrink = shrink;
    s->scale = 0;
    return true;
}

int vpass_launch(const u8 *in, u8 *out, int n, const SepSpec &spec, const SepWindow &w, hipStream_t st) {
    VPassArgs a{};
    a.in = in;
    a.out = out;
    a.row_bytes = w.out_w * w.bands;
    a.in_pitch = w.in_pitch;
    a.in_base = w.in_base;
    a.in_img = w.in_img;
    a.out_img = static_cast<long long>(a.row_bytes) * w.out_h;
    a.hl = w.in_len;
    a.oy0 = w.o0;
    a.oh = w.out_h;
    a.tp = make_taps(spec);
    const int taps = a.tp.taps;
    const double s = spec.mode == kSepReduce ? spec.shrink : 1.0;
    if (a.in_img >= 0x7fffffffLL) return MIPX_EUNSUPPORTED;
    a.col_blocks = (a.row_bytes + 1023) / 1024;
    // staged input rows per block (1 KiB each); MIPX_VP_ROWS overrides for A/B runs
    const char *erb = tune_env("MIPX_VP_ROWS");
    // 24 rows measured best at 9-17 taps (v12_vpass_ab.log, v14/ab_vpass_rows_blur.log); taller
    // masks need room for several output rows per block (25 taps: 40 rows 2.6 vs 1.7 TB/s,
    // v14/ab_vpass_budget.log)
    const int kRowBudget = (erb && *erb) ? std::max(8, std::atoi(erb)) : std::max(24, taps + 15);
    constexpr int kRowMax = 60;
    int kr = taps >= kRowBudget ? 1 : static_cast<int>(std::floor((kRowBudget - taps - 1) / s)) + 1;
    kr = std::max(1, std::min({kr, 32, a.oh}));
    auto rows_for = [&](int k) {  // conv: taps read in 4s
        return static_cast<int>(std::ceil((k - 1) * s)) + taps + 2 + (spec.mode == kSepConv ? 2 : 0);
    };
    while (kr > 1 && rows_for(kr) > kRowMax) --kr;  // stay on the staged path when one row fits
    a.kr = kr;
    a.lrows = rows_for(kr);
    a.kr_blocks = (a.oh + kr - 1) / kr;
    const dim3 blk(256);
    const size_t lds = static_cast<size_t>(a.lrows) * kVStride * 4 + static_cast<size_t>(kr) * taps * 4 + kr * 4 +
                       static_cast<size_t>(std::max({(taps + 3) / 4 + 4 * ((taps + 6) / 4), kr * std::max((taps + 1) / 2, kVpPairs)}) + 4) * 4;
    if (a.lrows > kRowMax || lds > 64 * 1024) {  // very tall masks: gather through L1
        const dim3 grid((a.row_bytes + 1023) / 1024, a.oh, n);
        if (spec.mode == kSepReduce) hipLaunchKernelGGL(k_vpass_gather<kSepReduce>, grid, blk, 0, st, a);
        else hipLaunchKernelGGL(k_vpass_gather<kSepConv>, grid, blk, 0, st, a);
        return launch_check("k_vpass_gather");
    }
    const long long blocks = static_cast<long long>(a.col_blocks) * a.kr_blocks * n;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    const uintptr_t ip = reinterpret_cast<uintptr_t>(in);
    bool al16 = (ip % 16) == 0 && (a.in_pitch % 16) == 0 && (a.in_base % 16) == 0 && (a.in_img % 16) == 0;
    bool al4 = (ip % 4) == 0 && (a.in_pitch % 4) == 0 && (a.in_base % 4) == 0 && (a.in_img % 4) == 0;
    const char *edm = tune_env("MIPX_VP_DMA");  // A/B: cap the DMA width (16 / 4 / 0)
    if (edm && *edm) {
        const int cap = std::atoi(edm);
        al16 = al16 && cap >= 16;
        al4 = al4 && cap >= 4;
    }
    const char *evf = tune_env("MIPX_VP_FAST");  // A/B: 0 keeps k_vpass's generic reduce loop
    const int tp2 = (taps + 1) / 2;
    const bool vfast = spec.mode == kSepReduce && a.tp.dot && !(evf && *evf == '0') &&
                       tp2 <= kVpPairs && a.row_bytes % 4 == 0 && a.out_img % 4 == 0 &&
                       reinterpret_cast<uintptr_t>(out) % 4 == 0 && a.out_img < 0x7fffffffLL;
    const dim3 grid(static_cast<unsigned>(blocks));
    if (vfast && al4) {
        const size_t lv = static_cast<size_t>(a.lrows) * kVStride * 4 + static_cast<size_t>(kr) * (kVpPairs + 1) * 4;
#define MIPX_VR(T_)                                                                                     \
    case T_:                                                                                            \
        if (al16) hipLaunchKernelGGL((k_vreduce<T_, 16>), grid, blk, lv, st, a);                        \
        else hipLaunchKernelGGL((k_vreduce<T_, 4>), grid, blk, lv, st, a);                              \
        break;
        switch (tp2) {
            MIPX_VR(2) MIPX_VR(3) MIPX_VR(4) MIPX_VR(5) MIPX_VR(6) MIPX_VR(7) MIPX_VR(8)
            default: return MIPX_EUNSUPPORTED;
        }
#undef MIPX_VR
        return launch_check("k_vreduce");
    }
#define MIPX_VP(MODE)                                                                                   \
    if (al16) hipLaunchKernelGGL((k_vpass<MODE, 16>), grid, blk, lds, st, a);                           \
    else if (al4) hipLaunchKernelGGL((k_vpass<MODE, 4>), grid, blk, lds, st, a);                        \
    else hipLaunchKernelGGL((k_vpass<MODE, 0>), grid, blk, lds, st, a);
    if (spec.mode == kSepReduce) {
        MIPX_VP(kSepReduce)
    } else {
        MIPX_VP(kSepConv)
    }
#undef MIPX_VP
    return launch_check("k_vpass");
}

int hpass_launch(const u8 *in, u8 *out, int n, const SepSpec &spec, const SepWindow &w, hipStream_t st) {
    const int b = w.bands;
    HPassArgs a{};
    a.in = in;
    a.out = out;
    a.in_pitch = w.in_pitch;
    a.in_base = w.in_base;
    a.in_img = w.in_img;
    a.out_img = static_cast<long long>(w.out_w) * w.out_h * b;
    a.wl = w.in_len;
    a.rows = w.out_h;
    a.ox0 = w.o0;
    a.ow = w.out_w;
    a.tp = make_taps(spec);
    a.x_blocks = (a.ow + 255) / 256;
    constexpr int kTReg = 16;
    const bool treg = a.tp.phased && a.tp.taps <= kTReg;
    a.ntab = treg ? 0 : (((a.tp.phased ? kTransformScale + 1 : 1) * a.tp.taps + 3) & ~3);
    if (spec.mode != kSepReduce) a.ntab += 4 * ((a.tp.taps + 6) / 4);  // conv: packed phase-shifted tap sets
    const double s = a.tp.phased ? spec.shrink : 1.0;
    a.span_max = (static_cast<int>(std::ceil(255 * s)) + a.tp.taps + 2 + 64 + 3) & ~3;  // 16-byte rows
    const char *erp = tune_env("MIPX_HP_REPACK");
    a.repack4 = !(erp && *erp == '0');
    const char *ep3 = tune_env("MIPX_HP_PACK3");
    // A/B (profiles/r01/v18/pack3_ab.jsonl): packed stores win 7% on reduceh / 2.4 and
    // lose 3% on / 1.6 and on the two-pass blur, so they are on for shrinks >= 2 only
    a.pack3 = ep3 && *ep3 ? *ep3 != '0' : (spec.mode == kSepReduce && spec.shrink >= 2.0);
    a.raw_max = (a.span_max * b + 8 + 3) / 4 + 64;
    if (a.in_img >= 0x7fffffffLL) return MIPX_EUNSUPPORTED;
    const bool dw = b == 4 && (a.in_pitch % 4) == 0 && (a.in_base % 4) == 0 && (a.in_img % 4) == 0 && aligned4(in);
    const char *ehd = tune_env("MIPX_HP_DMA");  // A/B: cap the DMA width (16 / 4)
    const bool dw16 = dw && (a.in_pitch % 16) == 0 && (a.in_base % 16) == 0 && (a.in_img % 16) == 0 &&
                      (reinterpret_cast<uintptr_t>(in) % 16) == 0 && !(ehd && *ehd && std::atoi(ehd) < 16);
    if (dw16) {  // rows staged in whole 256-pixel dwordx4 waves from a 4-pixel-aligned origin
        const int span_px = static_cast<int>(std::ceil(255 * s)) + a.tp.taps + 2;
        const int per_row = ((span_px + 3 + 3) / 4 + 63) / 64;
        a.span_max = ((a.tp.taps + 4 + per_row * 256 + 4) + 3) & ~3;
    }
    if (b == 4 && !aligned4(out)) return MIPX_EINVAL;
    auto lds_for = [&](int rb) {
        return (static_cast<size_t>(a.ntab) + static_cast<size_t>(rb) * a.span_max +
                (!dw ? static_cast<size_t>(rb) * a.raw_max : 0)) * 4;
    };
    const int dwv = dw16 ? 16 : dw ? 4 : 0;
    constexpr size_t kLdsBudget = 40 * 1024;
    int rb = 8;
    while (rb > 1 && lds_for(rb) > kLdsBudget) rb >>= 1;
    if (lds_for(rb) > 64 * 1024) {
        if (spec.mode != kSepReduce) return MIPX_EUNSUPPORTED;
        dim3 grid(a.x_blocks, a.rows, n);
        MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL(k_hpass_gather<B_>, grid, dim3(256), 0, st, a));
        return launch_check("k_hpass_gather");
    }
    a.rb_blocks = (a.rows + rb - 1) / rb;
    const long long blocks = static_cast<long long>(a.x_blocks) * a.rb_blocks * n;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    const size_t lds = lds_for(rb);
    const dim3 grid(static_cast<unsigned>(blocks)), blk(256);
    const char *ehf = tune_env("MIPX_HP_FAST");  // A/B: 0 keeps k_hpass's reduce path
    const int tp2 = (a.tp.taps + 1) / 2;
    if (spec.mode == kSepReduce && treg && a.tp.dot && (b == 3 || b == 4) && tp2 <= kVpPairs &&
        !(ehf && *ehf == '0') && a.out_img < 0x7fffffffLL) {
        int nt = 0;
        a.pairs = device_reduce_pairs(spec.shrink, &nt, &a.tpa);
        if (!a.pairs || nt != a.tp.taps) return MIPX_EDEVICE;
        a.rbn = rb;
#define MIPX_HR(B_, DW_, T_) hipLaunchKernelGGL((k_hreduce<B_, DW_, T_>), grid, blk, lds, st, a)
#define MIPX_HRT(B_, DW_)                                                                                 \
    switch (tp2) {                                                                                      \
        case 2: MIPX_HR(B_, DW_, 2); break;                                                             \
        case 3: MIPX_HR(B_, DW_, 3); break;                                                             \
        case 4: MIPX_HR(B_, DW_, 4); break;                                                             \
        case 5: MIPX_HR(B_, DW_, 5); break;                                                             \
        case 6: MIPX_HR(B_, DW_, 6); break;                                                             \
        case 7: MIPX_HR(B_, DW_, 7); break;                                                             \
        default: MIPX_HR(B_, DW_, 8); break;                                                            \
    }
        if (b == 3) { MIPX_HRT(3, 0) }
        else if (dwv == 16) { MIPX_HRT(4, 16) }
        else if (dwv == 4) { MIPX_HRT(4, 4) }
        else { MIPX_HRT(4, 0) }
#undef MIPX_HRT
#undef MIPX_HR
        return launch_check("k_hreduce");
    }
#define MIPX_HP3(RB_, MODE_, DW_, TR_) \
    MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_hpass<B_, RB_, MODE_, DW_, TR_>), grid, blk, lds, st, a))
#define MIPX_HPW(RB_, MODE_, TR_)                                       \
    if (dwv == 16) { MIPX_HP3(RB_, MODE_, 16, TR_) }                    \
    else if (dwv == 4) { MIPX_HP3(RB_, MODE_, 4, TR_) }                 \
    else { MIPX_HP3(RB_, MODE_, 0, TR_) }
#define MIPX_HP2(RB_)                                                   \
    if (spec.mode == kSepReduce) {                                      \
        if (treg) { MIPX_HPW(RB_, kSepReduce, kTReg) }                  \
        else { MIPX_HPW(RB_, kSepReduce, 0) }                           \
    } else {                                                            \
        MIPX_HPW(RB_, kSepConv, 0)                                      \
    }
    switch (rb) {
        case 8: MIPX_HP2(8) break;
        case 4: MIPX_HP2(4) break;
        case 2: MIPX_HP2(2) break;
        default: MIPX_HP2(1) break;
    }
#undef MIPX_HP2
#undef MIPX_HPW
#undef MIPX_HP3
    return launch_check("k_hpass");
}

// k_rmf2: 3- / 4-band images with rows of any alignment, <= 16 taps each way;
// MIPX_EUNSUPPORTED otherwise (the caller runs another path).  MIPX_RMFMA=0 turns it
// off (A/B); MIPX_RMF2_XW=64/128 forces the column width, MIPX_RMF2_HT=0/1 the tap
// hoisting; MIPX_RMF2_UNALIGNED=0 keeps unaligned rows off it (as when the device
// fails the unaligned direct-to-LDS probe, lds_dma_unaligned_ok()).
int reduce_mfma_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double hs, double vs, int ox0, int oy0,
                       int ow, int oh, hipStream_t st) {
    const char *e = tune_env("MIPX_RMFMA");
    if (e && *e == '0') return MIPX_EUNSUPPORTED;
    const long long in_img = img_bytes(w, h, b), out_img = img_bytes(ow, oh, b);
    if ((b != 3 && b != 4) || !(hs > 1.0) || !(vs > 1.0) || in_img >= 0x7fffffffLL || out_img >= 0x7fffffffLL)
        return MIPX_EUNSUPPORTED;
    // rows of any alignment: a direct-to-LDS dword load honours a byte offset that is
    // not a multiple of 4 (scripts/probe/lds_dma_unaligned.hip, profiles/r02/
    // lds_dma_unaligned.jsonl); the device is probed once (lds_dma_unaligned_ok) and
    // unaligned rows stay off k_rmf2 if it fails
    const bool rows_aligned = (w * b) % 4 == 0 && reinterpret_cast<uintptr_t>(in) % 4 == 0;
    const char *eu = tune_env("MIPX_RMF2_UNALIGNED");
    if (!rows_aligned && ((eu && *eu == '0') || !lds_dma_unaligned_ok())) return MIPX_EUNSUPPORTED;
    SepSpec sh, sv;
    if (!sep_spec_reduce(hs, &sh) || !sep_spec_reduce(vs, &sv)) return MIPX_EDEVICE;
    if (sh.taps > 16 || sv.taps > 16) return MIPX_EUNSUPPORTED;
    RmArgs a{};
    a.in = in;
    a.out = out;
    a.w = w;
    a.h = h;
    a.ox0 = ox0;
    a.oy0 = oy0;
    a.ow = ow;
    a.oh = oh;
    a.in_img = in_img;
    a.out_img = out_img;
    a.th = make_taps(sh);
    a.tv = make_taps(sv);
    int nt = 0;
    a.tab = device_reduce_i8(hs, &nt, &a.tsum);
    if (!a.tab || nt != sh.taps) return MIPX_EDEVICE;
    a.tabv = device_reduce_i8(vs, &nt, &a.tsumv);
    if (!a.tabv || nt != sv.taps) return MIPX_EDEVICE;
    a.y_blocks = (oh + kRmRows - 1) / kRmRows;
    a.nks = (static_cast<int>(std::ceil(15 * hs)) + sh.taps + 16 + 63) / 64;
    if (a.nks > 4 || static_cast<int>(std::ceil((kRmRows - 1) * vs)) + sv.taps > 64) return MIPX_EUNSUPPORTED;
    a.direct = (ow * b) % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 4 == 0;
    // 128- or 64-pixel columns; staged rows at the narrowest stride whose (dwords mod 64)
    // / 4 is odd, so a transposed read's 8 rows x 2 halves hit 16 distinct bank pairs.
    // The smaller the LDS, the more workgroups share a CU (<= 32 KB: 5).
    const char *xe = tune_env("MIPX_RMF2_XW");
    const int xw_only = xe ? std::atoi(xe) : 0;
    size_t l2 = 0;
    int xw = 0;
    const int lrows2 = static_cast<int>(std::ceil((kRmRows - 1) * vs)) + sv.taps + 1;
    for (const int x : {128, 64}) {
        if (xw_only && x != xw_only) continue;
        const int sp = static_cast<int>(std::ceil((x - 1) * hs)) + sh.taps + 4;  // >= hi - org + 1
        int rsd = (b * (sp / 4 + 1) + 3) & ~3;
        while (((rsd & 63) >> 2) % 2 == 0) rsd += 4;
        const int pw = (sp + 15) & ~15;
        const int rw = b * pw + ((b * pw / 16) % 2 == 0 ? 16 : 0);
        const int iw = ((b * sp + 15) & ~15) + 16;
        const size_t lx = static_cast<size_t>(3 * x + 3 * kRmRows) * 4 +
                          std::max(static_cast<size_t>(lrows2) * rsd * 4, static_cast<size_t>(kRmRows) * (iw + rw) + 64 + 16);
        if (b * sp > 16 * 4 * kRmMaxCt || x * b + 4 > iw) continue;
        if (xw == 0 || (l2 > 32 * 1024 && lx < l2)) {
            xw = x, l2 = lx, a.rsd = rsd, a.plane_w = pw, a.row_w = rw, a.iw = iw;
            a.x_blocks = (ow + x - 1) / x;
        }
    }
    // RGB and RGBA (cfg_rmf2_ab.jsonl: C3 / C4 / C5 +2.7 / +1.7 / +0.2 % over the RGB-only
    // default once the narrow stride took 1024^2 RGBA / 1.333 to 6 workgroups)
    if (xw == 0 || l2 > 40 * 1024) return MIPX_EUNSUPPORTED;
    const long long blocks2 = static_cast<long long>(a.x_blocks) * a.y_blocks * n;
    if (!grid_ok(blocks2)) return MIPX_EINVAL;
    const dim3 grid2(static_cast<unsigned>(blocks2)), blk(256);
    // HT: tap fragments loaded while the staged rows are in flight.  ht_ab.jsonl: RGBA
    // -5 % (1024^2 / 1.333 1.308 -> 1.246 ms, 1080p / 1.6 0.288 -> 0.275), RGB flat (+-2 %,
    // the extra registers cost what the hidden latency saves)
    const char *he = tune_env("MIPX_RMF2_HT");
    const bool ht = (he && *he) ? *he != '0' : b == 4;
#define MIPX_RMF2_GO(HT_)                                                                 \
    if (b == 3) {                                                                         \
        if (xw == 128) hipLaunchKernelGGL((k_rmf2<3, 128, HT_>), grid2, blk, l2, st, a);  \
        else hipLaunchKernelGGL((k_rmf2<3, 64, HT_>), grid2, blk, l2, st, a);             \
    } else {                                                                              \
        if (xw == 128) hipLaunchKernelGGL((k_rmf2<4, 128, HT_>), grid2, blk, l2, st, a);  \
        else hipLaunchKernelGGL((k_rmf2<4, 64, HT_>), grid2, blk, l2, st, a);             \
    }
    if (ht) {
        MIPX_RMF2_GO(1)
    } else {
        MIPX_RMF2_GO(0)
    }
#undef MIPX_RMF2_GO
    return launch_check("k_rmf2");
}

// Fused reducev -> reduceh of the output window [ox0, ox0 + ow) x [oy0, oy0 + oh);
// MIPX_EUNSUPPORTED when the tile would not fit LDS (caller runs two passes).
int reduce_fused_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double hs, double vs, int ox0, int oy0,
                        int ow, int oh, hipStream_t st) {
    // Measured (profiles/r01/v11_fused_ab.log): the fused launch wins on small
    // images (<= ~0.5 MB, the thumbnail / smartcrop / post-shrink shapes) and loses
    // to the two DMA-staged passes on large ones.  MIPX_FUSED_REDUCE=0/1 forces it.
    const char *ef = tune_env("MIPX_FUSED_REDUCE");
    if (ef && *ef) {
        if (ef[0] == '0') return MIPX_EUNSUPPORTED;
    } else if (img_bytes(w, h, b) > 512 * 1024) {
        return MIPX_EUNSUPPORTED;
    }
    SepSpec sh, sv;
    if (!sep_spec_reduce(hs, &sh) || !sep_spec_reduce(vs, &sv)) return MIPX_EDEVICE;
    if (sh.taps > kFMaxTaps || sv.taps > 40) return MIPX_EUNSUPPORTED;
    FusedArgs a{};
    a.in = in;
    a.out = out;
    a.w = w;
    a.h = h;
    a.in_pitch = w * b;
    a.in_img = img_bytes(w, h, b);
    a.out_img = img_bytes(ow, oh, b);
    a.ox0 = ox0;
    a.oy0 = oy0;
    a.ow = ow;
    a.oh = oh;
    a.tv = make_taps(sv);
    a.thz = make_taps(sh);
    if (a.in_img >= 0x7fffffffLL) return MIPX_EUNSUPPORTED;
    a.span_max = static_cast<int>(std::ceil((kFW - 1) * hs)) + sh.taps + 2;
    a.raw_stride = ((a.span_max * b + 3 + 3) / 4 + 63) / 64 * 64 + 1;  // DMA chunks of 64 dwords + alignbyte spill
    constexpr size_t kBudget = 48 * 1024;
    auto lds_for = [&](int th) {
        const int lrows = static_cast<int>(std::ceil((th - 1) * vs)) + sv.taps + 2;
        return (static_cast<size_t>(lrows) * a.raw_stride + static_cast<size_t>(th) * a.span_max) * 4 +
               static_cast<size_t>(th) * (sv.taps + 1) * 4;
    };
    int th = 32;
    while (th > 4 && lds_for(th) > kBudget) th -= 4;
    if (lds_for(th) > 64 * 1024) return MIPX_EUNSUPPORTED;
    th = std::min(th, oh);
    a.th = th;
    a.lrows = static_cast<int>(std::ceil((th - 1) * vs)) + sv.taps + 2;
    a.x_blocks = (ow + kFW - 1) / kFW;
    a.y_blocks = (oh + th - 1) / th;
    const long long blocks = static_cast<long long>(a.x_blocks) * a.y_blocks * n;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    const size_t lds = lds_for(th);
    MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL(k_reduce_fused<B_>, dim3(static_cast<unsigned>(blocks)), dim3(256), lds,
                                              st, a));
    return launch_check("k_reduce_fused");
}

}  // namespace mipx
