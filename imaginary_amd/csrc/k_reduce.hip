// k_reduce.hip — libvips vips_reduce (Lanczos3) on gfx950.
//
// reduce.c runs reducev then reduceh with a uchar intermediate; every tap is a
// 12-bit integer (matrixi, truncated) and each uchar result is
// (sum + 2048) >> 12 clipped (reduceh.cpp / reducev.cpp / templates.h,
// restated in oracle/vips_ref.c).  Sums stay exact in fp32 (< 2^24), so the
// kernels are bit-identical to the integer C path.
//
//  * k_reduce2x2     fused reducev -> reduceh for shrink 2 x 2 (north star C2)
//  * any other shrink: the generic separable passes of k_sep.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "device_common.h"

namespace mipx {
namespace {

using namespace dev;

// ===========================================================================
// Lanczos3 reduce by exactly 2 x 2, fused reducev -> reduceh (the north-star
// kernel: 4K -> 1080p).
//
// At shrink 2 with the corner convention every output samples phase 0, whose
// 13-tap mask has zeros at the odd integer positions of the Lanczos lobe and is
// symmetric, so output o = c0 * p[2o] + c1 * (p[2o-1] + p[2o+1])
//                      + c3 * (p[2o-3] + p[2o+3]) + c5 * (p[2o-5] + p[2o+5]).
// The host verifies that shape on the actual integer table before choosing
// this kernel, so the arithmetic is exactly libvips' 13-tap sum.
//
// One workgroup = a strip of TW output pixels x a band of rows.
//  * Vertical pass: lane t owns dword t of the strip's input bytes (channel
//    agnostic) and walks down the band with the six odd rows of the current
//    window in a static register ring (slot = odd-row index mod 6, unrolled
//    by 12); each input byte is loaded and converted once.  The rounded uchar
//    intermediate (libvips materialises it between reducev and reduceh) is
//    packed back to a dword and written to LDS in input byte order: one
//    conflict-free ds_write_b32 per lane and row.
//  * Horizontal pass: an item is K output pixels of one row; it reads the
//    13-dword byte window it needs (ds_read_b64: lane stride 6 dwords for RGB,
//    conflict-free; ds_read_b128 for RGBA, stride 4 dwords), converts each
//    byte once and stores 12 (RGB) / 8 (RGBA) contiguous output bytes.
// The intermediate never touches HBM, and the LDS image is 7.5 KB per
// workgroup, so occupancy is set by registers, not LDS.
// ===========================================================================
constexpr int kR = 12;           // output rows per LDS chunk (2 ring periods)
// WIDE level (variant bits 6 / 7): 128 << WIDE threads and strips 2x / 4x as
// wide (less relative halo, longer contiguous row segments, fewer workgroups)
// TIGHT (variant bit 8, WIDE 1 only): rows 264 dwords apart (== 8 mod 64) instead of 288,
// 25.3 instead of 27.6 KB of LDS, so 6 workgroups share a CU instead of 5 (r02 A/B)
template <int WIDE, int TIGHT = 0>
struct R2T {
    static constexpr int kThreads = 128 << WIDE;
    static constexpr int kPitch = WIDE == 2 ? 544 : WIDE == 1 ? (TIGHT ? 264 : 288) : 160;  // LDS dwords per row
};

template <int B, int WIDE = 0, int TIGHT = 0>
struct R2 {
    static constexpr int kThreads = R2T<WIDE, TIGHT>::kThreads;
    static constexpr int kPitch = R2T<WIDE, TIGHT>::kPitch;
    static constexpr int TW = B == 3 ? 80 << WIDE : WIDE == 0 ? 56 : 60 << WIDE;  // output pixels per strip
    static constexpr int NPX = 2 * TW + 9;           // intermediate px 2x0-5 .. 2x0+2TW+3
    static constexpr int K = B == 3 ? 4 : 2;         // output pixels per horizontal item
    static constexpr int OFF0 = B == 3 ? 1 : 0;      // B*(2x0-5) - floor4(B*(2x0-5))
    static constexpr int ND = (B * NPX + OFF0 + 3) / 4;  // dwords per row
    static_assert(ND <= kThreads && ND <= kPitch, "strip too wide");
    static_assert(((TW / K) * K) == TW, "items must tile the strip");
    static_assert((B * 2 * K) % 8 == 0, "window start must be 8-byte aligned");
};

struct Reduce2Args {
    const u8 *in;
    u8 *out;
    int w, h, ow, oh;
    int n_strips, n_bands, band_rows;  // band_rows multiple of kR
    // computed output region (demand-driven execution, mipx_runtime.cpp plan_demand):
    // strips from s_base, bands from row y_base (a multiple of kR), clipped at x_end /
    // y_end; the full image is s_base = y_base = 0, x_end = ow, y_end = oh
    int s_base, y_base, x_end, y_end;
    long long in_img, out_img;
    // taps pre-scaled by 1/4096 (exact: powers of two); the bias 2^-13 turns the
    // exact chain into RNE(sum/4096 + 2^-13) == floor(sum/4096 + 0.5) at the cvt
    float c0, c1, c3, c5, bias;
    int remap;       // XCD-aware tile order (MIPX_R2_REMAP=0 disables, for A/B)
    int band_major;  // tile order inside an XCD range (MIPX_R2_ORDER=1: bands fastest)
};

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v cvt4_once(uint32_t v) {
    return f4v{ubyte_once<0>(v), ubyte_once<1>(v), ubyte_once<2>(v), ubyte_once<3>(v)};
}
__device__ __forceinline__ f2v lo2(f4v v) { return __builtin_shufflevector(v, v, 0, 1); }
__device__ __forceinline__ f2v hi2(f4v v) { return __builtin_shufflevector(v, v, 2, 3); }

// c0 e + c1 (m1 + p1) + c3 (m3 + p3) + c5 (m5 + p5) with pre-scaled taps and the
// bias: every partial is exact on a 1/8192 grid below 2^9, so the result is
// exactly sum/4096 + 2^-13
__device__ __forceinline__ float tap7(float c0, float c1, float c3, float c5, float bias, float e, float m1,
                                      float p1, float m3, float p3, float m5, float p5) {
    float acc = __builtin_fmaf(c0, e, bias);
    acc = __builtin_fmaf(c1, m1 + p1, acc);
    acc = __builtin_fmaf(c3, m3 + p3, acc);
    return __builtin_fmaf(c5, m5 + p5, acc);
}
// the same chain on two columns at once (v_pk_fma_f32 / v_pk_add_f32): each lane
// of the pair sees exactly the scalar operation sequence, so results are identical
__device__ __forceinline__ f2v tap7v(f2v c0, f2v c1, f2v c3, f2v c5, f2v bias, f2v e, f2v m1, f2v p1, f2v m3,
                                     f2v p3, f2v m5, f2v p5) {
    f2v acc = __builtin_elementwise_fma(c0, e, bias);
    acc = __builtin_elementwise_fma(c1, m1 + p1, acc);
    acc = __builtin_elementwise_fma(c3, m3 + p3, acc);
    return __builtin_elementwise_fma(c5, m5 + p5, acc);
}
// v_cvt_pk_u8_f32 rounds to nearest-even and saturates to 0..255; on the
// 1/4096 grid RNE(sum/4096 + 2^-13) == floor(sum/4096 + 0.5) (no ties occur)
__device__ __forceinline__ uint32_t pack4b(float a, float b, float c, float d) {
    uint32_t v = __builtin_amdgcn_cvt_pk_u8_f32(a, 0, 0u);
    v = __builtin_amdgcn_cvt_pk_u8_f32(b, 1, v);
    v = __builtin_amdgcn_cvt_pk_u8_f32(c, 2, v);
    return __builtin_amdgcn_cvt_pk_u8_f32(d, 3, v);
}

template <int B, int R, bool PF, bool PK, bool MEM, int LAUX, bool NTS, int WIDE, int TIGHT>
__device__ __forceinline__ void reduce2_tile(const Reduce2Args &a, int img, int strip, int band,
                                             uint32_t *lds) {
    using G = R2<B, WIDE, TIGHT>;
    constexpr int kThreads = G::kThreads, kPitch = G::kPitch;
    constexpr int TW = G::TW, K = G::K;
    const int tid = threadIdx.x;
    const int x0 = (a.s_base + strip) * TW;
    const int row_bytes = a.w * B;
    const int px0 = 2 * x0 - 5;          // first intermediate pixel of the strip
    const int base = (B * px0) & ~3;     // floor to a dword (two's complement)
    const int byte0 = base + 4 * tid;
    const bool vlane = tid < G::ND && byte0 >= 0 && byte0 + 4 <= row_bytes;
    // raw buffer loads: per-lane byte offset in voffset, row offset in soffset;
    // lanes outside the row get an out-of-range voffset and read 0
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<u8 *>(a.in + img * a.in_img), 0, static_cast<int>(a.in_img), 0x00020000);
    const uint32_t voff = vlane ? static_cast<uint32_t>(byte0) : 0x80000000u;
    const int y0 = a.y_base + band * a.band_rows;
    const int y1 = min(y0 + a.band_rows, a.y_end);
    const float c0 = a.c0, c1 = a.c1, c3 = a.c3, c5 = a.c5, bias = a.bias;
    // strip pixels outside the image (COPY edge): LDS pixels [0, nl) copy pixel 0,
    // [fr, fr_end] copy pixel w-1; filled after each vertical pass
    const int nl = px0 < 0 ? -px0 : 0;
    const int x_last = min(x0 + TW, a.x_end) - 1;
    const int fr = a.w - px0;                                   // LDS index of pixel w
    const int fr_end = min(2 * x_last + 5 - px0, G::NPX - 1);   // last LDS pixel read
    const int nr = fr_end >= fr ? fr_end - fr + 1 : 0;
    const bool edge = nl > 0 || nr > 0;

    auto load_row = [&](int r) -> uint32_t {
        r = clampi(r, 0, a.h - 1);
        return static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, r * row_bytes, LAUX));
    };

    // odd-row ring: slot s holds odd row 2m+1 with m = s (mod 6); y0 % 6 == 0
    f4v ring[6];
    ring[3] = cvt4_once(load_row(2 * (y0 - 3) + 1));
    ring[4] = cvt4_once(load_row(2 * (y0 - 2) + 1));
    ring[5] = cvt4_once(load_row(2 * (y0 - 1) + 1));
    ring[0] = cvt4_once(load_row(2 * y0 + 1));
    ring[1] = cvt4_once(load_row(2 * (y0 + 1) + 1));
    ring[2] = f4v{0.f, 0.f, 0.f, 0.f};

    uint32_t odd[R], even[R];
    if (PF) {
#pragma unroll
        for (int u = 0; u < R; ++u) {
            odd[u] = load_row(2 * (y0 + u + 2) + 1);
            even[u] = load_row(2 * (y0 + u));
        }
    }
    int buf = 0;
    for (int yc = y0; yc < y1; yc += R, buf ^= 1) {
        uint32_t *L = lds + buf * (R * kPitch);
        // ---- vertical pass: R intermediate rows -> LDS (packed uchar) ----
        if (!PF) {
#pragma unroll
            for (int u = 0; u < R; ++u) {
                odd[u] = load_row(2 * (yc + u + 2) + 1);
                even[u] = load_row(2 * (yc + u));
            }
        }
        const bool more = yc + R < y1;
#pragma unroll
        for (int u = 0; u < R; ++u) {
            uint32_t d;
            if (MEM) {  // diagnostic: same loads / LDS / stores, no arithmetic
                d = odd[u] + even[u];
                if (PF && more) {
                    odd[u] = load_row(2 * (yc + R + u + 2) + 1);
                    even[u] = load_row(2 * (yc + R + u));
                }
            } else {
                ring[(u + 2) % 6] = cvt4_once(odd[u]);
                const f4v e = cvt4_once(even[u]);
                if (PF && more) {  // rotate: this register now fetches the next chunk's row
                    odd[u] = load_row(2 * (yc + R + u + 2) + 1);
                    even[u] = load_row(2 * (yc + R + u));
                }
                const f4v m5 = ring[(u + 3) % 6], m3 = ring[(u + 4) % 6], m1 = ring[(u + 5) % 6];
                const f4v p1 = ring[u % 6], p3 = ring[(u + 1) % 6], p5 = ring[(u + 2) % 6];
                if (PK) {
                    const f2v C0 = {c0, c0}, C1 = {c1, c1}, C3 = {c3, c3}, C5 = {c5, c5}, BI = {bias, bias};
                    const f2v a = tap7v(C0, C1, C3, C5, BI, lo2(e), lo2(m1), lo2(p1), lo2(m3), lo2(p3), lo2(m5),
                                        lo2(p5));
                    const f2v b = tap7v(C0, C1, C3, C5, BI, hi2(e), hi2(m1), hi2(p1), hi2(m3), hi2(p3), hi2(m5),
                                        hi2(p5));
                    d = pack4b(a.x, a.y, b.x, b.y);
                } else {
                    d = pack4b(tap7(c0, c1, c3, c5, bias, e.x, m1.x, p1.x, m3.x, p3.x, m5.x, p5.x),
                               tap7(c0, c1, c3, c5, bias, e.y, m1.y, p1.y, m3.y, p3.y, m5.y, p5.y),
                               tap7(c0, c1, c3, c5, bias, e.z, m1.z, p1.z, m3.z, p3.z, m5.z, p5.z),
                               tap7(c0, c1, c3, c5, bias, e.w, m1.w, p1.w, m3.w, p3.w, m5.w, p5.w));
                }
            }
            if (G::ND >= kThreads || tid < G::ND) L[u * kPitch + tid] = d;
        }
        if (edge) {  // replicate the edge pixels (EXTEND_COPY) inside the LDS image
            __syncthreads();
            u8 *Lb = reinterpret_cast<u8 *>(L);
            const int nfill = nl + nr;
            for (int i = tid; i < R * nfill * B; i += kThreads) {
                const int u = i / (nfill * B);
                const int rem = i - u * nfill * B;
                const int f = rem / B, c = rem - f * B;
                const int dst = f < nl ? f : fr + (f - nl);
                const int srcp = f < nl ? nl : fr - 1;
                Lb[u * kPitch * 4 + B * dst + G::OFF0 + c] = Lb[u * kPitch * 4 + B * srcp + G::OFF0 + c];
            }
        }
        __syncthreads();
        // ---- horizontal pass: K output pixels per item, one channel at a time ----
        constexpr int items_per_row = TW / K;
        for (int it = tid; it < R * items_per_row; it += kThreads) {
            const int u = it / items_per_row;
            const int j = it - u * items_per_row;
            const int x = x0 + K * j;
            const int y = yc + u;
            if (y >= a.y_end || x >= a.x_end) continue;
            const uint32_t *row = L + u * kPitch;
            constexpr int W0 = (B * 2 * K) / 4;  // window start (dwords) per item
            uint32_t win[13];
            if (B == 3) {
                const uint2 *r2 = reinterpret_cast<const uint2 *>(row + W0 * j);
#pragma unroll
                for (int q = 0; q < 6; ++q) {
                    const uint2 dd = r2[q];
                    win[2 * q] = dd.x;
                    win[2 * q + 1] = dd.y;
                }
                win[12] = row[W0 * j + 12];
            } else {
                const uint4 *r4 = reinterpret_cast<const uint4 *>(row + W0 * j);
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const uint4 dd = r4[q];
                    win[4 * q] = dd.x, win[4 * q + 1] = dd.y, win[4 * q + 2] = dd.z, win[4 * q + 3] = dd.w;
                }
                win[12] = row[W0 * j + 12];
            }
            float o[K][B];
            if (MEM) {  // diagnostic: skip the arithmetic, keep the LDS reads and stores
#pragma unroll
                for (int k = 0; k < K; ++k)
#pragma unroll
                    for (int c = 0; c < B; ++c) o[k][c] = __uint_as_float(win[(k * B + c) % 13] & 0x437f0000u);
            } else
#pragma unroll
            for (int c = 0; c < B; ++c) {
                // px[t]: intermediate pixel 2x - 5 + t of channel c
                float px[2 * K + 9];
#pragma unroll
                for (int t = 0; t < 2 * K + 9; ++t) {
                    const int lb = B * t + c + G::OFF0;
                    const uint32_t dd = win[lb >> 2];
                    switch (lb & 3) {
                        case 0: px[t] = ubyte_once<0>(dd); break;
                        case 1: px[t] = ubyte_once<1>(dd); break;
                        case 2: px[t] = ubyte_once<2>(dd); break;
                        default: px[t] = ubyte_once<3>(dd); break;
                    }
                }
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int m = 2 * k + 5;
                    o[k][c] = tap7(c0, c1, c3, c5, bias, px[m], px[m - 1], px[m + 1], px[m - 3], px[m + 3],
                                   px[m - 5], px[m + 5]);
                }
            }
            u8 *q = a.out + img * a.out_img + (static_cast<size_t>(y) * a.ow + x) * B;
            const bool full = x + K <= a.ow;
            if (B == 3) {
                const uint32_t d0 = pack4b(o[0][0], o[0][1], o[0][2], o[1][0]);
                const uint32_t d1 = pack4b(o[1][1], o[1][2], o[2][0], o[2][1]);
                const uint32_t d2 = pack4b(o[2][2], o[3][0], o[3][1], o[3][2]);
                if (full && (reinterpret_cast<uintptr_t>(q) & 3u) == 0) {
                    if (NTS) {
                        typedef uint32_t u3v __attribute__((ext_vector_type(3)));
                        __builtin_nontemporal_store(u3v{d0, d1, d2}, reinterpret_cast<u3v *>(q));
                    } else {
                        *reinterpret_cast<uint3 *>(q) = uint3{d0, d1, d2};
                    }
                } else {
                    const uint32_t dd[3] = {d0, d1, d2};
                    const int nb = (full ? K : a.ow - x) * B;
                    for (int i = 0; i < nb; ++i) q[i] = static_cast<u8>(dd[i >> 2] >> (8 * (i & 3)));
                }
            } else {
                const uint32_t d0 = pack4b(o[0][0], o[0][1], o[0][2], o[0][3]);
                const uint32_t d1 = pack4b(o[1][0], o[1][1], o[1][2], o[1][3]);
                uint32_t *q32 = reinterpret_cast<uint32_t *>(q);
                if (full && (reinterpret_cast<uintptr_t>(q) & 7u) == 0) {
                    *reinterpret_cast<uint2 *>(q) = uint2{d0, d1};
                } else {
                    q32[0] = d0;
                    if (full) q32[1] = d1;
                }
            }
        }
        // double-buffered LDS: the next vertical pass writes the other buffer, whose
        // readers all finished before this chunk's barrier
    }
}

// The centre sampling convention's 2 x 2 reduce is k_reduce2m (k_reduce2m.hip); its
// all-VALU predecessor k_reduce2c (r04, 1.84-1.88 ms per C2 step) was removed once the
// matrix-core kernel beat it, its measurements are under profiles/r04/reduce2c/.

// Variant bits (A/B in one process via MIPX_R2_VARIANT; default = best measured):
// bit 0: R = 6 (else 12), bit 1: register prefetch of the next chunk,
// bit 2: packed-FP32 vertical taps, bit 3: memory-only diagnostic (not exact),
// bit 4: non-temporal loads, bit 5: non-temporal stores, bit 6: 256-thread
// workgroups over strips twice as wide, bit 7: 512-thread workgroups over
// strips four times as wide.  Measured in
// profiles/r01/v7_variants_ab.log: the memory-only build is no faster than the
// full one (the arithmetic is hidden), packed math and nt hints lose.
template <int B, int VAR>
__global__ void __launch_bounds__(R2T<(VAR & 128) ? 2 : (VAR & 64) ? 1 : 0>::kThreads) k_reduce2x2(Reduce2Args a) {
    constexpr int WIDE = (VAR & 128) ? 2 : (VAR & 64) ? 1 : 0;
    constexpr int TIGHT = (VAR & 256) ? 1 : 0;
    constexpr int kPitch = R2T<WIDE, TIGHT>::kPitch;
    constexpr int R = (VAR & 1) ? 6 : 12;
    constexpr bool PF = (VAR & 2) != 0;
    constexpr bool PK = (VAR & 4) != 0;
    constexpr bool MEM = (VAR & 8) != 0;
    constexpr int LAUX = (VAR & 16) ? 2 : 0;  // bit 4: non-temporal loads (cache policy nt)
    constexpr bool NTS = (VAR & 32) != 0;     // bit 5: non-temporal stores
    __shared__ uint32_t lds[2 * R * kPitch];
    const uint32_t t = a.remap ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    int strip, band, img;
    if (a.band_major) {  // tiles ordered (img, strip, band): vertical neighbours adjacent
        band = t % a.n_bands;
        const int rest = t / a.n_bands;
        strip = rest % a.n_strips;
        img = rest / a.n_strips;
    } else {             // (img, band, strip): horizontal neighbours adjacent
        strip = t % a.n_strips;
        const int rest = t / a.n_strips;
        band = rest % a.n_bands;
        img = rest / a.n_bands;
    }
    reduce2_tile<B, R, PF, PK, MEM, LAUX, NTS, WIDE, TIGHT>(a, img, strip, band, lds);
}


}  // namespace

// ===========================================================================
// launchers
// ===========================================================================
int reducev_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double vshrink, hipStream_t st) {
    SepSpec spec;
    if (!sep_spec_reduce(vshrink, &spec)) return MIPX_EDEVICE;
    SepWindow win{};
    win.bands = b;
    win.in_pitch = w * b;
    win.in_base = 0;
    win.in_img = img_bytes(w, h, b);
    win.in_len = h;
    win.o0 = 0;
    win.out_w = w;
    win.out_h = out_size_reduce(h, vshrink);
    return vpass_launch(in, out, n, spec, win, st);
}

int reduceh_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double hshrink, hipStream_t st) {
    SepSpec spec;
    if (!sep_spec_reduce(hshrink, &spec)) return MIPX_EDEVICE;
    SepWindow win{};
    win.bands = b;
    win.in_pitch = w * b;
    win.in_base = 0;
    win.in_img = img_bytes(w, h, b);
    win.in_len = w;
    win.o0 = 0;
    win.out_w = out_size_reduce(w, hshrink);
    win.out_h = h;
    return hpass_launch(in, out, n, spec, win, st);
}

// Both shrinks > 1 in one launch, output window [ox0, ox0 + ow) x [oy0, oy0 + oh):
// the column walker k_rcol (matrix cores, LDS row ring; dword-aligned input rows,
// <= 16 taps) first, then k_rmf2 (matrix cores, rows of any alignment), then the
// small-image strip walker and fused kernel (> 16 taps); MIPX_EUNSUPPORTED leaves it
// to the two separable passes.  MIPX_RCOL=0 / MIPX_RMFMA=0 turn the first two off
// (A/B); MIPX_RSTRIP=1 puts the strip walker first.
int reduce_one_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double hs, double vs, int ox0, int oy0,
                      int ow, int oh, hipStream_t st) {
    const char *ef = tune_env("MIPX_RSTRIP");
    const bool strip_first = ef && *ef == '1';
    if (strip_first) {
        const int se = reduce_strip_launch(in, out, n, w, h, b, hs, vs, ox0, oy0, ow, oh, st);
        if (se != MIPX_EUNSUPPORTED) return se;
    }
    const char *ec = tune_env("MIPX_RCOL");
    if (!(ec && *ec == '0')) {
        const int ce = reduce_col_launch(in, out, n, w, h, b, hs, vs, ox0, oy0, ow, oh, st);
        if (ce != MIPX_EUNSUPPORTED) return ce;
    }
    const int me = reduce_mfma_launch(in, out, n, w, h, b, hs, vs, ox0, oy0, ow, oh, st);
    if (me != MIPX_EUNSUPPORTED) return me;
    if (!strip_first) {
        const int se = reduce_strip_launch(in, out, n, w, h, b, hs, vs, ox0, oy0, ow, oh, st);
        if (se != MIPX_EUNSUPPORTED) return se;
    }
    return reduce_fused_launch(in, out, n, w, h, b, hs, vs, ox0, oy0, ow, oh, st);
}

// vips_reduce followed by vips_extract_area(left, top, ow, oh): only the
// window's output rows (vertical pass) and columns (horizontal pass) are
// computed.  Every output is the same sum over the same input pixels, so the
// result is identical to reduce-then-extract, minus the discarded work and the
// extract pass.  ws: n * w * oh * b bytes when both shrinks are > 1.
int reduce_window_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double hs, double vs, int left,
                         int top, int ow, int oh, void *ws, size_t ws_bytes, hipStream_t st) {
    const int rw = hs > 1.0 ? out_size_reduce(w, hs) : w;
    const int rh = vs > 1.0 ? out_size_reduce(h, vs) : h;
    if (left < 0 || top < 0 || ow <= 0 || oh <= 0 || left + ow > rw || top + oh > rh) return MIPX_EINVAL;
    const long long in_img = img_bytes(w, h, b);
    SepSpec sv, sh;
    if (vs > 1.0 && !sep_spec_reduce(vs, &sv)) return MIPX_EDEVICE;
    if (hs > 1.0 && !sep_spec_reduce(hs, &sh)) return MIPX_EDEVICE;
    if (vs > 1.0 && hs > 1.0) {
        const int fe = reduce_one_launch(in, out, n, w, h, b, hs, vs, left, top, ow, oh, st);
        if (fe != MIPX_EUNSUPPORTED) return fe;
        const size_t need = align_up(static_cast<size_t>(n) * w * oh * b);
        if (!ws || ws_bytes < need) return MIPX_EINVAL;
        u8 *tmp = static_cast<u8 *>(ws);
        const SepWindow v{b, w * b, 0, in_img, h, top, w, oh};
        int e = vpass_launch(in, tmp, n, sv, v, st);
        if (e) return e;
        const SepWindow hw{b, w * b, 0, img_bytes(w, oh, b), w, left, ow, oh};
        return hpass_launch(tmp, out, n, sh, hw, st);
    }
    if (vs > 1.0) {
        const SepWindow v{b, w * b, static_cast<long long>(left) * b, in_img, h, top, ow, oh};
        return vpass_launch(in, out, n, sv, v, st);
    }
    if (hs > 1.0) {
        const SepWindow hw{b, w * b, static_cast<long long>(top) * w * b, in_img, w, left, ow, oh};
        return hpass_launch(in, out, n, sh, hw, st);
    }
    return extract_launch(in, out, n, w, h, b, left, top, ow, oh, st);
}

// Is the phase-0 mask of shrink 2 the 7-nonzero symmetric shape the fused
// kernel hard-wires?  Returns the four distinct taps.
bool reduce2_taps(float c[4]) {
    std::vector<int> t;
    reduce_table(2.0, t);
    const int n = reduce_points(2.0);
    if (n != 13) return false;
    const int *r = t.data();  // phase 0
    static const int zero[] = {1, 3, 7, 9, 11, 12};
    for (int z : zero)
        if (r[z] != 0) return false;
    if (r[4] != r[6] || r[2] != r[8] || r[0] != r[10]) return false;
    c[0] = static_cast<float>(r[5]);
    c[1] = static_cast<float>(r[4]);
    c[2] = static_cast<float>(r[2]);
    c[3] = static_cast<float>(r[0]);
    return true;
}

// The centre convention's phase-64 mask: 12 non-zero taps symmetric about 5.5 and a
// zero tap 12 (k_reduce2m).  Returns t_0..t_5.
bool reduce2c_taps(float t[6]) {
    std::vector<int> tab;
    reduce_table(2.0, tab);
    const int n = reduce_points(2.0);
    if (n != 13) return false;
    const int *r = tab.data() + 64 * n;
    if (r[12] != 0) return false;
    for (int i = 0; i < 6; ++i) {
        if (r[i] != r[11 - i]) return false;
        t[i] = static_cast<float>(r[i]);
    }
    return true;
}


// Fused path applies to shrink exactly 2 x 2 on 3- or 4-band images whose rows
// are dword aligned: k_reduce2x2 at the corner convention, k_reduce2m at the centre one.
bool reduce2_eligible(const u8 *in, int w, int h, int b, double hs, double vs) {
    if (hs != 2.0 || vs != 2.0) return false;
    const char *e2 = tune_env("MIPX_REDUCE2");  // 0: leave 2 x 2 to the generic reduce (A/B)
    if (e2 && *e2 == '0') return false;
    if (b != 3 && b != 4) return false;
    if ((w * b) % 4 != 0 || (reinterpret_cast<uintptr_t>(in) % 4) != 0) return false;
    if (w < 8 || h < 8) return false;
    if (reduce_centre()) {
        static const bool centre_ok = [] { float t[6]; return reduce2c_taps(t); }();
        return centre_ok;
    }
    static const bool shape_ok = [] { float c[4]; return reduce2_taps(c); }();
    return shape_ok;
}

// k_reduce2x2 build variant.  Only the shipped one (66) is compiled now; the r01 / r02
// A/B builds (strip widths, register prefetch, LDS row strides) are recorded under
// profiles/r01 and profiles/r02 (scripts/ab_reduce.py, in git history, ran them).  r06's
// cache-policy A/B compiled 66 | 16 / 32 / 48 (82 / 98 / 114: non-temporal loads / stores /
// both, the LAUX / NTS parameters of reduce2_tile) as extra cases here: -15 % / +0.2 % /
// -14 % (profiles/r06/c2_nt_ab.jsonl), so none is kept.
constexpr int kR2Default = 66;  // wide strips, R = 12 + register prefetch: measured best (profiles/r01/v10_wide_ab.log)
int reduce2_variant() {
    const char *e = tune_env("MIPX_R2_VARIANT");
    if (!e || !*e) return kR2Default;
    const int v = std::atoi(e);
    switch (v) {
        case 66: return v;
        default: return kR2Default;
    }
}

int reduce2_launch(const u8 *in, u8 *out, int n, int w, int h, int b, hipStream_t st) {
    return reduce2_window_launch(in, out, n, w, h, b, 0, 0, out_size_reduce(w, 2.0), out_size_reduce(h, 2.0), st);
}

// Only the output region [x0, x1) x [y0, y1) is computed (rounded out to whole
// strips and 12-row chunks); the rest of the full-size output is left as it was.
// Every computed pixel is the same sum as in the full launch.
int reduce2_window_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int x0, int y0, int x1, int y1,
                          hipStream_t st) {
    if (reduce_centre()) {  // k_reduce2m: both passes on the matrix cores
        float tf[6];
        if (!reduce2c_taps(tf)) return MIPX_EINVAL;
        int taps[12];
        for (int i = 0; i < 6; ++i) taps[i] = taps[11 - i] = static_cast<int>(tf[i]);
        return reduce2m_window_launch(in, out, n, w, h, b, x0, y0, x1, y1, taps, st);
    }
    float c[4];
    if (!reduce2_taps(c)) return MIPX_EINVAL;
    Reduce2Args a{};
    a.in = in;
    a.out = out;
    a.w = w;
    a.h = h;
    a.ow = out_size_reduce(w, 2.0);
    a.oh = out_size_reduce(h, 2.0);
    if (x0 < 0 || y0 < 0 || x1 > a.ow || y1 > a.oh || x0 >= x1 || y0 >= y1) return MIPX_EINVAL;
    const int var = reduce2_variant();
    const int wl = (var & 128) ? 2 : (var & 64) ? 1 : 0;
    const int tw = b == 3 ? (wl == 2 ? R2<3, 2>::TW : wl == 1 ? R2<3, 1>::TW : R2<3>::TW)
                          : (wl == 2 ? R2<4, 2>::TW : wl == 1 ? R2<4, 1>::TW : R2<4>::TW);
    a.s_base = x0 / tw;
    a.x_end = x1;
    a.y_base = y0 / kR * kR;
    a.y_end = y1;
    a.n_strips = (x1 + tw - 1) / tw - a.s_base;
    const int chunks = (y1 - a.y_base + kR - 1) / kR;
    // rows per workgroup: 2 chunks of 12 (measured best, profiles/r01/geom_ab.log; MIPX_R2_BAND overrides)
    const char *eb = tune_env("MIPX_R2_BAND");
    const int cpb = (eb && *eb) ? std::max(1, std::atoi(eb)) : 2;
    const int chunks_per_band = std::max(1, std::min(chunks, cpb));
    a.band_rows = chunks_per_band * kR;
    a.n_bands = (y1 - a.y_base + a.band_rows - 1) / a.band_rows;
    a.in_img = img_bytes(w, h, b);
    a.out_img = img_bytes(a.ow, a.oh, b);
    a.c0 = c[0] / 4096.0f;
    a.c1 = c[1] / 4096.0f;
    a.c3 = c[2] / 4096.0f;
    a.c5 = c[3] / 4096.0f;
    a.bias = 1.0f / 8192.0f;
    const char *er = tune_env("MIPX_R2_REMAP");
    a.remap = (er && *er) ? std::atoi(er) : 1;
    const char *eo = tune_env("MIPX_R2_ORDER");
    a.band_major = (eo && *eo) ? std::atoi(eo) : 0;
    const long long tiles = static_cast<long long>(a.n_strips) * a.n_bands * n;
    if (tiles > 0x7fffffffLL) return MIPX_EINVAL;
    dim3 grid(static_cast<unsigned>(tiles));
#define MIPX_R2(V)                                                                                      \
    case V: {                                                                                           \
        const dim3 blk(R2T<(V & 128) ? 2 : (V & 64) ? 1 : 0>::kThreads);                                                   \
        if (b == 3) hipLaunchKernelGGL((k_reduce2x2<3, V>), grid, blk, 0, st, a);                       \
        else hipLaunchKernelGGL((k_reduce2x2<4, V>), grid, blk, 0, st, a);                              \
        break;                                                                                          \
    }
    switch (var) {
        MIPX_R2(66)
        default: return MIPX_EINVAL;
    }
#undef MIPX_R2
    return launch_check("k_reduce2x2");
}


}  // namespace mipx
