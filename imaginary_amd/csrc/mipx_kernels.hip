// mipx_kernels.hip — hand-written gfx950 kernels of the pixel-transform engine.
//
// Each kernel replaces one libvips 8.12.2 operation that bimg.Resize runs for
// imaginary.  All of them are HBM-bound byte/integer
// work: no MFMA.  Integer libvips arithmetic is carried in fp32 where every
// intermediate is an integer below 2^24, so the results are bit-identical to
// the integer C paths restated in oracle/vips_ref.c.
//
// Batches: n equally sized images packed back to back; the image index rides
// in blockIdx.z (generic kernels) or in the XCD-remapped tile index (fused
// Lanczos3 kernel).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mipx_internal.h"

namespace {

using namespace mipx;
using u8 = uint8_t;

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }

// byte k of a dword as float: the backend selects v_cvt_f32_ubyte{k}
template <int K>
__device__ __forceinline__ float ubyte_f(uint32_t v) {
    return static_cast<float>((v >> (8 * K)) & 0xffu);
}

// (sum + 2048) >> 12 clipped to 0..255, with sum an exact integer in fp32.
// sum / 4096 + 0.5 is exact (|sum| < 2^21), so floor() reproduces the
// arithmetic shift of libvips' unsigned_fixed_round().
__device__ __forceinline__ float fixed_round_f(float sum) {
    const float v = floorf(__builtin_fmaf(sum, 1.0f / 4096.0f, 0.5f));
    return __builtin_amdgcn_fmed3f(v, 0.0f, 255.0f);
}
__device__ __forceinline__ uint32_t fixed_round_u(float sum) {
    return static_cast<uint32_t>(fixed_round_f(sum));
}

// XCD-aware block remap (bijective for any grid, cdna_hip_programming.md §5):
// blocks b, b+8, b+16... share an XCD; give each XCD a contiguous tile range so
// neighbouring strips (which share halo bytes) meet in the same L2.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nb) {
    const uint32_t xcd = b & 7u, q = nb >> 3, r = nb & 7u;
    const uint32_t base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (b >> 3);
}

// ===========================================================================
// Lanczos3 reduce, generic shrink (libvips reducev.cpp / reduceh.cpp)
// ===========================================================================
struct ReduceGeom {
    double shrink;
    int pad;     // n/2 - 1: the EXTEND_COPY border libvips embeds before sampling
    int taps;
};

// Vertical: one block row = one output row (phase uniform per block, taps in
// SGPRs); each thread owns 4 consecutive bytes of the row (channel-agnostic).
template <bool DWORD>
__global__ void __launch_bounds__(256) k_reducev_generic(
    const u8 *__restrict__ in, u8 *__restrict__ out, int row_bytes, int h, int oh,
    ReduceGeom g, const float *__restrict__ tab, long long in_img, long long out_img) {
    const int y = blockIdx.y;
    const int img = blockIdx.z;
    const int j = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (j >= row_bytes) return;
    const double Y = y * g.shrink;
    const int iy = static_cast<int>(Y);
    const int sy = static_cast<int>(Y * 256.0);
    const int ty = ((sy & 255) + 1) >> 1;
    const float *c = tab + ty * g.taps;
    const u8 *src = in + img * in_img;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    const bool full = j + 4 <= row_bytes;
    for (int i = 0; i < g.taps; ++i) {
        const int r = clampi(iy + i - g.pad, 0, h - 1);
        const u8 *p = src + static_cast<size_t>(r) * row_bytes + j;
        const float ci = c[i];
        if (DWORD) {
            const uint32_t v = *reinterpret_cast<const uint32_t *>(p);
            a0 = __builtin_fmaf(ci, ubyte_f<0>(v), a0);
            a1 = __builtin_fmaf(ci, ubyte_f<1>(v), a1);
            a2 = __builtin_fmaf(ci, ubyte_f<2>(v), a2);
            a3 = __builtin_fmaf(ci, ubyte_f<3>(v), a3);
        } else {
            a0 = __builtin_fmaf(ci, static_cast<float>(p[0]), a0);
            if (full) {
                a1 = __builtin_fmaf(ci, static_cast<float>(p[1]), a1);
                a2 = __builtin_fmaf(ci, static_cast<float>(p[2]), a2);
                a3 = __builtin_fmaf(ci, static_cast<float>(p[3]), a3);
            } else {
                if (j + 1 < row_bytes) a1 = __builtin_fmaf(ci, static_cast<float>(p[1]), a1);
                if (j + 2 < row_bytes) a2 = __builtin_fmaf(ci, static_cast<float>(p[2]), a2);
            }
        }
    }
    u8 *q = out + img * out_img + static_cast<size_t>(y) * row_bytes + j;
    if (DWORD) {
        const uint32_t v = fixed_round_u(a0) | (fixed_round_u(a1) << 8) |
                           (fixed_round_u(a2) << 16) | (fixed_round_u(a3) << 24);
        *reinterpret_cast<uint32_t *>(q) = v;
    } else {
        q[0] = fixed_round_u(a0);
        if (j + 1 < row_bytes) q[1] = fixed_round_u(a1);
        if (j + 2 < row_bytes) q[2] = fixed_round_u(a2);
        if (j + 3 < row_bytes) q[3] = fixed_round_u(a3);
    }
    (void)oh;
}

// Horizontal: one thread per output pixel (all bands); the per-pixel phase
// row of the table is read through L1.
template <int B>
__global__ void __launch_bounds__(256) k_reduceh_generic(
    const u8 *__restrict__ in, u8 *__restrict__ out, int w, int ow, ReduceGeom g,
    const float *__restrict__ tab, long long in_img, long long out_img) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int img = blockIdx.z;
    if (x >= ow) return;
    const double X = x * g.shrink;
    const int ix = static_cast<int>(X);
    const int sx = static_cast<int>(X * 256.0);
    const int tx = ((sx & 255) + 1) >> 1;
    const float *c = tab + tx * g.taps;
    const u8 *row = in + img * in_img + static_cast<size_t>(y) * w * B;
    float acc[B];
#pragma unroll
    for (int z = 0; z < B; ++z) acc[z] = 0.f;
    for (int i = 0; i < g.taps; ++i) {
        const int col = clampi(ix + i - g.pad, 0, w - 1);
        const float ci = c[i];
        const u8 *p = row + col * B;
#pragma unroll
        for (int z = 0; z < B; ++z) acc[z] = __builtin_fmaf(ci, static_cast<float>(p[z]), acc[z]);
    }
    u8 *q = out + img * out_img + (static_cast<size_t>(y) * ow + x) * B;
#pragma unroll
    for (int z = 0; z < B; ++z) q[z] = fixed_round_u(acc[z]);
}

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
constexpr int kThreads = 128;
constexpr int kPitch = 160;      // LDS dwords per intermediate row (== 32 mod 64)

template <int B>
struct R2 {
    static constexpr int TW = B == 3 ? 80 : 56;     // output pixels per strip
    static constexpr int NPX = 2 * TW + 9;           // intermediate px 2x0-5 .. 2x0+2TW+3
    static constexpr int K = B == 3 ? 4 : 2;         // output pixels per horizontal item
    static constexpr int OFF0 = B == 3 ? 1 : 0;      // B*(2x0-5) - floor4(B*(2x0-5))
    static constexpr int ND = (B * NPX + OFF0 + 3) / 4;  // dwords per row
    static_assert(ND <= kThreads && ND <= kPitch, "strip too wide");
    static_assert((B * 2 * K) % 8 == 0, "window start must be 8-byte aligned");
};

struct Reduce2Args {
    const u8 *in;
    u8 *out;
    int w, h, ow, oh;
    int n_strips, n_bands, band_rows;  // band_rows multiple of kR
    long long in_img, out_img;
    // taps pre-scaled by 1/4096 (exact: powers of two); the bias 2^-13 turns the
    // exact chain into RNE(sum/4096 + 2^-13) == floor(sum/4096 + 0.5) at the cvt
    float c0, c1, c3, c5, bias;
};

// byte k of a dword as float, opaque to instcombine so that a row converted
// once is reused by every output it feeds (otherwise (float)a + (float)b is
// folded into (float)(a + b): one convert per use instead of per byte)
template <int K>
__device__ __forceinline__ float ubyte_once(uint32_t v) {
    float f = ubyte_f<K>(v);
    asm("" : "+v"(f));
    return f;
}
__device__ __forceinline__ float4 cvt4_once(uint32_t v) {
    return float4{ubyte_once<0>(v), ubyte_once<1>(v), ubyte_once<2>(v), ubyte_once<3>(v)};
}

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
// v_cvt_pk_u8_f32 rounds to nearest-even and saturates to 0..255; on the
// 1/4096 grid RNE(sum/4096 + 2^-13) == floor(sum/4096 + 0.5) (no ties occur)
__device__ __forceinline__ uint32_t pack4b(float a, float b, float c, float d) {
    uint32_t v = __builtin_amdgcn_cvt_pk_u8_f32(a, 0, 0u);
    v = __builtin_amdgcn_cvt_pk_u8_f32(b, 1, v);
    v = __builtin_amdgcn_cvt_pk_u8_f32(c, 2, v);
    return __builtin_amdgcn_cvt_pk_u8_f32(d, 3, v);
}

template <int B, int R, bool PF>
__device__ __forceinline__ void reduce2_tile(const Reduce2Args &a, int img, int strip, int band,
                                             uint32_t *lds) {
    using G = R2<B>;
    constexpr int TW = G::TW, K = G::K;
    const int tid = threadIdx.x;
    const int x0 = strip * TW;
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
    const int y0 = band * a.band_rows;
    const int y1 = min(y0 + a.band_rows, a.oh);
    const float c0 = a.c0, c1 = a.c1, c3 = a.c3, c5 = a.c5, bias = a.bias;
    // strip pixels outside the image (COPY edge): LDS pixels [0, nl) copy pixel 0,
    // [fr, fr_end] copy pixel w-1; filled after each vertical pass
    const int nl = px0 < 0 ? -px0 : 0;
    const int x_last = min(x0 + TW, a.ow) - 1;
    const int fr = a.w - px0;                                   // LDS index of pixel w
    const int fr_end = min(2 * x_last + 5 - px0, G::NPX - 1);   // last LDS pixel read
    const int nr = fr_end >= fr ? fr_end - fr + 1 : 0;
    const bool edge = nl > 0 || nr > 0;

    auto load_row = [&](int r) -> uint32_t {
        r = clampi(r, 0, a.h - 1);
        return static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, r * row_bytes, 0));
    };

    // odd-row ring: slot s holds odd row 2m+1 with m = s (mod 6); y0 % 6 == 0
    float4 ring[6];
    ring[3] = cvt4_once(load_row(2 * (y0 - 3) + 1));
    ring[4] = cvt4_once(load_row(2 * (y0 - 2) + 1));
    ring[5] = cvt4_once(load_row(2 * (y0 - 1) + 1));
    ring[0] = cvt4_once(load_row(2 * y0 + 1));
    ring[1] = cvt4_once(load_row(2 * (y0 + 1) + 1));
    ring[2] = float4{0.f, 0.f, 0.f, 0.f};

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
            ring[(u + 2) % 6] = cvt4_once(odd[u]);
            const float4 e = cvt4_once(even[u]);
            if (PF && more) {  // rotate: this register now fetches the next chunk's row
                odd[u] = load_row(2 * (yc + R + u + 2) + 1);
                even[u] = load_row(2 * (yc + R + u));
            }
            const float4 m5 = ring[(u + 3) % 6], m3 = ring[(u + 4) % 6], m1 = ring[(u + 5) % 6];
            const float4 p1 = ring[u % 6], p3 = ring[(u + 1) % 6], p5 = ring[(u + 2) % 6];
            const uint32_t d = pack4b(tap7(c0, c1, c3, c5, bias, e.x, m1.x, p1.x, m3.x, p3.x, m5.x, p5.x),
                                      tap7(c0, c1, c3, c5, bias, e.y, m1.y, p1.y, m3.y, p3.y, m5.y, p5.y),
                                      tap7(c0, c1, c3, c5, bias, e.z, m1.z, p1.z, m3.z, p3.z, m5.z, p5.z),
                                      tap7(c0, c1, c3, c5, bias, e.w, m1.w, p1.w, m3.w, p3.w, m5.w, p5.w));
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
            if (y >= a.oh || x >= a.ow) continue;
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
                    *reinterpret_cast<uint3 *>(q) = uint3{d0, d1, d2};
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

// Variant bits (A/B in one process via MIPX_R2_VARIANT; default = best measured):
// bit 0: R = 6 (else 12), bit 1: register prefetch of the next chunk.
template <int B, int VAR>
__global__ void __launch_bounds__(kThreads) k_reduce2x2(Reduce2Args a) {
    constexpr int R = (VAR & 1) ? 6 : 12;
    constexpr bool PF = (VAR & 2) != 0;
    __shared__ uint32_t lds[2 * R * kPitch];
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int strip = t % a.n_strips;
    const int rest = t / a.n_strips;
    const int band = rest % a.n_bands;
    const int img = rest / a.n_bands;
    reduce2_tile<B, R, PF>(a, img, strip, band, lds);
}

// ===========================================================================
// box shrink (libvips shrinkv.c then shrinkh.c): shrinkv rounds each column
// mean to uchar, shrinkh averages those; partial blocks read the COPY border.
// ===========================================================================
template <int B>
__global__ void __launch_bounds__(256) k_shrink(const u8 *__restrict__ in, u8 *__restrict__ out,
                                                int w, int h, int ow, int oh, int hs, int vs,
                                                long long in_img, long long out_img) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int img = blockIdx.z;
    if (x >= ow) return;
    const u8 *src = in + img * in_img;
    int hsum[B];
#pragma unroll
    for (int z = 0; z < B; ++z) hsum[z] = 0;
    for (int c = 0; c < hs; ++c) {
        const int col = min(x * hs + c, w - 1);
        int vsum[B];
#pragma unroll
        for (int z = 0; z < B; ++z) vsum[z] = 0;
        for (int k = 0; k < vs; ++k) {
            const int row = min(y * vs + k, h - 1);
            const u8 *p = src + (static_cast<size_t>(row) * w + col) * B;
#pragma unroll
            for (int z = 0; z < B; ++z) vsum[z] += p[z];
        }
#pragma unroll
        for (int z = 0; z < B; ++z) hsum[z] += (vsum[z] + vs / 2) / vs;
    }
    u8 *q = out + img * out_img + (static_cast<size_t>(y) * ow + x) * B;
#pragma unroll
    for (int z = 0; z < B; ++z) q[z] = static_cast<u8>((hsum[z] + hs / 2) / hs);
    (void)oh;
}

// ===========================================================================
// geometric remaps (libvips embed.c / extract.c / rot.c / flip.c) — bit-exact
// byte moves.  One thread per output pixel.
// ===========================================================================
enum RemapKind { kEmbed = 0, kRot90, kRot180, kRot270, kFlipH, kFlipV };

struct RemapArgs {
    const u8 *in;
    u8 *out;
    int w, h, ow, oh;
    int x, y, extend;
    u8 fill[4];
    long long in_img, out_img;
    const int *origins;  // extract with per-image (left, top) from the device (smartcrop)
};

__device__ __forceinline__ int pmod(int a, int m) {
    const int r = a % m;
    return r < 0 ? r + m : r;
}

template <int B, int KIND>
__global__ void __launch_bounds__(256) k_remap(RemapArgs a) {
    const int X = blockIdx.x * blockDim.x + threadIdx.x;
    const int Y = blockIdx.y;
    const int img = blockIdx.z;
    if (X >= a.ow) return;
    int sx = 0, sy = 0;
    bool use_fill = false;
    if (KIND == kEmbed) {
        int ox = a.x, oy = a.y;
        if (a.origins) {  // extract at a device-computed origin == embed at (-l, -t)
            ox = -a.origins[2 * img];
            oy = -a.origins[2 * img + 1];
        }
        sx = X - ox;
        sy = Y - oy;
        if (sx < 0 || sx >= a.w || sy < 0 || sy >= a.h) {
            switch (a.extend) {
                case MIPX_EXTEND_COPY:
                    sx = clampi(sx, 0, a.w - 1);
                    sy = clampi(sy, 0, a.h - 1);
                    break;
                case MIPX_EXTEND_REPEAT:
                    sx = pmod(sx, a.w);
                    sy = pmod(sy, a.h);
                    break;
                case MIPX_EXTEND_MIRROR: {
                    const int u = pmod(sx, 2 * a.w), v = pmod(sy, 2 * a.h);
                    sx = u < a.w ? u : 2 * a.w - 1 - u;
                    sy = v < a.h ? v : 2 * a.h - 1 - v;
                    break;
                }
                default: use_fill = true;
            }
        }
    } else if (KIND == kRot90) {
        sx = Y;
        sy = a.h - 1 - X;
    } else if (KIND == kRot180) {
        sx = a.w - 1 - X;
        sy = a.h - 1 - Y;
    } else if (KIND == kRot270) {
        sx = a.w - 1 - Y;
        sy = X;
    } else if (KIND == kFlipH) {
        sx = a.w - 1 - X;
        sy = Y;
    } else {
        sx = X;
        sy = a.h - 1 - Y;
    }
    u8 *q = a.out + img * a.out_img + (static_cast<size_t>(Y) * a.ow + X) * B;
    if (use_fill) {
#pragma unroll
        for (int z = 0; z < B; ++z) q[z] = a.fill[z];
        return;
    }
    const u8 *p = a.in + img * a.in_img + (static_cast<size_t>(sy) * a.w + sx) * B;
#pragma unroll
    for (int z = 0; z < B; ++z) q[z] = p[z];
}

// extract: row copies, 16 bytes per lane where the rows allow it
__global__ void __launch_bounds__(256) k_extract_rows(const u8 *__restrict__ in, u8 *__restrict__ out,
                                                      int in_row_bytes, int out_row_bytes,
                                                      int left_bytes, int top,
                                                      long long in_img, long long out_img) {
    const int y = blockIdx.y;
    const int img = blockIdx.z;
    const u8 *src = in + img * in_img + static_cast<size_t>(top + y) * in_row_bytes + left_bytes;
    u8 *dst = out + img * out_img + static_cast<size_t>(y) * out_row_bytes;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < out_row_bytes; j += gridDim.x * blockDim.x)
        dst[j] = src[j];
}

// ===========================================================================
// gaussian blur (libvips convi.c, separable integer mask, COPY edges):
// out = (sum + (scale + 1) / 2) / scale, clipped.  Horizontal pass then
// vertical pass with a uchar intermediate (vips_convsep).
// ===========================================================================
constexpr int kMaxMask = 255;
struct ConvArgs {
    const u8 *in;
    u8 *out;
    int w, h, n, scale, rounding;
    long long img_bytes;
    int mask[kMaxMask];
};

template <int B, bool VERT>
__global__ void __launch_bounds__(256) k_convi(ConvArgs a) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int img = blockIdx.z;
    if (x >= a.w) return;
    const u8 *src = a.in + img * a.img_bytes;
    const int half = a.n / 2;
    int sum[B];
#pragma unroll
    for (int z = 0; z < B; ++z) sum[z] = 0;
    for (int i = 0; i < a.n; ++i) {
        const int sx = VERT ? x : clampi(x + i - half, 0, a.w - 1);
        const int sy = VERT ? clampi(y + i - half, 0, a.h - 1) : y;
        const u8 *p = src + (static_cast<size_t>(sy) * a.w + sx) * B;
        const int m = a.mask[i];
#pragma unroll
        for (int z = 0; z < B; ++z) sum[z] += m * p[z];
    }
    u8 *q = a.out + img * a.img_bytes + (static_cast<size_t>(y) * a.w + x) * B;
#pragma unroll
    for (int z = 0; z < B; ++z) q[z] = static_cast<u8>(clampi((sum[z] + a.rounding) / a.scale, 0, 255));
}

// ===========================================================================
// watermark image blend (bimg vips_watermark_image): alpha 255 appended where
// missing; mask = (uchar)(wm_alpha * opacity); ifthenelse blend
// (m * a + (255 - m) * b + 128) / 255 over every band.
// ===========================================================================
template <int BI, int WB, int BO>
__global__ void __launch_bounds__(256) k_watermark(const u8 *__restrict__ base, const u8 *__restrict__ wm,
                                                   u8 *__restrict__ out, int w, int h, int ww, int wh,
                                                   int left, int top, float opacity,
                                                   long long base_img, long long out_img) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int img = blockIdx.z;
    if (x >= w) return;
    const u8 *p = base + img * base_img + (static_cast<size_t>(y) * w + x) * BI;
    int b[BO], av[BO];
#pragma unroll
    for (int z = 0; z < BO; ++z) b[z] = z < BI ? p[z] : 255;
    int m = 0;
    const int wx = x - left, wy = y - top;
    if (wx >= 0 && wx < ww && wy >= 0 && wy < wh) {
        const u8 *s = wm + (static_cast<size_t>(wy) * ww + wx) * WB;
#pragma unroll
        for (int z = 0; z < BO; ++z) av[z] = z < WB ? s[z] : 255;
        const float f = __fadd_rn(__fmul_rn(static_cast<float>(av[BO - 1]), opacity), 0.0f);
        m = f < 0.f ? 0 : (f > 255.f ? 255 : static_cast<int>(f));
    } else {
#pragma unroll
        for (int z = 0; z < BO; ++z) av[z] = 0;
    }
    u8 *q = out + img * out_img + (static_cast<size_t>(y) * w + x) * BO;
#pragma unroll
    for (int z = 0; z < BO; ++z) q[z] = static_cast<u8>((m * av[z] + (255 - m) * b[z] + 128) / 255);
    (void)h;
}


// ===========================================================================
// smartcrop attention scorer (libvips smartcrop.c vips_smartcrop_attention) on
// the ~32 px image vips_resize() produced.  One workgroup per image; the exact
// IEEE operation order of the libvips float/double pipeline, no contraction:
//   XYZ  (sRGB LUT -> scRGB x100 -> 3x3 matrix in double)
//   edge = |5 * Laplacian(Y)|            (convf: double sum)
//   skin = Y > 5 ? 100 - 100 * |XYZ/|XYZ| - (0.78, 0.57, 0.44)| : 0
//   sat  = Y > 5 ? Lab a : 0             (cbrt LUT with linear interpolation)
//   score = (edge + skin) + sat, gaussblur(sigma) (integer mask, double sums),
//   argmax (first in raster order), crop centred on it and clipped.
// ===========================================================================
constexpr int kScoreMaxPx = 4096;
struct ScoreArgs {
    const u8 *small;  // n images sw x sh x bands
    int *origins;     // n (left, top)
    int sw, sh, bands;
    int in_w, in_h, crop_w, crop_h;
    long long small_img;
    const float *v2y;   // 256
    const float *cbrt;  // kQuantElements
    int n_mask, mask_scale;
    int mask[kMaxMask];
};

__device__ __forceinline__ float lab_cbrt(const float *tab, float v, double white) {
    const float nq = static_cast<float>(static_cast<double>(__fmul_rn(100000.0f, v)) / white);
    const int i = clampi(static_cast<int>(nq), 0, kQuantElements - 2);
    const float f = __fsub_rn(nq, static_cast<float>(i));
    return __fadd_rn(tab[i], __fmul_rn(f, __fsub_rn(tab[i + 1], tab[i])));
}

__global__ void __launch_bounds__(256) k_smartcrop_score(ScoreArgs a) {
    __shared__ float sY[kScoreMaxPx];
    __shared__ float sA[kScoreMaxPx];
    __shared__ float sB[kScoreMaxPx];
    __shared__ float sC[kScoreMaxPx];
    __shared__ float wmax[4];
    __shared__ int widx[4];
    const int img = blockIdx.x;
    const int W = a.sw, H = a.sh, N = W * H;
    const u8 *src = a.small + img * a.small_img;
    // pass 1: Y into sY, skin into sA, sat into sB
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const u8 *p = src + static_cast<size_t>(i) * a.bands;
        const float R = __fmul_rn(a.v2y[p[0]], 100.0f);
        const float G = __fmul_rn(a.v2y[p[1]], 100.0f);
        const float Bc = __fmul_rn(a.v2y[p[2]], 100.0f);
        const float X = static_cast<float>(__dadd_rn(__dadd_rn(__dmul_rn(0.4124, R), __dmul_rn(0.3576, G)), __dmul_rn(0.1805, Bc)));
        const float Y = static_cast<float>(__dadd_rn(__dadd_rn(__dmul_rn(0.2126, R), __dmul_rn(0.7152, G)), __dmul_rn(0.0722, Bc)));
        const float Z = static_cast<float>(__dadd_rn(__dadd_rn(__dmul_rn(0.0193, R), __dmul_rn(0.1192, G)), __dmul_rn(0.9505, Bc)));
        sY[i] = Y;
        float sq = __fmul_rn(X, X);
        sq = __fadd_rn(sq, __fmul_rn(Y, Y));
        sq = __fadd_rn(sq, __fmul_rn(Z, Z));
        const float mag = static_cast<float>(sqrt(static_cast<double>(sq)));
        const float nx = mag == 0.0f ? 0.0f : __fdiv_rn(X, mag);
        const float ny = mag == 0.0f ? 0.0f : __fdiv_rn(Y, mag);
        const float nz = mag == 0.0f ? 0.0f : __fdiv_rn(Z, mag);
        const float dx = __fadd_rn(nx, -0.78f), dy = __fadd_rn(ny, -0.57f), dz = __fadd_rn(nz, -0.44f);
        float d2 = __fmul_rn(dx, dx);
        d2 = __fadd_rn(d2, __fmul_rn(dy, dy));
        d2 = __fadd_rn(d2, __fmul_rn(dz, dz));
        const float dist = static_cast<float>(sqrt(static_cast<double>(d2)));
        const bool bright = static_cast<double>(Y) > 5.0;
        sA[i] = bright ? __fadd_rn(__fmul_rn(-100.0f, dist), 100.0f) : 0.0f;
        const float cbx = lab_cbrt(a.cbrt, X, 95.047), cby = lab_cbrt(a.cbrt, Y, 100.0);
        sB[i] = bright ? static_cast<float>(500.0 * static_cast<double>(__fsub_rn(cbx, cby))) : 0.0f;
    }
    __syncthreads();
    // pass 2: score = (edge + skin) + sat into sC
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const int y = i / W, x = i - y * W;
        double acc = 0.0;
        acc = __dadd_rn(acc, -1.0 * sY[clampi(y - 1, 0, H - 1) * W + x]);
        acc = __dadd_rn(acc, -1.0 * sY[y * W + clampi(x - 1, 0, W - 1)]);
        acc = __dadd_rn(acc, 4.0 * sY[i]);
        acc = __dadd_rn(acc, -1.0 * sY[y * W + clampi(x + 1, 0, W - 1)]);
        acc = __dadd_rn(acc, -1.0 * sY[clampi(y + 1, 0, H - 1) * W + x]);
        const float edge = fabsf(__fadd_rn(__fmul_rn(5.0f, static_cast<float>(acc / 1.0 + 0.0)), 0.0f));
        sC[i] = __fadd_rn(__fadd_rn(edge, sA[i]), sB[i]);
    }
    __syncthreads();
    // pass 3: horizontal blur sC -> sB, vertical blur sB -> argmax
    const int half = a.n_mask / 2;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const int y = i / W, x = i - y * W;
        double s = 0.0;
        for (int t = 0; t < a.n_mask; ++t)
            s = __dadd_rn(s, static_cast<double>(a.mask[t]) * sC[y * W + clampi(x + t - half, 0, W - 1)]);
        sB[i] = static_cast<float>(s / a.mask_scale + 0.0);
    }
    __syncthreads();
    float best = -INFINITY;
    int bidx = 0x7fffffff;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const int y = i / W, x = i - y * W;
        double s = 0.0;
        for (int t = 0; t < a.n_mask; ++t)
            s = __dadd_rn(s, static_cast<double>(a.mask[t]) * sB[clampi(y + t - half, 0, H - 1) * W + x]);
        const float v = static_cast<float>(s / a.mask_scale + 0.0);
        if (v > best) { best = v; bidx = i; }  // i ascends per thread: first max kept
    }
    // argmax across the workgroup: larger value wins, ties -> smaller index
    for (int off = 32; off > 0; off >>= 1) {
        const float ob = __shfl_xor(best, off);
        const int oi = __shfl_xor(bidx, off);
        if (ob > best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
    }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { wmax[wave] = best; widx[wave] = bidx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < static_cast<int>(blockDim.x >> 6); ++k)
            if (wmax[k] > best || (wmax[k] == best && widx[k] < bidx)) { best = wmax[k]; bidx = widx[k]; }
        const int xp = bidx % W, yp = bidx / W;
        const double hscale = 32.0 / a.in_w, vscale = 32.0 / a.in_h;
        double l = xp / hscale - a.crop_w / 2, t = yp / vscale - a.crop_h / 2;
        const double lmax = a.in_w - a.crop_w, tmax = a.in_h - a.crop_h;
        l = l > lmax ? lmax : l;
        t = t > tmax ? tmax : t;
        a.origins[2 * img] = static_cast<int>(l < 0 ? 0 : l);
        a.origins[2 * img + 1] = static_cast<int>(t < 0 ? 0 : t);
    }
}

// ===========================================================================
// host launchers
// ===========================================================================
inline long long img_bytes(int w, int h, int b) { return static_cast<long long>(w) * h * b; }

template <template <int> class K>
struct Bands;  // (unused helper tag)

#define MIPX_DISPATCH_BANDS(b, ...)                      \
    switch (b) {                                         \
        case 1: { constexpr int B_ = 1; __VA_ARGS__; } break; \
        case 2: { constexpr int B_ = 2; __VA_ARGS__; } break; \
        case 3: { constexpr int B_ = 3; __VA_ARGS__; } break; \
        case 4: { constexpr int B_ = 4; __VA_ARGS__; } break; \
        default: return MIPX_EINVAL;                     \
    }

int launch_check(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, what);
    return MIPX_OK;
}

bool geom_ok(int n, int w, int h, int b) { return n > 0 && w > 0 && h > 0 && b >= 1 && b <= 4 && n <= 65535; }

int reducev_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double vshrink, hipStream_t st) {
    int taps = 0;
    const float *tab = device_reduce_table(vshrink, &taps);
    if (!tab) return MIPX_EDEVICE;
    const int oh = out_size_reduce(h, vshrink);
    const int row_bytes = w * b;
    ReduceGeom g{vshrink, taps / 2 - 1, taps};
    const int groups = (row_bytes + 3) / 4;
    dim3 grid((groups + 255) / 256, oh, n);
    const bool dword = (row_bytes % 4) == 0 && (reinterpret_cast<uintptr_t>(in) % 4) == 0 &&
                       (reinterpret_cast<uintptr_t>(out) % 4) == 0;
    if (dword)
        hipLaunchKernelGGL(k_reducev_generic<true>, grid, dim3(256), 0, st, in, out, row_bytes, h, oh, g, tab,
                           img_bytes(w, h, b), img_bytes(w, oh, b));
    else
        hipLaunchKernelGGL(k_reducev_generic<false>, grid, dim3(256), 0, st, in, out, row_bytes, h, oh, g, tab,
                           img_bytes(w, h, b), img_bytes(w, oh, b));
    return launch_check("k_reducev_generic");
}

int reduceh_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double hshrink, hipStream_t st) {
    int taps = 0;
    const float *tab = device_reduce_table(hshrink, &taps);
    if (!tab) return MIPX_EDEVICE;
    const int ow = out_size_reduce(w, hshrink);
    ReduceGeom g{hshrink, taps / 2 - 1, taps};
    dim3 grid((ow + 255) / 256, h, n);
    MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL(k_reduceh_generic<B_>, grid, dim3(256), 0, st, in, out, w, ow, g,
                                              tab, img_bytes(w, h, b), img_bytes(ow, h, b)));
    return launch_check("k_reduceh_generic");
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

// Fused path applies to shrink exactly 2 x 2 on 3- or 4-band images whose rows
// are dword aligned.
bool reduce2_eligible(const u8 *in, int w, int h, int b, double hs, double vs) {
    if (hs != 2.0 || vs != 2.0) return false;
    if (b != 3 && b != 4) return false;
    if ((w * b) % 4 != 0 || (reinterpret_cast<uintptr_t>(in) % 4) != 0) return false;
    if (w < 8 || h < 8) return false;
    static const bool shape_ok = [] { float c[4]; return reduce2_taps(c); }();
    return shape_ok;
}

// MIPX_R2_VARIANT overrides the default variant of k_reduce2x2 for A/B runs
// (scripts/ab_reduce.py); read per launch so one process can interleave them.
constexpr int kR2Default = 2;  // R = 12 + register prefetch: measured best (profiles/r01/v5_variants_ab.log)
int reduce2_variant() {
    const char *e = std::getenv("MIPX_R2_VARIANT");
    if (!e || !*e) return kR2Default;
    const int v = std::atoi(e);
    return (v >= 0 && v <= 3) ? v : kR2Default;
}

int reduce2_launch(const u8 *in, u8 *out, int n, int w, int h, int b, hipStream_t st) {
    float c[4];
    if (!reduce2_taps(c)) return MIPX_EINVAL;
    Reduce2Args a{};
    a.in = in;
    a.out = out;
    a.w = w;
    a.h = h;
    a.ow = out_size_reduce(w, 2.0);
    a.oh = out_size_reduce(h, 2.0);
    const int tw = b == 3 ? R2<3>::TW : R2<4>::TW;
    a.n_strips = (a.ow + tw - 1) / tw;
    const int chunks = (a.oh + kR - 1) / kR;
    const int chunks_per_band = std::max(1, std::min(chunks, 15));
    a.band_rows = chunks_per_band * kR;
    a.n_bands = (a.oh + a.band_rows - 1) / a.band_rows;
    a.in_img = img_bytes(w, h, b);
    a.out_img = img_bytes(a.ow, a.oh, b);
    a.c0 = c[0] / 4096.0f;
    a.c1 = c[1] / 4096.0f;
    a.c3 = c[2] / 4096.0f;
    a.c5 = c[3] / 4096.0f;
    a.bias = 1.0f / 8192.0f;
    const long long tiles = static_cast<long long>(a.n_strips) * a.n_bands * n;
    if (tiles > 0x7fffffffLL) return MIPX_EINVAL;
    dim3 grid(static_cast<unsigned>(tiles));
    const int var = reduce2_variant();
#define MIPX_R2(V)                                                                           \
    case V:                                                                                  \
        if (b == 3) hipLaunchKernelGGL((k_reduce2x2<3, V>), grid, dim3(kThreads), 0, st, a); \
        else hipLaunchKernelGGL((k_reduce2x2<4, V>), grid, dim3(kThreads), 0, st, a);        \
        break;
    switch (var) {
        MIPX_R2(0) MIPX_R2(1) MIPX_R2(2) MIPX_R2(3)
        default: return MIPX_EINVAL;
    }
#undef MIPX_R2
    return launch_check("k_reduce2x2");
}

int shrink_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int hs, int vs, hipStream_t st) {
    const int ow = out_size_shrink(w, hs), oh = out_size_shrink(h, vs);
    dim3 grid((ow + 255) / 256, oh, n);
    MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL(k_shrink<B_>, grid, dim3(256), 0, st, in, out, w, h, ow, oh, hs, vs,
                                              img_bytes(w, h, b), img_bytes(ow, oh, b)));
    return launch_check("k_shrink");
}

int remap_launch(int kind, RemapArgs a, int b, int n, hipStream_t st) {
    dim3 grid((a.ow + 255) / 256, a.oh, n);
#define MIPX_REMAP(KIND)                                                                  \
    MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_remap<B_, KIND>), grid, dim3(256), 0, st, a))
    switch (kind) {
        case kEmbed: MIPX_REMAP(kEmbed); break;
        case kRot90: MIPX_REMAP(kRot90); break;
        case kRot180: MIPX_REMAP(kRot180); break;
        case kRot270: MIPX_REMAP(kRot270); break;
        case kFlipH: MIPX_REMAP(kFlipH); break;
        case kFlipV: MIPX_REMAP(kFlipV); break;
        default: return MIPX_EINVAL;
    }
#undef MIPX_REMAP
    return launch_check("k_remap");
}

int convi_launch(const u8 *in, u8 *out, int n, int w, int h, int b, const std::vector<int> &mask, int scale,
                 bool vert, hipStream_t st) {
    ConvArgs a{};
    a.in = in;
    a.out = out;
    a.w = w;
    a.h = h;
    a.n = static_cast<int>(mask.size());
    a.scale = scale;
    a.rounding = (scale + 1) / 2;
    a.img_bytes = img_bytes(w, h, b);
    for (int i = 0; i < a.n; ++i) a.mask[i] = mask[i];
    dim3 grid((w + 255) / 256, h, n);
    if (vert) {
        MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_convi<B_, true>), grid, dim3(256), 0, st, a));
    } else {
        MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_convi<B_, false>), grid, dim3(256), 0, st, a));
    }
    return launch_check("k_convi");
}

size_t align_up(size_t v) { return (v + 255) & ~static_cast<size_t>(255); }

}  // namespace

// ===========================================================================
// C-ABI: per-op entry points
// ===========================================================================
namespace mipx {

size_t op_workspace_bytes(int op, int n, int w, int h, int bands, double p0, double p1) {
    if (n <= 0 || w <= 0 || h <= 0 || bands <= 0) return 0;
    switch (op) {
        case MIPX_OP_REDUCE: {  // generic path: reducev intermediate
            if (p1 <= 1.0) return 0;
            const int oh = out_size_reduce(h, p1);
            return align_up(static_cast<size_t>(n) * w * oh * bands);
        }
        case MIPX_OP_BLUR: return align_up(static_cast<size_t>(n) * w * h * bands);
        case MIPX_OP_SMARTCROP: {
            ResizeSchedule s;
            if (resize_schedule(w, h, 32.0 / w, 32.0 / h, s)) return 0;
            const size_t a = align_up(static_cast<size_t>(n) * s.w1 * s.h1 * bands);
            const size_t b = align_up(static_cast<size_t>(n) * s.w1 * s.h2 * bands);
            const size_t c = align_up(static_cast<size_t>(n) * s.w2 * s.h2 * bands);
            return a + b + c + align_up(static_cast<size_t>(n) * 2 * sizeof(int));
        }
        default: return 0;
    }
    (void)p0;
}

int smartcrop_origins(const u8 *in, int *origins, int n, int w, int h, int b, int cw, int ch, void *ws,
                      size_t ws_bytes, hipStream_t st, u8 **small_out = nullptr) {
    if (b < 3) return MIPX_EUNSUPPORTED;
    if (cw <= 0 || ch <= 0 || cw > w || ch > h) return MIPX_EINVAL;
    ResizeSchedule s;
    int e = resize_schedule(w, h, 32.0 / w, 32.0 / h, s);
    if (e) return e;
    if (s.w2 * s.h2 > kScoreMaxPx) return MIPX_EUNSUPPORTED;
    const size_t need = op_workspace_bytes(MIPX_OP_SMARTCROP, n, w, h, b, cw, ch);
    if (!ws || ws_bytes < need) return MIPX_EINVAL;
    u8 *p0 = static_cast<u8 *>(ws);
    u8 *p1 = p0 + align_up(static_cast<size_t>(n) * s.w1 * s.h1 * b);
    u8 *p2 = p1 + align_up(static_cast<size_t>(n) * s.w1 * s.h2 * b);
    const u8 *cur = in;
    if (s.shrink_h > 1 || s.shrink_v > 1) {
        if ((e = shrink_launch(cur, p0, n, w, h, b, s.shrink_h, s.shrink_v, st))) return e;
        cur = p0;
    }
    if (s.reduce_v > 1.0) {
        if ((e = reducev_launch(cur, p1, n, s.w1, s.h1, b, s.reduce_v, st))) return e;
        cur = p1;
    }
    if (s.reduce_h > 1.0) {
        if ((e = reduceh_launch(cur, p2, n, s.w1, s.h2, b, s.reduce_h, st))) return e;
        cur = p2;
    }
    const double hscale = 32.0 / w, vscale = 32.0 / h;
    double sigma = std::sqrt(std::pow(cw * hscale, 2) + std::pow(ch * vscale, 2)) / 10;
    if (sigma < 1.0) sigma = 1.0;
    std::vector<int> mask;
    int scale = 0;
    const int nm = gaussmat(sigma, 0.2, mask, scale);
    if (nm < 0 || nm > kMaxMask) return MIPX_EUNSUPPORTED;
    const float *tabs = device_colour_tables();
    if (!tabs) return MIPX_EDEVICE;
    ScoreArgs a{};
    a.small = cur;
    a.origins = origins;
    a.sw = s.w2;
    a.sh = s.h2;
    a.bands = b;
    a.in_w = w;
    a.in_h = h;
    a.crop_w = cw;
    a.crop_h = ch;
    a.small_img = img_bytes(s.w2, s.h2, b);
    a.v2y = tabs;
    a.cbrt = tabs + 256;
    a.n_mask = nm;
    a.mask_scale = scale;
    for (int i = 0; i < nm; ++i) a.mask[i] = mask[i];
    hipLaunchKernelGGL(k_smartcrop_score, dim3(n), dim3(256), 0, st, a);
    if (small_out) *small_out = const_cast<u8 *>(cur);
    return launch_check("k_smartcrop_score");
}

int smartcrop_extract(const u8 *in, u8 *out, int n, int w, int h, int b, int cw, int ch, void *ws,
                      size_t ws_bytes, hipStream_t st) {
    const size_t need = op_workspace_bytes(MIPX_OP_SMARTCROP, n, w, h, b, cw, ch);
    if (!ws || ws_bytes < need) return MIPX_EINVAL;
    int *origins = reinterpret_cast<int *>(static_cast<u8 *>(ws) + need - align_up(static_cast<size_t>(n) * 2 * sizeof(int)));
    int e = smartcrop_origins(in, origins, n, w, h, b, cw, ch, ws, ws_bytes, st);
    if (e) return e;
    RemapArgs a{};
    a.in = in;
    a.out = out;
    a.w = w;
    a.h = h;
    a.ow = cw;
    a.oh = ch;
    a.extend = MIPX_EXTEND_BLACK;
    a.in_img = img_bytes(w, h, b);
    a.out_img = img_bytes(cw, ch, b);
    a.origins = origins;
    return remap_launch(kEmbed, a, b, n, st);
}

}  // namespace mipx

extern "C" {

size_t mipx_op_workspace_bytes(int32_t op, int32_t n, int32_t w, int32_t h, int32_t bands, double p0,
                               double p1) {
    return mipx::op_workspace_bytes(op, n, w, h, bands, p0, p1);
}

int mipx_op_reducev(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                    double vshrink, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands) || !(vshrink >= 1.0)) return MIPX_EINVAL;
    if (vshrink == 1.0)
        MIPX_HIP(hipMemcpyAsync(d_out, d_in, static_cast<size_t>(n) * w * h * bands, hipMemcpyDeviceToDevice,
                                mipx::as_stream(stream)));
    else
        return reducev_launch(d_in, d_out, n, w, h, bands, vshrink, mipx::as_stream(stream));
    return MIPX_OK;
}

int mipx_op_reduceh(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                    double hshrink, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands) || !(hshrink >= 1.0)) return MIPX_EINVAL;
    if (hshrink == 1.0)
        MIPX_HIP(hipMemcpyAsync(d_out, d_in, static_cast<size_t>(n) * w * h * bands, hipMemcpyDeviceToDevice,
                                mipx::as_stream(stream)));
    else
        return reduceh_launch(d_in, d_out, n, w, h, bands, hshrink, mipx::as_stream(stream));
    return MIPX_OK;
}

int mipx_op_reduce(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                   double hshrink, double vshrink, void *d_ws, size_t ws_bytes, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands) || !(hshrink >= 1.0) || !(vshrink >= 1.0))
        return MIPX_EINVAL;
    hipStream_t st = mipx::as_stream(stream);
    if (reduce2_eligible(d_in, w, h, bands, hshrink, vshrink)) return reduce2_launch(d_in, d_out, n, w, h, bands, st);
    if (vshrink == 1.0) return mipx_op_reduceh(d_in, d_out, n, w, h, bands, hshrink, stream);
    if (hshrink == 1.0) return mipx_op_reducev(d_in, d_out, n, w, h, bands, vshrink, stream);
    const size_t need = mipx::op_workspace_bytes(MIPX_OP_REDUCE, n, w, h, bands, hshrink, vshrink);
    if (!d_ws || ws_bytes < need) return MIPX_EINVAL;
    uint8_t *t = static_cast<uint8_t *>(d_ws);
    int e = reducev_launch(d_in, t, n, w, h, bands, vshrink, st);
    if (e) return e;
    return reduceh_launch(t, d_out, n, w, mipx::out_size_reduce(h, vshrink), bands, hshrink, st);
}

int mipx_op_shrink(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                   int32_t hshrink, int32_t vshrink, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands) || hshrink < 1 || vshrink < 1) return MIPX_EINVAL;
    return shrink_launch(d_in, d_out, n, w, h, bands, hshrink, vshrink, mipx::as_stream(stream));
}

int mipx_op_embed(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands, int32_t x,
                  int32_t y, int32_t ow, int32_t oh, int32_t extend, const int32_t *bg, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands) || ow <= 0 || oh <= 0) return MIPX_EINVAL;
    RemapArgs a{};
    a.in = d_in;
    a.out = d_out;
    a.w = w;
    a.h = h;
    a.ow = ow;
    a.oh = oh;
    a.x = x;
    a.y = y;
    if (extend == MIPX_EXTEND_LAST) extend = MIPX_EXTEND_BACKGROUND;
    a.extend = extend;
    for (int z = 0; z < 4; ++z) a.fill[z] = 0;
    if (extend == MIPX_EXTEND_WHITE)
        for (int z = 0; z < 4; ++z) a.fill[z] = 255;
    if (extend == MIPX_EXTEND_BACKGROUND) {
        int b3[3] = {0, 0, 0};
        if (bg) b3[0] = bg[0], b3[1] = bg[1], b3[2] = bg[2];
        for (int z = 0; z < 4; ++z) a.fill[z] = static_cast<uint8_t>(std::min(255, std::max(0, b3[z < 3 ? z : 2])));
        if (bands == 4) a.fill[3] = 255;
        if (bands <= 2) a.fill[0] = static_cast<uint8_t>(std::min(255, std::max(0, b3[0]))), a.fill[1] = 255;
    }
    a.in_img = img_bytes(w, h, bands);
    a.out_img = img_bytes(ow, oh, bands);
    return remap_launch(kEmbed, a, bands, n, mipx::as_stream(stream));
}

int mipx_op_extract(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                    int32_t left, int32_t top, int32_t ow, int32_t oh, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands)) return MIPX_EINVAL;
    if (left < 0 || top < 0 || ow <= 0 || oh <= 0 || left + ow > w || top + oh > h) {
        mipx::set_error("bad extract area");
        return MIPX_EINVAL;
    }
    const int out_row = ow * bands;
    dim3 grid(std::min((out_row + 255) / 256, 64), oh, n);
    hipLaunchKernelGGL(k_extract_rows, grid, dim3(256), 0, mipx::as_stream(stream), d_in, d_out, w * bands, out_row,
                       left * bands, top, img_bytes(w, h, bands), img_bytes(ow, oh, bands));
    return launch_check("k_extract_rows");
}

int mipx_op_rot(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands, int32_t angle,
                void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands)) return MIPX_EINVAL;
    angle = ((angle % 360) + 360) % 360;
    RemapArgs a{};
    a.in = d_in;
    a.out = d_out;
    a.w = w;
    a.h = h;
    a.in_img = img_bytes(w, h, bands);
    a.out_img = a.in_img;
    hipStream_t st = mipx::as_stream(stream);
    switch (angle) {
        case 0:
            MIPX_HIP(hipMemcpyAsync(d_out, d_in, static_cast<size_t>(a.in_img) * n, hipMemcpyDeviceToDevice, st));
            return MIPX_OK;
        case 90: a.ow = h, a.oh = w; return remap_launch(kRot90, a, bands, n, st);
        case 180: a.ow = w, a.oh = h; return remap_launch(kRot180, a, bands, n, st);
        case 270: a.ow = h, a.oh = w; return remap_launch(kRot270, a, bands, n, st);
        default: return MIPX_EINVAL;
    }
}

int mipx_op_flip(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                 int32_t vertical, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands)) return MIPX_EINVAL;
    RemapArgs a{};
    a.in = d_in;
    a.out = d_out;
    a.w = w;
    a.h = h;
    a.ow = w;
    a.oh = h;
    a.in_img = img_bytes(w, h, bands);
    a.out_img = a.in_img;
    return remap_launch(vertical ? kFlipV : kFlipH, a, bands, n, mipx::as_stream(stream));
}

int mipx_op_gaussblur(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                      double sigma, double min_ampl, void *d_ws, size_t ws_bytes, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands)) return MIPX_EINVAL;
    std::vector<int> mask;
    int scale = 0;
    const int nm = mipx::gaussmat(sigma, min_ampl, mask, scale);
    if (nm < 0) return MIPX_EINVAL;
    if (nm > kMaxMask) {
        mipx::set_error("gaussblur mask of %d taps exceeds %d", nm, kMaxMask);
        return MIPX_EUNSUPPORTED;
    }
    const size_t need = mipx::op_workspace_bytes(MIPX_OP_BLUR, n, w, h, bands, sigma, min_ampl);
    if (!d_ws || ws_bytes < need) return MIPX_EINVAL;
    hipStream_t st = mipx::as_stream(stream);
    uint8_t *t = static_cast<uint8_t *>(d_ws);
    int e = convi_launch(d_in, t, n, w, h, bands, mask, scale, false, st);
    if (e) return e;
    return convi_launch(t, d_out, n, w, h, bands, mask, scale, true, st);
}

int mipx_op_watermark(const uint8_t *d_base, const uint8_t *d_wm, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                      int32_t bands, int32_t ww, int32_t wh, int32_t wb, int32_t left, int32_t top, float opacity,
                      void *stream) {
    if (!d_base || !d_wm || !d_out || !geom_ok(n, w, h, bands) || ww <= 0 || wh <= 0 || wb < 1 || wb > 4)
        return MIPX_EINVAL;
    const int bo = (bands == 2 || bands > 3) ? bands : bands + 1;
    const int wo = (wb == 2 || wb > 3) ? wb : wb + 1;
    if (bo != wo) return MIPX_EUNSUPPORTED;
    dim3 grid((w + 255) / 256, h, n);
    hipStream_t st = mipx::as_stream(stream);
    const long long bi = img_bytes(w, h, bands), oi = img_bytes(w, h, bo);
#define MIPX_WM(BI, WB, BO)                                                                                   \
    hipLaunchKernelGGL((k_watermark<BI, WB, BO>), grid, dim3(256), 0, st, d_base, d_wm, d_out, w, h, ww, wh, left, \
                       top, opacity, bi, oi)
    if (bo == 4) {
        if (bands == 3 && wb == 3) MIPX_WM(3, 3, 4);
        else if (bands == 3 && wb == 4) MIPX_WM(3, 4, 4);
        else if (bands == 4 && wb == 3) MIPX_WM(4, 3, 4);
        else MIPX_WM(4, 4, 4);
    } else {  // grey: 1 or 2 bands -> 2
        if (bands == 1 && wb == 1) MIPX_WM(1, 1, 2);
        else if (bands == 1 && wb == 2) MIPX_WM(1, 2, 2);
        else if (bands == 2 && wb == 1) MIPX_WM(2, 1, 2);
        else MIPX_WM(2, 2, 2);
    }
#undef MIPX_WM
    return launch_check("k_watermark");
}

int mipx_op_smartcrop_origin(const uint8_t *d_in, int32_t *d_origins, int32_t n, int32_t w, int32_t h, int32_t bands,
                             int32_t cw, int32_t ch, void *d_ws, size_t ws_bytes, void *stream) {
    if (!d_in || !d_origins || !geom_ok(n, w, h, bands)) return MIPX_EINVAL;
    return mipx::smartcrop_origins(d_in, d_origins, n, w, h, bands, cw, ch, d_ws, ws_bytes, mipx::as_stream(stream));
}

}  // extern "C"
