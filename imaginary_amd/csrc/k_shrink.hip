// k_shrink.hip — libvips vips_shrink (integer box) on gfx950.
//
// shrink.c runs shrinkv then shrinkh; each pass is (sum + n/2) / n to uchar,
// output size VIPS_ROUND(in / n), partial blocks at the far edge read the
// EXTEND_COPY border (restated in oracle/vips_ref.c).
//
// A block = one output row x TWS output pixels.  Phase 1 (shrinkv): lanes own
// dwords of the block's input byte span, sum the vs rows (dword buffer loads,
// every input byte read once) and write the rounded column means to LDS.
// Phase 2 (shrinkh): one lane per output pixel averages hs LDS pixels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "device_common.h"

namespace mipx {
namespace {

using namespace dev;

struct ShrinkArgs {
    const u8 *in;
    u8 *out;
    int w, h, ow, oh, hs, vs, tws, x_blocks;
    int ry, y_blocks, lstride;  // k_shrink_x4: output rows per block, row blocks, LDS dwords per row
    // computed output region (demand-driven execution): column blocks from xb0, rows
    // from y_base, clipped at x_end / y_end (full image: 0, 0, ow, oh)
    int xb0, y_base, x_end, y_end;
    float inv_hs, inv_vs;
    long long in_img, out_img;
};

template <int B>
__global__ void __launch_bounds__(256) k_shrink_lds(ShrinkArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    u8 *col = reinterpret_cast<u8 *>(smem);
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int xb = t % a.x_blocks;
    const int rest = t / a.x_blocks;
    const int y = a.y_base + rest % (a.y_end - a.y_base);
    const int img = rest / (a.y_end - a.y_base);
    const int x0 = (a.xb0 + xb) * a.tws;
    const int nx = min(a.tws, a.x_end - x0);
    const int row_bytes = a.w * B;
    const int span = nx * a.hs * B;           // bytes of the input span, COPY-extended
    const int sb = x0 * a.hs * B;             // first byte (may extend past the row)
    const u8 *src = a.in + img * a.in_img;
    const __amdgpu_buffer_rsrc_t rs = image_rsrc(src, a.in_img);
    const bool aligned_rows = (row_bytes & 3) == 0;
    // ---- phase 1: vertical sums, 4 byte-columns per lane ----
    for (int d = threadIdx.x * 4; d < span; d += 1024) {
        const int g = sb + d;
        const bool whole = aligned_rows && g + 4 <= row_bytes;  // dword inside the row
        uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        int off[4];
        if (!whole) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int gb = g + k;
                const int p = gb / B, c = gb - p * B;
                off[k] = min(p, a.w - 1) * B + c;  // COPY border beyond the last pixel
            }
        }
        if (whole) {  // batches of 8 independent row loads in flight
            for (int k0 = 0; k0 < a.vs; k0 += 8) {
                uint32_t v[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int r = min(y * a.vs + min(k0 + q, a.vs - 1), a.h - 1);
                    v[q] = static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(rs, g, r * row_bytes, 0));
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    if (k0 + q < a.vs) {
                        s0 += v[q] & 0xff;
                        s1 += (v[q] >> 8) & 0xff;
                        s2 += (v[q] >> 16) & 0xff;
                        s3 += v[q] >> 24;
                    }
                }
            }
        }
        for (int k = 0; k < a.vs && !whole; ++k) {
            const int r = min(y * a.vs + k, a.h - 1);
            {
                const u8 *p = src + static_cast<size_t>(r) * row_bytes;
                s0 += p[off[0]];
                s1 += p[off[1]];
                s2 += p[off[2]];
                s3 += p[off[3]];
            }
        }
        const uint32_t half = a.vs / 2;
        const uint32_t m = div_floor(static_cast<float>(s0 + half), a.inv_vs) |
                           (div_floor(static_cast<float>(s1 + half), a.inv_vs) << 8) |
                           (div_floor(static_cast<float>(s2 + half), a.inv_vs) << 16) |
                           (div_floor(static_cast<float>(s3 + half), a.inv_vs) << 24);
        smem[d >> 2] = m;
    }
    __syncthreads();
    // ---- phase 2: horizontal means ----
    const int x = threadIdx.x;
    if (x >= nx) return;
    const u8 *c = col + x * a.hs * B;
    uint32_t acc[B];
#pragma unroll
    for (int z = 0; z < B; ++z) acc[z] = 0;
    for (int j = 0; j < a.hs; ++j)
#pragma unroll
        for (int z = 0; z < B; ++z) acc[z] += c[j * B + z];
    u8 *q = a.out + img * a.out_img + (static_cast<size_t>(y) * a.ow + x0 + x) * B;
    const uint32_t half = a.hs / 2;
#pragma unroll
    for (int z = 0; z < B; ++z) q[z] = static_cast<u8>(div_floor(static_cast<float>(acc[z] + half), a.inv_hs));
}

// Rows dword aligned and vs <= 257: lanes own 16-byte chunks of the span
// (buffer_load_dwordx4, 4x the bytes in flight per instruction) and sum byte
// columns as packed u16 pairs (bytes 0/2 and 1/3 of each dword: every column
// sum <= 257 * 255 < 2^16, so the pairs never carry into each other).
template <int B, bool ROWS>
__global__ void __launch_bounds__(256) k_shrink_x4(ShrinkArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    u8 *col = reinterpret_cast<u8 *>(smem);
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int xb = t % a.x_blocks;
    const int rest = t / a.x_blocks;
    const int yb = rest % a.y_blocks;
    const int img = rest / a.y_blocks;
    const int x0 = (a.xb0 + xb) * a.tws;
    const int nx = min(a.tws, a.x_end - x0);
    const int row_bytes = a.w * B;
    const int span = nx * a.hs * B;
    const int sb = x0 * a.hs * B;  // multiple of 4: x0 is a multiple of tws >= 4
    const u8 *src = a.in + img * a.in_img;
    const __amdgpu_buffer_rsrc_t rs = image_rsrc(src, a.in_img);
    const uint32_t half = a.vs / 2;
    const int y0 = a.y_base + (ROWS ? yb * a.ry : yb);
    const int ny = ROWS ? min(a.ry, a.y_end - y0) : 1;
    // phase 1: 16 bytes x vs rows -> 16 rounded column means in LDS
    auto chunk = [&](int yy, int d) {
        const int g = sb + d;
        const int r0 = (y0 + yy) * a.vs;
        uint32_t m[4];
        if (g + 16 <= row_bytes) {
            uint32_t lo[4] = {0u, 0u, 0u, 0u}, hi[4] = {0u, 0u, 0u, 0u};
            for (int k0 = 0; k0 < a.vs; k0 += 8) {
                typedef uint32_t u4v __attribute__((ext_vector_type(4)));
                u4v v[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int r = min(r0 + min(k0 + q, a.vs - 1), a.h - 1);
                    v[q] = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(rs, g, r * row_bytes, 0));
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    if (k0 + q < a.vs) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            lo[j] += v[q][j] & 0x00ff00ffu;
                            hi[j] += (v[q][j] >> 8) & 0x00ff00ffu;
                        }
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                m[j] = div_floor(static_cast<float>((lo[j] & 0xffffu) + half), a.inv_vs) |
                       (div_floor(static_cast<float>((hi[j] & 0xffffu) + half), a.inv_vs) << 8) |
                       (div_floor(static_cast<float>((lo[j] >> 16) + half), a.inv_vs) << 16) |
                       (div_floor(static_cast<float>((hi[j] >> 16) + half), a.inv_vs) << 24);
            }
        } else {  // the chunk reaches past the row end: COPY border, byte by byte
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t sum[4] = {0u, 0u, 0u, 0u};
                int off[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int gb = g + 4 * j + k;
                    const int p = gb / B, c = gb - p * B;
                    off[k] = min(p, a.w - 1) * B + c;
                }
                for (int k = 0; k < a.vs; ++k) {
                    const u8 *p = src + static_cast<size_t>(min(r0 + k, a.h - 1)) * row_bytes;
#pragma unroll
                    for (int b = 0; b < 4; ++b) sum[b] += p[off[b]];
                }
                m[j] = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) m[j] |= div_floor(static_cast<float>(sum[b] + half), a.inv_vs) << (8 * b);
            }
        }
        *reinterpret_cast<uint4 *>(smem + yy * a.lstride + (d >> 2)) = uint4{m[0], m[1], m[2], m[3]};
    };
    const uint32_t hh = a.hs / 2;
    // phase 2: one output pixel -> hs LDS pixels averaged
    auto pixel = [&](int yy, int x) {
        const u8 *c = col + yy * a.lstride * 4 + x * a.hs * B;
        uint32_t acc[B];
#pragma unroll
        for (int z = 0; z < B; ++z) acc[z] = 0;
        for (int j = 0; j < a.hs; ++j)
#pragma unroll
            for (int z = 0; z < B; ++z) acc[z] += c[j * B + z];
        u8 *q = a.out + img * a.out_img + (static_cast<size_t>(y0 + yy) * a.ow + x0 + x) * B;
#pragma unroll
        for (int z = 0; z < B; ++z) q[z] = static_cast<u8>(div_floor(static_cast<float>(acc[z] + hh), a.inv_hs));
    };
    if (!ROWS) {
        for (int d = threadIdx.x * 16; d < span; d += 4096) chunk(0, d);
        __syncthreads();
        if (static_cast<int>(threadIdx.x) < nx) pixel(0, threadIdx.x);
        return;
    }
    // several output rows: (row, chunk) items stepped by 256 without a division per item
    const int chunks = (span + 15) >> 4;
    const int dy = 256 / chunks, dq = 256 - dy * chunks;
    int yy = threadIdx.x / chunks, q = threadIdx.x - yy * chunks;
    for (; yy < ny; yy += dy, q += dq, yy += q >= chunks ? 1 : 0, q -= q >= chunks ? chunks : 0) chunk(yy, q * 16);
    __syncthreads();
    const int py = 256 / nx, px = 256 - py * nx;
    int y2 = threadIdx.x / nx, x2 = threadIdx.x - y2 * nx;
    for (; y2 < ny; y2 += py, x2 += px, y2 += x2 >= nx ? 1 : 0, x2 -= x2 >= nx ? nx : 0) pixel(y2, x2);
}

// Small factors (S <= 4, both axes) without LDS: a lane makes 4 output pixels of one
// row from the S x 4 S input pixels under them, held in registers (S rows of S B
// dwords, loaded as 16/8/4-byte buffer loads), vertical means first (shrinkv), then
// horizontal (shrinkh), each (sum + S/2) / S like shrink.c.  Consecutive lanes take
// consecutive quads of a row, so a wave streams 64 * 4 S B contiguous bytes per input
// row.  The k_shrink_x4 path stages every row through LDS and reads it back a byte at a
// time; at S = 2 / 3 that ran at 37 % of HBM (C5 r02).
template <int B, int S>
__device__ __forceinline__ void load_row_words(const __amdgpu_buffer_rsrc_t &rs, int off, int roff, uint32_t *w) {
    constexpr int N = S * B;  // dwords per lane and row
    int i = 0;
#pragma unroll
    for (; i + 4 <= N; i += 4) {
        typedef uint32_t u4v __attribute__((ext_vector_type(4)));
        const u4v v = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 4 * i, roff, 0));
        w[i] = v[0], w[i + 1] = v[1], w[i + 2] = v[2], w[i + 3] = v[3];
    }
    if constexpr (N % 4 >= 2) {
        typedef uint32_t u2v __attribute__((ext_vector_type(2)));
        const u2v v = __builtin_bit_cast(u2v, __builtin_amdgcn_raw_buffer_load_b64(rs, off + 4 * i, roff, 0));
        w[i] = v[0], w[i + 1] = v[1];
        i += 2;
    }
    if constexpr (N % 2 == 1) w[i] = static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(rs, off + 4 * i, roff, 0));
}

template <int B, int S>
__global__ void __launch_bounds__(256) k_shrink_q(ShrinkArgs a) {
    constexpr int N = S * B;  // input dwords per lane and row: 4 S pixels
    const int nq = (a.x_end - 4 * a.xb0 + 3) >> 2;  // quads per computed output row (xb0 in quads here)
    const unsigned gq = blockIdx.x * 256u + threadIdx.x;  // quad within this image's window
    if (gq >= static_cast<unsigned>(nq) * static_cast<unsigned>(a.y_end - a.y_base)) return;
    const int img = blockIdx.y;
    const unsigned yr = gq / static_cast<unsigned>(nq);
    const int y = a.y_base + static_cast<int>(yr);
    const int xq = a.xb0 + static_cast<int>(gq - yr * nq);
    const int x = 4 * xq;
    const __amdgpu_buffer_rsrc_t rs = image_rsrc(a.in + img * a.in_img, a.in_img);
    const int row_bytes = a.w * B;
    uint8_t o[4 * B];
    if (x + 4 <= a.ow && S * (x + 4) <= a.w) {
        // ---- vertical means of the S rows, packed u16 pairs (sums <= 4 * 255) ----
        uint32_t lo[N], hi[N];
#pragma unroll
        for (int i = 0; i < N; ++i) lo[i] = hi[i] = 0u;
#pragma unroll
        for (int k = 0; k < S; ++k) {
            uint32_t w[N];
            load_row_words<B, S>(rs, S * x * B + min(S * y + k, a.h - 1) * row_bytes, 0, w);
#pragma unroll
            for (int i = 0; i < N; ++i) {
                lo[i] += w[i] & 0x00ff00ffu;
                hi[i] += (w[i] >> 8) & 0x00ff00ffu;
            }
        }
        uint8_t v[4 * N];  // the vertical means: 4 S pixels of the row
#pragma unroll
        for (int i = 0; i < N; ++i) {
            v[4 * i + 0] = static_cast<uint8_t>(((lo[i] & 0xffffu) + S / 2) / S);
            v[4 * i + 1] = static_cast<uint8_t>(((hi[i] & 0xffffu) + S / 2) / S);
            v[4 * i + 2] = static_cast<uint8_t>(((lo[i] >> 16) + S / 2) / S);
            v[4 * i + 3] = static_cast<uint8_t>(((hi[i] >> 16) + S / 2) / S);
        }
        // ---- horizontal means ----
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int c = 0; c < B; ++c) {
                uint32_t sum = 0;
#pragma unroll
                for (int k = 0; k < S; ++k) sum += v[(S * p + k) * B + c];
                o[p * B + c] = static_cast<uint8_t>((sum + S / 2) / S);
            }
    } else {  // the row's last quad: pixels past the image repeat its edge (COPY)
        const u8 *src = a.in + img * a.in_img;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int xo = min(x + p, a.ow - 1);
#pragma unroll
            for (int c = 0; c < B; ++c) {
                uint32_t sum = 0;
                for (int k = 0; k < S; ++k) {
                    const int xi = min(S * xo + k, a.w - 1);
                    uint32_t vs = 0;
                    for (int r = 0; r < S; ++r) vs += src[static_cast<size_t>(min(S * y + r, a.h - 1)) * row_bytes + xi * B + c];
                    sum += (vs + S / 2) / S;
                }
                o[p * B + c] = static_cast<uint8_t>((sum + S / 2) / S);
            }
        }
    }
    // ---- 4 B bytes out: one store when the row position is dword aligned; otherwise
    // a 1-3 byte head, B - 1 realigned dwords and a 1-3 byte tail ----
    u8 *q = a.out + img * a.out_img + (static_cast<size_t>(y) * a.ow + x) * B;
    const int np = min(4, a.ow - x);
    const int r = static_cast<int>(reinterpret_cast<uintptr_t>(q) & 3u);
    uint32_t d[B];
#pragma unroll
    for (int i = 0; i < B; ++i)
        d[i] = o[4 * i] | (static_cast<uint32_t>(o[4 * i + 1]) << 8) | (static_cast<uint32_t>(o[4 * i + 2]) << 16) |
               (static_cast<uint32_t>(o[4 * i + 3]) << 24);
    const __amdgpu_buffer_rsrc_t os = image_rsrc(a.out + img * a.out_img, a.out_img);
    const int qo = (y * a.ow + x) * B;
    if (np == 4 && r != 0) {
        const int hb = 4 - r;  // head bytes
        if (hb & 1) __builtin_amdgcn_raw_buffer_store_b8(static_cast<u8>(d[0]), os, qo, 0, 0);
        if (hb & 2)
            __builtin_amdgcn_raw_buffer_store_b16(static_cast<unsigned short>(d[0] >> (8 * (hb & 1))), os, qo + (hb & 1), 0, 0);
#pragma unroll
        for (int j = 0; j + 1 < B; ++j)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_alignbyte(d[j + 1], d[j], hb), os, qo + hb + 4 * j, 0, 0);
        const uint32_t tl = d[B - 1] >> (8 * hb);  // the last r bytes
        const int to = qo + 4 * B - r;
        if (r & 2) __builtin_amdgcn_raw_buffer_store_b16(static_cast<unsigned short>(tl), os, to, 0, 0);
        if (r & 1) __builtin_amdgcn_raw_buffer_store_b8(static_cast<u8>(tl >> (8 * (r & 2))), os, to + (r & 2), 0, 0);
    } else if (np == 4) {
        if constexpr (B == 3) {
            typedef int v3i_t __attribute__((ext_vector_type(3)));
            __builtin_amdgcn_raw_buffer_store_b96(v3i_t{static_cast<int>(d[0]), static_cast<int>(d[1]),
                                                        static_cast<int>(d[2])}, os, qo, 0, 0);
        } else {
            typedef int v4i_t __attribute__((ext_vector_type(4)));
            __builtin_amdgcn_raw_buffer_store_b128(v4i_t{static_cast<int>(d[0]), static_cast<int>(d[1]),
                                                         static_cast<int>(d[2]), static_cast<int>(d[3])}, os, qo, 0, 0);
        }
    } else {
        for (int i = 0; i < np * B; ++i) q[i] = o[i];
    }
}

// Larger factors (5 <= S <= 12, both axes equal, rows of any alignment): one output pixel per
// lane from its S x S box in registers, no LDS.  Each of the S rows is 3 x 16-byte loads from
// the box's dword-aligned-down start, realigned with v_alignbyte and summed as packed u16
// pairs; then the S column means of each channel are averaged (shrinkv, then shrinkh, each
// (sum + S/2) / S).  A wave streams 64 S B contiguous bytes of each row.
#ifndef MIPX_P1_UNROLL
#define MIPX_P1_UNROLL 4
#endif
template <int B, int S>
__global__ void __launch_bounds__(256) k_shrink_p1(ShrinkArgs a) {
    constexpr int NB = S * B;             // box bytes per row
    constexpr int ND = (NB + 3) / 4;      // realigned dwords
    constexpr int NL = (NB + 3 + 15) / 16;  // 16-byte loads per row (<= 3)
    static_assert(NL <= 3, "box too wide");
    const unsigned gq = blockIdx.x * 256u + threadIdx.x;  // pixel within this image's window
    const unsigned cols = static_cast<unsigned>(a.x_end - a.xb0);
    if (gq >= cols * static_cast<unsigned>(a.y_end - a.y_base)) return;
    const int img = blockIdx.y;
    const unsigned yr = gq / cols;
    const int y = a.y_base + static_cast<int>(yr);
    const int x = a.xb0 + static_cast<int>(gq - yr * cols);
    const int row_bytes = a.w * B;
    uint8_t o[B];
    if (S * (x + 1) <= a.w) {
        int delta = 0;
        const __amdgpu_buffer_rsrc_t rs = image_rsrc_aligned(a.in + img * a.in_img, a.in_img, &delta);
        uint32_t lo[ND], hi[ND];
#pragma unroll
        for (int i = 0; i < ND; ++i) lo[i] = hi[i] = 0u;
#pragma unroll MIPX_P1_UNROLL
        for (int k = 0; k < S; ++k) {
            const int off = delta + min(S * y + k, a.h - 1) * row_bytes + S * x * B;
            const int a4 = off & ~3, sh = off & 3;
            uint32_t t[4 * NL + 1];
#pragma unroll
            for (int j = 0; j < NL; ++j) {
                typedef uint32_t u4v __attribute__((ext_vector_type(4)));
                const u4v v = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(rs, a4 + 16 * j, 0, 0));
                t[4 * j] = v[0], t[4 * j + 1] = v[1], t[4 * j + 2] = v[2], t[4 * j + 3] = v[3];
            }
            t[4 * NL] = 0u;
#pragma unroll
            for (int i = 0; i < ND; ++i) {
                const uint32_t w = __builtin_amdgcn_alignbyte(t[i + 1], t[i], sh);
                lo[i] += w & 0x00ff00ffu;
                hi[i] += (w >> 8) & 0x00ff00ffu;
            }
        }
        uint32_t sum[B];
#pragma unroll
        for (int c = 0; c < B; ++c) sum[c] = 0u;
#pragma unroll
        for (int i = 0; i < ND; ++i) {
            const uint32_t m[4] = {((lo[i] & 0xffffu) + S / 2) / S, ((hi[i] & 0xffffu) + S / 2) / S,
                                   ((lo[i] >> 16) + S / 2) / S, ((hi[i] >> 16) + S / 2) / S};
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (4 * i + j < NB) sum[(4 * i + j) % B] += m[j];
        }
#pragma unroll
        for (int c = 0; c < B; ++c) o[c] = static_cast<uint8_t>((sum[c] + S / 2) / S);
    } else {  // the box reaches past the row end: COPY border, byte by byte
        const u8 *src = a.in + img * a.in_img;
#pragma unroll
        for (int c = 0; c < B; ++c) {
            uint32_t sum = 0;
            for (int k = 0; k < S; ++k) {
                const int xi = min(S * x + k, a.w - 1);
                uint32_t vs = 0;
                for (int r = 0; r < S; ++r) vs += src[static_cast<size_t>(min(S * y + r, a.h - 1)) * row_bytes + xi * B + c];
                sum += (vs + S / 2) / S;
            }
            o[c] = static_cast<uint8_t>((sum + S / 2) / S);
        }
    }
    u8 *q = a.out + img * a.out_img + (static_cast<size_t>(y) * a.ow + x) * B;
#pragma unroll
    for (int c = 0; c < B; ++c) q[c] = o[c];
}

}  // namespace

int shrink_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int hs, int vs, hipStream_t st) {
    return shrink_window_launch(in, out, n, w, h, b, hs, vs, 0, 0, out_size_shrink(w, hs), out_size_shrink(h, vs), st);
}

// Only the output region [x0, x1) x [y0, y1) of the full-size output is computed
// (columns rounded out to whole blocks); each computed pixel is the same box mean.
int shrink_window_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int hs, int vs, int x0, int y0, int x1,
                         int y1, hipStream_t st) {
    ShrinkArgs a{};
    a.in = in;
    a.out = out;
    a.w = w;
    a.h = h;
    a.ow = out_size_shrink(w, hs);
    a.oh = out_size_shrink(h, vs);
    if (x0 < 0 || y0 < 0 || x1 > a.ow || y1 > a.oh || x0 >= x1 || y0 >= y1) return MIPX_EINVAL;
    a.hs = hs;
    a.vs = vs;
    a.inv_hs = 1.0f / hs;
    a.inv_vs = 1.0f / vs;
    // output pixels per block: 256, fewer when the input span would exceed 32 KB
    int tws = 256;
    while (tws > 4 && static_cast<long long>(tws) * hs * b > 32768) tws >>= 1;
    if (static_cast<long long>(tws) * hs * b > 32768 || hs > 65535 || vs > 65535) {
        set_error("shrink %dx%d too large", hs, vs);
        return MIPX_EUNSUPPORTED;
    }
    a.tws = tws;
    a.xb0 = x0 / tws;
    a.x_end = x1;
    a.y_base = y0;
    a.y_end = y1;
    a.x_blocks = (x1 + tws - 1) / tws - a.xb0;
    a.in_img = img_bytes(w, h, b);
    a.out_img = img_bytes(a.ow, a.oh, b);
    if (a.in_img >= 0x7fffffffLL) return MIPX_EUNSUPPORTED;
    const long long blocks = static_cast<long long>(a.x_blocks) * (y1 - y0) * n;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    // S <= 4 on both axes, dword-aligned rows: the register-only quad kernel (MIPX_SHRINK_Q=0: off)
    const char *eq = tune_env("MIPX_SHRINK_Q");
    if (!(eq && *eq == '0') && hs == vs && hs >= 2 && hs <= 4 && (b == 3 || b == 4) && (w * b) % 4 == 0 && n <= 65535 &&
        a.in_img % 4 == 0 && (reinterpret_cast<uintptr_t>(in) & 3u) == 0) {
        ShrinkArgs q = a;
        q.xb0 = x0 / 4;  // in quads
        const long long quads = static_cast<long long>((x1 - 4 * q.xb0 + 3) / 4) * (y1 - y0);  // per image
        const dim3 g(static_cast<unsigned>((quads + 255) / 256), static_cast<unsigned>(n));  // image = blockIdx.y
#define MIPX_SQ(S_)                                                                                   \
    if (b == 3) hipLaunchKernelGGL((k_shrink_q<3, S_>), g, dim3(256), 0, st, q);                      \
    else hipLaunchKernelGGL((k_shrink_q<4, S_>), g, dim3(256), 0, st, q);
        if (hs == 2) { MIPX_SQ(2) } else if (hs == 3) { MIPX_SQ(3) } else { MIPX_SQ(4) }
#undef MIPX_SQ
        return launch_check("k_shrink_q");
    }
    // equal factors 5-12 (RGBA 5-10): one output pixel per lane from registers, 1.03-1.25x
    // k_shrink_x4 (profiles/r02/shrink_p1_ab.jsonl); MIPX_SHRINK_P1=0: off, =1: RGBA / 11 too
    const char *ep = tune_env("MIPX_SHRINK_P1");
    const int p1_rgba_max = (ep && *ep == '1') ? 11 : 10;
    if (!(ep && *ep == '0') && hs == vs && hs >= 5 && hs <= 12 && (b == 3 || (b == 4 && hs <= p1_rgba_max)) &&
        n <= 65535) {
        ShrinkArgs q = a;
        q.xb0 = x0;  // in pixels here
        const long long px = static_cast<long long>(x1 - x0) * (y1 - y0);  // per image (< 2^31: in_img is)
        const dim3 g(static_cast<unsigned>((px + 255) / 256), static_cast<unsigned>(n));
#define MIPX_SP(S_)                                                                                   \
    if (b == 3) hipLaunchKernelGGL((k_shrink_p1<3, S_>), g, dim3(256), 0, st, q);                     \
    else hipLaunchKernelGGL((k_shrink_p1<4, (S_ > 11 ? 11 : S_)>), g, dim3(256), 0, st, q);
        switch (hs) {
            case 5: MIPX_SP(5) break;
            case 6: MIPX_SP(6) break;
            case 7: MIPX_SP(7) break;
            case 8: MIPX_SP(8) break;
            case 9: MIPX_SP(9) break;
            case 10: MIPX_SP(10) break;
            case 11: MIPX_SP(11) break;
            default: MIPX_SP(12) break;
        }
#undef MIPX_SP
        return launch_check("k_shrink_p1");
    }
    const char *ex = tune_env("MIPX_SHRINK_X4");  // A/B: 0 selects the dword kernel
    const bool x4 = (w * b) % 4 == 0 && a.in_img % 4 == 0 && (reinterpret_cast<uintptr_t>(in) & 3u) == 0 &&
                    vs <= 257 && tws >= 4 && !(ex && *ex == '0');
    if (x4) {
        // output rows per block (small vs: enough to stream ~8 input rows), within 32 KB of LDS;
        // each row's chunks may run up to 16 bytes past its span (LDS rows rounded to whole chunks)
        a.lstride = static_cast<int>(((static_cast<size_t>(tws) * hs * b + 15) / 16 + 1) * 4);
        const char *ery = tune_env("MIPX_SHRINK_RY");
        // measured (profiles/r01/v14/ab_shrink_rows.log): only vs <= 3 gains from several rows per block
        int ry = (ery && *ery) ? std::max(1, std::atoi(ery)) : vs <= 3 ? (8 + vs - 1) / vs : 1;
        while (ry > 1 && static_cast<size_t>(ry) * a.lstride * 4 > 32768) --ry;
        a.ry = std::min(ry, y1 - y0);
        a.y_blocks = (y1 - y0 + a.ry - 1) / a.ry;
        const long long blocks4 = static_cast<long long>(a.x_blocks) * a.y_blocks * n;
        if (!grid_ok(blocks4)) return MIPX_EINVAL;
        const size_t lds16 = static_cast<size_t>(a.ry) * a.lstride * 4;
        if (a.ry > 1) {
            MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_shrink_x4<B_, true>), dim3(static_cast<unsigned>(blocks4)),
                                                      dim3(256), lds16, st, a));
        } else {
            MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_shrink_x4<B_, false>), dim3(static_cast<unsigned>(blocks4)),
                                                      dim3(256), lds16, st, a));
        }
        return launch_check("k_shrink_x4");
    }
    const size_t lds = ((static_cast<size_t>(tws) * hs * b + 3) / 4 + 1) * 4;
    MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL(k_shrink_lds<B_>, dim3(static_cast<unsigned>(blocks)), dim3(256), lds,
                                              st, a));
    return launch_check("k_shrink_lds");
}

}  // namespace mipx
