// k_geometry.hip — libvips vips_embed / vips_extract_area / vips_rot /
// vips_flip on gfx950: bit-exact byte moves.
//
//  * k_remap<B, EMBED|FLIPH|FLIPV|ROT180>: one lane per output pixel; embed
//    implements every VipsExtend mode (embed.c: COPY clamps, REPEAT tiles with
//    period W, MIRROR tiles the 2x2 [in, flip(in)] mosaic with period 2W,
//    BLACK / WHITE / BACKGROUND fill).  With `origins` set it is an extract at a
//    device-computed (left, top) — smartcrop needs no host round trip.
//  * k_rot90_px<B, CW, 64, TH>: 90 / 270 for 3- and 4-band images through a
//    pixel-major LDS tile (4 pixels per lane both ways); k_rot90_lds<B, CW, TH, T> for
//    1-2 bands; k_rot90t<B, CW> (32 x 32 tiles) past 2 GB per image.
//  * k_extract_rows: row copies, dword lanes when rows and offset allow.
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device_common.h"

namespace mipx {
namespace {

using namespace dev;

enum RemapKind { kEmbed = 0, kFlipH, kFlipV, kRot180 };

struct RemapArgs {
    const u8 *in;
    u8 *out;
    int w, h, ow, oh;
    int x, y, extend;
    u8 fill[4];
    long long in_img, out_img;
    const int *origins;  // extract with per-image (left, top) from the device (smartcrop)
    int q16;             // k_embed_rows: 16-byte source loads where the row offset is dword aligned
    int rpb;             // k_embed_rows: output rows per block
};

__device__ __forceinline__ uint32_t load_px(const u8 *p, int B) {
    uint32_t v = p[0];
    if (B > 1) v |= static_cast<uint32_t>(p[1]) << 8;
    if (B > 2) v |= static_cast<uint32_t>(p[2]) << 16;
    if (B > 3) v |= static_cast<uint32_t>(p[3]) << 24;
    return v;
}
__device__ __forceinline__ void store_px(u8 *q, uint32_t v, int B) {
    q[0] = static_cast<u8>(v);
    if (B > 1) q[1] = static_cast<u8>(v >> 8);
    if (B > 2) q[2] = static_cast<u8>(v >> 16);
    if (B > 3) q[3] = static_cast<u8>(v >> 24);
}

template <int B, int KIND>
__global__ void __launch_bounds__(256) k_remap(RemapArgs a) {
    const int X = blockIdx.x * blockDim.x + threadIdx.x;
    const int Y = blockIdx.y;
    const int img = blockIdx.z;
    if (X >= a.ow) return;
    int sx = X, sy = Y;
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
    } else if (KIND == kFlipH) {
        sx = a.w - 1 - X;
    } else if (KIND == kFlipV) {
        sy = a.h - 1 - Y;
    } else {  // kRot180
        sx = a.w - 1 - X;
        sy = a.h - 1 - Y;
    }
    u8 *q = a.out + img * a.out_img + (static_cast<size_t>(Y) * a.ow + X) * B;
    uint32_t v;
    if (use_fill) {
        v = a.fill[0] | (a.fill[1] << 8) | (a.fill[2] << 16) | (static_cast<uint32_t>(a.fill[3]) << 24);
    } else {
        const u8 *p = a.in + img * a.in_img + (static_cast<size_t>(sy) * a.w + sx) * B;
        v = B == 4 ? *reinterpret_cast<const uint32_t *>(p) : load_px(p, B);
    }
    if (B == 4) *reinterpret_cast<uint32_t *>(q) = v;
    else store_px(q, v, B);
}

// embed (and device-origin extract), 16 output bytes per lane.  Bytes whose
// pixels all come from one source row's interior are read as aligned dwords +
// v_alignbyte (any pixel offset, any band count); rows wholly outside in a
// fill mode store the fill pattern; border dwords resolve each byte through the
// extend mode.  Needs a dword aligned image base; bit-exact with k_remap<EMBED>.
__device__ __forceinline__ int extend_index(int v, int n, int ext) {  // -1 = fill
    const int c = clampi(v, 0, n - 1);
    const int r = pmod(v, n);
    const int u = pmod(v, 2 * n);
    const int m = u < n ? u : 2 * n - 1 - u;
    const int o = ext == MIPX_EXTEND_COPY ? c : ext == MIPX_EXTEND_REPEAT ? r : ext == MIPX_EXTEND_MIRROR ? m : -1;
    return (v >= 0 && v < n) ? v : o;
}

template <int B>
// fw: the fill bytes packed (byte c = fill[c]), so no per-lane index into the argument
// struct forces it into scratch memory
__device__ __forceinline__ void embed_fetch(const RemapArgs &a, uint32_t fw, int img, int Y, int j0, uint32_t v[4]) {
    int ox = a.x, oy = a.y;
    if (a.origins) {
        ox = -a.origins[2 * img];
        oy = -a.origins[2 * img + 1];
    }
    const int sy = extend_index(Y - oy, a.h, a.extend);
    const u8 *src = a.in + img * a.in_img;
    const __amdgpu_buffer_rsrc_t rs = image_rsrc(src, a.in_img);
    if (sy < 0) {  // fill row: the pattern, phase j mod B
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            uint32_t w = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) w |= ((fw >> (8 * ((j0 + 4 * d + k) % B))) & 0xffu) << (8 * k);
            v[d] = w;
        }
    } else if (j0 / B - ox >= 0 && (j0 + 15) / B - ox < a.w) {  // interior: shifted row copy
        const int o = sy * a.w * B + (j0 - ox * B);
        const int o4 = o & ~3, sh = o & 3;
        if (sh == 0 && a.q16) {  // dword-aligned source: one 16-byte load (r02: was 5 dword loads)
            typedef uint32_t u4v __attribute__((ext_vector_type(4)));
            const u4v t = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
            v[0] = t[0], v[1] = t[1], v[2] = t[2], v[3] = t[3];
        } else {
            uint32_t w[5];
#pragma unroll
            for (int d = 0; d < 5; ++d) w[d] = static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(rs, o4 + 4 * d, 0, 0));
#pragma unroll
            for (int d = 0; d < 4; ++d) v[d] = __builtin_amdgcn_alignbyte(w[d + 1], w[d], sh);  // (hi:lo) >> 8 sh
        }
    } else {
        const long long rowb = static_cast<long long>(sy) * a.w * B;
#pragma unroll 1
        for (int d = 0; d < 4; ++d) {
            uint32_t w = 0;
            for (int k = 0; k < 4; ++k) {
                const int jb = j0 + 4 * d + k;
                const int px = jb / B, c = jb - px * B;
                const int sx = extend_index(px - ox, a.w, a.extend);
                const uint32_t byte = sx < 0 ? (fw >> (8 * c)) & 0xffu : src[rowb + static_cast<long long>(sx) * B + c];
                w |= byte << (8 * k);
            }
            v[d] = w;
        }
    }
}

template <int B, bool NT>
__device__ __forceinline__ void embed_put(const RemapArgs &a, int img, int Y, int j0, const uint32_t v[4]) {
    const int row_out = a.ow * B;
    const int nb = min(16, row_out - j0);
    u8 *q = a.out + img * a.out_img + static_cast<long long>(Y) * row_out + j0;
    if (nb == 16 && ((reinterpret_cast<uintptr_t>(q) & 15u) == 0)) {
        typedef uint32_t u4v __attribute__((ext_vector_type(4)));
        if (NT) __builtin_nontemporal_store(u4v{v[0], v[1], v[2], v[3]}, reinterpret_cast<u4v *>(q));
        else *reinterpret_cast<uint4 *>(q) = uint4{v[0], v[1], v[2], v[3]};
    } else if (nb == 16 && ((reinterpret_cast<uintptr_t>(q) & 3u) == 0)) {
        uint32_t *q32 = reinterpret_cast<uint32_t *>(q);
        q32[0] = v[0], q32[1] = v[1], q32[2] = v[2], q32[3] = v[3];
    } else {
        for (int k = 0; k < nb; ++k) q[k] = static_cast<u8>(v[k >> 2] >> (8 * (k & 3)));
    }
}

template <int B>
__device__ __forceinline__ void embed_chunk(const RemapArgs &a, uint32_t fw, int img, int Y, int j0) {
    uint32_t v[4];
    embed_fetch<B>(a, fw, img, Y, j0, v);
    embed_put<B, false>(a, img, Y, j0, v);
}

// a block: 4 KiB of a.rpb consecutive output rows (r02: 4 rows per block, so a
// border-fill row is not one 16-byte store per lane and wave; MIPX_EMBED_RPB=1 A/B)
template <int B>
__global__ void __launch_bounds__(256) k_embed_rows(RemapArgs a) {
    const int img = blockIdx.z;
    const int j0 = (blockIdx.x * 256 + threadIdx.x) * 16;
    if (j0 >= a.ow * B) return;
    const uint32_t fw = a.fill[0] | (a.fill[1] << 8) | (a.fill[2] << 16) | (static_cast<uint32_t>(a.fill[3]) << 24);
    const int y0 = blockIdx.y * a.rpb, y1 = min(y0 + a.rpb, a.oh);
    for (int Y = y0; Y < y1; ++Y) embed_chunk<B>(a, fw, img, Y, j0);
}

// r03: the same blocks with every row's 16 bytes fetched before any is stored (RPB loads in
// flight per lane instead of one), optionally non-temporal stores
template <int B, int RPB, bool NT>
__global__ void __launch_bounds__(256) k_embed_rows2(RemapArgs a) {
    const int img = blockIdx.z;
    const int j0 = (blockIdx.x * 256 + threadIdx.x) * 16;
    if (j0 >= a.ow * B) return;
    const uint32_t fw = a.fill[0] | (a.fill[1] << 8) | (a.fill[2] << 16) | (static_cast<uint32_t>(a.fill[3]) << 24);
    const int y0 = blockIdx.y * RPB;
    uint32_t v[RPB][4];
#pragma unroll
    for (int k = 0; k < RPB; ++k)
        if (y0 + k < a.oh) embed_fetch<B>(a, fw, img, y0 + k, j0, v[k]);
#pragma unroll
    for (int k = 0; k < RPB; ++k)
        if (y0 + k < a.oh) embed_put<B, NT>(a, img, y0 + k, j0, v[k]);
}

// flip H / flip V / rot 180 as row remaps: output row Y = source row sy
// (Y or h-1-Y), pixels mirrored for H / 180.  A block stages the source bytes
// of its 4 KiB output segment in LDS with dword loads (aligned-down start),
// then each lane gathers its 16 output bytes from LDS and stores them at once.
template <int B, bool MIRROR, bool NT>
__global__ void __launch_bounds__(256) k_flip_rows(const u8 *__restrict__ in, u8 *__restrict__ out, int w, int h,
                                                   int vflip, long long img_bytes_, int rpb) {
    __shared__ __attribute__((aligned(16))) uint32_t seg[1024 + 8];
    const int img = blockIdx.z;
    // rpb output rows per block (r02: 4, like k_embed_rows; MIPX_FLIP_RPB=1 is the r01 grid)
    for (int Y = blockIdx.y * rpb; Y < min((blockIdx.y + 1) * rpb, h); ++Y) {
    if (Y != blockIdx.y * rpb) __syncthreads();  // the previous row's gather is done with seg
    const int row_bytes = w * B;
    const int j0 = blockIdx.x * 4096;              // output byte range [j0, j1) of the row
    const int j1 = min(j0 + 4096, row_bytes);
    const int sy = vflip ? h - 1 - Y : Y;
    // source bytes: pixels mirrored -> [s0, s1)
    const int p0 = j0 / B, p1 = (j1 + B - 1) / B;  // output pixels touched
    const int s0 = MIRROR ? (w - p1) * B : p0 * B;
    const int s1 = MIRROR ? (w - p0) * B : p1 * B;
    int delta = 0;
    const u8 *src = in + img * img_bytes_;
    const __amdgpu_buffer_rsrc_t rs = image_rsrc_aligned(src, img_bytes_, &delta);
    const int abs0 = delta + sy * row_bytes + s0;
    const int a4 = abs0 & ~3, skew = abs0 - a4;
    const int nd = (s1 - s0 + skew + 3) >> 2;  // <= 1026
    {  // one dwordx4 per lane (all in flight at once), the <= 3 spill dwords by lanes 0-2
        const int t = threadIdx.x;
        if (4 * t < nd) {
            typedef uint32_t u4v __attribute__((ext_vector_type(4)));
            const u4v v = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(rs, a4 + 16 * t, 0, 0));
            *reinterpret_cast<uint4 *>(seg + 4 * t) = uint4{v[0], v[1], v[2], v[3]};
        }
        if (t < nd - 1024)
            seg[1024 + t] = static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(rs, a4 + 4096 + 4 * t, 0, 0));
    }
    __syncthreads();
    const u8 *sb = reinterpret_cast<const u8 *>(seg) + skew;
    const int jl = j0 + threadIdx.x * 16;
    if (jl >= j1) continue;
    const int nb = min(16, j1 - jl);
    uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if (k < nb) {
            const int jb = jl + k;
            const int px = jb / B, c = jb - px * B;
            const int sbyte = MIRROR ? (w - 1 - px) * B + c - s0 : jb - s0;
            v[k >> 2] |= static_cast<uint32_t>(sb[sbyte]) << (8 * (k & 3));
        }
    }
    u8 *q = out + img * img_bytes_ + static_cast<long long>(Y) * row_bytes + jl;
    if (nb == 16 && (reinterpret_cast<uintptr_t>(q) & 15u) == 0) {
        typedef uint32_t u4v __attribute__((ext_vector_type(4)));
        if (NT) __builtin_nontemporal_store(u4v{v[0], v[1], v[2], v[3]}, reinterpret_cast<u4v *>(q));
        else *reinterpret_cast<uint4 *>(q) = uint4{v[0], v[1], v[2], v[3]};
    } else {
        for (int k = 0; k < nb; ++k) q[k] = static_cast<u8>(v[k >> 2] >> (8 * (k & 3)));
    }
    }
}

// 90 / 270 via 64 x 64 pixel tiles.  Staging: every tile row de-skewed on the way
// into LDS (one b64 load per dword + v_alignbyte, all loads in flight before the
// LDS writes), so a staged row starts exactly at the tile's first pixel.  Gather:
// a task builds 4 output pixels from aligned LDS dword reads, packs them into B
// dwords (v_perm) and stores them as one aligned B-dword write.
// Flat grid, tiles x-fastest; xcd: blocks dealt so that each XCD walks a
// contiguous run of tiles (neighbouring tiles share the 128-byte lines that a
// 3-band tile edge splits, in one L2) instead of round robin.  TH: input rows
// per tile (= contiguous output pixels per output row of the tile).
template <int B, bool CW, int TH, int T>
__global__ void __launch_bounds__(256) k_rot90_lds(const u8 *__restrict__ in, u8 *__restrict__ out, int w, int h,
                                                   long long img_bytes_, int tiles_x, int tiles_y, int xcd, int q16,
                                                   int yfast) {
    constexpr int RS = (T * B + 3) / 4 + 1;  // dwords per staged row (+1: the unaligned pixel read spills)
    __shared__ uint32_t tile[TH * RS];
    const uint32_t t = xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    // yfast: consecutive blocks take consecutive input row bands = neighbouring output
    // column ranges of the same output rows, so split output lines complete in one L2
    int bx, by, img;
    if (yfast) {
        by = static_cast<int>(t % tiles_y);
        const int rest = static_cast<int>(t / tiles_y);
        bx = rest % tiles_x, img = rest / tiles_x;
    } else {
        bx = static_cast<int>(t % tiles_x);
        const int rest = static_cast<int>(t / tiles_x);
        by = rest % tiles_y, img = rest / tiles_y;
    }
    const int tx0 = bx * T, ty0 = by * TH;  // input tile origin
    const int tw = min(T, w - tx0), th = min(TH, h - ty0);
    int delta = 0;
    const u8 *src = in + img * img_bytes_;
    const __amdgpu_buffer_rsrc_t rs = image_rsrc_aligned(src, img_bytes_, &delta);
    const int nd = (tw * B + 3) >> 2;
    if (q16) {  // r02: 16 bytes of a row per item (one b128 + one b32 load, 4 alignbytes)
        const int nq = (nd + 3) >> 2;
        constexpr int kPer = (TH * (((T * B + 3) / 4 + 3) / 4) + 255) / 256;
        uint32_t v[kPer][4];
        int slot[kPer], cnt[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int i = threadIdx.x + 256 * k;
            slot[k] = -1;
            cnt[k] = 0;
            if (i < th * nq) {
                const int r = i / nq, q = i - r * nq;
                const int abs0 = delta + ((ty0 + r) * w + tx0) * B;
                const int o = (abs0 & ~3) + 16 * q;
                typedef uint32_t u4v __attribute__((ext_vector_type(4)));
                const u4v p = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
                const uint32_t e = static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(rs, o + 16, 0, 0));
                const int sh = abs0 & 3;
                v[k][0] = __builtin_amdgcn_alignbyte(p[1], p[0], sh);
                v[k][1] = __builtin_amdgcn_alignbyte(p[2], p[1], sh);
                v[k][2] = __builtin_amdgcn_alignbyte(p[3], p[2], sh);
                v[k][3] = __builtin_amdgcn_alignbyte(e, p[3], sh);
                slot[k] = r * RS + 4 * q;
                cnt[k] = min(4, nd - 4 * q);
            }
        }
#pragma unroll
        for (int k = 0; k < kPer; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (j < cnt[k]) tile[slot[k] + j] = v[k][j];
    } else {
        constexpr int kPer = (TH * ((T * B + 3) / 4) + 255) / 256;
        uint32_t v[kPer];
        int slot[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int i = threadIdx.x + 256 * k;
            slot[k] = -1;
            if (i < th * nd) {
                const int r = i / nd, d = i - r * nd;
                const int abs0 = delta + ((ty0 + r) * w + tx0) * B;
                typedef uint32_t u2v __attribute__((ext_vector_type(2)));
                const u2v p = __builtin_bit_cast(u2v, __builtin_amdgcn_raw_buffer_load_b64(rs, (abs0 & ~3) + 4 * d, 0, 0));
                v[k] = __builtin_amdgcn_alignbyte(p[1], p[0], abs0 & 3);
                slot[k] = r * RS + d;
            }
        }
#pragma unroll
        for (int k = 0; k < kPer; ++k)
            if (slot[k] >= 0) tile[slot[k]] = v[k];
    }
    __syncthreads();
    // output tile: th columns wide (output x <- input y), tw rows tall; 4 output pixels per task
    const int quads = (th + 3) >> 2;
    u8 *dst = out + img * img_bytes_;
    for (int task = threadIdx.x; task < tw * quads; task += 256) {
        const int orr = task / quads, q = task - orr * quads;
        const int icol = CW ? orr : tw - 1 - orr;  // output row within the tile -> input column
        int ox, oy;
        if (CW) {  // out(x, y) = in(y, h-1-x): output row oy = input col, output col ox = h-1-input row
            oy = tx0 + icol;
            ox = h - (ty0 + th);  // output column of the tile's first pixel (input row ty0 + th - 1)
        } else {   // out(x, y) = in(w-1-y, x): output row oy = w-1-input col, output col ox = input row
            oy = w - 1 - (tx0 + icol);
            ox = ty0;
        }
        const int px0 = 4 * q, npx = min(4, th - px0);
        uint32_t P[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int ir = CW ? th - 1 - min(px0 + k, th - 1) : min(px0 + k, th - 1);  // input row within the tile
            const int b0 = icol * B;
            const uint32_t *row = tile + ir * RS + (b0 >> 2);
            P[k] = B == 4 ? row[0] : __builtin_amdgcn_alignbyte(row[1], row[0], b0 & 3);
        }
        uint32_t o[B];
        if (B == 4) {
#pragma unroll
            for (int k = 0; k < B; ++k) o[k] = P[k];
        } else if (B == 3) {
            o[0] = __builtin_amdgcn_perm(P[1], P[0], 0x04020100u);
            o[1 % B] = __builtin_amdgcn_perm(P[2], P[1], 0x05040201u);
            o[2 % B] = __builtin_amdgcn_perm(P[3], P[2], 0x06050402u);
        } else if (B == 2) {
            o[0] = (P[0] & 0xffffu) | (P[1] << 16);
            o[1 % B] = (P[2] & 0xffffu) | (P[3] << 16);
        } else {
            o[0] = (P[0] & 0xffu) | ((P[1] & 0xffu) << 8) | ((P[2] & 0xffu) << 16) | (P[3] << 24);
        }
        u8 *qd = dst + (static_cast<long long>(oy) * h + ox + px0) * B;
        if (npx == 4 && (reinterpret_cast<uintptr_t>(qd) & 3u) == 0) {
            uint32_t *q32 = reinterpret_cast<uint32_t *>(qd);
#pragma unroll
            for (int k = 0; k < B; ++k) q32[k] = o[k];
        } else {
            for (int k = 0; k < npx * B; ++k) qd[k] = static_cast<u8>(o[k >> 2] >> (8 * (k & 3)));
        }
    }
}

// r03: 90 / 270 for 3- and 4-band images through a pixel-major LDS tile of TC input columns x TH
// input rows.  Staging: a lane loads 4 pixels (12 bytes) of an input row and writes them as
// 4 pixel dwords, each into its input column's run of TH dwords (slot = the pixel's place
// in the output row), in 4-slot groups XOR-swizzled by the lane's quad so that the 16
// quads of a row write 16 different bank groups.  Gather: a lane reads one 4-slot group
// with one ds_read_b128 (4 consecutive output pixels), packs them to 3 dwords and stores
// 12 bytes.  The 64 x 64 tiles of k_rot90_lds cap the same access pattern at 55 % of HBM
// in a memory-only replica, 64 x 128 tiles taken row-band fastest at 65 %
// (scripts/strip_probe.hip PROBE_ROT, profiles/r03/rot_probe.jsonl).
template <int B, bool CW, int TC, int TH>
__global__ void __launch_bounds__(256) k_rot90_px(const u8 *__restrict__ in, u8 *__restrict__ out, int w, int h,
                                                  long long img_bytes_, int tiles_x, int tiles_y, int yfast, int al) {
    constexpr int NQ = TC / 4, NG = TH / 4;
    static_assert(TC == 64 && TH % 16 == 0, "16 quads per tile row; whole 256-lane staging rounds");
    static_assert(B == 3 || B == 4, "4 pixels = B dwords");
    __shared__ __attribute__((aligned(16))) uint32_t tile[TC * TH];
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    int bx, by, img;
    if (yfast) {
        by = static_cast<int>(t % tiles_y);
        const int rest = static_cast<int>(t / tiles_y);
        bx = rest % tiles_x, img = rest / tiles_x;
    } else {
        bx = static_cast<int>(t % tiles_x);
        const int rest = static_cast<int>(t / tiles_x);
        by = rest % tiles_y, img = rest / tiles_y;
    }
    const int tx0 = bx * TC, ty0 = by * TH;
    const int tw = min(TC, w - tx0), th = min(TH, h - ty0);
    int delta = 0;
    const __amdgpu_buffer_rsrc_t rs = image_rsrc_aligned(in + img * img_bytes_, img_bytes_, &delta);
    constexpr int KP = TH * NQ / 256;
    uint32_t d[KP][B];
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        const int i = threadIdx.x + 256 * k, r = i / NQ, q = i % NQ;
        const int abs0 = delta + ((ty0 + r) * w + tx0 + 4 * q) * B;
        const bool live = r < th && 4 * q < tw;
        if (B == 4) {  // 4-band images are dword aligned (rot_launch): the 16 bytes are 4 pixels
            typedef uint32_t u4v __attribute__((ext_vector_type(4)));
            const u4v p = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(rs, live ? abs0 : 0x7ffffff0, 0, 0));
#pragma unroll
            for (int j = 0; j < B; ++j) d[k][j] = p[j];
        } else if (al) {  // rows and images on a dword: the 12 bytes are 3 dwords
            typedef uint32_t u3v __attribute__((ext_vector_type(3)));
            const u3v p = __builtin_bit_cast(u3v, __builtin_amdgcn_raw_buffer_load_b96(rs, live ? abs0 : 0x7ffffff0, 0, 0));
#pragma unroll
            for (int j = 0; j < 3; ++j) d[k][j] = p[j];
        } else {
            typedef uint32_t u4v __attribute__((ext_vector_type(4)));
            const u4v p = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(rs, live ? abs0 & ~3 : 0x7ffffff0, 0, 0));
            const int sh = abs0 & 3;
#pragma unroll
            for (int j = 0; j < B && j < 3; ++j) d[k][j] = __builtin_amdgcn_alignbyte(p[j + 1], p[j], sh);
        }
    }
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        const int i = threadIdx.x + 256 * k, r = i / NQ, q = i % NQ;
        if (r >= th || 4 * q >= tw) continue;
        const int s = CW ? th - 1 - r : r;  // slot: the pixel's place in its output row
        const int base = (4 * q) * TH + 4 * ((s >> 2) ^ (q & (NG - 1))) + (s & 3);
        if (B == 4) {
#pragma unroll
            for (int j = 0; j < 4; ++j) tile[base + j * TH] = d[k][j];
        } else {
            tile[base] = d[k][0];
            tile[base + TH] = __builtin_amdgcn_alignbyte(d[k][1], d[k][0], 3);
            tile[base + 2 * TH] = __builtin_amdgcn_alignbyte(d[k][2 % B], d[k][1], 2);
            tile[base + 3 * TH] = d[k][2 % B] >> 8;
        }
    }
    __syncthreads();
    const __amdgpu_buffer_rsrc_t dst = image_rsrc(out + img * img_bytes_, img_bytes_);
    const int ox = CW ? h - (ty0 + th) : ty0;  // output column of slot 0
#pragma unroll
    for (int k = 0; k < TC * NG / 256; ++k) {
        const int task = threadIdx.x + 256 * k, orr = task / NG, g = task % NG;
        if (orr >= tw || 4 * g >= th) continue;
        const int icol = CW ? orr : tw - 1 - orr;
        const int oy = CW ? tx0 + icol : w - 1 - (tx0 + icol);
        typedef uint32_t u4v __attribute__((ext_vector_type(4)));
        const u4v P = *reinterpret_cast<const u4v *>(tile + icol * TH + 4 * (g ^ ((icol >> 2) & (NG - 1))));
        const int off = (oy * h + ox + 4 * g) * B;
        if (B == 4) {
            if (4 * g + 4 <= th) {
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, P), dst, off, 0, 0);
            } else {
#pragma unroll
                for (int j = 0; j < 3; ++j)
                    if (4 * g + j < th) __builtin_amdgcn_raw_buffer_store_b32(P[j], dst, off + 4 * j, 0, 0);
            }
        } else {
            typedef uint32_t u3v __attribute__((ext_vector_type(3)));
            const u3v o{__builtin_amdgcn_perm(P[1], P[0], 0x04020100u), __builtin_amdgcn_perm(P[2], P[1], 0x05040201u),
                        __builtin_amdgcn_perm(P[3], P[2], 0x06050402u)};
            if (4 * g + 4 <= th) {
                __builtin_amdgcn_raw_buffer_store_b96(__builtin_bit_cast(u3v, o), dst, off, 0, 0);
            } else {
                const int nb = (th - 4 * g) * 3;
#pragma unroll
                for (int j = 0; j < 9; ++j)
                    if (j < nb) __builtin_amdgcn_raw_buffer_store_b8(static_cast<u8>(o[j >> 2] >> (8 * (j & 3))), dst, off + j, 0, 0);
            }
        }
    }
}

// 90 (CW) / 270 rotation: out(x, y) = in(y, H-1-x) for CW, in(W-1-y, x) for CCW.
// A block moves one 32 x 32 input tile; rows of the tile are read and rows of
// the transposed tile written, each coalesced.
template <int B, bool CW>
__global__ void __launch_bounds__(256) k_rot90t(const u8 *__restrict__ in, u8 *__restrict__ out, int w, int h,
                                                 long long img_bytes_) {
    __shared__ uint32_t tile[32][33];
    const int img = blockIdx.z;
    const int tx0 = blockIdx.x * 32, ty0 = blockIdx.y * 32;  // input tile origin
    const u8 *src = in + img * img_bytes_;
    u8 *dst = out + img * img_bytes_;
    for (int i = threadIdx.x; i < 32 * 32; i += 256) {
        const int r = i >> 5, c = i & 31;
        const int x = tx0 + c, y = ty0 + r;
        if (x < w && y < h) {
            const u8 *p = src + (static_cast<size_t>(y) * w + x) * B;
            tile[r][c] = B == 4 ? *reinterpret_cast<const uint32_t *>(p) : load_px(p, B);
        }
    }
    __syncthreads();
    // output is h wide, w tall; output row X_out = input column
    for (int i = threadIdx.x; i < 32 * 32; i += 256) {
        const int r = i >> 5, c = i & 31;  // r: output row within tile, c: output column within tile
        int ox, oy, ix, iy;
        if (CW) {   // out(ox, oy) = in(x = oy, y = h-1-ox)
            oy = tx0 + r;
            ix = oy;
            iy = ty0 + (31 - c);
            ox = h - 1 - iy;
        } else {    // out(ox, oy) = in(x = w-1-oy, y = ox)
            ix = tx0 + (31 - r);
            oy = w - 1 - ix;
            iy = ty0 + c;
            ox = iy;
        }
        if (ix < w && iy < h && ix >= tx0 && iy >= ty0) {
            const uint32_t v = tile[iy - ty0][ix - tx0];
            u8 *q = dst + (static_cast<size_t>(oy) * h + ox) * B;
            if (B == 4) *reinterpret_cast<uint32_t *>(q) = v;
            else store_px(q, v, B);
        }
    }
}

__global__ void __launch_bounds__(256) k_extract_rows(const u8 *__restrict__ in, u8 *__restrict__ out,
                                                      int in_row_bytes, int out_row_bytes, int left_bytes, int top,
                                                      long long in_img, long long out_img, int dword) {
    const int y = blockIdx.y;
    const int img = blockIdx.z;
    const u8 *src = in + img * in_img + static_cast<size_t>(top + y) * in_row_bytes + left_bytes;
    u8 *dst = out + img * out_img + static_cast<size_t>(y) * out_row_bytes;
    if (dword == 2) {  // non-temporal stores (the default; MIPX_EXTRACT_NT=0: plain, A/B)
        const uint32_t *s = reinterpret_cast<const uint32_t *>(src);
        uint32_t *d = reinterpret_cast<uint32_t *>(dst);
        for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < out_row_bytes / 4; j += gridDim.x * blockDim.x)
            __builtin_nontemporal_store(s[j], d + j);
    } else if (dword) {
        const uint32_t *s = reinterpret_cast<const uint32_t *>(src);
        uint32_t *d = reinterpret_cast<uint32_t *>(dst);
        for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < out_row_bytes / 4; j += gridDim.x * blockDim.x)
            d[j] = s[j];
    } else {
        for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < out_row_bytes; j += gridDim.x * blockDim.x)
            dst[j] = src[j];
    }
}

int remap_launch(int kind, const RemapArgs &a, int b, int n, hipStream_t st) {
    dim3 grid((a.ow + 255) / 256, a.oh, n);
#define MIPX_REMAP(KIND) \
    MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_remap<B_, KIND>), grid, dim3(256), 0, st, a))
    switch (kind) {
        case kEmbed: MIPX_REMAP(kEmbed); break;
        case kFlipH: MIPX_REMAP(kFlipH); break;
        case kFlipV: MIPX_REMAP(kFlipV); break;
        case kRot180: MIPX_REMAP(kRot180); break;
        default: return MIPX_EINVAL;
    }
#undef MIPX_REMAP
    return launch_check("k_remap");
}

bool aligned4(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 3u) == 0; }

// Device-to-device copy of a whole batch (a plan with no steps, flatten of an image without
// alpha, a 1.0 reduce, B_W of 1-2 bands): 4 x 16 bytes per lane in flight, consecutive
// lanes on consecutive 16-byte chunks; the bytes past the last whole chunk by block 0.
typedef uint32_t cp_u4 __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ void __launch_bounds__(256) k_copy16(const cp_u4 *__restrict__ in, cp_u4 *__restrict__ out, long long n16,
                                                const u8 *__restrict__ tin, u8 *__restrict__ tout, int tail) {
    const long long i0 = static_cast<long long>(blockIdx.x) * 1024 + threadIdx.x;
    cp_u4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (i0 + 256 * k < n16) v[k] = NT ? __builtin_nontemporal_load(in + i0 + 256 * k) : in[i0 + 256 * k];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (i0 + 256 * k >= n16) continue;
        if (NT) __builtin_nontemporal_store(v[k], out + i0 + 256 * k);
        else out[i0 + 256 * k] = v[k];
    }
    if (blockIdx.x == 0 && static_cast<int>(threadIdx.x) < tail) tout[threadIdx.x] = tin[threadIdx.x];
}

}  // namespace

int embed_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int x, int y, int ow, int oh, int extend,
                 const int *bg, const int *d_origins, hipStream_t st) {
    RemapArgs a{};
    a.in = in;
    a.out = out;
    a.w = w;
    a.h = h;
    a.ow = ow;
    a.oh = oh;
    a.x = x;
    a.y = y;
    if (extend == MIPX_EXTEND_LAST) extend = MIPX_EXTEND_BACKGROUND;  // bimg vipsEmbed: extend > 5
    a.extend = extend;
    for (int z = 0; z < 4; ++z) a.fill[z] = 0;
    if (extend == MIPX_EXTEND_WHITE)
        for (int z = 0; z < 4; ++z) a.fill[z] = 255;
    if (extend == MIPX_EXTEND_BACKGROUND) {
        int b3[3] = {0, 0, 0};
        if (bg) b3[0] = bg[0], b3[1] = bg[1], b3[2] = bg[2];
        for (int z = 0; z < 4; ++z) a.fill[z] = static_cast<uint8_t>(std::min(255, std::max(0, b3[z < 3 ? z : 2])));
        if (b == 4) a.fill[3] = 255;
        if (b <= 2) a.fill[0] = static_cast<uint8_t>(std::min(255, std::max(0, b3[0]))), a.fill[1] = 255;
    }
    a.in_img = img_bytes(w, h, b);
    a.out_img = img_bytes(ow, oh, b);
    a.origins = d_origins;
    const char *eq = tune_env("MIPX_EMBED_Q16");  // A/B: 0 keeps the 5-dword loads
    a.q16 = aligned4(in) && a.in_img % 4 == 0 && !(eq && *eq == '0');
    if (b == 4 && !(aligned4(in) && aligned4(out))) return MIPX_EINVAL;
    if (aligned4(in) && (a.in_img % 4) == 0 && a.in_img < 0x7fffffffLL && oh <= 65535) {
        const char *er = tune_env("MIPX_EMBED_RPB");
        a.rpb = (er && *er) ? std::max(1, std::atoi(er)) : 4;
        const char *ev = tune_env("MIPX_EMBED_V");  // 0: k_embed_rows; 1: fetch-all; 2: + nt stores (A/B)
        const int ver = ev && *ev ? *ev - '0' : 2;
        const dim3 grid((ow * b + 4095) / 4096, (oh + a.rpb - 1) / a.rpb, n);
        if (ver >= 1 && a.rpb == 4) {
            if (ver == 2) {
                MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_embed_rows2<B_, 4, true>), grid, dim3(256), 0, st, a));
            } else {
                MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_embed_rows2<B_, 4, false>), grid, dim3(256), 0, st, a));
            }
            return launch_check("k_embed_rows2");
        }
        MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL(k_embed_rows<B_>, grid, dim3(256), 0, st, a));
        return launch_check("k_embed_rows");
    }
    return remap_launch(kEmbed, a, b, n, st);
}

int flip_rows_launch(const u8 *in, u8 *out, int n, int w, int h, int b, bool mirror, bool vflip, hipStream_t st) {
    if (h > 65535) return MIPX_EUNSUPPORTED;
    const long long ib = img_bytes(w, h, b);
    if (ib >= 0x7fffffffLL) return MIPX_EUNSUPPORTED;
    const char *er = tune_env("MIPX_FLIP_RPB");
    const int rpb = (er && *er) ? std::max(1, std::atoi(er)) : 4;
    const dim3 grid((w * b + 4095) / 4096, (h + rpb - 1) / rpb, n);
    const char *en = tune_env("MIPX_FLIP_NT");  // 1: non-temporal stores (A/B)
    const bool nt = en && *en ? *en == '1' : true;
#define MIPX_FLIP(M_, NT_)                                                                                        \
    MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_flip_rows<B_, M_, NT_>), grid, dim3(256), 0, st, in, out, w, h, \
                                              vflip ? 1 : 0, ib, rpb))
    if (mirror) {
        if (nt) { MIPX_FLIP(true, true); } else { MIPX_FLIP(true, false); }
    } else {
        if (nt) { MIPX_FLIP(false, true); } else { MIPX_FLIP(false, false); }
    }
#undef MIPX_FLIP
    return launch_check("k_flip_rows");
}

int flip_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int vertical, hipStream_t st) {
    if (img_bytes(w, h, b) < 0x7fffffffLL && h <= 65535)
        return flip_rows_launch(in, out, n, w, h, b, !vertical, vertical != 0, st);
    RemapArgs a{};
    a.in = in;
    a.out = out;
    a.w = w;
    a.h = h;
    a.ow = w;
    a.oh = h;
    a.in_img = img_bytes(w, h, b);
    a.out_img = a.in_img;
    if (b == 4 && !(aligned4(in) && aligned4(out))) return MIPX_EINVAL;
    return remap_launch(vertical ? kFlipV : kFlipH, a, b, n, st);
}

int rot_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int angle, hipStream_t st) {
    angle = ((angle % 360) + 360) % 360;
    if (b == 4 && !(aligned4(in) && aligned4(out))) return MIPX_EINVAL;
    if (angle == 0) {
        return device_copy(out, in, static_cast<size_t>(img_bytes(w, h, b)) * n, st);
    }
    if (angle == 180 && img_bytes(w, h, b) < 0x7fffffffLL && h <= 65535)
        return flip_rows_launch(in, out, n, w, h, b, true, true, st);
    const char *epx = tune_env("MIPX_ROT_PX");  // 0: 3-band images on k_rot90_lds (A/B)
    // 4-band images too (profiles/r03/rot_px4_shrink_ntl_ab.jsonl: 1080p RGBA 4.00 -> 4.87 TB/s,
    // 12 MP 3.99 -> 4.67, 4K 5.05 -> 5.01); MIPX_ROT_PX4=0 keeps them on k_rot90_lds (A/B)
    const char *epx4 = tune_env("MIPX_ROT_PX4");
    const bool px4 = b == 4 && !(epx4 && *epx4 == '0');
    if ((angle == 90 || angle == 270) && (b == 3 || px4) && img_bytes(w, h, b) < 0x7fffffffLL && !(epx && *epx == '0')) {
        // input rows per tile (A/B, profiles/r03/rot_px_ab.jsonl): 128 where input rows are a
        // whole number of 128-byte lines (1080p / 4K: 5.0 TB/s against 4.6-4.9 at 32 / 64),
        // 64 where they end mid-line (12 MP, 12000 B: 4.7 against 4.5 at 128)
        const char *eph = tune_env("MIPX_ROT_PXH");
        const int th = eph && *eph ? std::atoi(eph) : (static_cast<long long>(w) * b) % 128 == 0 ? 128 : 64;
        const char *eo = tune_env("MIPX_ROT_ORDER");  // 1: input row bands fastest
        const int yfast = eo && *eo ? *eo == '1' : 1;
        const int tx = (w + 63) / 64, ty = (h + th - 1) / th;
        const long long nblk = static_cast<long long>(tx) * ty * n;
        if (nblk > 0x7fffffffLL) return MIPX_EUNSUPPORTED;
        const long long ib = img_bytes(w, h, b);
        const int al = aligned4(in) && (w * b) % 4 == 0;
        const dim3 grid(static_cast<unsigned>(nblk));
#define MIPX_ROTPX(CW_, TH_)                                                                                       \
    if (b == 3) hipLaunchKernelGGL((k_rot90_px<3, CW_, 64, TH_>), grid, dim3(256), 0, st, in, out, w, h, ib, tx, ty, yfast, al); \
    else hipLaunchKernelGGL((k_rot90_px<4, CW_, 64, TH_>), grid, dim3(256), 0, st, in, out, w, h, ib, tx, ty, yfast, al)
        if (th == 32) {
            if (angle == 90) { MIPX_ROTPX(true, 32); } else { MIPX_ROTPX(false, 32); }
        } else if (th == 64) {
            if (angle == 90) { MIPX_ROTPX(true, 64); } else { MIPX_ROTPX(false, 64); }
        } else {
            if (angle == 90) { MIPX_ROTPX(true, 128); } else { MIPX_ROTPX(false, 128); }
        }
#undef MIPX_ROTPX
        return launch_check("k_rot90_px");
    }
    if ((angle == 90 || angle == 270) && img_bytes(w, h, b) < 0x7fffffffLL) {
        const char *eth = tune_env("MIPX_ROT_TH");
        const int th = eth && *eth ? (std::atoi(eth) == 128 ? 128 : 64) : 64;
        // r03 A/B (profiles/r03/rot_ab.jsonl, same process): input rows a whole number of
        // 128-byte lines (1080p / 4K RGB, 4K RGBA) rotate fastest with 64-column tiles taken
        // row-band fastest (+4 / +9 / +8 %), rows that end mid-line (12 MP RGB: 12000 B)
        // with 128-column tiles column-fastest (+47 %)
        const bool line_rows = (static_cast<long long>(w) * b) % 128 == 0;
        const char *etc = tune_env("MIPX_ROT_T");  // input columns per tile: 64 / 128 (A/B)
        const int tc = th == 64 && (etc && *etc ? std::atoi(etc) == 128 : !line_rows) ? 128 : 64;
        const char *eo = tune_env("MIPX_ROT_ORDER");  // 1: input row bands fastest (A/B)
        const int yfast = eo && *eo ? *eo == '1' : line_rows;
        const int tx = (w + tc - 1) / tc, ty = (h + th - 1) / th;
        const long long nblk = static_cast<long long>(tx) * ty * n;
        if (nblk > 0x7fffffffLL) return MIPX_EUNSUPPORTED;
        const dim3 grid(static_cast<unsigned>(nblk));
        const long long ib = img_bytes(w, h, b);
        const char *ex = tune_env("MIPX_ROT_XCD");
        // A/B (profiles/r01/v18/rotxcd_ab.jsonl): contiguous runs win 3-8% on 4K RGB, where a
        // 64-pixel tile row (192 B) splits a 128-byte line, and lose 2% on RGBA (whole lines)
        const int xcd = ex && *ex ? (*ex != '0') : ((64 * b) % 128 != 0);
        const char *eq = tune_env("MIPX_ROT_Q16");  // A/B: 0 keeps the b64-per-dword staging
        const int q16 = !(eq && *eq == '0');
#define MIPX_ROT(CW_, TH_, T_)                                                                                 \
    MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_rot90_lds<B_, CW_, TH_, T_>), grid, dim3(256), 0, st, in, out, w, h, \
                                              ib, tx, ty, xcd, q16, yfast))
        if (th == 128) {
            if (angle == 90) { MIPX_ROT(true, 128, 64); } else { MIPX_ROT(false, 128, 64); }
        } else if (tc == 128) {
            if (angle == 90) { MIPX_ROT(true, 64, 128); } else { MIPX_ROT(false, 64, 128); }
        } else {
            if (angle == 90) { MIPX_ROT(true, 64, 64); } else { MIPX_ROT(false, 64, 64); }
        }
#undef MIPX_ROT
        return launch_check("k_rot90_lds");
    }
    if (angle == 180) {
        RemapArgs a{};
        a.in = in;
        a.out = out;
        a.w = a.ow = w;
        a.h = a.oh = h;
        a.in_img = a.out_img = img_bytes(w, h, b);
        return remap_launch(kRot180, a, b, n, st);
    }
    if (angle != 90 && angle != 270) return MIPX_EINVAL;
    dim3 grid((w + 31) / 32, (h + 31) / 32, n);
    const long long ib = img_bytes(w, h, b);
    if (angle == 90) {
        MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_rot90t<B_, true>), grid, dim3(256), 0, st, in, out, w, h, ib));
    } else {
        MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_rot90t<B_, false>), grid, dim3(256), 0, st, in, out, w, h, ib));
    }
    return launch_check("k_rot90t");
}

int device_copy(void *dst, const void *src, size_t bytes, hipStream_t st) {
    const char *ec = tune_env("MIPX_COPY");  // 0: hipMemcpyAsync (A/B)
    if (bytes == 0) return MIPX_OK;
    // A/B (profiles/r03/copy_ab.jsonl): k_copy16 with non-temporal loads and stores moves 4K /
    // 1080p / 12 MP RGB batches at 6.2-6.3 TB/s against 5.2-5.3 for hipMemcpyAsync (5.6-5.7 with
    // plain stores); a 16 MB batch, which the caches hold, copies faster through hipMemcpyAsync
    const bool small = bytes < (64u << 20) && !(ec && *ec);
    if (small || (ec && *ec == '0') || ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15u) ||
        bytes / 16 / 1024 >= 0x7fffffffULL) {
        MIPX_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
        return MIPX_OK;
    }
    const long long n16 = static_cast<long long>(bytes / 16);
    const int tail = static_cast<int>(bytes % 16);
    const dim3 grid(static_cast<unsigned>(std::max(1LL, (n16 + 1023) / 1024)));
    const u8 *tin = static_cast<const u8 *>(src) + 16 * n16;
    u8 *tout = static_cast<u8 *>(dst) + 16 * n16;
    if (ec && *ec == '2')  // plain (temporal) loads and stores (A/B)
        hipLaunchKernelGGL(k_copy16<false>, grid, dim3(256), 0, st, static_cast<const cp_u4 *>(src), static_cast<cp_u4 *>(dst),
                           n16, tin, tout, tail);
    else
        hipLaunchKernelGGL(k_copy16<true>, grid, dim3(256), 0, st, static_cast<const cp_u4 *>(src), static_cast<cp_u4 *>(dst),
                           n16, tin, tout, tail);
    return launch_check("k_copy16");
}

int extract_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int left, int top, int ow, int oh,
                   hipStream_t st) {
    const int in_row = w * b, out_row = ow * b, lb = left * b;
    const int dword = (in_row % 4 == 0) && (out_row % 4 == 0) && (lb % 4 == 0) && aligned4(in) && aligned4(out);
    // any other alignment: an embed whose window lies inside the image (every byte from the
    // interior path, 16 bytes per lane) rather than one byte per thread
    if (!dword && (b != 4 || (aligned4(in) && aligned4(out))))
        return embed_launch(in, out, n, w, h, b, -left, -top, ow, oh, MIPX_EXTEND_COPY, nullptr, nullptr, st);
    dim3 grid(std::max(1, std::min((out_row / (dword ? 4 : 1) + 255) / 256, 64)), oh, n);
    // non-temporal stores by default: 4K RGB -> 2000x1500 +11 %, 1080p -> 1000x700 +57 %, 12 MP
    // RGBA -> 3001x2000 +9 % (profiles/r04/extract_nt_ab.jsonl); MIPX_EXTRACT_NT=0 keeps plain stores (A/B)
    const char *en = tune_env("MIPX_EXTRACT_NT");
    const int mode = dword && !(en && *en == '0') ? 2 : dword;
    hipLaunchKernelGGL(k_extract_rows, grid, dim3(256), 0, st, in, out, in_row, out_row, lb, top, img_bytes(w, h, b),
                       img_bytes(ow, oh, b), mode);
    return launch_check("k_extract_rows");
}

}  // namespace mipx
