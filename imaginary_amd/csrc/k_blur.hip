// k_blur.hip — libvips vips_gaussblur on gfx950.
//
// gaussblur.c builds the integer separable mask (vips_gaussmat, precision
// integer: rint(20 exp(-x^2 / 2 sigma^2)), scale = sum) and convsep.c runs the
// horizontal 1 x n mask then the vertical one through convi.c: uchar result
// (sum + (scale + 1) / 2) / scale, clipped, edges EXTEND_COPY, uchar
// intermediate (restated in oracle/vips_ref.c).  Both passes are the generic
// separable kernels of k_sep.hip (k_hpass -> k_vpass, conv rounding).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <vector>

#include "device_common.h"

namespace mipx {
using dev::u8;

namespace {

using namespace dev;

// ===========================================================================
// k_blur2d<B, NQ>: both convsep passes in one launch.  A block = up to 256
// output pixels (one per lane) x kb output rows of one image, walked one 4-row
// quad at a time:
//   * the 4 input rows of the next quad (horizontal halo included, COPY edge by
//     clamped columns / rows) are loaded into registers while the current quad
//     computes, then written to LDS as 4-pixel groups already transposed
//     (dword c = channel c of 4 pixels);
//   * each lane runs the horizontal mask for its pixel on the 4 rows (NQ groups
//     x B v_dot4 per row, with the lane's phase-shifted tap set), rounds like
//     convi, and transposes its 4 results to one dword per channel;
//   * those quads enter a register ring of NQ quads, and output row 4Q + k is
//     NQ x B v_dot4 against the uniform tap set k.
// The uchar intermediate never leaves the lane that made it: no LDS round trip
// for the vertical pass and no HBM intermediate (libvips materialises one; the
// values are the same).
// ===========================================================================
constexpr int kB2MaxQ = 12;              // taps <= 4 * kB2MaxQ - 6 (sigma <= 12.5 at min_ampl 0.2)
constexpr int kB2MaxG = 64 + kB2MaxQ + 1;  // staged groups per row

struct Blur2DArgs {
    const u8 *in;
    u8 *out;
    int in_pitch;                // bytes between input rows
    long long in_base;           // byte offset of the window origin in an image
    long long in_img, out_img;
    int w, h;                    // window = output size (COPY clamp range)
    int bw, kb;                  // output pixels / rows per block
    int x_blocks, y_blocks;
    int pad, padg;               // taps / 2, and pad rounded up to a whole group
    int out_al4;                 // output rows start dword aligned (B == 4 dword stores)
    uint32_t rnd, mag;           // convi rounding: (acc + rnd) / scale == mulhi(acc + rnd, mag)
    float inv, fofs;             // the same in fp32: floor(acc * inv + fofs), fofs = (rnd + 0.5) * inv
    uint32_t cph[4][kB2MaxQ];    // tap set p: group j, byte b holds tap 4j + b - p
};

struct B2Raw {
    uint32_t d[8];
};

__device__ __forceinline__ long long b2_row(int delta, const Blur2DArgs &a, int r) {
    return delta + a.in_base + static_cast<long long>(r) * a.in_pitch;
}

// issue the loads of the 4-pixel group starting at column x of window row r.
// Both branches assign every slot in the same order (a store whose index
// depends on the branch would push raw[] to scratch).
template <int B>
__device__ __forceinline__ void b2_load(const __amdgpu_buffer_rsrc_t rs, long long row, int w, int x, B2Raw &raw) {
    uint32_t v[8];
    if (x >= 0 && x + 3 < w) {  // interior: 4B bytes as dwords from the aligned-down start (+1 when skewed)
        const int off = static_cast<int>(row + static_cast<long long>(x) * B);
        const int a4 = off & ~3;
        if (B == 4) {
            const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, a4, 0, 0);
            v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
        } else if (B == 3) {
            const auto q = __builtin_amdgcn_raw_buffer_load_b96(rs, a4, 0, 0);
            v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = 0u;
        } else if (B == 2) {
            const auto q = __builtin_amdgcn_raw_buffer_load_b64(rs, a4, 0, 0);
            v[0] = q[0]; v[1] = q[1]; v[2] = 0u; v[3] = 0u;
        } else {
            v[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, a4, 0, 0);
            v[1] = 0u; v[2] = 0u; v[3] = 0u;
        }
        v[4] = (off & 3) ? __builtin_amdgcn_raw_buffer_load_b32(rs, a4 + 4 * B, 0, 0) : 0u;
        if (B < 4) { v[B] = v[4]; v[4] = 0u; }
        v[5] = 0u; v[6] = 0u; v[7] = 0u;
    } else {  // edge group: each pixel from its clamped column, the 2 dwords covering it
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int off = static_cast<int>(row + static_cast<long long>(clampi(x + i, 0, w - 1)) * B);
            v[2 * i] = __builtin_amdgcn_raw_buffer_load_b32(rs, off & ~3, 0, 0);
            v[2 * i + 1] = (off & 3) + B > 4 ? __builtin_amdgcn_raw_buffer_load_b32(rs, (off & ~3) + 4, 0, 0) : 0u;
        }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) raw.d[i] = v[i];
}

// the loaded group as 4 pixel slots (u32 per pixel, channel c in byte c), transposed
template <int B>
__device__ __forceinline__ uint4 b2_finish(long long row, int w, int x, const B2Raw &raw) {
    uint32_t s[4];
    if (x >= 0 && x + 3 < w) {
        const int sh = static_cast<int>(row + static_cast<long long>(x) * B) & 3;
        uint32_t e[4];
#pragma unroll
        for (int i = 0; i < B; ++i) e[i] = __builtin_amdgcn_alignbyte(raw.d[i + 1], raw.d[i], sh);
        if (B == 4) {
            s[0] = e[0]; s[1] = e[1]; s[2] = e[2]; s[3] = e[3];
        } else if (B == 3) {  // p0 = e0[0..2], p1 = e0[3] e1[0..1], p2 = e1[2..3] e2[0], p3 = e2[1..3]
            s[0] = e[0];
            s[1] = __builtin_amdgcn_alignbyte(e[1], e[0], 3);
            s[2] = __builtin_amdgcn_alignbyte(e[2], e[1], 2);
            s[3] = e[2] >> 8;
        } else if (B == 2) {
            s[0] = e[0]; s[1] = e[0] >> 16; s[2] = e[1]; s[3] = e[1] >> 16;
        } else {
            s[0] = e[0]; s[1] = e[0] >> 8; s[2] = e[0] >> 16; s[3] = e[0] >> 24;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int sh = static_cast<int>(row + static_cast<long long>(clampi(x + i, 0, w - 1)) * B) & 3;
            s[i] = __builtin_amdgcn_alignbyte(raw.d[2 * i + 1], raw.d[2 * i], sh);
        }
    }
    uint32_t t[4];
    transpose4x4(s[0], s[1], s[2], s[3], t);
    return make_uint4(t[0], t[1], t[2], t[3]);
}

// (acc + (scale + 1) / 2) / scale: with mag = ceil(2^32 / scale) the high word of
// the product is the exact quotient for every acc + rnd < 2^32 / scale, and the
// masks are non-negative, so acc <= 255 * scale keeps it below 256 (scale <= 4096).
__device__ __forceinline__ uint32_t b2_round(uint32_t acc, const Blur2DArgs &a) {
    return __umulhi(acc + a.rnd, a.mag);
}
// The same in three full-rate fp32 ops (v_mul_hi_u32 is quarter rate): every
// (acc + rnd + 0.5) / scale sits at least 0.5 / scale from an integer, far above
// the error of one fma and one rounded constant (< 2^-15 below 256), so the floor
// is exact; v_cvt_pk_u8_f32 then packs the exact integer into byte C.
template <int C>
__device__ __forceinline__ uint32_t b2_pack_f(uint32_t acc, const Blur2DArgs &a, uint32_t prev) {
    const float v = floorf(__builtin_fmaf(static_cast<float>(acc), a.inv, a.fofs));
    return __builtin_amdgcn_cvt_pk_u8_f32(v, C, prev);
}
template <int B, bool FR>
__device__ __forceinline__ uint32_t b2_pack(const uint32_t *acc, const Blur2DArgs &a) {
    uint32_t m = 0;
    if (FR) {
        m = b2_pack_f<0>(acc[0], a, 0u);
        if (B > 1) m = b2_pack_f<1>(acc[1], a, m);
        if (B > 2) m = b2_pack_f<2>(acc[2], a, m);
        if (B > 3) m = b2_pack_f<3>(acc[3], a, m);
    } else {
#pragma unroll
        for (int c = 0; c < B; ++c) m |= b2_round(acc[c], a) << (8 * c);
    }
    return m;
}

template <int B, int NQ, bool FR>
__global__ void __launch_bounds__(256) k_blur2d(Blur2DArgs a) {
    __shared__ uint4 stg[4][kB2MaxG];
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int xb = t % a.x_blocks;
    const int rest = t / a.x_blocks;
    const int yb = rest % a.y_blocks;
    const int img = rest / a.y_blocks;
    const int tid = threadIdx.x;
    const int x0 = xb * a.bw, y0 = yb * a.kb;
    const int nx = min(a.bw, a.w - x0), ny = min(a.kb, a.h - y0);
    const int base = x0 - a.padg;                              // column of staged group 0
    const int ng = ((nx - 1 + a.padg - a.pad) >> 2) + NQ;      // groups per staged row
    const int nitems = 4 * ng;                                 // (row, group) items per quad
    int delta = 0;
    const __amdgpu_buffer_rsrc_t rs = image_rsrc_aligned(a.in + img * a.in_img, a.in_img, &delta);
    // this lane's output column, first group and horizontal tap set
    const int o = tid + a.padg - a.pad;
    const int g0 = o >> 2, ph = o & 3;
    uint32_t hc[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j)
        hc[j] = ph == 0 ? a.cph[0][j] : ph == 1 ? a.cph[1][j] : ph == 2 ? a.cph[2][j] : a.cph[3][j];
    const int nq_out = (ny + 3) >> 2;
    const int nq_mid = nq_out + NQ - 1;
    const int m0 = y0 - a.pad;                                 // window row of quad 0, row 0
    // ---- prefetch quad 0 ----
    B2Raw raw[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int it = tid + 256 * u;
        if (it < nitems) {
            const int r = it / ng, g = it - r * ng;
            b2_load<B>(rs, b2_row(delta, a, clampi(m0 + r, 0, a.h - 1)), a.w, base + 4 * g, raw[u]);
        }
    }
    uint32_t ring[NQ][B];
#pragma unroll
    for (int j = 0; j < NQ; ++j)
#pragma unroll
        for (int c = 0; c < B; ++c) ring[j][c] = 0u;
    u8 *dst = a.out + img * a.out_img + (static_cast<long long>(y0) * a.w + x0 + tid) * B;
    const bool active = tid < nx;
    for (int q = 0; q < nq_mid; ++q) {
        // ---- stage quad q (loaded last iteration), prefetch quad q + 1 ----
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int it = tid + 256 * u;
            if (it < nitems) {
                const int r = it / ng, g = it - r * ng;
                stg[r][g] = b2_finish<B>(b2_row(delta, a, clampi(m0 + 4 * q + r, 0, a.h - 1)), a.w, base + 4 * g,
                                         raw[u]);
            }
        }
        __syncthreads();
        if (q + 1 < nq_mid) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int it = tid + 256 * u;
                if (it < nitems) {
                    const int r = it / ng, g = it - r * ng;
                    b2_load<B>(rs, b2_row(delta, a, clampi(m0 + 4 * (q + 1) + r, 0, a.h - 1)), a.w, base + 4 * g,
                               raw[u]);
                }
            }
        }
        // ---- horizontal pass: this lane's pixel on the quad's 4 rows ----
        uint32_t mid[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            uint32_t acc[B];
#pragma unroll
            for (int c = 0; c < B; ++c) acc[c] = 0u;
#pragma unroll
            for (int j = 0; j < NQ; ++j) {
                const uint4 v = stg[r][min(g0 + j, kB2MaxG - 1)];
                const uint32_t vc[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int c = 0; c < B; ++c) acc[c] = __builtin_amdgcn_udot4(vc[c], hc[j], acc[c], false);
            }
            mid[r] = b2_pack<B, FR>(acc, a);
        }
        __syncthreads();  // stg is rewritten next iteration
        // ---- the quad joins the ring: one dword per channel, 4 rows ----
#pragma unroll
        for (int j = 0; j + 1 < NQ; ++j)
#pragma unroll
            for (int c = 0; c < B; ++c) ring[j][c] = ring[j + 1][c];
        {
            uint32_t tr[4];
            transpose4x4(mid[0], mid[1], mid[2], mid[3], tr);
#pragma unroll
            for (int c = 0; c < B; ++c) ring[NQ - 1][c] = tr[c];
        }
        if (q < NQ - 1 || !active) continue;
        // ---- vertical pass: output rows 4Q .. 4Q + 3 ----
        const int Q = q - (NQ - 1);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int y = 4 * Q + k;
            if (y >= ny) break;
            uint32_t acc[B];
#pragma unroll
            for (int c = 0; c < B; ++c) acc[c] = 0u;
#pragma unroll
            for (int j = 0; j < NQ; ++j)
#pragma unroll
                for (int c = 0; c < B; ++c) acc[c] = __builtin_amdgcn_udot4(ring[j][c], a.cph[k][j], acc[c], false);
            u8 *p = dst + static_cast<long long>(y) * a.w * B;
            const uint32_t ov = b2_pack<B, FR>(acc, a);
            if (B == 4 && a.out_al4) {
                *reinterpret_cast<uint32_t *>(p) = ov;
            } else {
#pragma unroll
                for (int c = 0; c < B; ++c) p[c] = static_cast<u8>(ov >> (8 * c));
            }
        }
    }
}


// k_bmf (r02: both convsep passes on the matrix cores, 128-pixel blocks) was removed in
// r04: k_bcol (k_bcol.hip) takes every image k_bmf could (RGB / RGBA, <= 33 taps, dword
// rows) and is faster there (profiles/r03/bcol_*); its records stay under profiles/r02-r03.

}  // namespace

// Fused blur of the (left, top, ow x oh) window; MIPX_EUNSUPPORTED when the
// mask is too tall for the register ring (the caller runs the two passes).
// MIPX_BLUR2D=0 disables it (A/B), MIPX_BLUR2D_ROWS sets the rows per block.
int blur2d_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int left, int top, int ow, int oh,
                  const std::vector<int> &mask, int scale, hipStream_t st) {
    const char *ef = tune_env("MIPX_BLUR2D");
    if (ef && *ef == '0') return MIPX_EUNSUPPORTED;
    const int taps = static_cast<int>(mask.size());
    const int nq = (taps + 6) >> 2;
    if (nq > kB2MaxQ || scale <= 0 || scale > 4096) return MIPX_EUNSUPPORTED;
    for (int m : mask)
        if (m < 0 || m > 255) return MIPX_EUNSUPPORTED;
    Blur2DArgs a{};
    a.in = in;
    a.out = out;
    a.in_pitch = w * b;
    a.in_base = (static_cast<long long>(top) * w + left) * b;
    a.in_img = img_bytes(w, h, b);
    a.out_img = img_bytes(ow, oh, b);
    if (a.in_img >= 0x7fffffffLL - 16) return MIPX_EUNSUPPORTED;
    a.w = ow;
    a.h = oh;
    const int xblk = (ow + 255) / 256;
    a.bw = ((ow + xblk - 1) / xblk + 3) & ~3;
    const char *er = tune_env("MIPX_BLUR2D_ROWS");
    int kb = (er && *er) ? std::atoi(er) : 128;  // 64: +5 %, 32: +14 % (v17/ab_blur2d_c3.log)
    kb = std::max(4, std::min(kb, 1024)) & ~3;
    a.kb = std::min(kb, (oh + 3) & ~3);
    a.x_blocks = (ow + a.bw - 1) / a.bw;
    a.y_blocks = (oh + a.kb - 1) / a.kb;
    a.pad = taps / 2;
    a.padg = (a.pad + 3) & ~3;
    a.out_al4 = (reinterpret_cast<uintptr_t>(out) & 3u) == 0;
    a.rnd = static_cast<uint32_t>((scale + 1) / 2);
    a.mag = static_cast<uint32_t>(((1ULL << 32) + scale - 1) / scale);
    a.inv = 1.0f / static_cast<float>(scale);
    a.fofs = (static_cast<float>(a.rnd) + 0.5f) * a.inv;
    const char *efr = tune_env("MIPX_BLUR2D_FROUND");
    const bool fr = efr && *efr == '1';  // fp32 rounding: 2-3 % slower (v17/ab_blur2d_fround_*.log)
    for (int p = 0; p < 4; ++p)
        for (int j = 0; j < kB2MaxQ; ++j) {
            uint32_t v = 0;
            for (int bb = 0; bb < 4; ++bb) {
                const int tp = 4 * j + bb - p;
                if (tp >= 0 && tp < taps) v |= static_cast<uint32_t>(mask[tp]) << (8 * bb);
            }
            a.cph[p][j] = v;
        }
    const long long blocks = static_cast<long long>(a.x_blocks) * a.y_blocks * n;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    const dim3 grid(static_cast<unsigned>(blocks)), blk(256);
#define MIPX_B2(NQ_)                                                                                  \
    if (fr) { MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_blur2d<B_, NQ_, true>), grid, blk, 0, st, a)) } \
    else { MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_blur2d<B_, NQ_, false>), grid, blk, 0, st, a)) }
    switch (nq) {
        case 1:
        case 2: MIPX_B2(2) break;
        case 3: MIPX_B2(3) break;
        case 4: MIPX_B2(4) break;
        case 5: MIPX_B2(5) break;
        case 6: MIPX_B2(6) break;
        case 7: MIPX_B2(7) break;
        case 8: MIPX_B2(8) break;
        case 9: MIPX_B2(9) break;
        case 10: MIPX_B2(10) break;
        case 11: MIPX_B2(11) break;
        default: MIPX_B2(12) break;
    }
#undef MIPX_B2
    return launch_check("k_blur2d");
}

int blur_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double sigma, double min_ampl, void *ws,
                size_t ws_bytes, hipStream_t st) {
    return blur_window_launch(in, out, n, w, h, b, 0, 0, w, h, sigma, min_ampl, ws, ws_bytes, st);
}

// gaussblur of the (left, top, ow x oh) window of each w x h image: the extract
// that precedes a blur in a plan folds into the horizontal pass (the blur's
// COPY edge is the window's edge, exactly as after vips_extract_area).
int blur_window_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int left, int top, int ow, int oh,
                       double sigma, double min_ampl, void *ws, size_t ws_bytes, hipStream_t st) {
    SepSpec spec;
    std::vector<int> mask;
    int scale = 0;
    if (gaussmat(sigma, min_ampl, mask, scale) < 0) return MIPX_EINVAL;
    const int ec = blur_col_launch(in, out, n, w, h, b, left, top, ow, oh, mask, scale, st);
    if (ec != MIPX_EUNSUPPORTED) return ec;
    const int ef = blur2d_launch(in, out, n, w, h, b, left, top, ow, oh, mask, scale, st);
    if (ef != MIPX_EUNSUPPORTED) return ef;
    if (!sep_spec_gauss(sigma, min_ampl, &spec)) return MIPX_EDEVICE;
    const size_t need = align_up(static_cast<size_t>(n) * ow * oh * b);
    if (!ws || ws_bytes < need) return MIPX_EINVAL;
    u8 *tmp = static_cast<u8 *>(ws);
    SepWindow hw{};
    hw.bands = b;
    hw.in_pitch = w * b;
    hw.in_base = (static_cast<long long>(top) * w + left) * b;
    hw.in_img = img_bytes(w, h, b);
    hw.in_len = ow;
    hw.o0 = 0;
    hw.out_w = ow;
    hw.out_h = oh;
    int e = hpass_launch(in, tmp, n, spec, hw, st);
    if (e) return e;
    SepWindow vw{};
    vw.bands = b;
    vw.in_pitch = ow * b;
    vw.in_base = 0;
    vw.in_img = img_bytes(ow, oh, b);
    vw.in_len = oh;
    vw.o0 = 0;
    vw.out_w = ow;
    vw.out_h = oh;
    return vpass_launch(tmp, out, n, spec, vw, st);
}

}  // namespace mipx
