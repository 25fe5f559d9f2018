// k_smartcrop.hip — libvips vips_smartcrop(INTERESTING_ATTENTION) on gfx950.
//
// smartcrop.c vips_smartcrop_attention: vips_resize() to ~32 px, then on that
// tiny image: sRGB -> scRGB -> XYZ, edge = |5 Laplacian(Y)|, skin score, Lab
// saturation, both masked to Y > 5, summed, gaussblur(sigma), argmax, crop
// centred there and clipped.  The resize runs on the shrink / reduce kernels;
// the scorer is one workgroup per image that keeps the exact IEEE operation
// order of the libvips float/double pipeline (explicit _rn intrinsics, no
// contraction), so the crop origin is identical to the oracle's; the origin
// stays on the device and the extract reads it there.
#include <hip/hip_runtime.h>

#include <cmath>
#include <vector>

#include "device_common.h"

namespace mipx {
namespace {

using namespace dev;

constexpr int kMaxMask = 255;

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
    const float nq = static_cast<float>(static_cast<double>(fmul_rn(100000.0f, v)) / white);
    const int i = clampi(static_cast<int>(nq), 0, kQuantElements - 2);
    const float f = fsub_rn(nq, static_cast<float>(i));
    return fadd_rn(tab[i], fmul_rn(f, fsub_rn(tab[i + 1], tab[i])));
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
        const float R = fmul_rn(a.v2y[p[0]], 100.0f);
        const float G = fmul_rn(a.v2y[p[1]], 100.0f);
        const float Bc = fmul_rn(a.v2y[p[2]], 100.0f);
        const float X = static_cast<float>(dadd_rn(dadd_rn(dmul_rn(0.4124, R), dmul_rn(0.3576, G)), dmul_rn(0.1805, Bc)));
        const float Y = static_cast<float>(dadd_rn(dadd_rn(dmul_rn(0.2126, R), dmul_rn(0.7152, G)), dmul_rn(0.0722, Bc)));
        const float Z = static_cast<float>(dadd_rn(dadd_rn(dmul_rn(0.0193, R), dmul_rn(0.1192, G)), dmul_rn(0.9505, Bc)));
        sY[i] = Y;
        float sq = fmul_rn(X, X);
        sq = fadd_rn(sq, fmul_rn(Y, Y));
        sq = fadd_rn(sq, fmul_rn(Z, Z));
        const float mag = static_cast<float>(sqrt(static_cast<double>(sq)));
        const float nx = mag == 0.0f ? 0.0f : fdiv_rn(X, mag);
        const float ny = mag == 0.0f ? 0.0f : fdiv_rn(Y, mag);
        const float nz = mag == 0.0f ? 0.0f : fdiv_rn(Z, mag);
        const float dx = fadd_rn(nx, -0.78f), dy = fadd_rn(ny, -0.57f), dz = fadd_rn(nz, -0.44f);
        float d2 = fmul_rn(dx, dx);
        d2 = fadd_rn(d2, fmul_rn(dy, dy));
        d2 = fadd_rn(d2, fmul_rn(dz, dz));
        const float dist = static_cast<float>(sqrt(static_cast<double>(d2)));
        const bool bright = static_cast<double>(Y) > 5.0;
        sA[i] = bright ? fadd_rn(fmul_rn(-100.0f, dist), 100.0f) : 0.0f;
        const float cbx = lab_cbrt(a.cbrt, X, 95.047), cby = lab_cbrt(a.cbrt, Y, 100.0);
        sB[i] = bright ? static_cast<float>(500.0 * static_cast<double>(fsub_rn(cbx, cby))) : 0.0f;
    }
    __syncthreads();
    // pass 2: score = (edge + skin) + sat into sC
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const int y = i / W, x = i - y * W;
        double acc = 0.0;
        acc = dadd_rn(acc, -1.0 * sY[clampi(y - 1, 0, H - 1) * W + x]);
        acc = dadd_rn(acc, -1.0 * sY[y * W + clampi(x - 1, 0, W - 1)]);
        acc = dadd_rn(acc, 4.0 * sY[i]);
        acc = dadd_rn(acc, -1.0 * sY[y * W + clampi(x + 1, 0, W - 1)]);
        acc = dadd_rn(acc, -1.0 * sY[clampi(y + 1, 0, H - 1) * W + x]);
        const float edge = fabsf(fadd_rn(fmul_rn(5.0f, static_cast<float>(acc / 1.0 + 0.0)), 0.0f));
        sC[i] = fadd_rn(fadd_rn(edge, sA[i]), sB[i]);
    }
    __syncthreads();
    // pass 3: horizontal blur sC -> sB, vertical blur sB -> argmax
    const int half = a.n_mask / 2;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const int y = i / W, x = i - y * W;
        double s = 0.0;
        for (int t = 0; t < a.n_mask; ++t)
            s = dadd_rn(s, static_cast<double>(a.mask[t]) * sC[y * W + clampi(x + t - half, 0, W - 1)]);
        sB[i] = static_cast<float>(s / a.mask_scale + 0.0);
    }
    __syncthreads();
    float best = -INFINITY;
    int bidx = 0x7fffffff;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const int y = i / W, x = i - y * W;
        double s = 0.0;
        for (int t = 0; t < a.n_mask; ++t)
            s = dadd_rn(s, static_cast<double>(a.mask[t]) * sB[clampi(y + t - half, 0, H - 1) * W + x]);
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


}  // namespace

size_t smartcrop_workspace_bytes(int n, int w, int h, int bands) {
    ResizeSchedule s;
    if (resize_schedule(w, h, 32.0 / w, 32.0 / h, s)) return 0;
    const size_t a = align_up(static_cast<size_t>(n) * s.w1 * s.h1 * bands);
    const size_t b = align_up(static_cast<size_t>(n) * s.w1 * s.h2 * bands);
    const size_t c = align_up(static_cast<size_t>(n) * s.w2 * s.h2 * bands);
    return a + b + c + align_up(static_cast<size_t>(n) * 2 * sizeof(int));
}

int smartcrop_origins(const u8 *in, int *origins, int n, int w, int h, int b, int cw, int ch, void *ws,
                      size_t ws_bytes, hipStream_t st) {
    if (b < 3) return MIPX_EUNSUPPORTED;
    if (cw <= 0 || ch <= 0 || cw > w || ch > h) return MIPX_EINVAL;
    ResizeSchedule s;
    int e = resize_schedule(w, h, 32.0 / w, 32.0 / h, s);
    if (e) return e;
    if (s.w2 * s.h2 > kScoreMaxPx) return MIPX_EUNSUPPORTED;
    const size_t need = smartcrop_workspace_bytes(n, w, h, b);
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
    return launch_check("k_smartcrop_score");
}

int smartcrop_extract(const u8 *in, u8 *out, int n, int w, int h, int b, int cw, int ch, void *ws,
                      size_t ws_bytes, hipStream_t st) {
    const size_t need = smartcrop_workspace_bytes(n, w, h, b);
    if (!ws || ws_bytes < need) return MIPX_EINVAL;
    int *origins = reinterpret_cast<int *>(static_cast<u8 *>(ws) + need - align_up(static_cast<size_t>(n) * 2 * sizeof(int)));
    int e = smartcrop_origins(in, origins, n, w, h, b, cw, ch, ws, ws_bytes, st);
    if (e) return e;
    return embed_launch(in, out, n, w, h, b, 0, 0, cw, ch, MIPX_EXTEND_BLACK, nullptr, origins, st);
}

}  // namespace mipx
