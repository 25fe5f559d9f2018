// k_affine.hip — libvips vips_affine (bicubic interpolator) and vips_zoom on
// gfx950.  bimg reaches them for Enlarge (image.go:202, vipsAffine with the
// default bicubic interpolator and o.Extend) and Zoom (image.go:286,
// vips_zoom(zoom + 1)).
//
// Affine (scale only, as bimg uses it): output pixel (x, y) samples input
// X = (x + 0.5) / xscale - 0.5 (centre convention, affine.c), shifted by the
// interpolator's window offset 1; phase ((int(X*256) & 255) + 1) >> 1 of the
// 129-entry Catmull-Rom table (x 4096, truncated), 4 x 4 window through the
// input embed's extend mode.  uchar arithmetic as bicubic.cpp: each of the 4
// rows -> (sum + 2048) >> 12, then the column of those -> (sum + 2048) >> 12,
// clipped — all int32 (restated in oracle/vips_ref.c ref_affine).
#include <hip/hip_runtime.h>

#include <cmath>

#include "device_common.h"

namespace mipx {
namespace {

using namespace dev;

struct AffineArgs {
    const u8 *in;
    u8 *out;
    int w, h, ow, oh, extend, fill;
    double xscale, yscale;
    const int *tab;  // 129 x 4
    long long in_img, out_img;
};

__device__ __forceinline__ int extend_idx(int v, int n, int ext) {  // -1 = fill
    const int c = clampi(v, 0, n - 1);
    const int r = pmod(v, n);
    const int u = pmod(v, 2 * n);
    const int m = u < n ? u : 2 * n - 1 - u;
    const int o = ext == MIPX_EXTEND_COPY ? c : ext == MIPX_EXTEND_REPEAT ? r : ext == MIPX_EXTEND_MIRROR ? m : -1;
    return (v >= 0 && v < n) ? v : o;
}

__device__ __forceinline__ double affine_pos(int o, double scale) { return (o + 0.5) / scale - 0.5 + 1.0; }
__device__ __forceinline__ int ufr(int v) { return (v + (kInterpScale >> 1)) >> kInterpShift; }

template <int B>
__global__ void __launch_bounds__(256) k_affine(AffineArgs a) {
    __shared__ int tab[(kTransformScale + 1) * 4];
    for (int i = threadIdx.x; i < (kTransformScale + 1) * 4; i += 256) tab[i] = a.tab[i];
    __syncthreads();
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int y = blockIdx.y;
    const int img = blockIdx.z;
    if (x >= a.ow) return;
    const double Y = affine_pos(y, a.yscale);
    const int iy = static_cast<int>(Y);
    const int ty = ((static_cast<int>(Y * 256.0) & 255) + 1) >> 1;
    const double X = affine_pos(x, a.xscale);
    const int ix = static_cast<int>(X);
    const int tx = ((static_cast<int>(X * 256.0) & 255) + 1) >> 1;
    const int *cx = tab + tx * 4, *cy = tab + ty * 4;
    int rows[4], cols[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        rows[j] = extend_idx(iy - 2 + j, a.h, a.extend);
        cols[j] = extend_idx(ix - 2 + j, a.w, a.extend);
    }
    const u8 *src = a.in + img * a.in_img;
    u8 *q = a.out + img * a.out_img + (static_cast<long long>(y) * a.ow + x) * B;
#pragma unroll
    for (int c = 0; c < B; ++c) {
        int r[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            int sum = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int p = (rows[j] < 0 || cols[i] < 0)
                                  ? a.fill
                                  : src[(static_cast<long long>(rows[j]) * a.w + cols[i]) * B + c];
                sum += cx[i] * p;
            }
            r[j] = ufr(sum);
        }
        const int v = ufr(cy[0] * r[0] + cy[1] * r[1] + cy[2] * r[2] + cy[3] * r[3]);
        q[c] = static_cast<u8>(clampi(v, 0, 255));
    }
}

// vips_zoom: 16 output bytes per lane, each the byte of the replicated pixel
template <int B>
__global__ void __launch_bounds__(256) k_zoom(const u8 *__restrict__ in, u8 *__restrict__ out, int w, int ow,
                                              int xf, int yf, long long in_img, long long out_img) {
    const int Y = blockIdx.y;
    const int img = blockIdx.z;
    const int row_out = ow * B;
    const int j0 = (blockIdx.x * 256 + threadIdx.x) * 16;
    if (j0 >= row_out) return;
    const u8 *src = in + img * in_img + static_cast<long long>(Y / yf) * w * B;
    u8 *q = out + img * out_img + static_cast<long long>(Y) * row_out + j0;
    const int nb = min(16, row_out - j0);
    uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if (k < nb) {
            const int jb = j0 + k;
            const int px = jb / B, c = jb - px * B;
            v[k >> 2] |= static_cast<uint32_t>(src[(px / xf) * B + c]) << (8 * (k & 3));
        }
    }
    if (nb == 16 && (reinterpret_cast<uintptr_t>(q) & 15u) == 0) {
        *reinterpret_cast<uint4 *>(q) = uint4{v[0], v[1], v[2], v[3]};
    } else {
        for (int k = 0; k < nb; ++k) q[k] = static_cast<u8>(v[k >> 2] >> (8 * (k & 3)));
    }
}

}  // namespace

int affine_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double xs, double ys, int extend,
                  hipStream_t st) {
    AffineArgs a{};
    a.in = in;
    a.out = out;
    a.w = w;
    a.h = h;
    a.ow = static_cast<int>(std::ceil(w * xs));
    a.oh = static_cast<int>(std::ceil(h * ys));
    if (extend > 5) extend = MIPX_EXTEND_BACKGROUND;
    a.extend = extend;
    a.fill = extend == MIPX_EXTEND_WHITE ? 255 : 0;  // affine background defaults to black
    a.xscale = xs;
    a.yscale = ys;
    a.tab = device_bicubic_table();
    if (!a.tab) return MIPX_EDEVICE;
    a.in_img = img_bytes(w, h, b);
    a.out_img = img_bytes(a.ow, a.oh, b);
    if (a.oh > 65535) return MIPX_EUNSUPPORTED;
    const dim3 grid((a.ow + 255) / 256, a.oh, n);
    MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL(k_affine<B_>, grid, dim3(256), 0, st, a));
    return launch_check("k_affine");
}

int zoom_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int xf, int yf, hipStream_t st) {
    const int ow = w * xf, oh = h * yf;
    if (oh > 65535) return MIPX_EUNSUPPORTED;
    const dim3 grid((ow * b + 4095) / 4096, oh, n);
    MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL(k_zoom<B_>, grid, dim3(256), 0, st, in, out, w, ow, xf, yf,
                                              img_bytes(w, h, b), img_bytes(ow, oh, b)));
    return launch_check("k_zoom");
}

}  // namespace mipx
