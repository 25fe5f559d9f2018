// k_colour.hip — the end-of-pipeline colour ops bimg runs before encode:
//  * vips_flatten(background) (bimg imageFlatten: PNG input, non-black
//    background, an alpha band): out = (p * a + bg * (255 - a)) / 255 in int
//    arithmetic, alpha dropped (conversion/flatten.c);
//  * vips_colourspace sRGB -> B_W (bimg vipsPreSave, imaginary colorspace=bw,
//    params.go:392): sRGB LUT -> scRGB, Y = 0.2126 R + 0.7152 G + 0.0722 B in
//    double, back through the 8-bit Y -> sRGB LUT with linear interpolation,
//    rint; alpha passes through (colour/sRGB2scRGB.c, scRGB2BW.c).  The float
//    steps keep libvips' operation order with explicit _rn intrinsics (no
//    contraction), so results match the oracle bit for bit.
#include <hip/hip_runtime.h>

#include "device_common.h"

namespace mipx {
namespace {

using namespace dev;

template <int B>
__global__ void __launch_bounds__(256) k_flatten(const u8 *__restrict__ in, u8 *__restrict__ out, long long npx,
                                                 int bg0, int bg1, int bg2) {
    const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= npx) return;
    const u8 *p = in + i * B;
    u8 *q = out + i * (B - 1);
    const int alpha = p[B - 1], nalpha = 255 - alpha;
    const int bg[3] = {bg0, bg1, bg2};
#pragma unroll
    for (int c = 0; c < B - 1; ++c) q[c] = static_cast<u8>((p[c] * alpha + bg[c] * nalpha) / 255);
}

template <int B>
__global__ void __launch_bounds__(256) k_bw(const u8 *__restrict__ in, u8 *__restrict__ out, long long npx,
                                            const float *__restrict__ v2y, const float *__restrict__ y2v) {
    __shared__ float sv2y[256];
    __shared__ float sy2v[257];
    for (int i = threadIdx.x; i < 256; i += 256) sv2y[i] = v2y[i];
    for (int i = threadIdx.x; i < 257; i += 256) sy2v[i] = y2v[i];
    __syncthreads();
    const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= npx) return;
    constexpr int OB = B == 4 ? 2 : 1;
    const u8 *p = in + i * B;
    const float R = sv2y[p[0]], G = sv2y[p[1]], Bl = sv2y[p[2]];
    const double yd = dadd_rn(dadd_rn(dmul_rn(0.2126, R), dmul_rn(0.7152, G)), dmul_rn(0.0722, Bl));
    const float Y = static_cast<float>(yd);
    const float Yf = fmul_rn(Y, 255.0f);
    const int k = clampi(static_cast<int>(Yf), 0, 255);
    const float f = fsub_rn(Yf, static_cast<float>(k));
    const float v = fadd_rn(sy2v[k], fmul_rn(f, fsub_rn(sy2v[k + 1], sy2v[k])));
    u8 *q = out + i * OB;
    q[0] = static_cast<u8>(clampi(static_cast<int>(rintf(v)), 0, 255));
    if (OB == 2) q[1] = p[3];
}

}  // namespace

int flatten_launch(const u8 *in, u8 *out, int n, int w, int h, int b, const int *bg, hipStream_t st) {
    const long long npx = static_cast<long long>(n) * w * h;
    if (b != 2 && b != 4) {  // no alpha band: vips_flatten is a copy
        return device_copy(out, in, static_cast<size_t>(npx) * b, st);
    }
    const int c0 = clampi_host(bg[0]), c1 = clampi_host(bg[1]), c2 = clampi_host(bg[2]);
    const dim3 grid(static_cast<unsigned>((npx + 255) / 256));
    if (b == 2) hipLaunchKernelGGL(k_flatten<2>, grid, dim3(256), 0, st, in, out, npx, c0, c1, c2);
    else hipLaunchKernelGGL(k_flatten<4>, grid, dim3(256), 0, st, in, out, npx, c0, c1, c2);
    return launch_check("k_flatten");
}

int bw_launch(const u8 *in, u8 *out, int n, int w, int h, int b, hipStream_t st) {
    const long long npx = static_cast<long long>(n) * w * h;
    if (b < 3) {  // 1-2 bands are already B_W
        return device_copy(out, in, static_cast<size_t>(npx) * b, st);
    }
    const float *t = device_colour_tables();
    if (!t) return MIPX_EDEVICE;
    const dim3 grid(static_cast<unsigned>((npx + 255) / 256));
    if (b == 3) hipLaunchKernelGGL(k_bw<3>, grid, dim3(256), 0, st, in, out, npx, t, t + 256 + kQuantElements);
    else hipLaunchKernelGGL(k_bw<4>, grid, dim3(256), 0, st, in, out, npx, t, t + 256 + kQuantElements);
    return launch_check("k_bw");
}

}  // namespace mipx
