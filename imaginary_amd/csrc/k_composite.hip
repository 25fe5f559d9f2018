// k_composite.hip — bimg vips_watermark_image on gfx950 (bimg v1.1.9 vips.h):
// alpha 255 band-joined where missing, the watermark embedded BLACK at
// (left, top) on a canvas of the base size, mask = (uchar)(wm_alpha * opacity)
// (vips_linear1 + vips_cast, truncating), ifthenelse blend
// (m * a + (255 - m) * b + 128) / 255 on every band (restated in
// oracle/vips_ref.c).  One lane per output pixel; bit-exact.
#include <hip/hip_runtime.h>

#include "device_common.h"

namespace mipx {
namespace {

using namespace dev;

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
        const float f = fadd_rn(fmul_rn(static_cast<float>(av[BO - 1]), opacity), 0.0f);
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



}  // namespace

int watermark_launch(const u8 *d_base, const u8 *d_wm, u8 *d_out, int n, int w, int h, int bands, int ww, int wh,
                     int wb, int left, int top, float opacity, hipStream_t st) {
    const int bo = (bands == 2 || bands > 3) ? bands : bands + 1;
    const int wo = (wb == 2 || wb > 3) ? wb : wb + 1;
    if (bo != wo) return MIPX_EUNSUPPORTED;
    dim3 grid((w + 255) / 256, h, n);
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


}  // namespace mipx
