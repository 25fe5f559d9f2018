// k_blur.hip — libvips vips_gaussblur on gfx950.
//
// gaussblur.c builds the integer separable mask (vips_gaussmat, precision
// integer: rint(20 exp(-x^2 / 2 sigma^2)), scale = sum) and convsep.c runs the
// horizontal 1 x n mask then the vertical one through convi.c: uchar result
// (sum + (scale + 1) / 2) / scale, clipped, edges EXTEND_COPY, uchar
// intermediate (restated in oracle/vips_ref.c).  Both passes are the generic
// separable kernels of k_sep.hip (k_hpass -> k_vpass, conv rounding).
#include <hip/hip_runtime.h>

#include <vector>

#include "device_common.h"

namespace mipx {
using dev::u8;

int blur_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double sigma, double min_ampl, void *ws,
                size_t ws_bytes, hipStream_t st) {
    return blur_window_launch(in, out, n, w, h, b, 0, 0, w, h, sigma, min_ampl, ws, ws_bytes, st);
}

// gaussblur of the (left, top, ow x oh) window of each w x h image: the extract
// that precedes a blur in a plan folds into the horizontal pass (the blur's
// COPY edge is the window's edge, exactly as after vips_extract_area).
int blur_window_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int left, int top, int ow, int oh,
                       double sigma, double min_ampl, void *ws, size_t ws_bytes, hipStream_t st) {
    (void)h;
    SepSpec spec;
    std::vector<int> mask;
    int scale = 0;
    if (gaussmat(sigma, min_ampl, mask, scale) < 0) return MIPX_EINVAL;
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
