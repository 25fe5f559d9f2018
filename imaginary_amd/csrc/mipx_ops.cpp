// mipx_ops.cpp — C-ABI per-op entry points (include/mipx.h mipx_op_*): argument
// checks, workspace accounting and dispatch to the kernel launchers.  Each
// entry point replaces one libvips operation.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "device_common.h"
#include "mipx_internal.h"

namespace mipx {

size_t op_workspace_bytes(int op, int n, int w, int h, int bands, double p0, double p1) {
    if (n <= 0 || w <= 0 || h <= 0 || bands <= 0) return 0;
    switch (op) {
        case MIPX_OP_REDUCE: {  // generic path: reducev intermediate
            if (!(p1 > 1.0) || !(p0 > 1.0)) return 0;
            const int oh = out_size_reduce(h, p1);
            return align_up(static_cast<size_t>(n) * w * oh * bands);
        }
        case MIPX_OP_BLUR: return align_up(static_cast<size_t>(n) * w * h * bands);
        case MIPX_OP_SMARTCROP: return smartcrop_workspace_bytes(n, w, h, bands);
        default: return 0;
    }
}

}  // namespace mipx

using namespace mipx;

extern "C" {

size_t mipx_op_workspace_bytes(int32_t op, int32_t n, int32_t w, int32_t h, int32_t bands, double p0, double p1) {
    return op_workspace_bytes(op, n, w, h, bands, p0, p1);
}

int mipx_op_reducev(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                    double vshrink, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands) || !(vshrink >= 1.0)) return MIPX_EINVAL;
    const SamplingScope sampling;  // one convention for the whole call
    if (vshrink == 1.0) {
        return device_copy(d_out, d_in, static_cast<size_t>(n) * w * h * bands, as_stream(stream));
    }
    return reducev_launch(d_in, d_out, n, w, h, bands, vshrink, as_stream(stream));
}

int mipx_op_reduceh(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                    double hshrink, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands) || !(hshrink >= 1.0)) return MIPX_EINVAL;
    const SamplingScope sampling;  // one convention for the whole call
    if (hshrink == 1.0) {
        return device_copy(d_out, d_in, static_cast<size_t>(n) * w * h * bands, as_stream(stream));
    }
    return reduceh_launch(d_in, d_out, n, w, h, bands, hshrink, as_stream(stream));
}

int mipx_op_reduce(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                   double hshrink, double vshrink, void *d_ws, size_t ws_bytes, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands) || !(hshrink >= 1.0) || !(vshrink >= 1.0))
        return MIPX_EINVAL;
    const SamplingScope sampling;  // one convention for the whole call (the enclosing plan step's, if any)
    hipStream_t st = as_stream(stream);
    if (reduce2_eligible(d_in, w, h, bands, hshrink, vshrink)) return reduce2_launch(d_in, d_out, n, w, h, bands, st);
    if (vshrink == 1.0) return mipx_op_reduceh(d_in, d_out, n, w, h, bands, hshrink, stream);
    if (hshrink == 1.0) return mipx_op_reducev(d_in, d_out, n, w, h, bands, vshrink, stream);
    {  // both axes: one fused launch, intermediate in LDS
        const int e = reduce_one_launch(d_in, d_out, n, w, h, bands, hshrink, vshrink, 0, 0,
                                        out_size_reduce(w, hshrink), out_size_reduce(h, vshrink), st);
        if (e != MIPX_EUNSUPPORTED) return e;
    }
    const size_t need = op_workspace_bytes(MIPX_OP_REDUCE, n, w, h, bands, hshrink, vshrink);
    if (!d_ws || ws_bytes < need) return MIPX_EINVAL;
    uint8_t *t = static_cast<uint8_t *>(d_ws);
    int e = reducev_launch(d_in, t, n, w, h, bands, vshrink, st);
    if (e) return e;
    return reduceh_launch(t, d_out, n, w, out_size_reduce(h, vshrink), bands, hshrink, st);
}

int mipx_op_shrink(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                   int32_t hshrink, int32_t vshrink, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands) || hshrink < 1 || vshrink < 1) return MIPX_EINVAL;
    return shrink_launch(d_in, d_out, n, w, h, bands, hshrink, vshrink, as_stream(stream));
}

int mipx_op_embed(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands, int32_t x,
                  int32_t y, int32_t ow, int32_t oh, int32_t extend, const int32_t *bg, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands) || ow <= 0 || oh <= 0) return MIPX_EINVAL;
    int b3[3] = {0, 0, 0};
    if (bg) b3[0] = bg[0], b3[1] = bg[1], b3[2] = bg[2];
    return embed_launch(d_in, d_out, n, w, h, bands, x, y, ow, oh, extend, b3, nullptr, as_stream(stream));
}

int mipx_op_extract(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                    int32_t left, int32_t top, int32_t ow, int32_t oh, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands)) return MIPX_EINVAL;
    if (left < 0 || top < 0 || ow <= 0 || oh <= 0 || left + ow > w || top + oh > h) {
        set_error("bad extract area %d,%d %dx%d of %dx%d", left, top, ow, oh, w, h);
        return MIPX_EINVAL;
    }
    return extract_launch(d_in, d_out, n, w, h, bands, left, top, ow, oh, as_stream(stream));
}

int mipx_op_rot(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands, int32_t angle,
                void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands)) return MIPX_EINVAL;
    return rot_launch(d_in, d_out, n, w, h, bands, angle, as_stream(stream));
}

int mipx_op_flip(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                 int32_t vertical, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands)) return MIPX_EINVAL;
    return flip_launch(d_in, d_out, n, w, h, bands, vertical, as_stream(stream));
}

int mipx_op_gaussblur(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                      double sigma, double min_ampl, void *d_ws, size_t ws_bytes, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands)) return MIPX_EINVAL;
    return blur_launch(d_in, d_out, n, w, h, bands, sigma, min_ampl, d_ws, ws_bytes, as_stream(stream));
}

int mipx_op_watermark(const uint8_t *d_base, const uint8_t *d_wm, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                      int32_t bands, int32_t ww, int32_t wh, int32_t wb, int32_t left, int32_t top, float opacity,
                      void *stream) {
    if (!d_base || !d_wm || !d_out || !geom_ok(n, w, h, bands) || ww <= 0 || wh <= 0 || wb < 1 || wb > 4)
        return MIPX_EINVAL;
    return watermark_launch(d_base, d_wm, d_out, n, w, h, bands, ww, wh, wb, left, top, opacity, as_stream(stream));
}

int mipx_op_affine(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands, double xscale,
                   double yscale, int32_t extend, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands) || !(xscale > 0) || !(yscale > 0)) return MIPX_EINVAL;
    return affine_launch(d_in, d_out, n, w, h, bands, xscale, yscale, extend, as_stream(stream));
}

int mipx_op_zoom(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands, int32_t xfac,
                 int32_t yfac, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands) || xfac < 1 || yfac < 1) return MIPX_EINVAL;
    return zoom_launch(d_in, d_out, n, w, h, bands, xfac, yfac, as_stream(stream));
}

int mipx_op_flatten(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                    const int32_t *bg, void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands)) return MIPX_EINVAL;
    int b3[3] = {0, 0, 0};
    if (bg) b3[0] = bg[0], b3[1] = bg[1], b3[2] = bg[2];
    return flatten_launch(d_in, d_out, n, w, h, bands, b3, as_stream(stream));
}

int mipx_op_colourspace_bw(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h, int32_t bands,
                           void *stream) {
    if (!d_in || !d_out || !geom_ok(n, w, h, bands)) return MIPX_EINVAL;
    return bw_launch(d_in, d_out, n, w, h, bands, as_stream(stream));
}

int mipx_op_smartcrop_origin(const uint8_t *d_in, int32_t *d_origins, int32_t n, int32_t w, int32_t h, int32_t bands,
                             int32_t cw, int32_t ch, void *d_ws, size_t ws_bytes, void *stream) {
    if (!d_in || !d_origins || !geom_ok(n, w, h, bands)) return MIPX_EINVAL;
    const SamplingScope sampling;  // one convention for the whole call
    return smartcrop_origins(d_in, d_origins, n, w, h, bands, cw, ch, d_ws, ws_bytes, as_stream(stream));
}

}  // extern "C"
