// mipx_planner.cpp — host-side geometry planner and coefficient tables.
//
// The planner re-states bimg v1.1.9's resizer (resizer.go: rotateAndFlipImage,
// normalizeOperation, imageCalculations, calculateShrink, calculateResidual,
// shrinkOnLoad, shouldTransformImage, transformImage, extractOrEmbedImage,
// calculateCrop, applyEffects, watermarkImageWithAnotherImage) so that the
// engine runs exactly the libvips operation sequence bimg.Resize would run for
// the bimg.Options imaginary builds (reference options.go:128-172, image.go:115-
// 377).  Output geometry is pinned by the reference's own dimension tests
// (image_test.go:8-179, server_test.go:42-366); see tests/test_planner.py.
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "mipx_internal.h"

namespace mipx {

// ---- Lanczos3 tables (libvips resample/reduce*.cpp, templates.h) -----------
int reduce_points(double shrink) { return static_cast<int>(2 * std::rint(3.0 * shrink) + 1); }

static double lanczos3(double x) {
    if (x == 0.0) return 1.0;
    if (x < -3.0 || x > 3.0) return 0.0;
    const double pix = M_PI * x;
    return 3.0 * std::sin(pix) * std::sin(pix / 3.0) / (pix * pix);
}

// Row `phase` of vips_reduce_make_mask(): tap i at (i - (n-2)/2 - x) / shrink,
// normalised to sum 1, then matrixi = matrixf * 4096 with C truncation.
void reduce_table(double shrink, std::vector<int> &t) {
    const int n = reduce_points(shrink);
    t.assign(static_cast<size_t>(n) * (kTransformScale + 1), 0);
    std::vector<double> f(n);
    for (int phase = 0; phase <= kTransformScale; ++phase) {
        const double x = static_cast<float>(phase) / kTransformScale;
        double sum = 0.0;
        for (int i = 0; i < n; ++i) {
            f[i] = lanczos3((i - (n - 2) / 2 - x) / shrink);
            sum += f[i];
        }
        for (int i = 0; i < n; ++i) {
            f[i] /= sum;
            t[static_cast<size_t>(phase) * n + i] = static_cast<int>(f[i] * kInterpScale);
        }
    }
}

static int vips_round(double v) {
    return static_cast<int>(v < 0.0 ? std::ceil(v - 0.5) : std::floor(v + 0.5));
}
int out_size_reduce(int in, double shrink) { return vips_round(in / shrink); }
int out_size_shrink(int in, int shrink) {
    const int o = vips_round(static_cast<double>(in) / shrink);
    return o < 1 ? 1 : o;
}

// ---- gaussmat (libvips create/gaussmat.c, integer precision) ---------------
int gaussmat(double sigma, double min_ampl, std::vector<int> &mask, int &scale) {
    if (!(sigma > 0.0)) return MIPX_EINVAL;
    const double sig2 = 2.0 * sigma * sigma;
    const double mx = 8.0 * sigma;
    const int max_x = static_cast<int>(mx > 5000 ? 5000 : mx);
    int x = 0;
    for (; x < max_x; ++x)
        if (std::exp(-static_cast<double>(x * x) / sig2) < min_ampl) break;
    if (x >= 5000) return MIPX_EINVAL;
    const int width = 2 * (x - 1 > 0 ? x - 1 : 0) + 1;
    mask.resize(width);
    int sum = 0;
    for (int i = 0; i < width; ++i) {
        const int xo = i - width / 2;
        mask[i] = static_cast<int>(std::rint(20.0 * std::exp(-static_cast<double>(xo * xo) / sig2)));
        sum += mask[i];
    }
    scale = sum == 0 ? 1 : sum;
    return width;
}

// ---- colour LUTs (libvips colour/colour.c calcul_tables, XYZ2Lab.c) ---------
namespace {
struct ColourTables {
    float v2y[256];
    std::vector<float> cbrt;
    ColourTables() : cbrt(kQuantElements) {
        for (int i = 0; i < 256; ++i) {
            const float f = static_cast<float>(i) / 255;
            float v;
            if (f <= 0.04045) v = f / 12.92;
            else v = std::pow((f + 0.055) / 1.055, 2.4);
            v2y[i] = v;
        }
        for (int i = 0; i < kQuantElements; ++i) {
            const float y = static_cast<double>(i) / kQuantElements;
            cbrt[i] = y < 0.008856 ? 7.787 * y + (16.0 / 116.0) : std::cbrt(y);
        }
    }
};
const ColourTables &colour() {
    static ColourTables t;
    return t;
}
}  // namespace
const float *v2y8_table() { return colour().v2y; }

// 8-bit linear Y -> sRGB, 257 entries (the last repeated for the interpolation)
const float *y2v8_table() {
    static const std::vector<float> t = [] {
        std::vector<float> v(257);
        for (int i = 0; i < 256; ++i) {
            const float f = i / 255.0f;
            float e;
            if (f <= 0.0031308f) e = 12.92f * f;
            else e = static_cast<float>(1.055 * std::pow(f, 1.0 / 2.4) - 0.055);
            v[i] = 255.0f * e;
        }
        v[256] = v[255];
        return v;
    }();
    return t.data();
}

// vips_interpolate_bicubic matrixi: Catmull-Rom (templates.h
// calculate_coefficients_catmull) x 4096, truncated; 129 phases x 4
void bicubic_table(int *t) {
    for (int x = 0; x <= kTransformScale; ++x) {
        const double p = static_cast<float>(x) / kTransformScale;
        const double cr1 = 1. - p, cr2 = -.5 * p, cr3 = cr1 * cr2;
        const double cone = cr1 * cr3, cfou = p * cr3, cr4 = cfou - cone;
        const double ctwo = cr1 - cr4 + cfou, cthr = p - cfou + cr4;
        const double c[4] = {cone, ctwo, cthr, cfou};
        for (int i = 0; i < 4; ++i) t[x * 4 + i] = static_cast<int>(c[i] * kInterpScale);
    }
}
const float *cbrt_table() { return colour().cbrt.data(); }

// vips_resize(): integer shrink floor(1 / (2 scale)), then residual reducev/h.
int resize_schedule(int w, int h, double hscale, double vscale, ResizeSchedule &s) {
    auto int_shrink = [](double scale) {
        if (scale > 1.0) return 1;
        const int v = static_cast<int>(std::floor(1.0 / (scale * 2)));
        return v < 1 ? 1 : v;
    };
    s.shrink_h = int_shrink(hscale);
    s.shrink_v = int_shrink(vscale);
    s.w1 = w;
    s.h1 = h;
    if (s.shrink_h > 1 || s.shrink_v > 1) {
        s.w1 = out_size_shrink(w, s.shrink_h);
        s.h1 = out_size_shrink(h, s.shrink_v);
        hscale *= s.shrink_h;
        vscale *= s.shrink_v;
    }
    if (hscale < 1.0 / s.w1) hscale = 1.0 / s.w1;
    if (vscale < 1.0 / s.h1) vscale = 1.0 / s.h1;
    if (hscale > 1.0 || vscale > 1.0) return MIPX_EUNSUPPORTED;  // upsizing: affine
    s.reduce_v = vscale < 1.0 ? 1.0 / vscale : 1.0;
    s.reduce_h = hscale < 1.0 ? 1.0 / hscale : 1.0;
    s.h2 = s.reduce_v > 1.0 ? out_size_reduce(s.h1, s.reduce_v) : s.h1;
    s.w2 = s.reduce_h > 1.0 ? out_size_reduce(s.w1, s.reduce_h) : s.w1;
    return MIPX_OK;
}

}  // namespace mipx

// ---------------------------------------------------------------------------
// Planner
// ---------------------------------------------------------------------------
namespace {

using mipx::out_size_reduce;
using mipx::out_size_shrink;

bool has_alpha(int bands) { return bands == 2 || bands > 3; }

// bimg roundFloat
int round_float(double f) {
    return f < 0 ? static_cast<int>(std::ceil(f - 0.5)) : static_cast<int>(std::floor(f + 0.5));
}

class PlanBuilder {
   public:
    explicit PlanBuilder(mipx_plan *p) : p_(p) { std::memset(p_, 0, sizeof(*p_)); }

    int push(int op) {
        if (p_->n_steps >= MIPX_MAX_STEPS) return MIPX_EINVAL;
        mipx_step &s = p_->steps[p_->n_steps++];
        std::memset(&s, 0, sizeof(s));
        s.op = op;
        return MIPX_OK;
    }
    mipx_step &last() { return p_->steps[p_->n_steps - 1]; }
    void geom(int w, int h, int b) {
        last().out_w = w;
        last().out_h = h;
        last().out_bands = b;
        w_ = w;
        h_ = h;
        b_ = b;
    }
    void start(int w, int h, int b) { w_ = w, h_ = h, b_ = b; }
    int w() const { return w_; }
    int h() const { return h_; }
    int b() const { return b_; }
    mipx_plan *plan() { return p_; }

   private:
    mipx_plan *p_;
    int w_ = 0, h_ = 0, b_ = 0;
};

// bimg calculateRotationAndFlip: EXIF orientation -> (rotation, flip)
void exif_rotation(int orientation, int *rot, bool *flip) {
    *rot = 0;
    *flip = false;
    switch (orientation) {
        case 6: *rot = 90; break;
        case 3: *rot = 180; break;
        case 8: *rot = 270; break;
        case 2: *flip = true; break;
        case 7: *flip = true; *rot = 270; break;
        case 4: *flip = true; *rot = 180; break;
        case 5: *flip = true; *rot = 90; break;
        default: break;
    }
}

// bimg getAngle + vips_rotate_bridge: drop the remainder mod 90, cap at 270.
int normalise_angle(int rotate) {
    int a = rotate - rotate % 90;
    if (a > 270) a = 270;
    return ((a % 360) + 360) % 360;
}

}  // namespace

extern "C" int mipx_fit_dimension(int32_t iw, int32_t ih, int32_t fw, int32_t fh, int32_t *ow,
                                  int32_t *oh) {
    // imaginary image.go:190-200 calculateDestinationFitDimension
    if (!ow || !oh || iw <= 0 || ih <= 0) return MIPX_EINVAL;
    if (static_cast<int64_t>(iw) * fh > static_cast<int64_t>(fw) * ih)
        fh = static_cast<int32_t>(std::round(static_cast<double>(fw) * ih / iw));
    else
        fw = static_cast<int32_t>(std::round(static_cast<double>(fh) * iw / ih));
    *ow = fw;
    *oh = fh;
    return MIPX_OK;
}

extern "C" int mipx_plan_make(const mipx_opts *opts, const mipx_input *in, mipx_plan *plan) {
    if (!opts || !in || !plan) return MIPX_EINVAL;
    if (in->w <= 0 || in->h <= 0 || in->bands <= 0 || in->bands > 4) {
        mipx::set_error("mipx_plan_make: bad input geometry %dx%dx%d", in->w, in->h, in->bands);
        return MIPX_EINVAL;
    }
    mipx_opts o = *opts;  // bimg passes Options by value through the resizer
    PlanBuilder pb(plan);

    // rotateAndFlipImage: EXIF consulted only when no explicit rotation.
    int rotate = o.rotate;
    bool flip = o.flip != 0, flop = o.flop != 0;
    if (!o.no_auto_rotate && o.rotate <= 0) {
        int r;
        bool f;
        exif_rotation(in->orientation, &r, &f);
        if (f) flip = true;
        if (r > 0 && rotate == 0) rotate = r;
    }
    const int angle = rotate > 0 ? normalise_angle(rotate) : 0;
    const bool swap = angle == 90 || angle == 270;

    // normalizeOperation sees the caller's Rotate (rotateAndFlipImage got a copy).
    if (!o.force && !o.crop && !o.embed && !o.enlarge && o.rotate == 0 &&
        (o.width > 0 || o.height > 0))
        o.force = 1;

    // Geometry decisions use the full-size, rotated image (inWidth/inHeight).
    const int iw = swap ? in->h : in->w;
    const int ih = swap ? in->w : in->h;

    // imageCalculations
    double factor = 1.0;
    const double xf = static_cast<double>(iw) / o.width;
    const double yf = static_cast<double>(ih) / o.height;
    if (o.width > 0 && o.height > 0) {
        factor = o.crop ? std::fmin(xf, yf) : std::fmax(xf, yf);
    } else if (o.width > 0) {
        if (o.crop) {
            o.height = ih;
        } else {
            factor = xf;
            o.height = round_float(static_cast<double>(ih) / factor);
        }
    } else if (o.height > 0) {
        if (o.crop) {
            o.width = iw;
        } else {
            factor = yf;
            o.width = round_float(static_cast<double>(iw) / factor);
        }
    } else {
        o.width = iw;
        o.height = ih;
    }
    // calculateShrink (default bicubic interpolator: window 4) / calculateResidual
    double shrink_f = factor >= 2 ? std::floor(factor * 3.0 / 4.0) : std::floor(factor);
    int shrink = static_cast<int>(shrink_f < 1 ? 1 : shrink_f);
    double residual = static_cast<double>(shrink) / factor;
    if (!o.enlarge && !o.force && iw < o.width && ih < o.height) {
        factor = 1.0;
        shrink = 1;
        residual = 0;
        o.width = iw;
        o.height = ih;
    }
    // shrinkOnLoad (host codec: libjpeg / libwebp scale 2, 4, 8)
    plan->load_shrink = 1;
    if ((in->type == MIPX_TYPE_JPEG || in->type == MIPX_TYPE_WEBP) && shrink >= 2) {
        const int sol = shrink >= 8 ? 8 : (shrink >= 4 ? 4 : 2);
        factor /= sol;
        plan->load_shrink = sol;
        factor = std::fmax(factor, 1.0);
        shrink = static_cast<int>(std::floor(factor));
        residual = static_cast<double>(shrink) / factor;
    }
    int dw = in->w, dh = in->h;
    if (plan->load_shrink > 1) {
        const int s = plan->load_shrink;
        dw = in->decoded_w > 0 ? in->decoded_w : (in->w + s - 1) / s;
        dh = in->decoded_h > 0 ? in->decoded_h : (in->h + s - 1) / s;
    }
    plan->in_w = dw;
    plan->in_h = dh;
    plan->in_bands = in->bands;
    pb.start(dw, dh, in->bands);

    if (angle != 0) {
        pb.push(MIPX_OP_ROT);
        pb.last().a[0] = angle;
        pb.geom(swap ? pb.h() : pb.w(), swap ? pb.w() : pb.h(), pb.b());
    }
    if (flip) {
        pb.push(MIPX_OP_FLIP);
        pb.last().a[0] = 0;
        pb.geom(pb.w(), pb.h(), pb.b());
    }
    if (flop) {
        pb.push(MIPX_OP_FLIP);
        pb.last().a[0] = 1;
        pb.geom(pb.w(), pb.h(), pb.b());
    }
    // zoomImage: vips_zoom(zoom + 1) after shrink-on-load and rotation
    if (o.zoom > 0) {
        const int z = o.zoom + 1;
        if (static_cast<double>(pb.w()) * z * pb.h() * z * pb.b() > 2147483647.0) {
            mipx::set_error("zoom %d of %dx%d is too large", z, pb.w(), pb.h());
            return MIPX_EINVAL;
        }
        pb.push(MIPX_OP_ZOOM);
        pb.last().a[0] = z;
        pb.last().a[1] = z;
        pb.geom(pb.w() * z, pb.h() * z, pb.b());
    }

    const bool transform = o.force || (o.width > 0 && o.width != iw) ||
                           (o.height > 0 && o.height != ih) || o.area_width > 0 ||
                           o.area_height > 0;
    if (transform) {
        // transformImage
        if (shrink > 1) {  // shrinkImage: residual recomputed from the shrunk size
            pb.push(MIPX_OP_SHRINK);
            pb.last().a[0] = shrink;
            pb.last().a[1] = shrink;
            pb.geom(out_size_shrink(pb.w(), shrink), out_size_shrink(pb.h(), shrink), pb.b());
            const double rx = static_cast<double>(o.width) / pb.w();
            const double ry = static_cast<double>(o.height) / pb.h();
            residual = o.crop ? std::fmax(rx, ry) : std::fmin(rx, ry);
        }
        double rx = residual, ry = residual;
        if (o.force) {
            rx = static_cast<double>(o.width) / pb.w();
            ry = static_cast<double>(o.height) / pb.h();
        }
        if (o.force || residual != 0) {
            if (rx < 1 && ry < 1) {
                pb.push(MIPX_OP_REDUCE);
                pb.last().d[0] = 1.0 / rx;
                pb.last().d[1] = 1.0 / ry;
                pb.last().a[7] = mipx::reduce_sampling_now();  // the plan keeps its convention (ABI v6)
                pb.geom(out_size_reduce(pb.w(), 1.0 / rx), out_size_reduce(pb.h(), 1.0 / ry),
                        pb.b());
            } else if (!(rx == 1.0 && ry == 1.0)) {
                // vipsAffine(residualx, residualy, bicubic, o.Extend): output = the
                // transformed input rectangle (vips__transform_set_area)
                const double ow = std::ceil(pb.w() * rx), oh = std::ceil(pb.h() * ry);
                if (ow * oh * pb.b() > 2147483647.0) {
                    mipx::set_error("affine output %.0fx%.0f is too large", ow, oh);
                    return MIPX_EINVAL;
                }
                pb.push(MIPX_OP_AFFINE);
                pb.last().d[0] = rx;
                pb.last().d[1] = ry;
                pb.last().a[0] = o.extend > 5 ? MIPX_EXTEND_BACKGROUND : o.extend;
                pb.geom(static_cast<int>(ow), static_cast<int>(oh), pb.b());
            }
        }
        if (o.force) {
            o.crop = 0;
            o.embed = 0;
        }
        // extractOrEmbedImage
        const int cw = pb.w(), ch = pb.h();
        if (o.gravity == MIPX_GRAVITY_SMART || o.smart_crop) {
            if (!(cw <= o.width && ch <= o.height)) {
                pb.push(MIPX_OP_SMARTCROP);
                const int w = std::min(cw, o.width), h = std::min(ch, o.height);
                pb.last().a[0] = w;
                pb.last().a[1] = h;
                pb.last().a[7] = mipx::reduce_sampling_now();  // its scorer's downsize reduces
                pb.geom(w, h, pb.b());
            }
        } else if (o.crop) {
            if (!(cw <= o.width && ch <= o.height)) {
                const int w = std::min(cw, o.width), h = std::min(ch, o.height);
                int l = 0, t = 0;  // calculateCrop
                switch (o.gravity) {
                    case MIPX_GRAVITY_NORTH: l = (cw - o.width + 1) / 2; break;
                    case MIPX_GRAVITY_EAST:
                        l = cw - o.width;
                        t = (ch - o.height + 1) / 2;
                        break;
                    case MIPX_GRAVITY_SOUTH:
                        l = (cw - o.width + 1) / 2;
                        t = ch - o.height;
                        break;
                    case MIPX_GRAVITY_WEST: t = (ch - o.height + 1) / 2; break;
                    default:
                        l = (cw - o.width + 1) / 2;
                        t = (ch - o.height + 1) / 2;
                }
                l = std::max(l, 0);
                t = std::max(t, 0);
                if (l + w > cw || t + h > ch) return MIPX_EINVAL;
                pb.push(MIPX_OP_EXTRACT);
                int *a = pb.last().a;
                a[0] = l, a[1] = t, a[2] = w, a[3] = h;
                pb.geom(w, h, pb.b());
            }
        } else if (o.embed) {
            const int l = (o.width - cw) / 2, t = (o.height - ch) / 2;
            if (!(l == 0 && t == 0 && o.width == cw && o.height == ch)) {
                pb.push(MIPX_OP_EMBED);
                int *a = pb.last().a;
                a[0] = l, a[1] = t, a[2] = o.width, a[3] = o.height;
                a[4] = o.extend > 5 ? MIPX_EXTEND_BACKGROUND : o.extend;  // bimg vipsEmbed
                a[5] = o.background[0], a[6] = o.background[1], a[7] = o.background[2];
                pb.geom(o.width, o.height, pb.b());
            }
        } else if (o.top != 0 || o.left != 0 || o.area_width != 0 || o.area_height != 0) {
            // bimg 1.1.9: `if o.AreaWidth == 0 { o.AreaHeight = o.Width }` sets the
            // height, so a zero AreaWidth stays zero and the extract is an error
            // (PARITY_ASSUMPTIONS.md #11)
            int aw = o.area_width, ah = o.area_height;
            if (aw == 0) ah = o.width;
            if (ah == 0) ah = o.height;
            if (aw == 0 || ah == 0) {
                mipx::set_error("Extract area width/height params are required");
                return MIPX_EINVAL;
            }
            if (o.left < 0 || o.top < 0 || o.left + aw > cw || o.top + ah > ch) {
                mipx::set_error("bad extract area %d,%d %dx%d of %dx%d", o.left, o.top, aw, ah, cw, ch);
                return MIPX_EINVAL;
            }
            pb.push(MIPX_OP_EXTRACT);
            int *a = pb.last().a;
            a[0] = o.left, a[1] = o.top, a[2] = aw, a[3] = ah;
            pb.geom(aw, ah, pb.b());
        }
    }
    // applyEffects: vips_gaussblur_bridge passes NULL before "min_ampl", so
    // libvips' default min_ampl 0.2 always applies (PARITY_ASSUMPTIONS.md).
    if (o.sigma > 0 || o.min_ampl > 0) {
        if (!(o.sigma > 0)) {
            mipx::set_error("gaussblur with sigma 0 is not implemented");
            return MIPX_EUNSUPPORTED;
        }
        pb.push(MIPX_OP_BLUR);
        pb.last().d[0] = o.sigma;
        pb.last().d[1] = 0.2;
        pb.geom(pb.w(), pb.h(), pb.b());
    }
    // watermarkImageWithAnotherImage (opacity 0 -> 1)
    if (o.wm_enable) {
        const int bb = has_alpha(pb.b()) ? pb.b() : pb.b() + 1;
        const int wb = has_alpha(in->wm_bands) ? in->wm_bands : in->wm_bands + 1;
        if (bb != wb || in->wm_w <= 0 || in->wm_h <= 0) {
            mipx::set_error("watermark bands %d vs image bands %d", wb, bb);
            return MIPX_EUNSUPPORTED;
        }
        pb.push(MIPX_OP_WATERMARK);
        pb.last().a[0] = o.wm_left;
        pb.last().a[1] = o.wm_top;
        pb.last().a[2] = in->wm_w;
        pb.last().a[3] = in->wm_h;
        pb.last().a[4] = in->wm_bands;
        pb.last().d[0] = o.wm_opacity == 0.0f ? 1.0 : static_cast<double>(o.wm_opacity);
        pb.geom(pb.w(), pb.h(), bb);
    }
    // imageFlatten: PNG input, non-black background, an alpha band
    if (in->type == MIPX_TYPE_PNG && (o.background[0] || o.background[1] || o.background[2]) && has_alpha(pb.b())) {
        pb.push(MIPX_OP_FLATTEN);
        pb.last().a[0] = o.background[0];
        pb.last().a[1] = o.background[1];
        pb.last().a[2] = o.background[2];
        pb.geom(pb.w(), pb.h(), pb.b() - 1);
    }
    // vipsPreSave: vips_colourspace to the requested interpretation
    if (o.interpretation == MIPX_INTERPRETATION_BW && pb.b() >= 3) {
        pb.push(MIPX_OP_BW);
        pb.geom(pb.w(), pb.h(), pb.b() == 4 ? 2 : 1);
    }
    plan->out_w = pb.w();
    plan->out_h = pb.h();
    plan->out_bands = pb.b();
    // libvips fails a resample whose output has no pixels ("image has shrunk to nothing"),
    // e.g. height=4 with force on a 16 px wide image: bimg derives width floor(16 / 92) = 0
    for (int i = 0; i < plan->n_steps; ++i) {
        const mipx_step &st = plan->steps[i];
        if (st.out_w <= 0 || st.out_h <= 0) return MIPX_EINVAL;
        if (st.op == MIPX_OP_REDUCE && !(std::isfinite(st.d[0]) && std::isfinite(st.d[1]))) return MIPX_EINVAL;
    }
    return MIPX_OK;
}

extern "C" int mipx_plan_chain(const mipx_plan *stages, int32_t n_stages, mipx_plan *out) {
    if (!stages || !out || n_stages <= 0) return MIPX_EINVAL;
    mipx_plan m{};
    m.load_shrink = stages[0].load_shrink;
    m.in_w = stages[0].in_w;
    m.in_h = stages[0].in_h;
    m.in_bands = stages[0].in_bands;
    int wm_stages = 0;
    for (int k = 0; k < n_stages; ++k) {
        const mipx_plan &s = stages[k];
        if (s.n_steps < 0 || s.n_steps > MIPX_MAX_STEPS) return MIPX_EINVAL;
        if (k > 0 && (s.load_shrink != 1 || s.in_w != stages[k - 1].out_w || s.in_h != stages[k - 1].out_h ||
                      s.in_bands != stages[k - 1].out_bands)) {
            mipx::set_error("mipx_plan_chain: stage %d takes %dx%dx%d (load_shrink %d), stage %d gives %dx%dx%d", k,
                            s.in_w, s.in_h, s.in_bands, s.load_shrink, k - 1, stages[k - 1].out_w,
                            stages[k - 1].out_h, stages[k - 1].out_bands);
            return MIPX_EINVAL;
        }
        bool wm = false;
        for (int i = 0; i < s.n_steps; ++i) wm |= s.steps[i].op == MIPX_OP_WATERMARK;
        wm_stages += wm;
        if (wm_stages > 1) {
            mipx::set_error("mipx_plan_chain: more than one watermark stage");
            return MIPX_EUNSUPPORTED;
        }
        if (m.n_steps + s.n_steps > MIPX_MAX_STEPS) {
            mipx::set_error("mipx_plan_chain: %d steps exceed MIPX_MAX_STEPS", m.n_steps + s.n_steps);
            return MIPX_EUNSUPPORTED;
        }
        for (int i = 0; i < s.n_steps; ++i) m.steps[m.n_steps++] = s.steps[i];
    }
    m.out_w = stages[n_stages - 1].out_w;
    m.out_h = stages[n_stages - 1].out_h;
    m.out_bands = stages[n_stages - 1].out_bands;
    *out = m;
    return MIPX_OK;
}
