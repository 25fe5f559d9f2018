/*
 * vips_ref.h — CPU ORACLE (test infrastructure only, never shipped, never on the
 * product path).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle.so.
 *
 * A plain-C restatement of the pixel arithmetic that imaginary reaches through
 * bimg.Resize (image.go:96) — bimg v1.1.9 (go.mod:6) driving libvips 8.12.2
 * (Dockerfile:5).  Neither bimg nor libvips is present in /root/reference or in
 * this container, so every function below restates the PUBLISHED upstream
 * algorithm; each upstream detail that changes results is a switch listed in
 * PARITY_ASSUMPTIONS.md.
 *
 * Parity status: the host planner (ref_plan) is PINNED by the reference's own
 * dimension tests (image_test.go:20-141, :160-167; server_test.go:69-366);
 * pixel values are "parity unpinned" — no reference test checks a pixel and no
 * libvips binary exists here.
 */
#ifndef VIPS_REF_H
#define VIPS_REF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* An interleaved, tightly packed uchar image (stride = w * bands). */
typedef struct {
    uint8_t *data;
    int w, h, bands;
} ref_img;

/* bimg enums (bimg v1.1.9 options.go / type.go, [U]). */
enum { REF_GRAVITY_CENTRE = 0, REF_GRAVITY_NORTH, REF_GRAVITY_EAST, REF_GRAVITY_SOUTH,
       REF_GRAVITY_WEST, REF_GRAVITY_SMART };
enum { REF_EXTEND_BLACK = 0, REF_EXTEND_COPY, REF_EXTEND_REPEAT, REF_EXTEND_MIRROR,
       REF_EXTEND_WHITE, REF_EXTEND_BACKGROUND, REF_EXTEND_LAST };
enum { REF_TYPE_UNKNOWN = 0, REF_TYPE_JPEG, REF_TYPE_WEBP, REF_TYPE_PNG, REF_TYPE_TIFF,
       REF_TYPE_GIF, REF_TYPE_PDF, REF_TYPE_SVG, REF_TYPE_MAGICK, REF_TYPE_HEIF,
       REF_TYPE_AVIF };

/* The subset of bimg.Options that options.go:128-172 and image.go set. */
typedef struct {
    int width, height;
    int area_width, area_height;
    int top, left;
    int crop, embed, enlarge, force;
    int no_auto_rotate;
    int rotate;          /* degrees, bimg.Angle */
    int flip, flop;
    int gravity;         /* REF_GRAVITY_* */
    int extend;          /* REF_EXTEND_* */
    int background[3];
    int zoom;
    double sigma, min_ampl;
    int smart_crop;
    /* watermark image (bimg WatermarkImage) */
    int wm_enable;
    int wm_left, wm_top;
    float wm_opacity;
    int interpretation;  /* bimg Interpretation at save: 0 = keep, REF_INTERPRETATION_BW */
} ref_opts;

#define REF_INTERPRETATION_BW 26  /* VIPS_INTERPRETATION_B_W (bimg InterpretationBW) */

typedef struct {
    int w, h, bands;     /* header size of the ENCODED input (pre shrink-on-load) */
    int type;            /* REF_TYPE_* — JPEG/WEBP enable codec shrink-on-load */
    int orientation;     /* EXIF orientation 0..8 */
    int decoded_w, decoded_h; /* size the host codec actually produced, 0 = ceil(w/s) */
    int wm_w, wm_h, wm_bands; /* decoded watermark size (when wm_enable) */
} ref_input;

enum {
    REF_OP_ROT = 1,      /* a[0] = angle (0/90/180/270, clockwise) */
    REF_OP_FLIP,         /* a[0] = 0 horizontal (mirror x), 1 vertical */
    REF_OP_SHRINK,       /* a[0] = hshrink, a[1] = vshrink (integers) */
    REF_OP_REDUCE,       /* d[0] = hshrink, d[1] = vshrink (>= 1) */
    REF_OP_EXTRACT,      /* a[0..3] = left, top, width, height */
    REF_OP_EMBED,        /* a[0..3] = x, y, width, height, a[4] = extend, a[5..7] = bg */
    REF_OP_SMARTCROP,    /* a[0..1] = width, height */
    REF_OP_BLUR,         /* d[0] = sigma, d[1] = min_ampl (effective) */
    REF_OP_WATERMARK,    /* a[0..1] = left, top; d[0] = opacity */
    REF_OP_AFFINE,       /* d[0] = xscale, d[1] = yscale; a[0] = extend (vips_affine bicubic) */
    REF_OP_ZOOM,         /* a[0] = xfac, a[1] = yfac (vips_zoom) */
    REF_OP_FLATTEN,      /* a[0..2] = background rgb (vips_flatten) */
    REF_OP_BW            /* vips_colourspace sRGB -> B_W */
};

#define REF_MAX_STEPS 16
typedef struct {
    int op;
    int a[8];
    double d[4];
    int out_w, out_h, out_bands;   /* image geometry after this step */
} ref_step;

typedef struct {
    int load_shrink;     /* codec shrink-on-load factor the host must apply (1,2,4,8) */
    int in_w, in_h, in_bands;   /* decoded input handed to the pixel engine */
    int out_w, out_h, out_bands;
    int n_steps;
    ref_step steps[REF_MAX_STEPS];
} ref_plan;

/* Error codes (negative). */
#define REF_OK 0
#define REF_EINVAL (-1)
#define REF_EUNSUPPORTED (-2)
#define REF_ENOMEM (-3)

/* ---- planner (bimg resizer.go restatement) ---- */
int ref_plan_make(const ref_opts *o, const ref_input *in, ref_plan *plan);
int ref_fit_dimension(int image_w, int image_h, int fit_w, int fit_h, int *out_w, int *out_h);

/* ---- resample: Lanczos3 reduce, box shrink ---- */
int ref_reduce_points(double shrink);
/* integer coefficient tables: 129 rows of n_point ints, returns n_point */
int ref_reduce_table(double shrink, int *table, int max_points);
int ref_reducev(const ref_img *in, ref_img *out, double vshrink);
int ref_reduceh(const ref_img *in, ref_img *out, double hshrink);
int ref_reduce(const ref_img *in, ref_img *out, double hshrink, double vshrink);
int ref_shrinkv(const ref_img *in, ref_img *out, int vshrink);
int ref_shrinkh(const ref_img *in, ref_img *out, int hshrink);
int ref_shrink(const ref_img *in, ref_img *out, int hshrink, int vshrink);
int ref_out_size_reduce(int in, double shrink);
int ref_out_size_shrink(int in, int shrink);

/* ---- conversion ---- */
int ref_embed(const ref_img *in, ref_img *out, int x, int y, int w, int h, int extend,
              const int bg[3]);
int ref_extract(const ref_img *in, ref_img *out, int left, int top, int w, int h);
int ref_rot(const ref_img *in, ref_img *out, int angle);
int ref_flip(const ref_img *in, ref_img *out, int vertical);

/* ---- convolution ---- */
int ref_gaussmat(double sigma, double min_ampl, int *mask, int max_width, int *scale);
int ref_gaussblur(const ref_img *in, ref_img *out, double sigma, double min_ampl);

/* ---- affine (bicubic) / zoom / flatten / colourspace ---- */
int ref_bicubic_table(int *table);  /* 129 x 4 truncated 12-bit Catmull-Rom taps */
int ref_affine(const ref_img *in, ref_img *out, double xscale, double yscale, int extend);
int ref_zoom(const ref_img *in, ref_img *out, int xfac, int yfac);
int ref_flatten(const ref_img *in, ref_img *out, const int bg[3]);
int ref_bw(const ref_img *in, ref_img *out);

/* ---- composite / smartcrop ---- */
int ref_watermark(const ref_img *base, const ref_img *wm, ref_img *out, int left, int top,
                  float opacity);
int ref_smartcrop_origin(const ref_img *in, int width, int height, int *left, int *top);

/* ---- whole plan execution ---- */
int ref_execute(const ref_plan *plan, const ref_img *in, const ref_img *wm, ref_img *out);

/* ---- CPU baseline (bench.py cpu_baseline leg): reduce a batch, OpenMP over images ---- */
int ref_reduce_batch(const uint8_t *const *in, uint8_t *const *out, int n, int w, int h,
                     int bands, double hshrink, double vshrink, int threads);

/* ---- CPU baseline (vips_fast.c, -O3 x86-64-v3): the same reduce, cache-friendly loop order ---- */
int ref_reduce_fast(const ref_img *in, ref_img *out, double hshrink, double vshrink);
int ref_reduce_fast_batch(const uint8_t *const *in, uint8_t *const *out, int n, int w, int h,
                          int bands, double hshrink, double vshrink, int threads);

/* parity switches (PARITY_ASSUMPTIONS.md); 0 = default assumption */
void ref_set_switch(const char *name, int value);
int ref_get_switch(const char *name);

void ref_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
