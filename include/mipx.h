/*
 * mipx.h — C-ABI of the MI355X pixel-transform engine (libmipx.so).
 *
 * Drop-in for the pixel work inside imaginary's Process() (reference
 * image.go:81-113): today Process calls bimg.Resize(buf, opts) (image.go:96),
 * which decodes, runs the libvips pixel ops and encodes in one call.  With the
 * engine, the host keeps libvips decode/encode and hands DECODED pixels plus a
 * plan (built from the same bimg.Options fields that options.go:128-172 and the
 * image.go operation wrappers set) to this library.  A Go shim binds these
 * entry points through cgo.
 *
 * Conventions
 *  - Every entry point returns 0 (MIPX_OK) or a negative MIPX_E* code; nothing
 *    aborts or throws across the ABI.  MIPX_EUNSUPPORTED means "the plan needs
 *    an op the engine does not implement": the caller falls back to
 *    bimg.Resize for that request (SURVEY.md §5 failure handling).
 *  - Images are interleaved uchar, `bands` 1..4, rows `stride` bytes apart
 *    (stride 0 = w * bands).
 *  - mipx_submit copies the input into pinned staging before it returns (cgo
 *    pointer rule: no Go pointer is retained); the output buffer must stay
 *    valid until mipx_wait returns a FINAL status for the ticket (anything but
 *    MIPX_ETIMEOUT) or mipx_cancel returns for it.  After MIPX_ETIMEOUT the
 *    request is still queued or running and will still write the output: wait
 *    again, or call mipx_cancel before freeing the buffer.
 *  - Plans are validated before use: every step's out_w/out_h/out_bands must be
 *    what its op makes from the previous step's geometry (MIPX_EINVAL otherwise),
 *    and a watermark image must have the watermark step's geometry.
 *  - All mipx_op_* / mipx_execute_dev entry points take DEVICE pointers to a
 *    batch of n equally sized images packed back to back, and a hipStream_t
 *    passed as void* (NULL = the device's default engine stream).  They only
 *    enqueue work; they never synchronise or allocate.
 *  - Thread-safe: mipx_submit / mipx_wait / mipx_process may be called from
 *    many threads (one goroutine per HTTP request).
 */
#ifndef MIPX_H
#define MIPX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIPX_ABI_VERSION 6

/* ---- error codes ---- */
#define MIPX_OK 0
#define MIPX_EINVAL (-1)         /* bad argument / geometry (libvips "bad extract area" etc.) */
#define MIPX_EUNSUPPORTED (-2)   /* op not implemented by the engine: fall back to bimg.Resize */
#define MIPX_ENOMEM (-3)
#define MIPX_ENODEV (-4)         /* no usable gfx950 device */
#define MIPX_EDEVICE (-5)        /* HIP runtime error (details: mipx_last_error()) */
#define MIPX_ETIMEOUT (-6)
#define MIPX_ENOTINIT (-7)
#define MIPX_ESTALE (-8)         /* unknown or already-waited ticket */
#define MIPX_EBUSY (-9)          /* refused while requests are queued or running */

/* ---- bimg enums (bimg v1.1.9 options.go / type.go) ---- */
enum { MIPX_GRAVITY_CENTRE = 0, MIPX_GRAVITY_NORTH, MIPX_GRAVITY_EAST, MIPX_GRAVITY_SOUTH,
       MIPX_GRAVITY_WEST, MIPX_GRAVITY_SMART };
enum { MIPX_EXTEND_BLACK = 0, MIPX_EXTEND_COPY, MIPX_EXTEND_REPEAT, MIPX_EXTEND_MIRROR,
       MIPX_EXTEND_WHITE, MIPX_EXTEND_BACKGROUND, MIPX_EXTEND_LAST };
enum { MIPX_TYPE_UNKNOWN = 0, MIPX_TYPE_JPEG, MIPX_TYPE_WEBP, MIPX_TYPE_PNG, MIPX_TYPE_TIFF,
       MIPX_TYPE_GIF, MIPX_TYPE_PDF, MIPX_TYPE_SVG, MIPX_TYPE_MAGICK, MIPX_TYPE_HEIF,
       MIPX_TYPE_AVIF };

/* Mirror of the bimg.Options subset set by options.go:128-172 (BimgOptions) and
 * the image.go wrappers (Resize 115, Fit 139, Enlarge 202, Extract 213, Crop 226,
 * SmartCrop 236, Rotate 247, Flip 267, Flop 273, Thumbnail 279, Zoom 286,
 * WatermarkImage 343, GaussianBlur 372).  Booleans are 0/1. */
typedef struct mipx_opts {
    int32_t width, height;          /* bimg Width/Height */
    int32_t area_width, area_height;/* bimg AreaWidth/AreaHeight (Extract, Zoom) */
    int32_t top, left;              /* bimg Top/Left */
    int32_t crop, embed, enlarge, force;
    int32_t no_auto_rotate;         /* bimg NoAutoRotate (options.go:137) */
    int32_t rotate;                 /* bimg Rotate: bimg.Angle(o.Rotate) (options.go:145) */
    int32_t flip, flop;
    int32_t gravity;                /* MIPX_GRAVITY_* */
    int32_t extend;                 /* MIPX_EXTEND_*; imaginary default ExtendCopy (params.go:342,356) */
    int32_t background[3];          /* options.go:151-153 */
    int32_t zoom;                   /* bimg Zoom (image.go:308) */
    double sigma, min_ampl;         /* bimg GaussianBlur (options.go:164-169) */
    int32_t smart_crop;             /* bimg SmartCrop */
    int32_t wm_enable;              /* WatermarkImage present (image.go:364-367) */
    int32_t wm_left, wm_top;
    float wm_opacity;               /* 0 -> 1.0 as bimg does */
    int32_t interpretation;         /* bimg Interpretation at save (options.go:142): 0 or
                                       sRGB = keep, MIPX_INTERPRETATION_BW = vips_colourspace B_W */
} mipx_opts;

#define MIPX_INTERPRETATION_SRGB 22 /* VIPS_INTERPRETATION_sRGB */
#define MIPX_INTERPRETATION_BW 26   /* VIPS_INTERPRETATION_B_W (params.go:392 colorspace=bw) */

/* What the host codec knows about the encoded input. */
typedef struct mipx_input {
    int32_t w, h, bands;            /* header size and bands of the encoded image */
    int32_t type;                   /* MIPX_TYPE_*; JPEG/WEBP allow shrink-on-load */
    int32_t orientation;            /* EXIF orientation 0..8 */
    int32_t decoded_w, decoded_h;   /* size the codec produced at plan.load_shrink (0 = ceil) */
    int32_t wm_w, wm_h, wm_bands;   /* decoded watermark image, when opts.wm_enable */
} mipx_input;

/* Plan steps: the libvips ops bimg would run, in order. */
enum {
    MIPX_OP_ROT = 1,     /* a[0] = angle 0/90/180/270 clockwise              (vips_rot) */
    MIPX_OP_FLIP,        /* a[0] = 0 horizontal mirror, 1 vertical           (vips_flip) */
    MIPX_OP_SHRINK,      /* a[0] = hshrink, a[1] = vshrink (integer box)     (vips_shrink) */
    MIPX_OP_REDUCE,      /* d[0] = hshrink, d[1] = vshrink, Lanczos3; a[7] = MIPX_SAMPLE_*  (vips_reduce) */
    MIPX_OP_EXTRACT,     /* a[0..3] = left, top, width, height               (vips_extract_area) */
    MIPX_OP_EMBED,       /* a[0..3] = x, y, w, h; a[4] = extend; a[5..7] bg  (vips_embed) */
    MIPX_OP_SMARTCROP,   /* a[0..1] = width, height, attention; a[7] = MIPX_SAMPLE_*  (vips_smartcrop) */
    MIPX_OP_BLUR,        /* d[0] = sigma, d[1] = min_ampl                    (vips_gaussblur) */
    MIPX_OP_WATERMARK,   /* a[0..1] = left, top; d[0] = opacity  (bimg vips_watermark_image) */
    MIPX_OP_AFFINE,      /* d[0] = xscale, d[1] = yscale, a[0] = extend; bicubic  (vips_affine) */
    MIPX_OP_ZOOM,        /* a[0] = xfac, a[1] = yfac                         (vips_zoom) */
    MIPX_OP_FLATTEN,     /* a[0..2] = background rgb                         (vips_flatten) */
    MIPX_OP_BW           /* sRGB -> B_W                                      (vips_colourspace) */
};

#define MIPX_MAX_STEPS 64   /* room for a merged /pipeline chain (mipx_plan_chain) */
typedef struct mipx_step {
    int32_t op;
    int32_t a[8];
    double d[4];
    int32_t out_w, out_h, out_bands;
} mipx_step;

typedef struct mipx_plan {
    int32_t load_shrink;            /* codec shrink-on-load the HOST applies (1,2,4,8) */
    int32_t in_w, in_h, in_bands;   /* decoded image the engine receives */
    int32_t out_w, out_h, out_bands;
    int32_t n_steps;
    mipx_step steps[MIPX_MAX_STEPS];
} mipx_plan;

typedef struct mipx_img {
    uint8_t *data;
    int32_t w, h, bands;
    int64_t stride;                 /* bytes between rows; 0 = w * bands */
} mipx_img;

typedef struct mipx_cfg {
    int32_t n_devices;              /* 0 = every visible device */
    int32_t device_ids[16];
    int64_t staging_bytes;          /* pinned staging kept cached for reuse; 0 = default (1 GiB) */
    int32_t max_batch;              /* requests fused into one launch; 0 = default (64) */
    int32_t batch_wait_us;          /* bounded wait for more requests; 0 = none */
    int32_t queues_per_device;      /* request queues (worker + 3 streams each) per device; 0 = 1 */
} mipx_cfg;

/* ---- library / devices ---- */
const char *mipx_version(void);
/* Build identity: the first 16 hex digits of the SHA-256 of the engine sources this
 * library was compiled from (imaginary_amd/csrc/ + include/mipx.h; imaginary_amd/srchash.py). */
const char *mipx_build_id(void);
int mipx_abi_version(void);
const char *mipx_strerror(int code);
const char *mipx_last_error(void);      /* thread-local detail of the last failure */
/* NULL = defaults.  Already up: MIPX_OK for NULL or the running configuration,
 * MIPX_EINVAL (with mipx_last_error) for a different one — mipx_shutdown first. */
int mipx_init(const mipx_cfg *cfg);
void mipx_shutdown(void);
int mipx_device_count(void);

/* ---- host planner (bimg resizer.go restated; callable without a GPU) ---- */
int mipx_plan_make(const mipx_opts *opts, const mipx_input *in, mipx_plan *plan);
/* /pipeline GPU-resident fusion (image.go:379-410 Pipeline): concatenate the plans of
 * a pipeline's stages (stage k planned on stage k-1's output, decoded intermediates)
 * into one plan, so the request path runs the chain with one upload, device-resident
 * intermediates and one download.  Stage k > 0 must take stage k-1's output geometry
 * and have load_shrink 1; at most one stage may carry a watermark step.
 * MIPX_EUNSUPPORTED when the chain exceeds MIPX_MAX_STEPS or has two watermark stages
 * (the caller then runs the stages one by one). */
int mipx_plan_chain(const mipx_plan *stages, int32_t n_stages, mipx_plan *out);
/* imaginary image.go:190 calculateDestinationFitDimension */
int mipx_fit_dimension(int32_t image_w, int32_t image_h, int32_t fit_w, int32_t fit_h,
                       int32_t *out_w, int32_t *out_h);

/* ---- request API (host buffers; pinned staging, per-device queues, batching) ---- */
int mipx_submit(int device, const mipx_plan *plan, const mipx_img *in, const mipx_img *wm,
                mipx_img *out, uint64_t *ticket);   /* device < 0 = least loaded */
int mipx_wait(uint64_t ticket, int timeout_ms);      /* timeout < 0 = forever */
/* Detach a submitted request's output: once this returns, the engine never writes
 * the caller's output buffer for `ticket` (a copy already under way completes
 * first) and the ticket is released.  MIPX_ESTALE for an unknown ticket. */
int mipx_cancel(uint64_t ticket);
int mipx_process(const mipx_plan *plan, const mipx_img *in, const mipx_img *wm,
                 mipx_img *out);                     /* submit + wait */
/* Batches launched and requests retired so far on `device`, summed over its
 * queues (batching telemetry).  mipx_submit(device >= 0) picks the least-loaded
 * queue of that device; device < 0 the least-loaded queue of all. */
int mipx_stats(int device, uint64_t *batches, uint64_t *requests);
int mipx_queue_count(void);                           /* 0 before mipx_init */
/* The dispatch rule of mipx_submit, callable without a GPU: the queue (index into
 * the n_queues arrays) with the fewest pending bytes among those of `device`
 * (device < 0: among all), first on ties; MIPX_EINVAL when none qualifies. */
int mipx_pick_queue(int32_t device, const int32_t *queue_device, const int64_t *pending_bytes,
                    int32_t n_queues);
int mipx_queue_stats(int queue, int32_t *device, uint64_t *batches, uint64_t *requests,
                     int64_t *pending_bytes);         /* pending = queued input bytes */

/* ---- device-resident batch API ---- */
size_t mipx_workspace_bytes(const mipx_plan *plan, int32_t n);
int mipx_execute_dev(const mipx_plan *plan, int32_t n, const uint8_t *d_in, uint8_t *d_out,
                     const uint8_t *d_wm, void *d_workspace, size_t workspace_bytes,
                     void *stream);

/* Per-op kernels (each replaces one libvips operation).  n images of w x h x bands
 * packed back to back in and out; output geometry follows the libvips rule. */
int mipx_op_reduce(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                   int32_t bands, double hshrink, double vshrink, void *d_workspace,
                   size_t workspace_bytes, void *stream);
int mipx_op_reducev(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                    int32_t bands, double vshrink, void *stream);
int mipx_op_reduceh(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                    int32_t bands, double hshrink, void *stream);
int mipx_op_shrink(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                   int32_t bands, int32_t hshrink, int32_t vshrink, void *stream);
int mipx_op_embed(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                  int32_t bands, int32_t x, int32_t y, int32_t out_w, int32_t out_h,
                  int32_t extend, const int32_t *background3, void *stream);
int mipx_op_extract(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                    int32_t bands, int32_t left, int32_t top, int32_t out_w, int32_t out_h,
                    void *stream);
int mipx_op_rot(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                int32_t bands, int32_t angle, void *stream);
int mipx_op_flip(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                 int32_t bands, int32_t vertical, void *stream);
int mipx_op_gaussblur(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                      int32_t bands, double sigma, double min_ampl, void *d_workspace,
                      size_t workspace_bytes, void *stream);
int mipx_op_watermark(const uint8_t *d_base, const uint8_t *d_wm, uint8_t *d_out, int32_t n,
                      int32_t w, int32_t h, int32_t bands, int32_t wm_w, int32_t wm_h,
                      int32_t wm_bands, int32_t left, int32_t top, float opacity, void *stream);
int mipx_op_affine(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                   int32_t bands, double xscale, double yscale, int32_t extend, void *stream);
int mipx_op_zoom(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                 int32_t bands, int32_t xfac, int32_t yfac, void *stream);
int mipx_op_flatten(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                    int32_t bands, const int32_t *background3, void *stream);
int mipx_op_colourspace_bw(const uint8_t *d_in, uint8_t *d_out, int32_t n, int32_t w, int32_t h,
                           int32_t bands, void *stream);
/* writes n (left, top) int32 pairs to d_origins */
int mipx_op_smartcrop_origin(const uint8_t *d_in, int32_t *d_origins, int32_t n, int32_t w,
                             int32_t h, int32_t bands, int32_t crop_w, int32_t crop_h,
                             void *d_workspace, size_t workspace_bytes, void *stream);
size_t mipx_op_workspace_bytes(int32_t op, int32_t n, int32_t w, int32_t h, int32_t bands,
                               double p0, double p1);

/* ---- parity settings (PARITY_ASSUMPTIONS.md) ----
 * The sampling convention of libvips' Lanczos3 reduce (reducev.cpp / reduceh.cpp;
 * PARITY_ASSUMPTIONS.md row 1): MIPX_SAMPLE_CORNER, output o samples X = o * shrink,
 * or MIPX_SAMPLE_CENTRE, X = (o + 0.5) * shrink - 0.5.  Output sizes do not depend on it.
 * ABI v6: mipx_plan_make records the process setting in every REDUCE and SMARTCROP step
 * (a[7]), and a plan always executes under the convention it recorded (a cached plan
 * keeps its convention when the setting changes later; a zeroed a[7] is the corner
 * convention, any value but 0 / 1 is MIPX_EINVAL).  The per-op entry points
 * (mipx_op_reduce, _reducev, _reduceh, _smartcrop_origin) read the setting once per call.
 * The setter returns MIPX_EINVAL for a value other than the two; it also returns
 * MIPX_EBUSY when it sees mipx_submit requests queued or running.  That refusal is
 * advisory, not a guarantee: it counts mipx_submit work only (not mipx_execute_dev or the
 * per-op calls on a caller's stream) and a submit may land just after the check.  Nothing
 * depends on it: a plan's own a[7] decides its convention.  Set the convention once at
 * start-up. */
#define MIPX_SAMPLE_CORNER 0
#define MIPX_SAMPLE_CENTRE 1
int mipx_set_reduce_sampling(int32_t convention);
int mipx_reduce_sampling(void);

/* ---- engine tuning (tests and benchmarks) ----
 * Kernel-selection knobs (MIPX_* environment variables, e.g. MIPX_RCOL=0 for the
 * previous generic reduce) are read once, on first use.  Every knob only chooses
 * among kernels that give identical bytes; none changes a result.
 * mipx_tuning_reload() re-reads them; call it only between launches (A/B scripts,
 * tests). */
int mipx_tuning_reload(void);

/* ---- device memory helpers (so a binding needs no other HIP wrapper) ---- */
int mipx_set_device(int device);
int mipx_dev_malloc(void **ptr, size_t bytes);
int mipx_dev_free(void *ptr);
int mipx_memcpy_h2d(void *d_dst, const void *h_src, size_t bytes);
int mipx_memcpy_d2h(void *h_dst, const void *d_src, size_t bytes);
int mipx_memset_dev(void *d_dst, int value, size_t bytes);
int mipx_stream_sync(void *stream);
int mipx_device_sync(void);
int mipx_stream_create(void **stream);
int mipx_stream_destroy(void *stream);
/* HIP events, for timing on the engine's stream */
int mipx_event_create(void **event);
int mipx_event_destroy(void *event);
int mipx_event_record(void *event, void *stream);
int mipx_event_elapsed_ms(void *start, void *stop, float *ms);

#ifdef __cplusplus
}
#endif
#endif /* MIPX_H */
