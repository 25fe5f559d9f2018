/*
 * vips_fast.c — CPU BASELINE (test infrastructure only, never shipped, never on
 * the product path; loaded by bench.py's cpu_baseline leg and tests/ only).
 *
 * The same libvips 8.12.2 Lanczos3 reduce as ref_reduce() in vips_ref.c
 * (reducev then reduceh, 12-bit integer taps, uchar intermediate, EXTEND_COPY
 * edges; reduce.c / reducev.cpp / reduceh.cpp restated), arranged the way an
 * optimised CPU build runs it, so the GPU is timed against a fair CPU figure:
 *
 *  - reducev walks each output row once: taps outer, row bytes inner, int32
 *    accumulators in a row buffer (contiguous, auto-vectorised at -O3);
 *  - reduceh walks rows in memory order, each output pixel's taps read from
 *    one cache-resident row;
 *  - OpenMP across images (each image single-threaded, as libvips' per-request
 *    concurrency 1 in imaginary), compiled -O3 for x86-64-v3 (AVX2).
 *
 * It shares the coefficient table with the oracle (ref_reduce_table), both
 * settings of the reduce_centre switch and the defaults of the others;
 * tests/test_oracle.py checks it is byte-identical to ref_reduce on random and
 * edge-case inputs under both sampling conventions.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "vips_ref.h"

#define TRANSFORM_SCALE 128

static inline int clampi_f(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
static inline int vround(double v) { return (int)floor(v + 0.5); }
static inline int phase_of(double X) { return (((int)(X * TRANSFORM_SCALE * 2) & (TRANSFORM_SCALE * 2 - 1)) + 1) >> 1; }
static inline unsigned char rnd12(int s) { return (unsigned char)clampi_f((s + 2048) >> 12, 0, 255); }
/* sample position: the corner convention o * s, or with the reduce_centre switch
 * (o + 0.5) * s - 0.5, as vips_ref.c reduce_pos */
static inline double pos_of(int o, double s) {
    return ref_get_switch("reduce_centre") ? (o + 0.5) * s - 0.5 : o * s;
}

static int reducev_fast(const unsigned char *in, int w, int h, int b, unsigned char *out, int oh, double vs,
                        const int *tab, int n, int *acc) {
    const int pad = n / 2 - 1;
    const size_t ne = (size_t)w * b;
    for (int y = 0; y < oh; y++) {
        const double Y = pos_of(y, vs);
        const int iy = (int)Y;
        const int *c = tab + phase_of(Y) * n;
        memset(acc, 0, ne * sizeof(int));
        for (int i = 0; i < n; i++) {
            const int ci = c[i];
            if (!ci) continue;
            const unsigned char *row = in + (size_t)clampi_f(iy + i - pad, 0, h - 1) * ne;
            for (size_t j = 0; j < ne; j++) acc[j] += ci * row[j];
        }
        unsigned char *q = out + (size_t)y * ne;
        for (size_t j = 0; j < ne; j++) q[j] = rnd12(acc[j]);
    }
    return 0;
}

static int reduceh_fast(const unsigned char *in, int w, int h, int b, unsigned char *out, int ow, double hs,
                        const int *tab, int n, int *cols, const int **coef) {
    const int pad = n / 2 - 1;
    for (int x = 0; x < ow; x++) {  /* per output column: first tap and mask, once */
        const double X = pos_of(x, hs);
        cols[x] = (int)X - pad;
        coef[x] = tab + phase_of(X) * n;
    }
    for (int y = 0; y < h; y++) {
        const unsigned char *p = in + (size_t)y * w * b;
        unsigned char *q = out + (size_t)y * ow * b;
        for (int x = 0; x < ow; x++) {
            const int s = cols[x];
            const int *c = coef[x];
            int sum[4] = {0, 0, 0, 0};
            if (s >= 0 && s + n <= w) {  /* interior: no clamping */
                const unsigned char *pp = p + (size_t)s * b;
                for (int i = 0; i < n; i++)
                    for (int z = 0; z < b; z++) sum[z] += c[i] * pp[i * b + z];
            } else {
                for (int i = 0; i < n; i++) {
                    const unsigned char *pp = p + (size_t)clampi_f(s + i, 0, w - 1) * b;
                    for (int z = 0; z < b; z++) sum[z] += c[i] * pp[z];
                }
            }
            for (int z = 0; z < b; z++) q[x * b + z] = rnd12(sum[z]);
        }
    }
    return 0;
}

/* One image into caller-owned buffers: mid (w x oh x b), acc (w x b ints),
 * cols / coef (ow entries).  Tables tv / th: ref_reduce_table. */
static void reduce_into(const unsigned char *in, int w, int h, int b, unsigned char *out, int ow, int oh,
                        double hs, double vs, const int *tv, int nv, const int *th, int nh, unsigned char *mid,
                        int *acc, int *cols, const int **coef) {
    if (vs == 1.0) memcpy(mid, in, (size_t)w * h * b);
    else reducev_fast(in, w, h, b, mid, oh, vs, tv, nv, acc);
    if (hs == 1.0) memcpy(out, mid, (size_t)w * oh * b);
    else reduceh_fast(mid, w, oh, b, out, ow, hs, th, nh, cols, coef);
}

typedef struct {
    int *tv, *th, nv, nh, ow, oh;
} fast_plan;

static int plan_fast(fast_plan *p, int w, int h, double hs, double vs) {
    p->oh = vs == 1.0 ? h : vround(h / vs);
    p->ow = hs == 1.0 ? w : vround(w / hs);
    if (p->ow < 1 || p->oh < 1) return REF_EINVAL;
    p->nv = ref_reduce_points(vs), p->nh = ref_reduce_points(hs);
    p->tv = (int *)malloc(sizeof(int) * p->nv * (TRANSFORM_SCALE + 1));
    p->th = (int *)malloc(sizeof(int) * p->nh * (TRANSFORM_SCALE + 1));
    if (!p->tv || !p->th) return REF_ENOMEM;
    ref_reduce_table(vs, p->tv, p->nv);
    ref_reduce_table(hs, p->th, p->nh);
    return REF_OK;
}

static int defaults_only(void) {
    return !(ref_get_switch("reduce_hfirst") || ref_get_switch("reduce_round_coeff"));
}

int ref_reduce_fast(const ref_img *in, ref_img *out, double hshrink, double vshrink) {
    if (hshrink < 1.0 || vshrink < 1.0 || in->bands < 1 || in->bands > 4) return REF_EINVAL;
    if (!defaults_only()) return ref_reduce(in, out, hshrink, vshrink);  /* the oracle itself */
    const int w = in->w, h = in->h, b = in->bands;
    fast_plan p = {0};
    int e = plan_fast(&p, w, h, hshrink, vshrink);
    unsigned char *mid = (unsigned char *)malloc((size_t)w * (p.oh > h ? p.oh : h) * b);
    int *acc = (int *)malloc(sizeof(int) * (size_t)w * b);
    int *cols = (int *)malloc(sizeof(int) * (p.ow > 0 ? p.ow : 1));
    const int **coef = (const int **)malloc(sizeof(int *) * (p.ow > 0 ? p.ow : 1));
    out->data = e ? NULL : (uint8_t *)malloc((size_t)p.ow * p.oh * b);
    if (!e && (!mid || !acc || !cols || !coef || !out->data)) e = REF_ENOMEM;
    if (!e) {
        out->w = p.ow, out->h = p.oh, out->bands = b;
        reduce_into(in->data, w, h, b, out->data, p.ow, p.oh, hshrink, vshrink, p.tv, p.nv, p.th, p.nh, mid, acc,
                    cols, coef);
    } else {
        free(out->data);
        out->data = NULL;
    }
    free(p.tv), free(p.th), free(mid), free(acc), free(cols), free(coef);
    return e;
}

/* bench.py cpu_baseline: reduce n images (pointers to w x h x b) straight into
 * the callers' outputs; OpenMP across images, each image single-threaded, every
 * thread reusing its own scratch (no per-image allocation or first-touch faults
 * in the timed loop). */
int ref_reduce_fast_batch(const uint8_t *const *in, uint8_t *const *out, int n, int w, int h, int bands,
                          double hshrink, double vshrink, int threads) {
    if (hshrink < 1.0 || vshrink < 1.0 || bands < 1 || bands > 4 || n < 1) return REF_EINVAL;
    if (!defaults_only()) return ref_reduce_batch(in, out, n, w, h, bands, hshrink, vshrink, threads);
    fast_plan p = {0};
    int err = plan_fast(&p, w, h, hshrink, vshrink);
    if (err) {
        free(p.tv), free(p.th);
        return err;
    }
#pragma omp parallel num_threads(threads) reduction(| : err)
    {
        unsigned char *mid = (unsigned char *)malloc((size_t)w * (p.oh > h ? p.oh : h) * bands);
        int *acc = (int *)malloc(sizeof(int) * (size_t)w * bands);
        int *cols = (int *)malloc(sizeof(int) * p.ow);
        const int **coef = (const int **)malloc(sizeof(int *) * p.ow);
        if (!mid || !acc || !cols || !coef) {
            err |= 1;
        } else {
#pragma omp for schedule(dynamic, 1)
            for (int i = 0; i < n; i++)
                reduce_into(in[i], w, h, bands, out[i], p.ow, p.oh, hshrink, vshrink, p.tv, p.nv, p.th, p.nh, mid,
                            acc, cols, coef);
        }
        free(mid), free(acc), free(cols), free(coef);
    }
    free(p.tv), free(p.th);
    return err ? REF_ENOMEM : REF_OK;
}
