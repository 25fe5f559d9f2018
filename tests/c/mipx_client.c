/*
 * mipx_client.c — a plain C consumer of include/mipx.h, the way the cgo shim that
 * replaces bimg.Resize at reference image.go:96 would bind it:
 * plan with mipx_plan_make, submit from several threads (one per "goroutine"),
 * wait, and byte-compare every result with the CPU oracle (liboracle.so, test
 * infrastructure only) running the oracle planner's plan for the same options.
 *
 *   mipx_client [threads] [requests_per_thread] [queues_per_device]
 *
 * Exit 0 = every output identical; 1 = mismatch or engine error; 77 = no device.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mipx.h"
#include "vips_ref.h"

typedef struct {
    int w, h, bands;
    int width, height, crop, embed, gravity;
    double sigma;
} spec_t;

/* three request shapes: reduce 2x2 (north star), generic reduce + crop, blur */
static const spec_t SPECS[] = {
    {320, 240, 3, 160, 120, 0, 1, 0, 0.0},
    {301, 203, 3, 120, 90, 1, 0, 0, 0.0},
    {160, 100, 4, 0, 0, 0, 0, 0, 2.0},
};
#define N_SPECS ((int)(sizeof(SPECS) / sizeof(SPECS[0])))

static mipx_plan g_plan[N_SPECS];
static ref_plan g_ref[N_SPECS];
static int g_requests = 16;
static int g_failures = 0;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

static uint32_t xorshift(uint32_t *s) {
    uint32_t x = *s;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    return *s = x;
}

static void fail(const char *what, int tid, int k, int code) {
    pthread_mutex_lock(&g_mu);
    fprintf(stderr, "thread %d request %d: %s (%d: %s; %s)\n", tid, k, what, code, mipx_strerror(code),
            mipx_last_error());
    ++g_failures;
    pthread_mutex_unlock(&g_mu);
}

static void *submitter(void *arg) {
    const int tid = (int)(intptr_t)arg;
    uint32_t seed = 0x9e3779b9u ^ (uint32_t)(tid * 7919 + 1);
    uint8_t **ins = calloc(g_requests, sizeof(uint8_t *));
    uint8_t **outs = calloc(g_requests, sizeof(uint8_t *));
    uint8_t **keep = calloc(g_requests, sizeof(uint8_t *));
    uint64_t *tickets = calloc(g_requests, sizeof(uint64_t));
    for (int k = 0; k < g_requests; ++k) {  /* submit everything first: requests overlap */
        const int si = (tid + k) % N_SPECS;
        const mipx_plan *p = &g_plan[si];
        const size_t ib = (size_t)p->in_w * p->in_h * p->in_bands;
        const size_t ob = (size_t)p->out_w * p->out_h * p->out_bands;
        ins[k] = malloc(ib);
        outs[k] = malloc(ob);
        for (size_t i = 0; i < ib; ++i) ins[k][i] = (uint8_t)xorshift(&seed);
        mipx_img in = {ins[k], p->in_w, p->in_h, p->in_bands, 0};
        mipx_img out = {outs[k], p->out_w, p->out_h, p->out_bands, 0};
        const int e = mipx_submit(-1, p, &in, NULL, &out, &tickets[k]);
        if (e) fail("mipx_submit", tid, k, e);
        /* the input is staged before submit returns (cgo rule): the caller may reuse
         * its buffer at once, so scribble on it and keep the real pixels aside */
        keep[k] = malloc(ib);
        memcpy(keep[k], ins[k], ib);
        memset(ins[k], 0xA5, ib);
    }
    for (int k = 0; k < g_requests; ++k) {
        const int si = (tid + k) % N_SPECS;
        const int e = mipx_wait(tickets[k], -1);
        if (e) {
            fail("mipx_wait", tid, k, e);
            continue;
        }
        const ref_plan *rp = &g_ref[si];
        ref_img rin = {keep[k], rp->in_w, rp->in_h, rp->in_bands};
        ref_img rout = {0};
        const int re = ref_execute(rp, &rin, NULL, &rout);
        if (re || rout.w != g_plan[si].out_w || rout.h != g_plan[si].out_h || rout.bands != g_plan[si].out_bands) {
            fail("oracle", tid, k, re);
        } else if (memcmp(rout.data, outs[k], (size_t)rout.w * rout.h * rout.bands) != 0) {
            fail("output differs from the oracle", tid, k, 0);
        }
        ref_free(rout.data);
    }
    for (int k = 0; k < g_requests; ++k) {
        free(ins[k]);
        free(keep[k]);
        free(outs[k]);
    }
    free(ins);
    free(keep);
    free(outs);
    free(tickets);
    return NULL;
}

int main(int argc, char **argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 4;
    g_requests = argc > 2 ? atoi(argv[2]) : 16;
    const int qpd = argc > 3 ? atoi(argv[3]) : 2;
    if (mipx_abi_version() != MIPX_ABI_VERSION) {
        fprintf(stderr, "ABI %d != header %d\n", mipx_abi_version(), MIPX_ABI_VERSION);
        return 1;
    }
    if (mipx_device_count() <= 0) {
        fprintf(stderr, "no device\n");
        return 77;
    }
    for (int i = 0; i < N_SPECS; ++i) {
        const spec_t *s = &SPECS[i];
        mipx_opts o;
        memset(&o, 0, sizeof o);
        o.width = s->width, o.height = s->height, o.crop = s->crop, o.embed = s->embed;
        o.gravity = s->gravity, o.sigma = s->sigma, o.extend = MIPX_EXTEND_COPY;
        mipx_input in;
        memset(&in, 0, sizeof in);
        in.w = s->w, in.h = s->h, in.bands = s->bands, in.type = MIPX_TYPE_PNG;
        int e = mipx_plan_make(&o, &in, &g_plan[i]);
        if (e) {
            fprintf(stderr, "mipx_plan_make spec %d: %d %s\n", i, e, mipx_last_error());
            return 1;
        }
        ref_opts ro;
        memset(&ro, 0, sizeof ro);
        ro.width = s->width, ro.height = s->height, ro.crop = s->crop, ro.embed = s->embed;
        ro.gravity = s->gravity, ro.sigma = s->sigma, ro.extend = REF_EXTEND_COPY;
        ref_input ri;
        memset(&ri, 0, sizeof ri);
        ri.w = s->w, ri.h = s->h, ri.bands = s->bands, ri.type = REF_TYPE_PNG;
        if (ref_plan_make(&ro, &ri, &g_ref[i]) != 0) {
            fprintf(stderr, "ref_plan_make spec %d failed\n", i);
            return 1;
        }
    }
    mipx_cfg cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.max_batch = 8;
    cfg.batch_wait_us = 500;
    cfg.queues_per_device = qpd;
    int e = mipx_init(&cfg);
    if (e) {
        fprintf(stderr, "mipx_init: %d %s\n", e, mipx_last_error());
        return 1;
    }
    pthread_t th[64];
    const int nt = threads < 64 ? threads : 64;
    for (int t = 0; t < nt; ++t) pthread_create(&th[t], NULL, submitter, (void *)(intptr_t)t);
    for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL);

    /* cancel: a detached request never writes the caller's buffer, even after it is freed */
    {
        const mipx_plan *p = &g_plan[0];
        const size_t ib = (size_t)p->in_w * p->in_h * p->in_bands;
        const size_t ob = (size_t)p->out_w * p->out_h * p->out_bands;
        uint8_t *in = calloc(1, ib), *out = malloc(ob);
        mipx_img mi = {in, p->in_w, p->in_h, p->in_bands, 0};
        mipx_img mo = {out, p->out_w, p->out_h, p->out_bands, 0};
        uint64_t t = 0;
        if ((e = mipx_submit(-1, p, &mi, NULL, &mo, &t)) != 0) fail("cancel submit", -1, 0, e);
        if ((e = mipx_cancel(t)) != 0) fail("mipx_cancel", -1, 0, e);
        free(out);
        free(in);
        if (mipx_wait(t, 0) != MIPX_ESTALE) fail("ticket live after cancel", -1, 0, 0);
        if (mipx_cancel(t) != MIPX_ESTALE) fail("second cancel", -1, 0, 0);
    }

    const int nq = mipx_queue_count();
    uint64_t total_req = 0, total_batches = 0;
    int busy_queues = 0;
    for (int q = 0; q < nq; ++q) {
        int32_t dev = -1;
        uint64_t b = 0, r = 0;
        int64_t pend = -1;
        if ((e = mipx_queue_stats(q, &dev, &b, &r, &pend)) != 0) fail("mipx_queue_stats", -1, q, e);
        printf("queue %d device %d batches %llu requests %llu pending_bytes %lld\n", q, dev,
               (unsigned long long)b, (unsigned long long)r, (long long)pend);
        total_req += r;
        total_batches += b;
        busy_queues += r > 0;
    }
    mipx_shutdown();
    /* the cancelled request is retired too, possibly after the stats were read */
    const uint64_t want = (uint64_t)nt * g_requests;
    if (total_req < want || total_req > want + 1) {
        fprintf(stderr, "retired %llu requests, submitted %llu\n", (unsigned long long)total_req,
                (unsigned long long)want);
        ++g_failures;
    }
    printf("%s: %d threads x %d requests, %d queues (%d used), %llu batches, build %s\n",
           g_failures ? "FAIL" : "ok", nt, g_requests, nq, busy_queues, (unsigned long long)total_batches,
           mipx_build_id());
    return g_failures ? 1 : 0;
}
