/*
 * mipx_e2e.c — request-path throughput from C, the way a cgo caller drives it
 * (one OS thread per in-flight goroutine): T threads each keep
 * `inflight` 4K RGB -> 1920x1080 requests outstanding (mipx_submit from host
 * memory, mipx_wait on the oldest), over pre-faulted caller buffers.  Prints one
 * JSON line: requests/s, host-link GB/s (pixels in + out), batches per queue.
 * Nothing Python sits between the callers and the engine, so the line is the
 * runtime's own rate for host-resident requests (bench_configs.py E2E measures
 * the same path from Python threads).
 *
 *   mipx_e2e [threads] [requests_per_thread] [queues_per_device] [inflight] [max_batch]
 *
 * Exit 0 = ok; 1 = engine error; 77 = no device.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mipx.h"

static mipx_plan g_plan;
static int g_requests = 64, g_inflight = 2, g_failures = 0;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_barrier_t g_start;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void fail(const char *what, int code) {
    pthread_mutex_lock(&g_mu);
    fprintf(stderr, "%s: %d %s (%s)\n", what, code, mipx_strerror(code), mipx_last_error());
    ++g_failures;
    pthread_mutex_unlock(&g_mu);
}

static void *caller(void *arg) {
    (void)arg;
    const size_t ib = (size_t)g_plan.in_w * g_plan.in_h * g_plan.in_bands;
    const size_t ob = (size_t)g_plan.out_w * g_plan.out_h * g_plan.out_bands;
    uint8_t **in = calloc(g_inflight, sizeof(uint8_t *)), **out = calloc(g_inflight, sizeof(uint8_t *));
    uint64_t *tk = calloc(g_inflight, sizeof(uint64_t));
    for (int s = 0; s < g_inflight; ++s) {  /* pre-faulted, like a server's reused request buffers */
        in[s] = malloc(ib);
        out[s] = malloc(ob);
        for (size_t i = 0; i < ib; ++i) in[s][i] = (uint8_t)(i * 131u + s);
        memset(out[s], 0, ob);
    }
    pthread_barrier_wait(&g_start);
    for (int k = 0; k < g_requests; ++k) {
        const int s = k % g_inflight;
        if (k >= g_inflight) {
            const int e = mipx_wait(tk[s], -1);
            if (e) fail("mipx_wait", e);
        }
        mipx_img mi = {in[s], g_plan.in_w, g_plan.in_h, g_plan.in_bands, 0};
        mipx_img mo = {out[s], g_plan.out_w, g_plan.out_h, g_plan.out_bands, 0};
        const int e = mipx_submit(-1, &g_plan, &mi, NULL, &mo, &tk[s]);
        if (e) fail("mipx_submit", e);
    }
    for (int k = g_requests > g_inflight ? g_requests - g_inflight : 0; k < g_requests; ++k) {
        const int e = mipx_wait(tk[k % g_inflight], -1);
        if (e) fail("mipx_wait", e);
    }
    pthread_barrier_wait(&g_start);
    for (int s = 0; s < g_inflight; ++s) {
        free(in[s]);
        free(out[s]);
    }
    free(in);
    free(out);
    free(tk);
    return NULL;
}

int main(int argc, char **argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 16;
    g_requests = argc > 2 ? atoi(argv[2]) : 64;
    const int qpd = argc > 3 ? atoi(argv[3]) : 1;
    g_inflight = argc > 4 ? atoi(argv[4]) : 2;
    const int max_batch = argc > 5 ? atoi(argv[5]) : 8;
    if (mipx_abi_version() != MIPX_ABI_VERSION) return 1;
    if (mipx_device_count() <= 0) {
        fprintf(stderr, "no device\n");
        return 77;
    }
    mipx_opts o;
    memset(&o, 0, sizeof o);
    o.width = 1920, o.height = 1080, o.extend = MIPX_EXTEND_COPY;
    mipx_input mi;
    memset(&mi, 0, sizeof mi);
    mi.w = 3840, mi.h = 2160, mi.bands = 3, mi.type = MIPX_TYPE_PNG;
    int e = mipx_plan_make(&o, &mi, &g_plan);
    if (e) {
        fprintf(stderr, "plan: %d %s\n", e, mipx_last_error());
        return 1;
    }
    mipx_cfg cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.max_batch = max_batch;
    cfg.queues_per_device = qpd;
    if ((e = mipx_init(&cfg)) != 0) {
        fprintf(stderr, "init: %d %s\n", e, mipx_last_error());
        return 1;
    }
    const int nt = threads < 256 ? threads : 256;
    pthread_t th[256];
    /* warm-up round (pinned pool growth, first launches) */
    {
        const int saved = g_requests;
        g_requests = g_inflight;
        pthread_barrier_init(&g_start, NULL, nt + 1);
        for (int t = 0; t < nt; ++t) pthread_create(&th[t], NULL, caller, NULL);
        pthread_barrier_wait(&g_start);
        pthread_barrier_wait(&g_start);
        for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL);
        pthread_barrier_destroy(&g_start);
        g_requests = saved;
    }
    uint64_t b0 = 0, r0 = 0;
    for (int q = 0; q < mipx_queue_count(); ++q) {
        int32_t d;
        uint64_t b, r;
        int64_t p;
        mipx_queue_stats(q, &d, &b, &r, &p);
        b0 += b, r0 += r;
    }
    pthread_barrier_init(&g_start, NULL, nt + 1);
    for (int t = 0; t < nt; ++t) pthread_create(&th[t], NULL, caller, NULL);
    pthread_barrier_wait(&g_start);
    const double t0 = now_s();
    pthread_barrier_wait(&g_start);
    const double t1 = now_s();
    for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL);
    pthread_barrier_destroy(&g_start);
    uint64_t b1 = 0, r1 = 0;
    for (int q = 0; q < mipx_queue_count(); ++q) {
        int32_t d;
        uint64_t b, r;
        int64_t p;
        mipx_queue_stats(q, &d, &b, &r, &p);
        b1 += b, r1 += r;
    }
    mipx_shutdown();
    const double n = (double)nt * g_requests, wall = t1 - t0;
    const double bytes = n * ((double)g_plan.in_w * g_plan.in_h * g_plan.in_bands +
                              (double)g_plan.out_w * g_plan.out_h * g_plan.out_bands);
    printf("{\"config\": \"E2E-C\", \"workload\": \"request path from C: 4K RGB -> %dx%d from host memory, %d caller "
           "threads x %d in flight, %d queue(s), max_batch %d\", \"images_per_sec\": %.1f, \"requests\": %.0f, "
           "\"wall_s\": %.4f, \"host_link_gbs\": %.2f, \"batches\": %llu, \"mean_batch\": %.2f, \"failures\": %d}\n",
           g_plan.out_w, g_plan.out_h, nt, g_inflight, qpd, max_batch, n / wall, n, wall, bytes / wall / 1e9,
           (unsigned long long)(b1 - b0), b1 > b0 ? (double)(r1 - r0) / (double)(b1 - b0) : 0.0, g_failures);
    return g_failures ? 1 : 0;
}
