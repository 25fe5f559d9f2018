// mipx_runtime.cpp — C-ABI runtime of libmipx.so: errors, device-resident
// coefficient tables, the plan executor, and the request path (pinned staging,
// one worker + stream per device, cross-request batching of identical plans).
//
// Reference seam: imaginary's Process() (image.go:81-113) calls bimg.Resize per
// HTTP request from one goroutine each.  Here every such
// request becomes mipx_submit(): its decoded pixels are copied into pinned
// memory before the call returns (cgo rule), requests with byte-identical plans
// queued on the same device are fused into one batched launch sequence, and
// mipx_wait() hands the result back.  Requests are independent, so multi-GPU is
// one queue per device with least-loaded dispatch — no collectives.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "mipx_internal.h"

namespace mipx {

// ---- errors -------------------------------------------------------------
static thread_local char g_err[512];

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int hip_fail(hipError_t e, const char *what) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return MIPX_EDEVICE;
}

// ---- device tables --------------------------------------------------------
namespace {
struct TableCache {
    std::mutex mu;
    std::map<std::pair<int, double>, std::pair<float *, int>> reduce;  // (device, shrink)
    std::map<int, float *> colour;
    std::map<int, int *> bicubic;
    std::map<std::tuple<int, double, double>, std::tuple<float *, int, int>> gauss;  // (device, sigma, min_ampl)
};
TableCache &tables() {
    static TableCache *t = new TableCache();  // leaked on purpose: outlives static dtors
    return *t;
}
}  // namespace

const float *device_reduce_table(double shrink, int *n_taps) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    TableCache &tc = tables();
    std::lock_guard<std::mutex> lk(tc.mu);
    auto key = std::make_pair(dev, shrink);
    auto it = tc.reduce.find(key);
    if (it != tc.reduce.end()) {
        *n_taps = it->second.second;
        return it->second.first;
    }
    std::vector<int> t;
    reduce_table(shrink, t);
    std::vector<float> f(t.begin(), t.end());
    float *d = nullptr;
    if (hipMalloc(&d, f.size() * sizeof(float)) != hipSuccess) return nullptr;
    if (hipMemcpy(d, f.data(), f.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return nullptr;
    }
    const int n = reduce_points(shrink);
    tc.reduce[key] = {d, n};
    *n_taps = n;
    return d;
}

const float *device_gauss_table(double sigma, double min_ampl, int *n_taps, int *scale) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    TableCache &tc = tables();
    std::lock_guard<std::mutex> lk(tc.mu);
    auto key = std::make_tuple(dev, sigma, min_ampl);
    auto it = tc.gauss.find(key);
    if (it != tc.gauss.end()) {
        *n_taps = std::get<1>(it->second);
        *scale = std::get<2>(it->second);
        return std::get<0>(it->second);
    }
    std::vector<int> mask;
    int sc = 0;
    const int n = gaussmat(sigma, min_ampl, mask, sc);
    if (n <= 0) return nullptr;
    std::vector<float> f(mask.begin(), mask.end());
    float *d = nullptr;
    if (hipMalloc(&d, f.size() * sizeof(float)) != hipSuccess) return nullptr;
    if (hipMemcpy(d, f.data(), f.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return nullptr;
    }
    tc.gauss[key] = std::make_tuple(d, n, sc);
    *n_taps = n;
    *scale = sc;
    return d;
}

bool sep_spec_gauss(double sigma, double min_ampl, SepSpec *s) {
    int taps = 0, scale = 0;
    s->tab = device_gauss_table(sigma, min_ampl, &taps, &scale);
    if (!s->tab) return false;
    s->taps = taps;
    s->mode = kSepConv;
    s->shrink = 1.0;
    s->scale = scale;
    return true;
}

const float *device_colour_tables() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    TableCache &tc = tables();
    std::lock_guard<std::mutex> lk(tc.mu);
    auto it = tc.colour.find(dev);
    if (it != tc.colour.end()) return it->second;
    std::vector<float> h(256 + kQuantElements + 257);
    std::memcpy(h.data(), v2y8_table(), 256 * sizeof(float));
    std::memcpy(h.data() + 256, cbrt_table(), kQuantElements * sizeof(float));
    std::memcpy(h.data() + 256 + kQuantElements, y2v8_table(), 257 * sizeof(float));
    float *d = nullptr;
    if (hipMalloc(&d, h.size() * sizeof(float)) != hipSuccess) return nullptr;
    if (hipMemcpy(d, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return nullptr;
    }
    tc.colour[dev] = d;
    return d;
}

const int *device_bicubic_table() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    TableCache &tc = tables();
    std::lock_guard<std::mutex> lk(tc.mu);
    auto it = tc.bicubic.find(dev);
    if (it != tc.bicubic.end()) return it->second;
    std::vector<int> t((kTransformScale + 1) * 4);
    bicubic_table(t.data());
    int *d = nullptr;
    if (hipMalloc(&d, t.size() * sizeof(int)) != hipSuccess) return nullptr;
    if (hipMemcpy(d, t.data(), t.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return nullptr;
    }
    tc.bicubic[dev] = d;
    return d;
}

void free_device_tables() {
    TableCache &tc = tables();
    std::lock_guard<std::mutex> lk(tc.mu);
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (auto &kv : tc.reduce) {
        (void)hipSetDevice(kv.first.first);
        (void)hipFree(kv.second.first);
    }
    for (auto &kv : tc.colour) {
        (void)hipSetDevice(kv.first);
        (void)hipFree(kv.second);
    }
    for (auto &kv : tc.bicubic) {
        (void)hipSetDevice(kv.first);
        (void)hipFree(kv.second);
    }
    tc.bicubic.clear();
    for (auto &kv : tc.gauss) {
        (void)hipSetDevice(std::get<0>(kv.first));
        (void)hipFree(std::get<0>(kv.second));
    }
    tc.reduce.clear();
    tc.colour.clear();
    tc.gauss.clear();
    (void)hipSetDevice(cur);
}

// ---- plan executor ------------------------------------------------------------
static size_t align256(size_t v) { return (v + 255) & ~static_cast<size_t>(255); }

struct ExecLayout {
    size_t buf_bytes = 0;  // each of the two ping-pong buffers
    size_t aux_bytes = 0;  // largest per-op workspace
    size_t total() const { return 2 * buf_bytes + aux_bytes; }
};

static int plan_layout(const mipx_plan *p, int n, ExecLayout *L) {
    if (!p || n <= 0 || p->n_steps < 0 || p->n_steps > MIPX_MAX_STEPS) return MIPX_EINVAL;
    int w = p->in_w, h = p->in_h, b = p->in_bands;
    size_t buf = 0, aux = 0;
    for (int i = 0; i < p->n_steps; ++i) {
        const mipx_step &s = p->steps[i];
        double p0 = 0, p1 = 0;
        if (s.op == MIPX_OP_REDUCE) p0 = s.d[0], p1 = s.d[1];
        if (s.op == MIPX_OP_BLUR) p0 = s.d[0], p1 = s.d[1];
        if (s.op == MIPX_OP_SMARTCROP) p0 = s.a[0], p1 = s.a[1];
        aux = std::max(aux, op_workspace_bytes(s.op, n, w, h, b, p0, p1));
        w = s.out_w, h = s.out_h, b = s.out_bands;
        if (w <= 0 || h <= 0 || b <= 0 || b > 4) return MIPX_EINVAL;
        if (i + 1 < p->n_steps) buf = std::max(buf, align256(static_cast<size_t>(n) * w * h * b));
    }
    if (w != p->out_w || h != p->out_h || b != p->out_bands) return MIPX_EINVAL;
    L->buf_bytes = buf;
    L->aux_bytes = align256(aux);
    return MIPX_OK;
}

int execute_plan(const mipx_plan *p, int n, const uint8_t *d_in, uint8_t *d_out, const uint8_t *d_wm,
                 void *d_ws, size_t ws_bytes, hipStream_t st) {
    ExecLayout L;
    int e = plan_layout(p, n, &L);
    if (e) return e;
    if (L.total() > 0 && (!d_ws || ws_bytes < L.total())) {
        set_error("workspace %zu < %zu bytes", ws_bytes, L.total());
        return MIPX_EINVAL;
    }
    uint8_t *bufA = static_cast<uint8_t *>(d_ws);
    uint8_t *bufB = bufA ? bufA + L.buf_bytes : nullptr;
    uint8_t *aux = bufA ? bufA + 2 * L.buf_bytes : nullptr;
    if (p->n_steps == 0) {
        MIPX_HIP(hipMemcpyAsync(d_out, d_in, static_cast<size_t>(n) * p->in_w * p->in_h * p->in_bands,
                                hipMemcpyDeviceToDevice, st));
        return MIPX_OK;
    }
    const uint8_t *cur = d_in;
    int w = p->in_w, h = p->in_h, b = p->in_bands;
    void *sv = st;
    for (int i = 0; i < p->n_steps; ++i) {
        const mipx_step &s = p->steps[i];
        uint8_t *dst = (i + 1 == p->n_steps) ? d_out : (cur == bufA ? bufB : bufA);
        // Peephole fusions (results identical to running the two ops):
        //  reduce -> extract : the reduce computes only the extract window
        //  extract -> blur   : the blur reads the window in place (COPY edge = window edge)
        if (i + 1 < p->n_steps && p->steps[i + 1].op == MIPX_OP_EXTRACT && s.op == MIPX_OP_REDUCE &&
            !reduce2_eligible(cur, w, h, b, s.d[0], s.d[1])) {
            const mipx_step &x = p->steps[i + 1];
            uint8_t *dst2 = (i + 2 == p->n_steps) ? d_out : (cur == bufA ? bufB : bufA);
            e = reduce_window_launch(cur, dst2, n, w, h, b, s.d[0], s.d[1], x.a[0], x.a[1], x.a[2], x.a[3], aux,
                                     L.aux_bytes, st);
            if (e) return e;
            cur = dst2;
            w = x.out_w, h = x.out_h, b = x.out_bands;
            ++i;
            continue;
        }
        if (i + 1 < p->n_steps && p->steps[i + 1].op == MIPX_OP_BLUR && s.op == MIPX_OP_EXTRACT) {
            const mipx_step &g = p->steps[i + 1];
            uint8_t *dst2 = (i + 2 == p->n_steps) ? d_out : (cur == bufA ? bufB : bufA);
            e = blur_window_launch(cur, dst2, n, w, h, b, s.a[0], s.a[1], s.a[2], s.a[3], g.d[0], g.d[1], aux,
                                   L.aux_bytes, st);
            if (e) return e;
            cur = dst2;
            w = g.out_w, h = g.out_h, b = g.out_bands;
            ++i;
            continue;
        }
        switch (s.op) {
            case MIPX_OP_ROT: e = mipx_op_rot(cur, dst, n, w, h, b, s.a[0], sv); break;
            case MIPX_OP_FLIP: e = mipx_op_flip(cur, dst, n, w, h, b, s.a[0], sv); break;
            case MIPX_OP_SHRINK: e = mipx_op_shrink(cur, dst, n, w, h, b, s.a[0], s.a[1], sv); break;
            case MIPX_OP_REDUCE:
                e = mipx_op_reduce(cur, dst, n, w, h, b, s.d[0], s.d[1], aux, L.aux_bytes, sv);
                break;
            case MIPX_OP_EXTRACT:
                e = mipx_op_extract(cur, dst, n, w, h, b, s.a[0], s.a[1], s.a[2], s.a[3], sv);
                break;
            case MIPX_OP_EMBED:
                e = mipx_op_embed(cur, dst, n, w, h, b, s.a[0], s.a[1], s.a[2], s.a[3], s.a[4], s.a + 5, sv);
                break;
            case MIPX_OP_SMARTCROP:
                e = smartcrop_extract(cur, dst, n, w, h, b, s.a[0], s.a[1], aux, L.aux_bytes, st);
                break;
            case MIPX_OP_BLUR:
                e = mipx_op_gaussblur(cur, dst, n, w, h, b, s.d[0], s.d[1], aux, L.aux_bytes, sv);
                break;
            case MIPX_OP_AFFINE: e = mipx_op_affine(cur, dst, n, w, h, b, s.d[0], s.d[1], s.a[0], sv); break;
            case MIPX_OP_ZOOM: e = mipx_op_zoom(cur, dst, n, w, h, b, s.a[0], s.a[1], sv); break;
            case MIPX_OP_FLATTEN: e = mipx_op_flatten(cur, dst, n, w, h, b, s.a, sv); break;
            case MIPX_OP_BW: e = mipx_op_colourspace_bw(cur, dst, n, w, h, b, sv); break;
            case MIPX_OP_WATERMARK:
                if (!d_wm) return MIPX_EINVAL;
                e = mipx_op_watermark(cur, d_wm, dst, n, w, h, b, s.a[2], s.a[3], s.a[4], s.a[0], s.a[1],
                                      static_cast<float>(s.d[0]), sv);
                break;
            default: e = MIPX_EINVAL;
        }
        if (e) return e;
        cur = dst;
        w = s.out_w, h = s.out_h, b = s.out_bands;
    }
    return MIPX_OK;
}

// ---- request path ----------------------------------------------------------------
//
// Per device: a worker thread forms batches and ENQUEUES them, a completer
// thread retires them.  Each batch occupies one of kSlots buffer slots and
// flows over three non-blocking streams chained by events:
//
//   s_h2d : pinned request inputs -> slot.d_in                 (ev_h2d)
//   s_exec: wait ev_h2d, run the plan  slot.d_in -> slot.d_out (ev_exec)
//   s_d2h : wait ev_exec, slot.d_out -> pinned slot.h_out      (ev_done)
//
// so batch k+1's upload overlaps batch k's kernels and batch k's download
// overlaps batch k+1's kernels.  A slot is reused only after the completer
// has seen its ev_done, so no buffer is overwritten while in flight.
namespace {

constexpr int kSlots = 2;

// Pinned host blocks reused across requests: hipHostMalloc / hipHostFree of a
// 25 MB block costs far more than the copy into it.
class PinnedPool {
   public:
    static size_t size_class(size_t n) {  // 1/16-power-of-two classes, >= 64 KiB
        const size_t floor_c = size_t(64) << 10;
        if (n <= floor_c) return floor_c;
        size_t p = 1;
        while (p < n) p <<= 1;
        const size_t step = p / 16;
        return (n + step - 1) / step * step;
    }
    uint8_t *get(size_t n, size_t *cap) {
        *cap = size_class(n);
        {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = free_.find(*cap);
            if (it != free_.end()) {
                uint8_t *p = it->second;
                free_.erase(it);
                cached_ -= *cap;
                return p;
            }
        }
        void *p = nullptr;
        if (hipHostMalloc(&p, *cap, hipHostMallocPortable) != hipSuccess) return nullptr;
        return static_cast<uint8_t *>(p);
    }
    void put(uint8_t *p, size_t cap) {
        if (!p) return;
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (cached_ + cap <= limit_) {
                free_.emplace(cap, p);
                cached_ += cap;
                return;
            }
        }
        (void)hipHostFree(p);
    }
    void set_limit(size_t l) {
        std::lock_guard<std::mutex> lk(mu_);
        limit_ = l;
    }
    void clear() {
        std::lock_guard<std::mutex> lk(mu_);
        for (auto &kv : free_) (void)hipHostFree(kv.second);
        free_.clear();
        cached_ = 0;
    }

   private:
    std::mutex mu_;
    std::multimap<size_t, uint8_t *> free_;
    size_t cached_ = 0, limit_ = size_t(1) << 30;
};
PinnedPool &pool() {
    static PinnedPool *p = new PinnedPool();  // leaked on purpose: outlives static dtors
    return *p;
}

// Host copies of the request path run on a few threads: one batch's outputs are
// copied out of pinned staging into the callers' buffers in ~1 MiB pieces, which
// also spreads the first-touch page faults of freshly allocated outputs.  The
// calling thread works too, so a call never waits on an idle pool.
class CopyPool {
public:
    explicit CopyPool(int n) {
        for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    void parallel_for(int n, const std::function<void(int)> &fn) {
        if (n <= 0) return;
        auto t = std::make_shared<Task>();
        t->fn = &fn;
        t->n = n;
        t->left = n;
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back(t);
        }
        cv_.notify_all();
        work(*t);
        std::unique_lock<std::mutex> lk(t->mu);
        t->cv.wait(lk, [&] { return t->left.load() == 0; });
    }

private:
    struct Task {
        const std::function<void(int)> *fn = nullptr;
        int n = 0;
        std::atomic<int> next{0}, left{0};
        std::mutex mu;
        std::condition_variable cv;
    };
    static void work(Task &t) {
        for (int i; (i = t.next.fetch_add(1)) < t.n;) {
            (*t.fn)(i);
            if (t.left.fetch_sub(1) == 1) {
                std::lock_guard<std::mutex> lk(t.mu);
                t.cv.notify_all();
            }
        }
    }
    void loop() {
        for (;;) {
            std::shared_ptr<Task> t;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return !q_.empty(); });
                t = q_.front();
                if (t->next.load() >= t->n) {  // exhausted: drop it and look again
                    q_.pop_front();
                    continue;
                }
            }
            work(*t);
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<Task>> q_;
};
CopyPool &copy_pool() {
    static CopyPool *p = new CopyPool(std::max(1u, std::min(8u, std::thread::hardware_concurrency() / 2)));  // leaked: threads live with the process
    return *p;
}

struct Job {
    uint64_t ticket = 0;
    mipx_plan plan{};
    std::vector<uint8_t> plan_key;   // bytes compared for batching
    uint8_t *pin_in = nullptr;       // pinned copy of the packed input (pool block)
    size_t in_bytes = 0, in_cap = 0;
    uint8_t *pin_wm = nullptr;
    size_t wm_bytes = 0, wm_cap = 0;
    mipx_img out{};
    size_t out_bytes = 0;
    int status = 1;                  // 1 = pending
    std::mutex mu;
    std::condition_variable cv;
};

struct Slot {
    uint8_t *d_in = nullptr, *d_out = nullptr, *d_wm = nullptr, *d_ws = nullptr;
    size_t in_cap = 0, out_cap = 0, wm_cap = 0, ws_cap = 0;
    uint8_t *h_out = nullptr;  // pinned output staging
    size_t h_out_cap = 0;
    hipEvent_t ev_h2d = nullptr, ev_exec = nullptr, ev_done = nullptr;
    bool busy = false;
    int status = 0;
    std::vector<std::shared_ptr<Job>> batch;
};

struct Device {
    int id = 0;
    hipStream_t s_h2d = nullptr, s_exec = nullptr, s_d2h = nullptr;
    std::thread worker, completer;
    std::mutex mu;  // request queue
    std::condition_variable cv;
    std::deque<std::shared_ptr<Job>> q;
    std::atomic<int64_t> pending_bytes{0};
    bool stop = false;
    std::mutex fmu;  // slots + in-flight FIFO
    std::condition_variable fcv;
    std::deque<int> inflight;
    bool worker_done = false;
    Slot slots[kSlots];
    std::atomic<uint64_t> batches{0}, requests{0};
};

struct Runtime {
    std::mutex mu;
    bool up = false;
    int max_batch = 64;
    int batch_wait_us = 0;
    std::vector<std::unique_ptr<Device>> devs;
    std::mutex jobs_mu;
    std::unordered_map<uint64_t, std::shared_ptr<Job>> jobs;
    std::atomic<uint64_t> next_ticket{1};
};
Runtime &rt() {
    static Runtime *r = new Runtime();
    return *r;
}

int grow(uint8_t **p, size_t *cap, size_t need) {
    if (need <= *cap) return MIPX_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    size_t sz = need + need / 4;
    MIPX_HIP(hipMalloc(p, sz));
    *cap = sz;
    return MIPX_OK;
}
int grow_host(uint8_t **p, size_t *cap, size_t need) {
    if (need <= *cap) return MIPX_OK;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    size_t sz = need + need / 4;
    MIPX_HIP(hipHostMalloc(reinterpret_cast<void **>(p), sz, hipHostMallocDefault));
    *cap = sz;
    return MIPX_OK;
}

void finish(const std::shared_ptr<Job> &j, int status) {
    std::lock_guard<std::mutex> lk(j->mu);
    j->status = status;
    j->cv.notify_all();
}

// Enqueue one batch on the slot's three-stream chain; never synchronises.
int launch_batch(Device &d, Slot &s) {
    auto &batch = s.batch;
    const mipx_plan &p = batch[0]->plan;
    const int n = static_cast<int>(batch.size());
    const size_t in1 = batch[0]->in_bytes, out1 = batch[0]->out_bytes;
    int e;
    if ((e = grow(&s.d_in, &s.in_cap, in1 * n))) return e;
    if ((e = grow(&s.d_out, &s.out_cap, out1 * n))) return e;
    if ((e = grow_host(&s.h_out, &s.h_out_cap, out1 * n))) return e;
    ExecLayout L;
    if ((e = plan_layout(&p, n, &L))) return e;
    if ((e = grow(&s.d_ws, &s.ws_cap, L.total() + 256))) return e;
    for (int i = 0; i < n; ++i)
        MIPX_HIP(hipMemcpyAsync(s.d_in + in1 * i, batch[i]->pin_in, in1, hipMemcpyHostToDevice, d.s_h2d));
    const uint8_t *wm = nullptr;
    if (batch[0]->pin_wm) {  // watermark is per request; batches share a byte-identical one
        if ((e = grow(&s.d_wm, &s.wm_cap, batch[0]->wm_bytes))) return e;
        MIPX_HIP(hipMemcpyAsync(s.d_wm, batch[0]->pin_wm, batch[0]->wm_bytes, hipMemcpyHostToDevice, d.s_h2d));
        wm = s.d_wm;
    }
    MIPX_HIP(hipEventRecord(s.ev_h2d, d.s_h2d));
    MIPX_HIP(hipStreamWaitEvent(d.s_exec, s.ev_h2d, 0));
    if ((e = execute_plan(&p, n, s.d_in, s.d_out, wm, s.d_ws, s.ws_cap, d.s_exec))) return e;
    MIPX_HIP(hipEventRecord(s.ev_exec, d.s_exec));
    MIPX_HIP(hipStreamWaitEvent(d.s_d2h, s.ev_exec, 0));
    MIPX_HIP(hipMemcpyAsync(s.h_out, s.d_out, out1 * n, hipMemcpyDeviceToHost, d.s_d2h));
    MIPX_HIP(hipEventRecord(s.ev_done, d.s_d2h));
    return MIPX_OK;
}

// Wait for a slot's batch, scatter its outputs to the callers, release it.
void retire_batch(Device &d, Slot &s) {
    int e = s.status;
    if (e == MIPX_OK) {
        const hipError_t he = hipEventSynchronize(s.ev_done);
        if (he != hipSuccess) e = hip_fail(he, "hipEventSynchronize(batch)");
    } else {  // a failed enqueue may have left work behind on any of the streams
        (void)hipStreamSynchronize(d.s_h2d);
        (void)hipStreamSynchronize(d.s_exec);
        (void)hipStreamSynchronize(d.s_d2h);
    }
    const size_t out1 = s.batch[0]->out_bytes;
    if (e == MIPX_OK && out1 > 0) {  // outputs -> callers, in row-aligned pieces of ~1 MiB
        const mipx_img &o0 = s.batch[0]->out;
        const size_t row = static_cast<size_t>(o0.w) * o0.bands;
        const int rows_per = static_cast<int>(std::max<size_t>(1, (size_t(1) << 20) / std::max<size_t>(1, row)));
        const int pieces = (o0.h + rows_per - 1) / rows_per;
        const int nb = static_cast<int>(s.batch.size());
        copy_pool().parallel_for(nb * pieces, [&](int k) {
            const int i = k / pieces, y0 = (k - i * pieces) * rows_per;
            const mipx_img &o = s.batch[i]->out;
            const int y1 = std::min(o.h, y0 + rows_per);
            const size_t stride = o.stride ? static_cast<size_t>(o.stride) : row;
            const uint8_t *src = s.h_out + out1 * i;
            if (stride == row) std::memcpy(o.data + y0 * row, src + y0 * row, (y1 - y0) * row);
            else
                for (int y = y0; y < y1; ++y) std::memcpy(o.data + y * stride, src + y * row, row);
        });
    }
    for (size_t i = 0; i < s.batch.size(); ++i) {
        auto &j = s.batch[i];
        d.pending_bytes -= static_cast<int64_t>(j->in_bytes);
        pool().put(j->pin_in, j->in_cap);
        j->pin_in = nullptr;
        pool().put(j->pin_wm, j->wm_cap);
        j->pin_wm = nullptr;
        finish(j, e);
    }
    d.batches += 1;
    d.requests += s.batch.size();
    s.batch.clear();
}

bool same_batch(const Job &a, const Job &b) {
    if (a.plan_key != b.plan_key || a.wm_bytes != b.wm_bytes) return false;
    if (a.pin_wm && std::memcmp(a.pin_wm, b.pin_wm, a.wm_bytes) != 0) return false;
    return true;
}

void worker_main(Device *d) {
    (void)hipSetDevice(d->id);
    Runtime &r = rt();
    for (;;) {
        std::vector<std::shared_ptr<Job>> batch;
        {
            std::unique_lock<std::mutex> lk(d->mu);
            d->cv.wait(lk, [&] { return d->stop || !d->q.empty(); });
            if (d->stop && d->q.empty()) break;
            if (r.batch_wait_us > 0 && static_cast<int>(d->q.size()) < r.max_batch)
                d->cv.wait_for(lk, std::chrono::microseconds(r.batch_wait_us),
                               [&] { return d->stop || static_cast<int>(d->q.size()) >= r.max_batch; });
            batch.push_back(d->q.front());
            d->q.pop_front();
            for (auto it = d->q.begin(); it != d->q.end() && static_cast<int>(batch.size()) < r.max_batch;) {
                if (same_batch(*batch[0], **it)) {
                    batch.push_back(*it);
                    it = d->q.erase(it);
                } else {
                    ++it;
                }
            }
        }
        int si = -1;
        {
            std::unique_lock<std::mutex> lk(d->fmu);
            d->fcv.wait(lk, [&] {
                for (const Slot &s : d->slots)
                    if (!s.busy) return true;
                return false;
            });
            for (int i = 0; i < kSlots && si < 0; ++i)
                if (!d->slots[i].busy) si = i;
            d->slots[si].busy = true;
        }
        Slot &s = d->slots[si];
        s.batch = std::move(batch);
        s.status = launch_batch(*d, s);
        {
            std::lock_guard<std::mutex> lk(d->fmu);
            d->inflight.push_back(si);
        }
        d->fcv.notify_all();
    }
    {
        std::lock_guard<std::mutex> lk(d->fmu);
        d->worker_done = true;
    }
    d->fcv.notify_all();
}

// Retires batches in submission order; exits once the worker is done and
// nothing is in flight.
void completer_main(Device *d) {
    (void)hipSetDevice(d->id);
    for (;;) {
        int si;
        {
            std::unique_lock<std::mutex> lk(d->fmu);
            d->fcv.wait(lk, [&] { return !d->inflight.empty() || d->worker_done; });
            if (d->inflight.empty()) return;
            si = d->inflight.front();
        }
        retire_batch(*d, d->slots[si]);
        {
            std::lock_guard<std::mutex> lk(d->fmu);
            d->inflight.pop_front();
            d->slots[si].busy = false;
        }
        d->fcv.notify_all();
    }
}

int pack_pinned(const mipx_img *img, uint8_t **dst, size_t *bytes, size_t *cap) {
    const size_t row = static_cast<size_t>(img->w) * img->bands;
    const size_t stride = img->stride ? static_cast<size_t>(img->stride) : row;
    *bytes = row * img->h;
    *dst = pool().get(*bytes, cap);
    if (!*dst) {
        set_error("pinned staging: hipHostMalloc(%zu) failed", *cap);
        return MIPX_ENOMEM;
    }
    if (stride == row) std::memcpy(*dst, img->data, *bytes);
    else
        for (int y = 0; y < img->h; ++y) std::memcpy(*dst + y * row, img->data + y * stride, row);
    return MIPX_OK;
}

void destroy_device(Device &d) {
    (void)hipSetDevice(d.id);
    for (Slot &s : d.slots) {
        (void)hipFree(s.d_in);
        (void)hipFree(s.d_out);
        (void)hipFree(s.d_wm);
        (void)hipFree(s.d_ws);
        if (s.h_out) (void)hipHostFree(s.h_out);
        if (s.ev_h2d) (void)hipEventDestroy(s.ev_h2d);
        if (s.ev_exec) (void)hipEventDestroy(s.ev_exec);
        if (s.ev_done) (void)hipEventDestroy(s.ev_done);
        s = Slot();
    }
    if (d.s_h2d) (void)hipStreamDestroy(d.s_h2d);
    if (d.s_exec) (void)hipStreamDestroy(d.s_exec);
    if (d.s_d2h) (void)hipStreamDestroy(d.s_d2h);
    d.s_h2d = d.s_exec = d.s_d2h = nullptr;
}

int create_device(Device &d) {
    MIPX_HIP(hipSetDevice(d.id));
    MIPX_HIP(hipStreamCreateWithFlags(&d.s_h2d, hipStreamNonBlocking));
    MIPX_HIP(hipStreamCreateWithFlags(&d.s_exec, hipStreamNonBlocking));
    MIPX_HIP(hipStreamCreateWithFlags(&d.s_d2h, hipStreamNonBlocking));
    for (Slot &s : d.slots) {
        MIPX_HIP(hipEventCreateWithFlags(&s.ev_h2d, hipEventDisableTiming));
        MIPX_HIP(hipEventCreateWithFlags(&s.ev_exec, hipEventDisableTiming));
        MIPX_HIP(hipEventCreateWithFlags(&s.ev_done, hipEventDisableTiming));
    }
    return MIPX_OK;
}

}  // namespace
}  // namespace mipx

// ===========================================================================
// C-ABI
// ===========================================================================
using namespace mipx;

extern "C" {

const char *mipx_version(void) { return "mipx 0.1.0 (gfx950)"; }
int mipx_abi_version(void) { return MIPX_ABI_VERSION; }
const char *mipx_last_error(void) { return g_err; }

const char *mipx_strerror(int code) {
    switch (code) {
        case MIPX_OK: return "ok";
        case MIPX_EINVAL: return "invalid argument";
        case MIPX_EUNSUPPORTED: return "operation not supported by the engine (fall back to bimg)";
        case MIPX_ENOMEM: return "out of memory";
        case MIPX_ENODEV: return "no usable gfx950 device";
        case MIPX_EDEVICE: return "HIP runtime error";
        case MIPX_ETIMEOUT: return "timed out";
        case MIPX_ENOTINIT: return "engine not initialised";
        case MIPX_ESTALE: return "unknown ticket";
        default: return "unknown error";
    }
}

int mipx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int mipx_init(const mipx_cfg *cfg) {
    Runtime &r = rt();
    std::lock_guard<std::mutex> lk(r.mu);
    if (r.up) return MIPX_OK;
    int ndev = mipx_device_count();
    if (ndev <= 0) {
        set_error("no HIP devices visible");
        return MIPX_ENODEV;
    }
    std::vector<int> ids;
    if (cfg && cfg->n_devices > 0) {
        for (int i = 0; i < cfg->n_devices && i < 16; ++i)
            if (cfg->device_ids[i] >= 0 && cfg->device_ids[i] < ndev) ids.push_back(cfg->device_ids[i]);
    } else {
        for (int i = 0; i < ndev; ++i) ids.push_back(i);
    }
    if (ids.empty()) return MIPX_ENODEV;
    r.max_batch = (cfg && cfg->max_batch > 0) ? cfg->max_batch : 64;
    r.batch_wait_us = (cfg && cfg->batch_wait_us > 0) ? cfg->batch_wait_us : 0;
    pool().set_limit((cfg && cfg->staging_bytes > 0) ? static_cast<size_t>(cfg->staging_bytes) : size_t(1) << 30);
    for (int id : ids) {
        auto d = std::make_unique<Device>();
        d->id = id;
        const int e = create_device(*d);
        if (e) {
            destroy_device(*d);
            for (auto &o : r.devs) destroy_device(*o);
            r.devs.clear();
            return e;
        }
        r.devs.push_back(std::move(d));
    }
    for (auto &d : r.devs) {
        d->worker = std::thread(worker_main, d.get());
        d->completer = std::thread(completer_main, d.get());
    }
    r.up = true;
    return MIPX_OK;
}

void mipx_shutdown(void) {
    Runtime &r = rt();
    std::lock_guard<std::mutex> lk(r.mu);
    if (!r.up) return;
    for (auto &d : r.devs) {
        {
            std::lock_guard<std::mutex> dl(d->mu);
            d->stop = true;
        }
        d->cv.notify_all();
    }
    for (auto &d : r.devs) {  // the worker drains the queue; the completer retires it
        if (d->worker.joinable()) d->worker.join();
        if (d->completer.joinable()) d->completer.join();
        destroy_device(*d);
    }
    r.devs.clear();
    pool().clear();
    free_device_tables();
    r.up = false;
}

int mipx_stats(int device, uint64_t *batches, uint64_t *requests) {
    Runtime &r = rt();
    std::lock_guard<std::mutex> lk(r.mu);
    if (!r.up) return MIPX_ENOTINIT;
    for (auto &d : r.devs)
        if (d->id == device) {
            if (batches) *batches = d->batches.load();
            if (requests) *requests = d->requests.load();
            return MIPX_OK;
        }
    return MIPX_EINVAL;
}

int mipx_submit(int device, const mipx_plan *plan, const mipx_img *in, const mipx_img *wm, mipx_img *out,
                uint64_t *ticket) {
    Runtime &r = rt();
    if (!plan || !in || !out || !ticket || !in->data || !out->data) return MIPX_EINVAL;
    if (in->w != plan->in_w || in->h != plan->in_h || in->bands != plan->in_bands) {
        set_error("input %dx%dx%d does not match plan %dx%dx%d", in->w, in->h, in->bands, plan->in_w, plan->in_h,
                  plan->in_bands);
        return MIPX_EINVAL;
    }
    if (out->w != plan->out_w || out->h != plan->out_h || out->bands != plan->out_bands) {
        set_error("output %dx%dx%d does not match plan %dx%dx%d", out->w, out->h, out->bands, plan->out_w,
                  plan->out_h, plan->out_bands);
        return MIPX_EINVAL;
    }
    bool needs_wm = false;
    for (int i = 0; i < plan->n_steps; ++i) needs_wm |= plan->steps[i].op == MIPX_OP_WATERMARK;
    if (needs_wm && (!wm || !wm->data)) return MIPX_EINVAL;
    Device *dev = nullptr;
    {
        std::lock_guard<std::mutex> lk(r.mu);
        if (!r.up) return MIPX_ENOTINIT;
        if (device >= 0) {
            for (auto &d : r.devs)
                if (d->id == device) dev = d.get();
            if (!dev) return MIPX_EINVAL;
        } else {  // least loaded by queued input bytes
            for (auto &d : r.devs)
                if (!dev || d->pending_bytes.load() < dev->pending_bytes.load()) dev = d.get();
        }
    }
    auto j = std::make_shared<Job>();
    j->plan = *plan;
    const uint8_t *pk = reinterpret_cast<const uint8_t *>(plan);
    j->plan_key.assign(pk, pk + sizeof(mipx_plan));
    int e = pack_pinned(in, &j->pin_in, &j->in_bytes, &j->in_cap);
    if (e) return e;
    if (needs_wm) {
        e = pack_pinned(wm, &j->pin_wm, &j->wm_bytes, &j->wm_cap);
        if (e) {
            pool().put(j->pin_in, j->in_cap);
            return e;
        }
    }
    j->out = *out;
    j->out_bytes = static_cast<size_t>(out->w) * out->h * out->bands;
    j->ticket = r.next_ticket.fetch_add(1);
    {
        std::lock_guard<std::mutex> lk(r.jobs_mu);
        r.jobs[j->ticket] = j;
    }
    dev->pending_bytes += static_cast<int64_t>(j->in_bytes);
    {
        std::lock_guard<std::mutex> lk(dev->mu);
        dev->q.push_back(j);
    }
    dev->cv.notify_one();
    *ticket = j->ticket;
    return MIPX_OK;
}

int mipx_wait(uint64_t ticket, int timeout_ms) {
    Runtime &r = rt();
    std::shared_ptr<Job> j;
    {
        std::lock_guard<std::mutex> lk(r.jobs_mu);
        auto it = r.jobs.find(ticket);
        if (it == r.jobs.end()) return MIPX_ESTALE;
        j = it->second;
    }
    std::unique_lock<std::mutex> lk(j->mu);
    auto done = [&] { return j->status != 1; };
    if (timeout_ms < 0) j->cv.wait(lk, done);
    else if (!j->cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), done)) return MIPX_ETIMEOUT;
    const int st = j->status;
    lk.unlock();
    std::lock_guard<std::mutex> jl(r.jobs_mu);
    r.jobs.erase(ticket);
    return st;
}

int mipx_process(const mipx_plan *plan, const mipx_img *in, const mipx_img *wm, mipx_img *out) {
    uint64_t t = 0;
    int e = mipx_submit(-1, plan, in, wm, out, &t);
    if (e) return e;
    return mipx_wait(t, -1);
}

size_t mipx_workspace_bytes(const mipx_plan *plan, int32_t n) {
    ExecLayout L;
    if (plan_layout(plan, n, &L)) return 0;
    return L.total();
}

int mipx_execute_dev(const mipx_plan *plan, int32_t n, const uint8_t *d_in, uint8_t *d_out, const uint8_t *d_wm,
                     void *d_ws, size_t ws_bytes, void *stream) {
    if (!plan || !d_in || !d_out || n <= 0) return MIPX_EINVAL;
    return execute_plan(plan, n, d_in, d_out, d_wm, d_ws, ws_bytes, as_stream(stream));
}

// ---- device helpers ----
int mipx_set_device(int device) {
    MIPX_HIP(hipSetDevice(device));
    return MIPX_OK;
}
int mipx_dev_malloc(void **ptr, size_t bytes) {
    if (!ptr) return MIPX_EINVAL;
    MIPX_HIP(hipMalloc(ptr, bytes));
    return MIPX_OK;
}
int mipx_dev_free(void *ptr) {
    MIPX_HIP(hipFree(ptr));
    return MIPX_OK;
}
int mipx_memcpy_h2d(void *d, const void *h, size_t bytes) {
    MIPX_HIP(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
    return MIPX_OK;
}
int mipx_memcpy_d2h(void *h, const void *d, size_t bytes) {
    MIPX_HIP(hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost));
    return MIPX_OK;
}
int mipx_memset_dev(void *d, int v, size_t bytes) {
    MIPX_HIP(hipMemset(d, v, bytes));
    return MIPX_OK;
}
int mipx_stream_sync(void *s) {
    MIPX_HIP(hipStreamSynchronize(as_stream(s)));
    return MIPX_OK;
}
int mipx_device_sync(void) {
    MIPX_HIP(hipDeviceSynchronize());
    return MIPX_OK;
}
int mipx_stream_create(void **s) {
    if (!s) return MIPX_EINVAL;
    hipStream_t st;
    MIPX_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    *s = st;
    return MIPX_OK;
}
int mipx_stream_destroy(void *s) {
    MIPX_HIP(hipStreamDestroy(as_stream(s)));
    return MIPX_OK;
}
int mipx_event_create(void **ev) {
    if (!ev) return MIPX_EINVAL;
    hipEvent_t e;
    MIPX_HIP(hipEventCreate(&e));
    *ev = e;
    return MIPX_OK;
}
int mipx_event_destroy(void *ev) {
    MIPX_HIP(hipEventDestroy(reinterpret_cast<hipEvent_t>(ev)));
    return MIPX_OK;
}
int mipx_event_record(void *ev, void *s) {
    MIPX_HIP(hipEventRecord(reinterpret_cast<hipEvent_t>(ev), as_stream(s)));
    return MIPX_OK;
}
int mipx_event_elapsed_ms(void *a, void *b, float *ms) {
    if (!ms) return MIPX_EINVAL;
    MIPX_HIP(hipEventSynchronize(reinterpret_cast<hipEvent_t>(b)));
    MIPX_HIP(hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(a), reinterpret_cast<hipEvent_t>(b)));
    return MIPX_OK;
}

}  // extern "C"
