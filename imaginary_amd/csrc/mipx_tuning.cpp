// mipx_tuning.cpp — kernel-selection knobs (MIPX_* environment variables) read once,
// and the parity settings (mipx_set_reduce_sampling).
//
// The launchers pick kernels and layouts by geometry; a few MIPX_* variables force
// an alternative for A/B runs and tests (e.g. MIPX_RCOL=0).  They are snapshotted
// from the environment on first use into an immutable map, so no launch calls
// getenv (which is not safe beside a concurrent setenv, and costs time on the
// small-image path).  mipx_tuning_reload() takes a new snapshot; old snapshots are
// kept alive, since a launcher on another thread may still hold one of their strings.
#include <atomic>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "mipx_internal.h"

extern char **environ;

namespace mipx {
namespace {

struct Snapshot {
    std::map<std::string, std::string> kv;
};
std::atomic<const Snapshot *> g_snap{nullptr};
std::mutex g_mu;
std::vector<std::unique_ptr<Snapshot>> &g_all() {
    static auto *v = new std::vector<std::unique_ptr<Snapshot>>();  // leaked on purpose: outlives static dtors
    return *v;
}

const Snapshot *take_snapshot_locked() {
    auto s = std::make_unique<Snapshot>();
    for (char **e = environ; e && *e; ++e) {
        if (std::strncmp(*e, "MIPX_", 5) != 0) continue;
        const char *eq = std::strchr(*e, '=');
        if (eq) s->kv.emplace(std::string(*e, static_cast<size_t>(eq - *e)), std::string(eq + 1));
    }
    const Snapshot *p = s.get();
    g_all().push_back(std::move(s));
    g_snap.store(p, std::memory_order_release);
    return p;
}

}  // namespace

const char *tune_env(const char *name) {
    const Snapshot *s = g_snap.load(std::memory_order_acquire);
    if (!s) {
        std::lock_guard<std::mutex> lk(g_mu);
        s = g_snap.load(std::memory_order_acquire);
        if (!s) s = take_snapshot_locked();
    }
    const auto it = s->kv.find(name);
    return it == s->kv.end() ? nullptr : it->second.c_str();
}

namespace {
std::atomic<int> g_sampling{MIPX_SAMPLE_CORNER};  // PARITY_ASSUMPTIONS.md row 1
thread_local int t_sampling = -1;                 // SamplingScope's convention; -1 = none
}  // namespace

bool reduce_centre() {
    const int t = t_sampling;
    return (t >= 0 ? t : g_sampling.load(std::memory_order_relaxed)) == MIPX_SAMPLE_CENTRE;
}

int reduce_sampling_now() { return g_sampling.load(std::memory_order_relaxed); }

SamplingScope::SamplingScope(int convention) : prev_(t_sampling) {
    t_sampling = convention == MIPX_SAMPLE_CENTRE ? MIPX_SAMPLE_CENTRE : MIPX_SAMPLE_CORNER;
}
SamplingScope::SamplingScope() : prev_(t_sampling) {
    if (prev_ < 0) t_sampling = g_sampling.load(std::memory_order_relaxed);
}
SamplingScope::~SamplingScope() { t_sampling = prev_; }

void tune_reload() {
    std::lock_guard<std::mutex> lk(g_mu);
    take_snapshot_locked();
}

}  // namespace mipx

namespace mipx {

int device_cu_count() {
    static std::mutex mu;
    static std::map<int, int> cus;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cus.find(dev);
    if (it != cus.end()) return it->second;
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
    cus.emplace(dev, n);
    return n;
}

int occupancy_per_cu(const void *fn, int threads, size_t lds, int fallback) {
    static std::mutex mu;
    static std::map<std::tuple<int, const void *, int, size_t>, int> occ;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fallback;
    const auto key = std::make_tuple(dev, fn, threads, lds);
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = occ.find(key);
        if (it != occ.end()) return it->second;
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, lds) != hipSuccess || per_cu < 1)
        per_cu = fallback;
    std::lock_guard<std::mutex> lk(mu);
    occ.emplace(key, per_cu);
    return per_cu;
}

}  // namespace mipx

extern "C" int mipx_set_reduce_sampling(int32_t convention) {
    if (convention != MIPX_SAMPLE_CORNER && convention != MIPX_SAMPLE_CENTRE) return MIPX_EINVAL;
    // plans record the convention they were made under (mipx_plan_make), so queued work
    // does not change; the setter still refuses while it sees mipx_submit requests queued
    // or running, so a caller does not believe its in-flight requests follow the new
    // setting.  Advisory only (mipx.h): no lock spans the check and the store, and work
    // outside mipx_submit is not counted; correctness rests on each plan's a[7]
    if (mipx::requests_in_flight() > 0) {
        mipx::set_error("mipx_set_reduce_sampling: %lld requests queued or running",
                        static_cast<long long>(mipx::requests_in_flight()));
        return MIPX_EBUSY;
    }
    mipx::g_sampling.store(convention, std::memory_order_relaxed);
    return MIPX_OK;
}

extern "C" int mipx_reduce_sampling(void) { return mipx::g_sampling.load(std::memory_order_relaxed); }

extern "C" int mipx_tuning_reload(void) {
    mipx::tune_reload();
    return MIPX_OK;
}
