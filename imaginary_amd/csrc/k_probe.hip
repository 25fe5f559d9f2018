// k_probe.hip — one-time device capability probes behind kernel choices.
//
// lds_dma_unaligned_ok(): k_rmf2 stages image rows whose pitch is not a multiple of
// 4 with direct-to-LDS dword buffer loads at byte offsets that are not multiples of
// 4.  gfx950 honours such offsets (scripts/probe/lds_dma_unaligned.hip,
// profiles/r02/lds_dma_unaligned.jsonl), but that is observed behaviour, not a
// documented guarantee, and a stricter buffer alignment mode would silently change
// the bytes.  So each device runs this check once (at mipx_init, or on first use);
// if any shift 1..3 differs from the unaligned dword, unaligned rows are kept off
// that kernel (the aligned kernels and the two separable passes take them).
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>

#include "device_common.h"

namespace mipx {
namespace {

typedef __attribute__((address_space(3))) void pr_lds_void;

__global__ void __launch_bounds__(64) k_probe_lds_dma(const uint8_t *src, uint32_t *dst) {
    __shared__ uint32_t buf[4][64];
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src), 0, 1024, 0x00020000);
    for (int s = 0; s < 4; ++s)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (pr_lds_void *)buf[s], 4, 4 * threadIdx.x + s, 0, 0, 0);
    __syncthreads();
    for (int s = 0; s < 4; ++s) dst[64 * s + threadIdx.x] = buf[s][threadIdx.x];
}

int run_probe() {
    uint8_t h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = static_cast<uint8_t>(i * 7 + 3);
    uint8_t *d = nullptr;
    uint32_t *o = nullptr;
    if (hipMalloc(&d, 1024) != hipSuccess) return -1;
    if (hipMalloc(&o, 256 * 4) != hipSuccess) {
        (void)hipFree(d);
        return -1;
    }
    uint32_t r[256];
    bool ok = hipMemcpy(d, h, 1024, hipMemcpyHostToDevice) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(k_probe_lds_dma, dim3(1), dim3(64), 0, 0, d, o);
        ok = hipGetLastError() == hipSuccess && hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost) == hipSuccess;
    }
    (void)hipFree(d);
    (void)hipFree(o);
    if (!ok) return -1;
    for (int s = 0; s < 4; ++s)
        for (int l = 0; l < 64; ++l) {
            const int b = 4 * l + s;
            const uint32_t want = h[b] | (h[b + 1] << 8) | (h[b + 2] << 16) | (static_cast<uint32_t>(h[b + 3]) << 24);
            if (r[64 * s + l] != want) return 0;
        }
    return 1;
}

}  // namespace

bool lds_dma_unaligned_ok() {
    const char *f = tune_env("MIPX_LDS_PROBE");  // "fail": behave as a device that fails it (tests)
    if (f && *f == 'f') return false;
    static std::mutex mu;
    static std::map<int, bool> *seen = new std::map<int, bool>();  // leaked: outlives static dtors
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    std::lock_guard<std::mutex> lk(mu);
    auto it = seen->find(dev);
    if (it != seen->end()) return it->second;
    const bool ok = run_probe() == 1;
    (*seen)[dev] = ok;
    return ok;
}

}  // namespace mipx
