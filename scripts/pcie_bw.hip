// Host link ceilings for the request path: pinned H2D, D2H, and both at once
// (separate streams), 256 MiB transfers, median of 5.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
int main() {
    const size_t N = 256u << 20;
    void *h1, *h2, *d1, *d2;
    CK(hipHostMalloc(&h1, N, 0)); CK(hipHostMalloc(&h2, N, 0));
    CK(hipMalloc(&d1, N)); CK(hipMalloc(&d2, N));
    hipStream_t s1, s2; CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto run = [&](int mode) {
        std::vector<float> v;
        for (int it = 0; it < 6; ++it) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a, s1));
            CK(hipStreamWaitEvent(s2, a, 0));
            if (mode != 1) CK(hipMemcpyAsync(d1, h1, N, hipMemcpyHostToDevice, s1));
            if (mode != 0) CK(hipMemcpyAsync(h2, d2, N, hipMemcpyDeviceToHost, s2));
            hipEvent_t e2; CK(hipEventCreate(&e2)); CK(hipEventRecord(e2, s2)); CK(hipStreamWaitEvent(s1, e2, 0));
            CK(hipEventRecord(b, s1)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b)); if (it) v.push_back(ms); CK(hipEventDestroy(e2));
        }
        std::sort(v.begin(), v.end());
        const double bytes = (mode == 2 ? 2.0 : 1.0) * N;
        printf("{\"mode\": \"%s\", \"ms\": %.3f, \"GBps\": %.1f}\n", mode == 0 ? "h2d" : mode == 1 ? "d2h" : "both", v[2], bytes / v[2] / 1e6);
        return 0;
    };
    for (int m = 0; m < 3; ++m) if (run(m)) return 1;
    return 0;
}
