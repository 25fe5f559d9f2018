// Calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// patterns of k_reduce2x2: per-lane dword buffer loads (reads) and per-lane
// 12-byte dwordx3 stores (writes), against known byte counts.  Run under
// rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE) in separate passes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void rd_dword(const uint8_t *p, size_t n, uint32_t *sink) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p), 0, 0x7fffffff, 0x00020000);
    uint32_t acc = 0;
    const size_t per_block = 4 * 256 * 64;  // 64 dword rows per block
    const size_t base = blockIdx.x * per_block;
    for (int i = 0; i < 64; ++i) {
        const size_t off = base + i * 1024 + threadIdx.x * 4;
        if (off + 4 <= n) acc += __builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)(off & 0xffffffff), 0, 0);
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}
__global__ void rd_dwordx4(const uint4 *p, size_t n16, uint32_t *sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        uint4 v = p[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}
__global__ void wr_dwordx3(uint8_t *p, size_t n12) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n12; i += (size_t)gridDim.x * 256)
        *reinterpret_cast<uint3 *>(p + 12 * i) = uint3{(uint32_t)i, 1u, 2u};
}

int main() {
    const size_t N = (size_t)1 << 31;  // 2 GiB, far beyond the 256 MiB Infinity Cache
    uint8_t *buf; uint32_t *sink;
    hipMalloc(&buf, N + 64);
    hipMalloc(&sink, 1 << 24);
    hipMemset(buf, 1, N);
    hipDeviceSynchronize();
    const size_t blocks = N / (4 * 256 * 64);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    float ms;
    hipEventRecord(a); rd_dword<<<(unsigned)blocks, 256>>>(buf, N, sink); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b); printf("rd_dword   bytes=%zu ms=%.3f GBps=%.1f\n", N, ms, N / ms / 1e6);
    hipEventRecord(a); rd_dwordx4<<<4096, 256>>>((const uint4 *)buf, N / 16, sink); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b); printf("rd_dwordx4 bytes=%zu ms=%.3f GBps=%.1f\n", N, ms, N / ms / 1e6);
    const size_t n12 = N / 12;
    hipEventRecord(a); wr_dwordx3<<<4096, 256>>>(buf, n12); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b); printf("wr_dwordx3 bytes=%zu ms=%.3f GBps=%.1f\n", n12 * 12, ms, n12 * 12 / ms / 1e6);
    hipFree(buf); hipFree(sink);
    return 0;
}
