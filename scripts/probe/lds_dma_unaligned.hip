// Probe: does a direct-to-LDS buffer_load_dword (raw_ptr_buffer_load_lds, 4 bytes)
// honour a byte offset that is not a multiple of 4?  Each lane loads the dword at
// byte 4 * lane + s (s = 0..3) of a byte ramp into LDS and writes it back out; the
// host compares with the unaligned ramp dword.  Prints one line per shift.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(3))) void lds_void;

__global__ void probe(const uint8_t *src, uint32_t *dst, int s) {
    __shared__ uint32_t buf[64];
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src), 0, 4096, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)buf, 4, 4 * threadIdx.x + s, 0, 0, 0);
    __syncthreads();
    dst[threadIdx.x] = buf[threadIdx.x];
    // the same through a plain buffer load for comparison
    dst[64 + threadIdx.x] = static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(rs, 4 * threadIdx.x + s, 0, 0));
}

int main() {
    uint8_t h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = static_cast<uint8_t>(i * 7 + 3);
    uint8_t *d;
    uint32_t *o;
    hipMalloc(&d, 4096);
    hipMalloc(&o, 128 * 4);
    hipMemcpy(d, h, 4096, hipMemcpyHostToDevice);
    for (int s = 0; s < 4; ++s) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, o, s);
        uint32_t r[128];
        hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
        int bad_lds = 0, bad_vgpr = 0;
        uint32_t first_lds = 0, want0 = 0;
        for (int l = 0; l < 64; ++l) {
            uint32_t want = h[4 * l + s] | (h[4 * l + s + 1] << 8) | (h[4 * l + s + 2] << 16) | (uint32_t(h[4 * l + s + 3]) << 24);
            if (l == 0) { first_lds = r[0]; want0 = want; }
            bad_lds += r[l] != want;
            bad_vgpr += r[64 + l] != want;
        }
        printf("{\"shift\": %d, \"lds_dma_mismatch\": %d, \"vgpr_load_mismatch\": %d, \"lane0_lds\": \"%08x\", \"want\": \"%08x\"}\n",
               s, bad_lds, bad_vgpr, first_lds, want0);
    }
    return 0;
}
