// Probe of ds_read_b64_tr_b8 (gfx950): which LDS bytes each lane receives for
// given per-lane addresses.  LDS byte a holds (a & 0xff) in pass 0 and (a >> 8) in
// pass 1, so the source address of every received byte is recovered exactly.
// Mode 0: lane l passes 8 l (contiguous 8-byte chunks); mode 1: within each 16-lane
// group, lane i passes (i & 7) * 256 + (i >> 3) * 8 + group * 16 (rows 256 B apart).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v2i __attribute__((ext_vector_type(2)));
__global__ void k(int *out, int pass, int mode) {
    __shared__ unsigned char s[8192];
    for (int i = threadIdx.x; i < 8192; i += 64) s[i] = (unsigned char)(pass ? (i >> 8) : i);
    __syncthreads();
    const int l = threadIdx.x, g = l >> 4, i = l & 15;
    const int addr = mode == 0 ? 8 * l : (i & 7) * 256 + (i >> 3) * 8 + g * 16;
    v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i *)(s + addr));
    out[l * 2] = r[0];
    out[l * 2 + 1] = r[1];
}
int main() {
    int *d, h0[128], h1[128];
    hipMalloc(&d, 512);
    for (int mode = 0; mode < 2; ++mode) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 0, mode);
        hipMemcpy(h0, d, 512, hipMemcpyDeviceToHost);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 1, mode);
        hipMemcpy(h1, d, 512, hipMemcpyDeviceToHost);
        printf("mode %d\n", mode);
        for (int l = 0; l < 64; ++l) {
            printf("lane %2d:", l);
            for (int b = 0; b < 8; ++b) {
                const int lo = (h0[l * 2 + b / 4] >> (8 * (b % 4))) & 255, hi = (h1[l * 2 + b / 4] >> (8 * (b % 4))) & 255;
                printf(" %4d", hi * 256 + lo);
            }
            printf("\n");
        }
    }
    return 0;
}
