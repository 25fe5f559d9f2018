// probe: v_cvt_pk_u8_f32 rounding and saturation on gfx950 (k_enlm epilogue choice)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
__global__ void k(const float *in, unsigned *out, int n) {
    const int i = threadIdx.x;
    if (i < n) out[i] = __builtin_amdgcn_cvt_pk_u8_f32(in[i], 0, 0u);
}
int main() {
    const float v[] = {-1.5f, -0.5f, -0.25f, 0.25f, 0.4999f, 0.5f, 0.5001f, 1.0f, 1.5f, 2.5f, 3.5f, 127.5f, 128.5f,
                       254.5f, 255.0f, 255.4f, 255.5f, 256.0f, 300.0f, 1e9f, -1e9f, NAN, 2.99999f, 7.75f};
    const int n = sizeof(v) / sizeof(v[0]);
    float *d; unsigned *o;
    if (hipMalloc(&d, sizeof(v)) || hipMalloc(&o, n * 4)) return 1;
    if (hipMemcpy(d, v, sizeof(v), hipMemcpyHostToDevice)) return 3;
    k<<<1, 64>>>(d, o, n);
    unsigned h[64];
    if (hipMemcpy(h, o, n * 4, hipMemcpyDeviceToHost)) return 2;
    for (int i = 0; i < n; ++i) printf("%g -> %u\n", v[i], h[i]);
    return 0;
}
