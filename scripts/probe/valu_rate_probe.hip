// Issue cost of candidate VALU instructions on gfx950 (k_reduce2c's arithmetic): one wave
// per SIMD, independent chains (8 accumulators) and one dependent chain, cycles per
// instruction from the cycle counter around an unrolled loop (the 5-waves-per-SIMD rows
// time each wave alone and under-count contention).  One JSON line per case.
// MODE 0 v_fma_f32, 1 v_dot2c_f32_f16, 2 v_fma_mix_f32 (f16 operand), 3 v_pk_add_u16,
// 4 v_pk_fma_f32, 5 v_perm_b32, 6 v_cvt_f32_ubyte0
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 h2v __attribute__((ext_vector_type(2)));

template <int MODE, int CH>
__global__ void k(float *out, unsigned seed, long long *cyc) {
    float acc[CH];
    for (int i = 0; i < CH; ++i) acc[i] = (float)(threadIdx.x + i);
    h2v a = __builtin_bit_cast(h2v, seed ^ threadIdx.x), b = __builtin_bit_cast(h2v, seed * 3u);
    float fa = (float)seed, fb = 1.0001f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef unsigned short u2 __attribute__((ext_vector_type(2)));
    unsigned ua[CH];
    f2 pa[CH];
    for (int i = 0; i < CH; ++i) ua[i] = seed + i * threadIdx.x, pa[i] = f2{acc[i], fa};
    const u2 ub = __builtin_bit_cast(u2, seed * 7u);
    const f2 pb = {fb, fa};
    const long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < 256; ++it) {
#pragma unroll
        for (int r = 0; r < 8 / CH; ++r)
#pragma unroll
            for (int i = 0; i < CH; ++i) {
                if (MODE == 0) acc[i] = __builtin_fmaf(fa, fb, acc[i]);
                else if (MODE == 1) acc[i] = __builtin_amdgcn_fdot2(a, b, acc[i], false);
                else if (MODE == 2)
                    asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(acc[i]) : "v"(a), "v"(fb));
                else if (MODE == 3)
                    asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(ua[i]) : "v"(__builtin_bit_cast(unsigned, ub)));
                else if (MODE == 4) pa[i] = __builtin_elementwise_fma(pa[i], pb, pa[i]);
                else if (MODE == 5)
                    asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(ua[i]) : "v"(seed), "v"(0x05010400u));
                else acc[i] += (float)(ua[i] & 0xff), ua[i] += 1;
            }
    }
    const long long t1 = __builtin_readcyclecounter();
    float s = 0;
    for (int i = 0; i < CH; ++i) s += acc[i] + (float)ua[i] + pa[i].x + pa[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, int CH>
void run(const char *name, int waves_per_simd) {
    const int blocks = 256 * waves_per_simd;  // 256 threads = 4 waves: one per SIMD
    float *out;
    long long *cyc;
    hipMalloc(&out, blocks * 256 * sizeof(float));
    hipMalloc(&cyc, blocks * sizeof(long long));
    hipLaunchKernelGGL((k<MODE, CH>), dim3(blocks), dim3(256), 0, 0, out, 12345u, cyc);
    hipLaunchKernelGGL((k<MODE, CH>), dim3(blocks), dim3(256), 0, 0, out, 12345u, cyc);
    hipDeviceSynchronize();
    long long *h = new long long[blocks];
    hipMemcpy(h, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < blocks; ++i) avg += h[i];
    avg /= blocks;
    printf("{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"cycles_per_instr\": %.2f}\n", name, CH,
           waves_per_simd, avg / (256.0 * 8));
    delete[] h;
    hipFree(out);
    hipFree(cyc);
}

int main() {
    for (int w : {1, 5}) {
        run<0, 8>("v_fma_f32", w);
        run<1, 8>("v_dot2c_f32_f16", w);
        run<2, 8>("v_fma_mix_f32", w);
        run<3, 8>("v_pk_add_u16", w);
        run<4, 8>("v_pk_fma_f32", w);
        run<5, 8>("v_perm_b32", w);
        run<6, 8>("v_cvt_f32_ubyte0+v_add (2 instr)", w);
        run<0, 1>("v_fma_f32", w);
        run<1, 1>("v_dot2c_f32_f16", w);
        run<2, 1>("v_fma_mix_f32", w);
    }
    return 0;
}
