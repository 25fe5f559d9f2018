// Probe of v_mfma_i32_16x16x64_i8 operand maps (exact integer data):
// A[m][k] = m*3 + k (mod 7) - 3, B[k][n] = (k*5 + n*11) mod 13 - 6, D = A.B checked on the host
// under the hypothesised maps: lane l holds A[l&15][16(l>>4)+j], B[16(l>>4)+j][l&15] (byte j),
// D[4(l>>4)+i][l&15] in register i.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k(const signed char *A, const signed char *B, int *D) {
    const int l = threadIdx.x;
    v4i a, b;
    signed char *pa = reinterpret_cast<signed char *>(&a), *pb = reinterpret_cast<signed char *>(&b);
    for (int j = 0; j < 16; ++j) {
        pa[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j];
        pb[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)];
    }
    v4i c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    for (int i = 0; i < 4; ++i) D[(4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
}
int main() {
    signed char A[16 * 64], B[64 * 16];
    int D[256], R[256];
    for (int m = 0; m < 16; ++m) for (int kk = 0; kk < 64; ++kk) A[m * 64 + kk] = (m * 3 + kk) % 7 - 3 + (m == kk ? 50 : 0);
    for (int kk = 0; kk < 64; ++kk) for (int n = 0; n < 16; ++n) B[kk * 16 + n] = (kk * 5 + n * 11) % 13 - 6 + (kk == 2 * n ? 70 : 0);
    for (int m = 0; m < 16; ++m) for (int n = 0; n < 16; ++n) { int s = 0; for (int kk = 0; kk < 64; ++kk) s += A[m * 64 + kk] * B[kk * 16 + n]; R[m * 16 + n] = s; }
    signed char *dA, *dB; int *dD;
    hipMalloc(&dA, sizeof A); hipMalloc(&dB, sizeof B); hipMalloc(&dD, sizeof D);
    hipMemcpy(dA, A, sizeof A, hipMemcpyHostToDevice); hipMemcpy(dB, B, sizeof B, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    hipMemcpy(D, dD, sizeof D, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) if (D[i] != R[i]) { if (bad < 5) printf("mismatch %d: %d vs %d\n", i, D[i], R[i]); ++bad; }
    printf("mfma_i32_16x16x64_i8 map: %s (%d bad)\n", bad ? "WRONG" : "ok", bad);
    return bad ? 1 : 0;
}
