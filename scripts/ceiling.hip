// Streaming-bandwidth ceilings on this MI355X for the C2 traffic shape:
// 256 images x 24,883,200 B read, 256 x 6,220,800 B written (4:1).
// Each kernel is warmed, then timed over 20 launches (median of 5 groups).
//   rd_x4      read-only, dwordx4 per lane, grid-stride, 4 loads in flight
//   copy_x4    1:1 copy, dwordx4
//   rd4wr1_x4  4:1 read:write, linear (each lane reads 4 x 16 B, writes 16 B)
//   rows_dw    the k_reduce2x2 tile walk with no arithmetic: 24-row bands x
//              1 KiB strips, dword loads, 480 B of each output row written
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void __launch_bounds__(256) rd_x4(const uint4 *p, size_t n16, uint32_t *sink) {
    uint32_t acc = 0;
    const size_t stride = static_cast<size_t>(gridDim.x) * 256;
    size_t i = blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
        acc += a.x ^ b.y ^ c.z ^ d.w;
    }
    for (; i < n16; i += stride) acc += p[i].x;
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(256) copy_x4(const uint4 *p, uint4 *q, size_t n16) {
    const size_t stride = static_cast<size_t>(gridDim.x) * 256;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) q[i] = p[i];
}

__global__ void __launch_bounds__(256) rd4wr1_x4(const uint4 *p, uint4 *q, size_t nout16) {
    const size_t stride = static_cast<size_t>(gridDim.x) * 256;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < nout16; i += stride) {
        const uint4 *s = p + 4 * (i - i % 256) + i % 256;  // 4 coalesced 4 KiB reads per wave-quad
        const uint4 a = s[0], b = s[256], c = s[512], d = s[768];
        q[i] = uint4{a.x ^ b.x, a.y ^ c.y, b.z ^ d.z, c.w ^ d.w};
    }
}

// 4:1 with two outputs per lane (8 loads in flight) and optional nt stores
template <bool NT>
__global__ void __launch_bounds__(256) rd4wr1_x4u2(const uint4 *p, uint4 *q, size_t nout16) {
    const size_t stride = static_cast<size_t>(gridDim.x) * 512;
    for (size_t i0 = blockIdx.x * 512 + threadIdx.x; i0 < nout16; i0 += stride) {
        const size_t i1 = i0 + 256;
        const uint4 *s0 = p + 4 * (i0 - i0 % 256) + i0 % 256;
        const uint4 *s1 = p + 4 * (i1 - i1 % 256) + i1 % 256;
        const uint4 a = s0[0], b = s0[256], c = s0[512], d = s0[768];
        const uint4 e = s1[0], f = s1[256], g = s1[512], h = s1[768];
        const uint4 o0{a.x ^ b.x, a.y ^ c.y, b.z ^ d.z, c.w ^ d.w}, o1{e.x ^ f.x, e.y ^ g.y, f.z ^ h.z, g.w ^ h.w};
        if (NT) {
            typedef uint32_t u4v __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(u4v{o0.x, o0.y, o0.z, o0.w}, reinterpret_cast<u4v *>(q + i0));
            if (i1 < nout16) __builtin_nontemporal_store(u4v{o1.x, o1.y, o1.z, o1.w}, reinterpret_cast<u4v *>(q + i1));
        } else {
            q[i0] = o0;
            if (i1 < nout16) q[i1] = o1;
        }
    }
}

// 4:1 with dword accesses: lane reads one dword from each of 4 rows (each row
// contiguous across the wave, 256 B per instruction) and writes one dword
__global__ void __launch_bounds__(256) rd4wr1_dw(const uint32_t *p, uint32_t *q, size_t nout) {
    const size_t stride = static_cast<size_t>(gridDim.x) * 256;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < nout; i += stride) {
        const uint32_t *s = p + 4 * (i - i % 256) + i % 256;
        q[i] = s[0] ^ s[256] ^ s[512] ^ s[768];
    }
}
// the same with 8 rows per lane in flight (2 outputs)
__global__ void __launch_bounds__(256) rd4wr1_dw2(const uint32_t *p, uint32_t *q, size_t nout) {
    const size_t stride = static_cast<size_t>(gridDim.x) * 512;
    for (size_t i0 = blockIdx.x * 512 + threadIdx.x; i0 < nout; i0 += stride) {
        const size_t i1 = i0 + 256;
        const uint32_t *s0 = p + 4 * (i0 - i0 % 256) + i0 % 256, *s1 = p + 4 * (i1 - i1 % 256) + i1 % 256;
        const uint32_t a = s0[0] ^ s0[256] ^ s0[512] ^ s0[768];
        const uint32_t b = i1 < nout ? (s1[0] ^ s1[256] ^ s1[512] ^ s1[768]) : 0u;
        q[i0] = a;
        if (i1 < nout) q[i1] = b;
    }
}

// C2's access pattern as a short-lived stream: one output dword (of a 1920x1080x3
// row) per lane from a 2 x 2 block of dwords in two rows of the 3840x2160x3 input
__global__ void __launch_bounds__(256) box2x2_dw(const uint32_t *p, uint32_t *q, long long nout) {
    const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= nout) return;
    constexpr int OPW = 1440, OPH = 1080, IPW = 2880;  // dwords per output / input row
    const long long img = i / (static_cast<long long>(OPW) * OPH);
    const int rem = static_cast<int>(i - img * OPW * OPH), y = rem / OPW, x = rem - y * OPW;
    const uint32_t *s = p + img * (static_cast<long long>(IPW) * 2 * OPH) + static_cast<long long>(2 * y) * IPW + 2 * x;
    q[i] = s[0] ^ s[1] ^ s[IPW] ^ s[IPW + 1];
}

// the same pattern at 16 B per lane: 2 output dwords (8 B stored) per lane from
// 4 input dwords of each of two rows, and 4 output dwords (16 B) from 8 + 8
__global__ void __launch_bounds__(256) box2x2_x2(const uint32_t *p, uint32_t *q, long long nout2) {
    const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= nout2) return;
    constexpr int OPW = 720, OPH = 1080, IPW = 2880;  // dword pairs per output row, dwords per input row
    const long long img = i / (static_cast<long long>(OPW) * OPH);
    const int rem = static_cast<int>(i - img * OPW * OPH), y = rem / OPW, x = rem - y * OPW;
    const uint4 *s = reinterpret_cast<const uint4 *>(p + img * (static_cast<long long>(IPW) * 2 * OPH) +
                                                     static_cast<long long>(2 * y) * IPW + 4 * x);
    const uint4 a = s[0], b = s[IPW / 4];
    reinterpret_cast<uint2 *>(q)[i] = uint2{a.x ^ a.y ^ b.x ^ b.y, a.z ^ a.w ^ b.z ^ b.w};
}
__global__ void __launch_bounds__(256) box2x2_x4(const uint32_t *p, uint32_t *q, long long nout4) {
    const long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= nout4) return;
    constexpr int OPW = 360, OPH = 1080, IPW = 2880;
    const long long img = i / (static_cast<long long>(OPW) * OPH);
    const int rem = static_cast<int>(i - img * OPW * OPH), y = rem / OPW, x = rem - y * OPW;
    const uint4 *s = reinterpret_cast<const uint4 *>(p + img * (static_cast<long long>(IPW) * 2 * OPH) +
                                                     static_cast<long long>(2 * y) * IPW + 8 * x);
    const uint4 a = s[0], b = s[1], c = s[IPW / 4], d = s[IPW / 4 + 1];
    reinterpret_cast<uint4 *>(q)[i] = uint4{a.x ^ a.y ^ c.x ^ c.y, a.z ^ a.w ^ c.z ^ c.w, b.x ^ b.y ^ d.x ^ d.y,
                                           b.z ^ b.w ^ d.z ^ d.w};
}

// k_reduce2x2 geometry, memory only: tile = (img, band, strip), strip fastest
__global__ void __launch_bounds__(256) rows_dw(const uint8_t *in, uint8_t *out, int w, int h, int n_strips,
                                               int n_bands, long long in_img, long long out_img) {
    const int t = blockIdx.x;
    const int strip = t % n_strips, rest = t / n_strips, band = rest % n_bands, img = rest / n_bands;
    const int row_bytes = w * 3, ow = w / 2, oh = h / 2;
    const int byte0 = ((3 * (2 * strip * 160 - 5)) & ~3) + 4 * threadIdx.x;
    const bool ok = threadIdx.x < 249 && byte0 >= 0 && byte0 + 4 <= row_bytes;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(in + img * in_img), 0,
                                                                       static_cast<int>(in_img), 0x00020000);
    const uint32_t voff = ok ? static_cast<uint32_t>(byte0) : 0x80000000u;
    const int y0 = band * 24, y1 = min(y0 + 24, oh);
    uint32_t acc = 0;
    for (int r = 2 * y0 - 5; r < 2 * y1 + 5; ++r) {
        const int rr = min(max(r, 0), h - 1);
        acc += __builtin_amdgcn_raw_buffer_load_b32(rs, voff, rr * row_bytes, 0);
        if ((r & 1) == 0 && r >= 2 * y0 && r < 2 * y1) {
            const int y = r / 2;
            const int ob = strip * 480 + threadIdx.x * 4;  // 480 output bytes per strip row (uncoalesced tail ignored)
            if (threadIdx.x < 120 && strip * 160 + threadIdx.x * 4 / 3 < ow)
                *reinterpret_cast<uint32_t *>(out + img * out_img + static_cast<long long>(y) * ow * 3 + ob) = acc;
        }
    }
}

template <class F>
static float time_it(F launch) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 5; ++i) launch();
    std::vector<float> v;
    for (int g = 0; g < 5; ++g) {
        hipEventRecord(a);
        for (int i = 0; i < 20; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        v.push_back(ms / 20);
    }
    std::sort(v.begin(), v.end());
    return v[2];
}

int main() {
    const int n = 256, W = 3840, H = 2160;
    const long long in_img = 1LL * W * H * 3, out_img = 1LL * (W / 2) * (H / 2) * 3;
    const size_t IN = n * in_img, OUT = n * out_img;
    uint8_t *in, *out;
    uint32_t *sink;
    CK(hipMalloc(&in, IN + 4096));
    CK(hipMalloc(&out, IN + 4096));
    CK(hipMalloc(&sink, 1 << 24));
    CK(hipMemset(in, 1, IN));
    CK(hipDeviceSynchronize());
    for (int grid : {4096, 16384, 65536}) {
        const float ms = time_it([&] { rd_x4<<<grid, 256>>>((const uint4 *)in, IN / 16, sink); });
        printf("{\"kernel\": \"rd_x4\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", grid, ms, IN / ms / 1e6);
    }
    for (int grid : {4096, 16384, 65536}) {
        const float ms = time_it([&] { copy_x4<<<grid, 256>>>((const uint4 *)in, (uint4 *)out, OUT * 4 / 16 / 2); });
        const double bytes = 2.0 * (OUT * 4 / 16 / 2) * 16;
        printf("{\"kernel\": \"copy_x4\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", grid, ms, bytes / ms / 1e6);
    }
    for (int grid : {16384, 65536, 262144}) {
        const size_t nout16 = (OUT / 16) / 256 * 256;
        const float ms = time_it([&] { rd4wr1_x4<<<grid, 256>>>((const uint4 *)in, (uint4 *)out, nout16); });
        const double bytes = 5.0 * nout16 * 16;
        printf("{\"kernel\": \"rd4wr1_x4\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", grid, ms, bytes / ms / 1e6);
    }
    for (int grid : {8192, 32768}) {
        const size_t nout16 = (OUT / 16) / 512 * 512;
        float ms = time_it([&] { rd4wr1_x4u2<false><<<grid, 256>>>((const uint4 *)in, (uint4 *)out, nout16); });
        printf("{\"kernel\": \"rd4wr1_x4u2\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", grid, ms, 5.0 * nout16 * 16 / ms / 1e6);
        ms = time_it([&] { rd4wr1_x4u2<true><<<grid, 256>>>((const uint4 *)in, (uint4 *)out, nout16); });
        printf("{\"kernel\": \"rd4wr1_x4u2_nt\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", grid, ms, 5.0 * nout16 * 16 / ms / 1e6);
    }
    for (int grid : {65536, 262144, 1048576}) {
        const size_t nout = (OUT / 4) / 256 * 256;
        float ms = time_it([&] { rd4wr1_dw<<<grid, 256>>>((const uint32_t *)in, (uint32_t *)out, nout); });
        printf("{\"kernel\": \"rd4wr1_dw\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", grid, ms, 5.0 * nout * 4 / ms / 1e6);
        ms = time_it([&] { rd4wr1_dw2<<<grid / 2, 256>>>((const uint32_t *)in, (uint32_t *)out, nout); });
        printf("{\"kernel\": \"rd4wr1_dw2\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", grid / 2, ms, 5.0 * nout * 4 / ms / 1e6);
    }
    {
        const long long nout = static_cast<long long>(n) * 1440 * 1080;
        const float ms = time_it([&] {
            box2x2_dw<<<static_cast<unsigned>((nout + 255) / 256), 256>>>((const uint32_t *)in, (uint32_t *)out, nout);
        });
        printf("{\"kernel\": \"box2x2_dw\", \"ms\": %.4f, \"GBps\": %.1f}\n", ms, (IN + OUT) / ms / 1e6);
    }
    {
        const long long nout2 = static_cast<long long>(n) * 720 * 1080;
        float ms = time_it([&] {
            box2x2_x2<<<static_cast<unsigned>((nout2 + 255) / 256), 256>>>((const uint32_t *)in, (uint32_t *)out, nout2);
        });
        printf("{\"kernel\": \"box2x2_x2\", \"ms\": %.4f, \"GBps\": %.1f}\n", ms, (IN + OUT) / ms / 1e6);
        const long long nout4 = static_cast<long long>(n) * 360 * 1080;
        ms = time_it([&] {
            box2x2_x4<<<static_cast<unsigned>((nout4 + 255) / 256), 256>>>((const uint32_t *)in, (uint32_t *)out, nout4);
        });
        printf("{\"kernel\": \"box2x2_x4\", \"ms\": %.4f, \"GBps\": %.1f}\n", ms, (IN + OUT) / ms / 1e6);
    }
    {
        const int n_strips = (W / 2 + 159) / 160, n_bands = (H / 2 + 23) / 24;
        const float ms = time_it([&] {
            rows_dw<<<n_strips * n_bands * n, 256>>>(in, out, W, H, n_strips, n_bands, in_img, out_img);
        });
        printf("{\"kernel\": \"rows_dw\", \"ms\": %.4f, \"GBps\": %.1f}\n", ms, (IN + OUT) / ms / 1e6);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
