// k_blur.hip — libvips vips_gaussblur on gfx950.
//
// gaussblur.c builds the integer separable mask (vips_gaussmat, precision
// integer: rint(20 exp(-x^2 / 2 sigma^2)), scale = sum) and convsep.c runs the
// horizontal 1 x n mask then the vertical one through convi.c: uchar result
// (sum + (scale + 1) / 2) / scale, clipped, edges EXTEND_COPY, uchar
// intermediate (restated in oracle/vips_ref.c).  Sums are exact in fp32.
//
//  * k_convi_h<B>: a block = 256 output pixels of one row; the n + 255 input
//    pixels it needs are staged once in LDS (one packed u32 per pixel).
//  * k_convi_v:    lanes own dword columns (channel agnostic); taps are dword
//    buffer loads down the column, consecutive rows on one XCD.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "device_common.h"

namespace mipx {
namespace {

using namespace dev;

constexpr int kMaxTaps = 255;

struct ConvArgs {
    const u8 *in;
    u8 *out;
    int w, h, n, x_blocks, col_blocks, row_bytes;
    float rounding, inv_scale;
    long long img_bytes;
    float m[kMaxTaps];
};

__device__ __forceinline__ uint32_t conv_round(float acc, const ConvArgs &a) {
    return min(div_floor(acc + a.rounding, a.inv_scale), 255u);
}

template <int B>
__global__ void __launch_bounds__(256) k_convi_h(ConvArgs a) {
    __shared__ uint32_t spx[256 + kMaxTaps];
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int xb = t % a.x_blocks;
    const int rest = t / a.x_blocks;
    const int y = rest % a.h;
    const int img = rest / a.h;
    const int half = a.n / 2;
    const int x0 = xb * 256;
    const int lo = x0 - half;
    const int span = min(256, a.w - x0) + a.n - 1;
    const u8 *row = a.in + img * a.img_bytes + static_cast<size_t>(y) * a.w * B;
    for (int p = threadIdx.x; p < span; p += 256) {
        const u8 *s = row + clampi(lo + p, 0, a.w - 1) * B;
        uint32_t v;
        if (B == 4) {
            v = *reinterpret_cast<const uint32_t *>(s);
        } else {
            v = s[0];
            if (B > 1) v |= static_cast<uint32_t>(s[1]) << 8;
            if (B > 2) v |= static_cast<uint32_t>(s[2]) << 16;
        }
        spx[p] = v;
    }
    __syncthreads();
    const int x = x0 + threadIdx.x;
    if (x >= a.w) return;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const uint32_t *sp = spx + threadIdx.x;
    for (int i = 0; i < a.n; ++i) {
        const uint32_t v = sp[i];
        const float m = a.m[i];
        acc[0] = __builtin_fmaf(m, ubyte_f<0>(v), acc[0]);
        if (B > 1) acc[1] = __builtin_fmaf(m, ubyte_f<1>(v), acc[1]);
        if (B > 2) acc[2] = __builtin_fmaf(m, ubyte_f<2>(v), acc[2]);
        if (B > 3) acc[3] = __builtin_fmaf(m, ubyte_f<3>(v), acc[3]);
    }
    u8 *q = a.out + img * a.img_bytes + (static_cast<size_t>(y) * a.w + x) * B;
    if (B == 4) {
        *reinterpret_cast<uint32_t *>(q) = conv_round(acc[0], a) | (conv_round(acc[1], a) << 8) |
                                           (conv_round(acc[2], a) << 16) | (conv_round(acc[3], a) << 24);
    } else {
#pragma unroll
        for (int z = 0; z < B; ++z) q[z] = static_cast<u8>(conv_round(acc[z], a));
    }
}

template <bool DWORD>
__global__ void __launch_bounds__(256) k_convi_v(ConvArgs a) {
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int cb = t % a.col_blocks;
    const int rest = t / a.col_blocks;
    const int y = rest % a.h;
    const int img = rest / a.h;
    const int j = (cb * 256 + threadIdx.x) * 4;
    if (j >= a.row_bytes) return;
    const int half = a.n / 2;
    const u8 *src = a.in + img * a.img_bytes;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const int nb = min(4, a.row_bytes - j);
    if (DWORD) {
        const __amdgpu_buffer_rsrc_t rs = image_rsrc(src, a.img_bytes);
        for (int i = 0; i < a.n; ++i) {
            const int r = clampi(y + i - half, 0, a.h - 1);
            const uint32_t v = static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(rs, j, r * a.row_bytes, 0));
            const float m = a.m[i];
            acc[0] = __builtin_fmaf(m, ubyte_f<0>(v), acc[0]);
            acc[1] = __builtin_fmaf(m, ubyte_f<1>(v), acc[1]);
            acc[2] = __builtin_fmaf(m, ubyte_f<2>(v), acc[2]);
            acc[3] = __builtin_fmaf(m, ubyte_f<3>(v), acc[3]);
        }
        *reinterpret_cast<uint32_t *>(a.out + img * a.img_bytes + static_cast<size_t>(y) * a.row_bytes + j) =
            conv_round(acc[0], a) | (conv_round(acc[1], a) << 8) | (conv_round(acc[2], a) << 16) |
            (conv_round(acc[3], a) << 24);
    } else {
        for (int i = 0; i < a.n; ++i) {
            const u8 *p = src + static_cast<size_t>(clampi(y + i - half, 0, a.h - 1)) * a.row_bytes + j;
            const float m = a.m[i];
            for (int k = 0; k < nb; ++k) acc[k] = __builtin_fmaf(m, static_cast<float>(p[k]), acc[k]);
        }
        u8 *q = a.out + img * a.img_bytes + static_cast<size_t>(y) * a.row_bytes + j;
        for (int k = 0; k < nb; ++k) q[k] = static_cast<u8>(conv_round(acc[k], a));
    }
}

}  // namespace

int blur_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double sigma, double min_ampl, void *ws,
                size_t ws_bytes, hipStream_t st) {
    std::vector<int> mask;
    int scale = 0;
    const int nm = gaussmat(sigma, min_ampl, mask, scale);
    if (nm < 0) return MIPX_EINVAL;
    if (nm > kMaxTaps) {
        set_error("gaussblur mask of %d taps exceeds %d", nm, kMaxTaps);
        return MIPX_EUNSUPPORTED;
    }
    const size_t need = align_up(static_cast<size_t>(n) * w * h * b);
    if (!ws || ws_bytes < need) return MIPX_EINVAL;
    if (b == 4 && ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out) |
                    reinterpret_cast<uintptr_t>(ws)) & 3u))
        return MIPX_EINVAL;
    ConvArgs a{};
    a.w = w;
    a.h = h;
    a.n = nm;
    a.row_bytes = w * b;
    a.x_blocks = (w + 255) / 256;
    a.col_blocks = (a.row_bytes / 4 + 1 + 255) / 256;
    a.rounding = static_cast<float>((scale + 1) / 2);
    a.inv_scale = 1.0f / scale;
    a.img_bytes = img_bytes(w, h, b);
    if (a.img_bytes >= 0x7fffffffLL) return MIPX_EUNSUPPORTED;
    for (int i = 0; i < nm; ++i) a.m[i] = static_cast<float>(mask[i]);
    u8 *tmp = static_cast<u8 *>(ws);
    // horizontal: in -> tmp
    a.in = in;
    a.out = tmp;
    long long blocks = static_cast<long long>(a.x_blocks) * h * n;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL(k_convi_h<B_>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st, a));
    int e = launch_check("k_convi_h");
    if (e) return e;
    // vertical: tmp -> out
    a.in = tmp;
    a.out = out;
    blocks = static_cast<long long>(a.col_blocks) * h * n;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    const bool dword = (a.row_bytes % 4) == 0 && ((reinterpret_cast<uintptr_t>(tmp) | reinterpret_cast<uintptr_t>(out)) & 3u) == 0;
    if (dword) hipLaunchKernelGGL(k_convi_v<true>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(k_convi_v<false>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st, a);
    return launch_check("k_convi_v");
}

}  // namespace mipx
