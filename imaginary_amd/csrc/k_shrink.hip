// k_shrink.hip — libvips vips_shrink (integer box) on gfx950.
//
// shrink.c runs shrinkv then shrinkh; each pass is (sum + n/2) / n to uchar,
// output size VIPS_ROUND(in / n), partial blocks at the far edge read the
// EXTEND_COPY border (restated in oracle/vips_ref.c).
//
// A block = one output row x TWS output pixels.  Phase 1 (shrinkv): lanes own
// dwords of the block's input byte span, sum the vs rows (dword buffer loads,
// every input byte read once) and write the rounded column means to LDS.
// Phase 2 (shrinkh): one lane per output pixel averages hs LDS pixels.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device_common.h"

namespace mipx {
namespace {

using namespace dev;

struct ShrinkArgs {
    const u8 *in;
    u8 *out;
    int w, h, ow, oh, hs, vs, tws, x_blocks;
    float inv_hs, inv_vs;
    long long in_img, out_img;
};

template <int B>
__global__ void __launch_bounds__(256) k_shrink_lds(ShrinkArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    u8 *col = reinterpret_cast<u8 *>(smem);
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int xb = t % a.x_blocks;
    const int rest = t / a.x_blocks;
    const int y = rest % a.oh;
    const int img = rest / a.oh;
    const int x0 = xb * a.tws;
    const int nx = min(a.tws, a.ow - x0);
    const int row_bytes = a.w * B;
    const int span = nx * a.hs * B;           // bytes of the input span, COPY-extended
    const int sb = x0 * a.hs * B;             // first byte (may extend past the row)
    const u8 *src = a.in + img * a.in_img;
    const __amdgpu_buffer_rsrc_t rs = image_rsrc(src, a.in_img);
    const bool aligned_rows = (row_bytes & 3) == 0;
    // ---- phase 1: vertical sums, 4 byte-columns per lane ----
    for (int d = threadIdx.x * 4; d < span; d += 1024) {
        const int g = sb + d;
        const bool whole = aligned_rows && g + 4 <= row_bytes;  // dword inside the row
        uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        int off[4];
        if (!whole) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int gb = g + k;
                const int p = gb / B, c = gb - p * B;
                off[k] = min(p, a.w - 1) * B + c;  // COPY border beyond the last pixel
            }
        }
        if (whole) {  // batches of 8 independent row loads in flight
            for (int k0 = 0; k0 < a.vs; k0 += 8) {
                uint32_t v[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int r = min(y * a.vs + min(k0 + q, a.vs - 1), a.h - 1);
                    v[q] = static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(rs, g, r * row_bytes, 0));
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    if (k0 + q < a.vs) {
                        s0 += v[q] & 0xff;
                        s1 += (v[q] >> 8) & 0xff;
                        s2 += (v[q] >> 16) & 0xff;
                        s3 += v[q] >> 24;
                    }
                }
            }
        }
        for (int k = 0; k < a.vs && !whole; ++k) {
            const int r = min(y * a.vs + k, a.h - 1);
            {
                const u8 *p = src + static_cast<size_t>(r) * row_bytes;
                s0 += p[off[0]];
                s1 += p[off[1]];
                s2 += p[off[2]];
                s3 += p[off[3]];
            }
        }
        const uint32_t half = a.vs / 2;
        const uint32_t m = div_floor(static_cast<float>(s0 + half), a.inv_vs) |
                           (div_floor(static_cast<float>(s1 + half), a.inv_vs) << 8) |
                           (div_floor(static_cast<float>(s2 + half), a.inv_vs) << 16) |
                           (div_floor(static_cast<float>(s3 + half), a.inv_vs) << 24);
        smem[d >> 2] = m;
    }
    __syncthreads();
    // ---- phase 2: horizontal means ----
    const int x = threadIdx.x;
    if (x >= nx) return;
    const u8 *c = col + x * a.hs * B;
    uint32_t acc[B];
#pragma unroll
    for (int z = 0; z < B; ++z) acc[z] = 0;
    for (int j = 0; j < a.hs; ++j)
#pragma unroll
        for (int z = 0; z < B; ++z) acc[z] += c[j * B + z];
    u8 *q = a.out + img * a.out_img + (static_cast<size_t>(y) * a.ow + x0 + x) * B;
    const uint32_t half = a.hs / 2;
#pragma unroll
    for (int z = 0; z < B; ++z) q[z] = static_cast<u8>(div_floor(static_cast<float>(acc[z] + half), a.inv_hs));
}

}  // namespace

int shrink_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int hs, int vs, hipStream_t st) {
    ShrinkArgs a{};
    a.in = in;
    a.out = out;
    a.w = w;
    a.h = h;
    a.ow = out_size_shrink(w, hs);
    a.oh = out_size_shrink(h, vs);
    a.hs = hs;
    a.vs = vs;
    a.inv_hs = 1.0f / hs;
    a.inv_vs = 1.0f / vs;
    // output pixels per block: 256, fewer when the input span would exceed 32 KB
    int tws = 256;
    while (tws > 4 && static_cast<long long>(tws) * hs * b > 32768) tws >>= 1;
    if (static_cast<long long>(tws) * hs * b > 32768 || hs > 65535 || vs > 65535) {
        set_error("shrink %dx%d too large", hs, vs);
        return MIPX_EUNSUPPORTED;
    }
    a.tws = tws;
    a.x_blocks = (a.ow + tws - 1) / tws;
    a.in_img = img_bytes(w, h, b);
    a.out_img = img_bytes(a.ow, a.oh, b);
    if (a.in_img >= 0x7fffffffLL) return MIPX_EUNSUPPORTED;
    const long long blocks = static_cast<long long>(a.x_blocks) * a.oh * n;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    const size_t lds = ((static_cast<size_t>(tws) * hs * b + 3) / 4 + 1) * 4;
    MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL(k_shrink_lds<B_>, dim3(static_cast<unsigned>(blocks)), dim3(256), lds,
                                              st, a));
    return launch_check("k_shrink_lds");
}

}  // namespace mipx
