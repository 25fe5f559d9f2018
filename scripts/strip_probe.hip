// Memory-only ceilings for the generic reduce's access pattern (k_rcol without the
// arithmetic): 64 x 1920x1080x3 images in, 1200x675x3 out (shrink 1.6).
//   strip  a block walks a vertical strip of SPX output pixels (span SPX * 1.6 + 11 input
//          pixels) down a segment of 16-row steps; each step loads the ~26 input rows it
//          adds with 16-byte buffer loads (the lane -> (row, chunk) map of k_rcol, two
//          steps in flight) and stores 16 output rows of the strip as dwords
//   band   the same rows, but a block owns a band of whole rows (every strip of the
//          image side by side): the row-major order of the two-pass kernels
// One JSON line per (pattern, strip width, steps per block).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t u4v __attribute__((ext_vector_type(4)));

struct P {
    const uint8_t *in;
    uint8_t *out;
    int w, h, ow, oh, strips, segs, seg_steps, ksteps, cpr, spx;
    long long in_img, out_img;
    float s;
};

__device__ __forceinline__ int grow(int k, float s) { return static_cast<int>(16 * k * s); }  // first input row of step k

// XCD-contiguous block order (as the engine's xcd_remap): XCD x walks t in its own range
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nb) {
    const uint32_t xcd = b & 7u, q = nb >> 3, r = nb & 7u;
    const uint32_t base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (b >> 3);
}

// MODE bit 0: XCD-contiguous order; bit 1: no loads; bit 2: no stores
template <int KM, int MODE>
__global__ void __launch_bounds__(256) strip(P a) {
    const int t = (MODE & 1) ? static_cast<int>(xcd_remap(blockIdx.x, gridDim.x)) : static_cast<int>(blockIdx.x);
    const int st = t % a.strips, rest = t / a.strips, seg = rest % a.segs, img = rest / a.segs;
    const int tid = threadIdx.x;
    const int pitch = a.w * 3;
    const int x0 = st * a.spx;
    const int b0 = (static_cast<int>(x0 * a.s) * 3 - 15) & ~15;
    const __amdgpu_buffer_rsrc_t src =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.in + img * a.in_img), 0, static_cast<int>(a.in_img), 0x00020000);
    const __amdgpu_buffer_rsrc_t dst =
        __builtin_amdgcn_make_buffer_rsrc(a.out + img * a.out_img, 0, static_cast<int>(a.out_img), 0x00020000);
    int rr[KM], cof[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        const int c = tid + 256 * j;
        rr[j] = c / a.cpr;
        cof[j] = b0 + 16 * (c - rr[j] * a.cpr);
    }
    const int ka = seg * a.seg_steps, kz = min(a.ksteps, ka + a.seg_steps);
    u4v v0[KM], v1[KM];
    uint32_t acc = 0;
    auto issue = [&](u4v *v, int k) {
        const int r0 = grow(k, a.s), r1 = grow(k + 1, a.s);
#pragma unroll
        for (int j = 0; j < KM; ++j)
            v[j] = (MODE & 2) ? u4v{0u, 0u, 0u, static_cast<uint32_t>(k)} : __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(
                                               src, rr[j] < r1 - r0 ? min(r0 + rr[j], a.h - 1) * pitch + cof[j] : 0x7ffffff0, 0, 0));
    };
    const int obw = a.spx * 3, nd = obw / 4;  // output dwords per strip row
    auto store = [&](int k) {
        if (MODE & 4) {
            if (acc == 0x9e3779b9u) __builtin_amdgcn_raw_buffer_store_b32(acc, dst, 0, 0, 0);
            return;
        }
        for (int i = tid; i < 16 * nd; i += 256) {
            const int r = i / nd, d = i - r * nd, y = 16 * k + r;
            const int off = y < a.oh && x0 + (4 * d) / 3 < a.ow ? (y * a.ow + x0) * 3 + 4 * d : 0x7ffffff0;
            __builtin_amdgcn_raw_buffer_store_b32(acc + i, dst, off, 0, 0);
        }
    };
    issue(v0, ka);
    issue(v1, ka + 1);
    for (int k = ka; k < kz; k += 2) {
#pragma unroll
        for (int j = 0; j < KM; ++j) acc ^= v0[j].x ^ v0[j].w;
        issue(v0, k + 2);
        store(k);
        if (k + 1 < kz) {
#pragma unroll
            for (int j = 0; j < KM; ++j) acc ^= v1[j].y ^ v1[j].z;
            issue(v1, k + 3);
            store(k + 1);
        }
    }
}

// k_bmf's access pattern, memory only: a block owns TW output pixels x TR output rows of
// one image (same-size output: the blur), loads its TR + HALO input rows of
// (TW + HALO) pixels with 16-byte loads (all issued, then used), stores its TR rows
struct T {
    const uint8_t *in;
    uint8_t *out;
    int w, h, tw, tr, halo, xb, yb;
    long long img;
};
template <int KM>
__global__ void __launch_bounds__(256) tile(T a) {
    const int t = static_cast<int>(xcd_remap(blockIdx.x, gridDim.x));
    const int xb = t % a.xb, rest = t / a.xb, yb = rest % a.yb, img = rest / a.yb;
    const int tid = threadIdx.x, pitch = a.w * 3;
    const int x0 = xb * a.tw, y0 = yb * a.tr;
    const int b0 = max(0, (x0 - a.halo / 2) * 3) & ~15;
    const int span = (a.tw + a.halo) * 3 + 16, cpr = (span + 15) / 16, L = a.tr + a.halo;
    const __amdgpu_buffer_rsrc_t src =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.in + img * a.img), 0, static_cast<int>(a.img), 0x00020000);
    const __amdgpu_buffer_rsrc_t dst = __builtin_amdgcn_make_buffer_rsrc(a.out + img * a.img, 0, static_cast<int>(a.img), 0x00020000);
    uint32_t acc = 0;
    u4v v[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        const int c = tid + 256 * j, r = c / cpr, col = c - r * cpr;
        const int row = min(max(y0 - a.halo / 2 + r, 0), a.h - 1);
        v[j] = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(src, r < L ? row * pitch + b0 + 16 * col : 0x7ffffff0, 0, 0));
    }
#pragma unroll
    for (int j = 0; j < KM; ++j) acc ^= v[j].x ^ v[j].w;
    const int nq = a.tw * 3 / 16;
    for (int i = tid; i < a.tr * nq; i += 256) {
        const int r = i / nq, q = i - r * nq, y = y0 + r;
        const int off = y < a.h && x0 * 3 + 16 * q + 16 <= pitch ? y * pitch + x0 * 3 + 16 * q : 0x7ffffff0;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, u4v{acc, acc + 1, acc + 2, acc + i}), dst, off, 0, 0);
    }
}

// rot 90's access pattern, memory only: a block owns a tile of TC input columns x TH input
// rows of one image (W x H x 3), loads its rows with 16-byte loads (LD 1: plus the b32 the
// engine adds for the de-skew), stores TC output rows of TH pixels at the transposed place:
// ST 0: 12 bytes per lane (the engine's 4-pixel tasks), ST 1: 16-byte pieces
struct R {
    const uint8_t *in;
    uint8_t *out;
    int w, h, tc, th, tx, ty, yfast;
    long long img;
};
template <int KM, int LD, int ST>
__global__ void __launch_bounds__(256) rot(R a) {
    const int t = static_cast<int>(xcd_remap(blockIdx.x, gridDim.x));
    int bx, by, img;
    if (a.yfast) { by = t % a.ty; const int rest = t / a.ty; bx = rest % a.tx; img = rest / a.tx; }
    else { bx = t % a.tx; const int rest = t / a.tx; by = rest % a.ty; img = rest / a.ty; }
    const int tid = threadIdx.x, pitch = a.w * 3;
    const int tx0 = bx * a.tc, ty0 = by * a.th;
    const int tw = min(a.tc, a.w - tx0), th = min(a.th, a.h - ty0);
    const __amdgpu_buffer_rsrc_t src =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.in + img * a.img), 0, static_cast<int>(a.img), 0x00020000);
    const __amdgpu_buffer_rsrc_t dst = __builtin_amdgcn_make_buffer_rsrc(a.out + img * a.img, 0, static_cast<int>(a.img), 0x00020000);
    const int nq = (tw * 3 + 15) / 16;
    uint32_t acc = 0;
    u4v v[KM];
    uint32_t e[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) {
        const int c = tid + 256 * j, r = c / nq, q = c - r * nq;
        const int off = r < th ? (ty0 + r) * pitch + ((tx0 * 3) & ~3) + 16 * q : 0x7ffffff0;
        v[j] = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(src, off, 0, 0));
        e[j] = LD ? static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(src, off + 16, 0, 0)) : 0u;
    }
#pragma unroll
    for (int j = 0; j < KM; ++j) acc ^= v[j].x ^ v[j].w ^ e[j];
    __syncthreads();
    const int ox = a.h - (ty0 + th);  // CW
    if (ST == 0) {
        const int quads = (th + 3) / 4;
        for (int i = tid; i < tw * quads; i += 256) {
            const int orr = i / quads, q = i - orr * quads;
            const int off = ((tx0 + orr) * a.h + ox + 4 * q) * 3;
            typedef uint32_t u3v __attribute__((ext_vector_type(3)));
            __builtin_amdgcn_raw_buffer_store_b96(__builtin_bit_cast(u3v, u3v{acc, acc + 1, acc + i}), dst, off, 0, 0);
        }
    } else {
        const int np = (th * 3 + 15) / 16;
        for (int i = tid; i < tw * np; i += 256) {
            const int orr = i / np, q = i - orr * np;
            const int off = ((tx0 + orr) * a.h + ox) * 3 + 16 * q;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, u4v{acc, acc + 1, acc + 2, acc + i}), dst, off, 0, 0);
        }
    }
}

template <class F>
static float time_it(F launch) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) launch();
    std::vector<float> v;
    for (int g = 0; g < 5; ++g) {
        hipEventRecord(a);
        for (int i = 0; i < 10; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        v.push_back(ms / 10);
    }
    std::sort(v.begin(), v.end());
    return v[2];
}

int main() {
    const int n = 64, W = 1920, H = 1080, OW = 1200, OH = 675;
    const float s = 1.6f;
    const long long in_img = 1LL * W * H * 3, out_img = 1LL * OW * OH * 3;
    uint8_t *in, *out;
    const long long cap = std::max(n * in_img, 32LL * 3840 * 2160 * 3);  // the rot probe's 32 x 4K RGB
    CK(hipMalloc(&in, cap + 4096));
    CK(hipMalloc(&out, cap + 4096));  // the tile pattern writes full-size images
    CK(hipMemset(in, 1, cap));
    CK(hipDeviceSynchronize());
    const double bytes = static_cast<double>(n) * (in_img + out_img);
    const int ksteps = (OH + 15) / 16;
    auto run = [&](const char *name, int spx, int ss, int mode) {
        const int span = static_cast<int>(spx * s) * 3 + 11 * 3 + 16;
        const int cpr = (span + 15) / 16;
        const int km = (26 * cpr + 255) / 256;
        P a{};
        a.in = in, a.out = out, a.w = W, a.h = H, a.ow = OW, a.oh = OH, a.s = s, a.spx = spx;
        a.strips = (OW + spx - 1) / spx, a.ksteps = ksteps, a.seg_steps = ss, a.segs = (ksteps + ss - 1) / ss;
        a.cpr = cpr, a.in_img = in_img, a.out_img = out_img;
        const unsigned blocks = static_cast<unsigned>(a.strips) * a.segs * n;
        float ms = -1;
#define SP_RUN(KM_) \
        if (mode == 0) ms = time_it([&] { strip<KM_, 0><<<blocks, 256>>>(a); }); \
        else if (mode == 1) ms = time_it([&] { strip<KM_, 1><<<blocks, 256>>>(a); }); \
        else if (mode == 3) ms = time_it([&] { strip<KM_, 3><<<blocks, 256>>>(a); }); \
        else if (mode == 5) ms = time_it([&] { strip<KM_, 5><<<blocks, 256>>>(a); });
        if (km <= 3) { SP_RUN(3) } else if (km <= 5) { SP_RUN(5) } else if (km <= 9) { SP_RUN(9) } else return;
        printf("{\"pattern\": \"%s\", \"spx\": %d, \"span_B\": %d, \"steps\": %d, \"mode\": %d, \"blocks\": %u, \"ms\": %.4f, \"GBps\": %.1f}\n",
               name, spx, 16 * cpr, ss, mode, blocks, ms, bytes / ms / 1e6);
        fflush(stdout);
    };
    if (getenv("PROBE_STRIP")) {
        for (int spx : {64, 128, 256}) {
            run("strip", spx, 11, 0);
            run("strip_xcd", spx, 11, 1);
            run("stores_only_xcd", spx, 11, 3);
            run("loads_only_xcd", spx, 11, 5);
        }
    }
    // the strip walk in k_bcol's geometry: in = out (shrink 1), 64 / 128-pixel strips
    if (getenv("PROBE_BLUR")) {
        for (int spx : {64, 128}) {
            const int span = spx * 3 + 24 * 3 + 16, cpr = (span + 15) / 16, km = (16 * cpr + 255) / 256;
            P a{};
            a.in = in, a.out = out, a.w = W, a.h = H, a.ow = W, a.oh = H, a.s = 1.0f, a.spx = spx;
            a.strips = (W + spx - 1) / spx, a.ksteps = (H + 15) / 16, a.seg_steps = 17, a.segs = (a.ksteps + 16) / 17;
            a.cpr = cpr, a.in_img = 1LL * W * H * 3, a.out_img = 1LL * W * H * 3;
            const unsigned blocks = static_cast<unsigned>(a.strips) * a.segs * n;
            float ms = -1;
            if (km <= 3) ms = time_it([&] { strip<3, 1><<<blocks, 256>>>(a); });
            else if (km <= 5) ms = time_it([&] { strip<5, 1><<<blocks, 256>>>(a); });
            printf("{\"pattern\": \"blur_strip_xcd\", \"spx\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", spx, ms,
                   2.0 * n * a.in_img / ms / 1e6);
            fflush(stdout);
        }
    }
    // rot 90 tiles on 32 x 4K RGB (the op survey's shape) and 16 x 12 MP RGB
    if (getenv("PROBE_ROT")) {
        for (int shape = 0; shape < 2; ++shape) {
            const int RW = shape ? 4000 : 3840, RH = shape ? 3000 : 2160, rn = shape ? 16 : 32;
            const long long img = 1LL * RW * RH * 3;
            if (rn * img > cap) continue;
            const double tb = 2.0 * rn * img;
            for (int tc : {64, 128})
                for (int thh : {32, 64, 128})
                    for (int yf = 0; yf < 2; ++yf)
                        for (int v = 0; v < 4; ++v) {
                            R a{};
                            a.in = in, a.out = out, a.w = RW, a.h = RH, a.tc = tc, a.th = thh, a.img = img, a.yfast = yf;
                            a.tx = (RW + tc - 1) / tc, a.ty = (RH + thh - 1) / thh;
                            const unsigned blocks = static_cast<unsigned>(a.tx) * a.ty * rn;
                            const int km = (thh * ((tc * 3 + 15) / 16) + 255) / 256;
                            float ms = -1;
#define ROT_RUN(KM_) \
                            if (v == 0) ms = time_it([&] { rot<KM_, 0, 0><<<blocks, 256>>>(a); }); \
                            else if (v == 1) ms = time_it([&] { rot<KM_, 1, 0><<<blocks, 256>>>(a); }); \
                            else if (v == 2) ms = time_it([&] { rot<KM_, 0, 1><<<blocks, 256>>>(a); }); \
                            else ms = time_it([&] { rot<KM_, 1, 1><<<blocks, 256>>>(a); });
                            if (km <= 2) { ROT_RUN(2) } else if (km <= 3) { ROT_RUN(3) } else if (km <= 6) { ROT_RUN(6) } else if (km <= 12) { ROT_RUN(12) } else continue;
#undef ROT_RUN
                            printf("{\"pattern\": \"rot90\", \"w\": %d, \"h\": %d, \"n\": %d, \"tc\": %d, \"th\": %d, \"yfast\": %d, \"ld_b32\": %d, \"st16\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
                                   RW, RH, rn, tc, thh, yf, v & 1, v >> 1, ms, tb / ms / 1e6);
                            fflush(stdout);
                        }
        }
        return 0;
    }
    // k_bmf tiles on 64 x 1080p RGB in = out (blur): 128 px x 16 / 32 / 48 rows, halo 0 / 12 / 16
    {
        const long long img = 1LL * W * H * 3;
        const double tb = 2.0 * n * img;
        for (int tr : {16, 32, 48})
            for (int halo : {0, 12, 16}) {
                T a{};
                a.in = in, a.out = out, a.w = W, a.h = H, a.tw = 128, a.tr = tr, a.halo = halo, a.img = img;
                a.xb = (W + 127) / 128, a.yb = (H + tr - 1) / tr;
                const unsigned blocks = static_cast<unsigned>(a.xb) * a.yb * n;
                const int cpr = ((128 + halo) * 3 + 16 + 15) / 16, km = ((tr + halo) * cpr + 255) / 256;
                float ms = -1;
                if (km <= 4) ms = time_it([&] { tile<4><<<blocks, 256>>>(a); });
                else if (km <= 8) ms = time_it([&] { tile<8><<<blocks, 256>>>(a); });
                else if (km <= 12) ms = time_it([&] { tile<12><<<blocks, 256>>>(a); });
                else continue;
                printf("{\"pattern\": \"bmf_tile\", \"tw\": 128, \"tr\": %d, \"halo\": %d, \"km\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
                       tr, halo, km, ms, tb / ms / 1e6);
                fflush(stdout);
            }
    }
    return 0;
}
