// device_common.h — helpers shared by the gfx950 kernels of libmipx.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mipx_internal.h"

namespace mipx {
namespace dev {

using u8 = uint8_t;

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }

__device__ __forceinline__ int pmod(int a, int m) {
    const int r = a % m;
    return r < 0 ? r + m : r;
}

// byte k of a dword as float: the backend selects v_cvt_f32_ubyte{k}
template <int K>
__device__ __forceinline__ float ubyte_f(uint32_t v) {
    return static_cast<float>((v >> (8 * K)) & 0xffu);
}

// The same, opaque to instcombine: a value converted once is reused by every
// tap it feeds (otherwise (float)a + (float)b folds into (float)(a + b), one
// convert per use instead of per byte).
template <int K>
__device__ __forceinline__ float ubyte_once(uint32_t v) {
    float f = ubyte_f<K>(v);
    asm("" : "+v"(f));
    return f;
}
__device__ __forceinline__ float opaque(float f) {
    asm("" : "+v"(f));
    return f;
}

// libvips unsigned_fixed_round for uchar: (sum + 2048) >> 12 clipped, with sum
// an exact integer in fp32 (|sum| < 2^21, so sum/4096 + 0.5 is exact).
__device__ __forceinline__ float fixed_round_f(float sum) {
    const float v = floorf(__builtin_fmaf(sum, 1.0f / 4096.0f, 0.5f));
    return __builtin_amdgcn_fmed3f(v, 0.0f, 255.0f);
}
__device__ __forceinline__ uint32_t fixed_round_u(float sum) { return static_cast<uint32_t>(fixed_round_f(sum)); }

// floor(a / n) for an exact integer 0 <= a < 2^24 given inv = 1.0f / n (n < 2^16):
// (a + 0.5) / n sits at least 0.5 / n from every integer, far above the fp32
// error of the product, so the floor is exact.
__device__ __forceinline__ uint32_t div_floor(float a, float inv) {
    return static_cast<uint32_t>(floorf((a + 0.5f) * inv));
}

// Conv masks (vips_gaussmat integer: every coefficient rint(20 * e^-x^2/2s^2),
// 0..20) fit packed u8, so 4 taps x 4 bytes are 8 v_perm_b32 (4 x 4 byte
// transpose) + 4 v_dot4_u32_u8, exact integer sums, instead of 16 byte
// conversions + 16 FMAs.  in[j] byte c -> out[c] byte j.
__device__ __forceinline__ void transpose4x4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t t[4]) {
    const uint32_t ab_lo = __builtin_amdgcn_perm(b, a, 0x05010400u);  // a0 b0 a1 b1
    const uint32_t ab_hi = __builtin_amdgcn_perm(b, a, 0x07030602u);  // a2 b2 a3 b3
    const uint32_t cd_lo = __builtin_amdgcn_perm(d, c, 0x05010400u);
    const uint32_t cd_hi = __builtin_amdgcn_perm(d, c, 0x07030602u);
    t[0] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x05040100u);  // a0 b0 c0 d0
    t[1] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x07060302u);
    t[2] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x05040100u);
    t[3] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x07060302u);
}
// XCD-aware block remap (bijective for any grid, cdna_hip_programming.md §5):
// blocks b, b+8, b+16... share an XCD; give each XCD a contiguous tile range so
// neighbouring tiles (which share halo bytes) meet in the same L2.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nb) {
    const uint32_t xcd = b & 7u, q = nb >> 3, r = nb & 7u;
    const uint32_t base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (b >> 3);
}

// Buffer descriptor over one image: out-of-range offsets read 0 (T8/T20).  The range
// check covers the VGPR offset (+ the instruction offset) only, NOT the SGPR offset, so
// any offset that can run past the image must ride in the VGPR operand (r02: a row
// address in the SGPR offset let a 1 x 23 RGB reduce read a shifted dword as 0 and let
// staging loads read past the last image of a batch).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t image_rsrc(const u8 *p, long long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<u8 *>(p), 0, static_cast<int>(bytes), 0x00020000);
}

// The same over the dword-aligned-down image base: *delta = p & 3 is added to
// every byte offset, so dword loads stay aligned for any image start.  Range
// checks are per dword (a dword straddling num_records reads 0), so the range
// is rounded up to the aligned word holding the image's last byte — never past
// it, so never into another page.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t image_rsrc_aligned(const u8 *p, long long bytes, int *delta) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    *delta = static_cast<int>(a & 3u);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<u8 *>(a & ~uintptr_t(3)), 0,
                                             static_cast<int>((bytes + *delta + 3) & ~3LL), 0x00020000);
}

// Individually rounded float ops for the kernels that restate libvips' float
// order of operations.  The HIP headers define __fmul_rn & co. as plain operators,
// which the backend may still fuse into FMAs; the pragma inside each body marks
// these operations non-contractable, so they stay separately rounded after inlining.
#define MIPX_RN_OP(name, T, op)                                   \
    __device__ __forceinline__ T name(T a, T b) {                 \
        _Pragma("clang fp contract(off)") return a op b;          \
    }
MIPX_RN_OP(fmul_rn, float, *)
MIPX_RN_OP(fadd_rn, float, +)
MIPX_RN_OP(fsub_rn, float, -)
MIPX_RN_OP(fdiv_rn, float, /)
MIPX_RN_OP(dmul_rn, double, *)
MIPX_RN_OP(dadd_rn, double, +)
#undef MIPX_RN_OP

// libvips reduce sample position of output o (reducev.cpp / reduceh.cpp): the corner
// convention X = o * shrink (the [U] default, PARITY_ASSUMPTIONS.md row 1) or, with
// the centre switch, X = (o + 0.5) * shrink - 0.5; separately rounded double ops, as
// oracle/vips_ref.c reduce_pos computes them
__device__ __forceinline__ double reduce_x(int o, double s, int centre) {
    return centre ? dadd_rn(dmul_rn(o + 0.5, s), -0.5) : dmul_rn(static_cast<double>(o), s);
}

}  // namespace dev

// ---- host-side helpers shared by the launchers ----
inline long long img_bytes(int w, int h, int b) { return static_cast<long long>(w) * h * b; }
inline int clampi_host(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
inline size_t align_up(size_t v) { return (v + 255) & ~static_cast<size_t>(255); }
inline int launch_check(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, what);
    return MIPX_OK;
}
inline bool geom_ok(int n, int w, int h, int b) {
    return n > 0 && w > 0 && h > 0 && b >= 1 && b <= 4 && n <= 65535;
}
// Blocks for a 1D-flattened grid (kept under the 2^31 grid limit).
inline bool grid_ok(long long blocks) { return blocks > 0 && blocks < 0x7fffffffLL; }

#define MIPX_DISPATCH_BANDS(b, ...)                               \
    switch (b) {                                                  \
        case 1: { constexpr int B_ = 1; __VA_ARGS__; } break;     \
        case 2: { constexpr int B_ = 2; __VA_ARGS__; } break;     \
        case 3: { constexpr int B_ = 3; __VA_ARGS__; } break;     \
        case 4: { constexpr int B_ = 4; __VA_ARGS__; } break;     \
        default: return MIPX_EINVAL;                              \
    }

}  // namespace mipx
