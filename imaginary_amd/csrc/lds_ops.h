// lds_ops.h — LDS accesses as inline asm with explicit lgkmcnt waits, shared by the
// column walkers (k_rcol.hip, k_bcol.hip): the loops count their own waits so that the
// compiler's waits stay on the global loads that are in flight on purpose.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mipx {
namespace dev {

typedef int rc_v4i __attribute__((ext_vector_type(4)));
typedef int rc_v2i __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void rc_lds_void;

// Workgroup barrier for LDS data: this wave's LDS reads and writes complete, then
// s_barrier; the "memory" clobber keeps the compiler from moving memory accesses across
// it.  Not __syncthreads(): its workgroup release fence would drain vmcnt(0), i.e. wait
// for the ring loads of the next two steps, which are in flight on purpose.
__device__ __forceinline__ void rc_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS accesses of the step loop as inline asm: the loop counts its own lgkmcnt waits
// (two tiles in flight per wait) and the compiler's waits stay on the global loads.
typedef uint32_t rc_u2 __attribute__((ext_vector_type(2)));
typedef uint32_t rc_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t rc_lds(const void *p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((rc_lds_void *)(const_cast<void *>(p))));
}
__device__ __forceinline__ uint32_t lds_rd32(uint32_t a) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
// 16 bytes at an 8-byte-aligned address in one instruction (2 x 8 bytes, adjacent)
__device__ __forceinline__ rc_u4 lds_rd2x64(uint32_t a) {
    rc_u4 v;
    asm volatile("ds_read2_b64 %0, %1 offset1:1" : "=v"(v) : "v"(a));
    return v;
}
// 16 bytes at an 8-byte-aligned address as two ds_read_b64 (2 LDS cycles each per the
// gfx950 rates, against 16 for one ds_read2_b64).  The halves stay separate values until
// after the caller's lgkm_wait_for: joined before the wait, the compiler could
// place the v_movs that build the 128-bit value ahead of s_waitcnt whenever it does not
// allocate both halves into one register tuple, and read stale LDS data.  rc_join after
// the wait.
struct rc_u2x2 {
    rc_u2 lo, hi;
};
__device__ __forceinline__ rc_u2x2 lds_rd64x2(uint32_t a) {
    rc_u2x2 v;
    asm volatile("ds_read_b64 %0, %1" : "=v"(v.lo) : "v"(a));
    asm volatile("ds_read_b64 %0, %1 offset:8" : "=v"(v.hi) : "v"(a));
    return v;
}
__device__ __forceinline__ rc_u2 lds_rd64(uint32_t a) {
    rc_u2 v;
    asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
// two dwords from a 4-byte aligned address (ds_read_b64 needs 8)
__device__ __forceinline__ rc_u2 lds_rd2x32(uint32_t a) {
    rc_u2 v;
    asm volatile("ds_read2_b32 %0, %1 offset1:1" : "=v"(v) : "v"(a));
    return v;
}
__device__ __forceinline__ rc_u4 rc_join(const rc_u2x2 &v) { return rc_u4{v.lo.x, v.lo.y, v.hi.x, v.hi.y}; }
__device__ __forceinline__ rc_u4 lds_rd128(uint32_t a) {
    rc_u4 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
__device__ __forceinline__ rc_v2i lds_tr8(uint32_t a) {
    rc_v2i v;
    asm volatile("ds_read_b64_tr_b8 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
__device__ __forceinline__ void lds_wr32(uint32_t a, uint32_t v) { asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory"); }
__device__ __forceinline__ void lds_wr128(uint32_t a, rc_u4 v) { asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory"); }
// 16 bytes at a 4-byte-aligned LDS address: two ds_write2_b32 (dwords 0, 1 / 2, 3)
__device__ __forceinline__ void lds_wr4x32(uint32_t a, rc_u4 v) {
    asm volatile("ds_write2_b32 %0, %1, %2 offset1:1" ::"v"(a), "v"(v.x), "v"(v.y) : "memory");
    asm volatile("ds_write2_b32 %0, %1, %2 offset0:2 offset1:3" ::"v"(a), "v"(v.z), "v"(v.w) : "memory");
}
// Lane -> (row, 16-byte chunk) for reading back a 16-row x 4-chunk tile with one
// ds_read_b128 per lane (r06).  The instruction serves 4 lane groups, {0-3, 12-15, 20-27},
// {4-11, 16-19, 28-31} and the same + 32: in 4-lane units q = (lane >> 2) & 7 those are
// the q of even / odd popcount, and q >> 1 numbers each set 0..3.  Group g reads rows g,
// g + 4, g + 8, g + 12, which sit on 4 disjoint 16-bank quarters whenever the row stride
// is an odd number of 16-byte units (the tiles' padded strides: 80 / 144 bytes); the
// plain lane -> (lane / 4, lane % 4) order put rows 0, 3, 5, 6 in one group, 2- to 3-way.
__device__ __forceinline__ void tile_rd_lane(int lane, int *row, int *chunk) {
    const int q = (lane >> 2) & 7;
    *row = 2 * (lane >> 5) + (__builtin_popcount(q) & 1) + 4 * (q >> 1);
    *chunk = lane & 3;
}
__device__ __forceinline__ void lgkm_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// The wait must also be a data dependence of the values it waits for: an asm read's
// result is an ordinary register to the compiler, which could otherwise schedule its
// first use between the read and a separate wait (no hardware interlock on LDS returns)
template <typename T>
__device__ __forceinline__ void rc_pin(T &v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void rc_pin(rc_u2x2 &v) {
    asm volatile("" : "+v"(v.lo));
    asm volatile("" : "+v"(v.hi));
}
template <int N, typename... T>
__device__ __forceinline__ void lgkm_wait_for(T &...v) {
    (rc_pin(v), ...);  // the values are live into the wait
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
    (rc_pin(v), ...);  // every later use reads the copy made after the wait
}

// (a0..3 + 2048) >> 12 clamped to 0..255 and packed (accumulators seeded with the
// rounding); v_ashr_pk_u8_i32 writes 16 bits, so the halves are joined by a perm.
// rc_round4s: the same minus 128 as signed bytes (seeds carry - 128 << 12): the
// intermediate in the pixel - 128 form the next pass multiplies
__device__ __forceinline__ uint32_t rc_round4(int a0, int a1, int a2, int a3) {
    uint32_t lo, hi;
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 12" : "=v"(lo) : "v"(a0), "v"(a1));
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 12" : "=v"(hi) : "v"(a2), "v"(a3));
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}
__device__ __forceinline__ uint32_t rc_round4s(int a0, int a1, int a2, int a3) {
    uint32_t lo, hi;
    asm("v_ashr_pk_i8_i32 %0, %1, %2, 12" : "=v"(lo) : "v"(a0), "v"(a1));
    asm("v_ashr_pk_i8_i32 %0, %1, %2, 12" : "=v"(hi) : "v"(a2), "v"(a3));
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

}  // namespace dev
}  // namespace mipx
