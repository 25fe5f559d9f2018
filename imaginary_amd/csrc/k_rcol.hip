// k_rcol.hip — the generic Lanczos3 reduce (libvips vips_reduce: reducev then
// reduceh, both shrinks in (1, 2.75), <= 16 taps each way) as a column walker on
// the i8 matrix cores.
//
// A block owns one strip of XW output pixels of one image and walks a segment of
// its output rows down the image, 16 rows per step:
//   * the input rows a step needs live in an LDS ring; each input row is loaded
//     once per segment (the vertical halo of a step is the previous step's rows),
//     by buffer loads into registers issued one step ahead and written to the ring
//     at the top of the next step, so the row loads overlap the block's own work;
//   * the vertical pass is k_rmf2's: per 16-byte column tile D[byte][row] =
//     A[byte][staged row] x B[staged row][row] on v_mfma_i32_16x16x64_i8, A from
//     two ds_read_b64_tr_b8, the 12-bit taps split c = 64 hi + lo, pixels as
//     p - 128 with the offset returned in the seed; the uchar intermediate goes to
//     LDS row-major (interleaved channels, still - 128);
//   * the horizontal pass runs on the interleaved bytes (no channel planes): a
//     unit is 16 consecutive output bytes x 16 rows, output byte o = B x + c takes
//     tap k at intermediate byte B (start(x) + k - org) + c, so its operand row is
//     a 16-byte window of the stride-B tap table (device_reduce_i8s).  These
//     operands depend on the column only, so they are loaded once per segment
//     and held in registers for every step; each step costs two ds_read_b64 and
//     two MFMAs per unit and K step, and the result is one output dword per lane.
// The COPY edge: rows clamp at the load; columns outside the image are gathered
// from the edge pixel at the load (only the chunks that hold them), so the
// vertical pass already produces the edge-extended intermediate.
//
// Results are bit-identical to reducev -> reduceh (oracle/vips_ref.c): the same
// integer sums in int32, the same rounding (>> 12 with 2048 folded into the seed)
// and clamping, the same positions (sep_position / vips_ref.c reduce_position).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "device_common.h"

namespace mipx {
namespace {

using namespace dev;

typedef int rc_v4i __attribute__((ext_vector_type(4)));
typedef int rc_v2i __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void rc_lds_void;

constexpr int kRcRows = 16;   // output rows per step (the MFMA N)

struct RcArgs {
    const u8 *in;
    u8 *out;
    int w, h;                 // input image
    int ox0, oy0, ow, oh;     // output window (op-output coordinates) and its size
    long long in_img, out_img;
    int strips, segs, seg_steps;
    int ring;                 // ring rows: a multiple of 16, >= the rows one step reads
    int rs;                   // ring row stride in dwords ((rs mod 64) / 4 odd)
    int iw;                   // intermediate row stride in bytes
    int vtaps, vpad, htaps, hpad;
    double vs, hs;
    const signed char *tabv;  // device_reduce_i8(vs): [129][hi, lo][kHmTabW]
    const int *sumv;          // its per-phase tap sums
    const signed char *tabh;  // device_reduce_i8s(hs, B): [129][hi, lo][kRsTabW]
    const int *sumh;
    const float *tabf;        // device_reduce_table(hs): [129][htaps] (edge operands, narrow images)
    const signed char *tabhf; // device_reduce_i8s_fold(hs, B): the COPY edge folded in
    int out_aligned;          // every output row starts on a dword
    int centre;               // MIPX_REDUCE_CENTRE: centre sampling convention
    unsigned long long *stamps;  // diagnostic (MIPX_RCOL_STAMPS=1): per block, cycles per step phase
};

// libvips reduce position (reducev.cpp / reduceh.cpp): X = reduce_x (o * shrink, or
// the centre convention), first tap floor(X) - pad, phase ((int)(X * 256) & 255 + 1) >> 1
__device__ __forceinline__ void rc_pos(int o, double s, int pad, int *start, int *phase, int centre) {
    const double X = reduce_x(o, s, centre);
    *start = static_cast<int>(X) - pad;
    *phase = ((static_cast<int>(X * 256.0) & 255) + 1) >> 1;
}

// Workgroup barrier for LDS data: this wave's LDS reads and writes complete, then
// s_barrier; the "memory" clobber keeps the compiler from moving memory accesses across
// it.  Not the fence builtins: with direct-to-LDS loads in flight, an LDS release fence
// makes the compiler drain vmcnt(0) — every load of the next steps (their ring rows go to
// slots nobody reads before a later counted wait).
__device__ __forceinline__ void rc_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// 8 bytes of a kHmTabW tap row from byte o (taps at kHmTabPad ..; zeros around)
__device__ __forceinline__ rc_v2i rc_taps8(const signed char *row, int o) {
    o = clampi(o, kHmTabPad - 8, kHmTabPad + 16);
    const uint32_t *p = reinterpret_cast<const uint32_t *>(row + (o & ~3));
    const int sh = o & 3;
    const uint32_t a = p[0], b = p[1], c = p[2];
    return rc_v2i{static_cast<int>(__builtin_amdgcn_alignbyte(b, a, sh)),
                  static_cast<int>(__builtin_amdgcn_alignbyte(c, b, sh))};
}

// 16 bytes of a kRsTabW stride-B tap row from byte o (any alignment)
__device__ __forceinline__ rc_v4i rc_frag16(const signed char *row, int o) {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(row + (o & ~3));
    const int sh = o & 3;
    const uint4 d = *reinterpret_cast<const uint4 *>(p);
    const uint32_t e = p[4];
    return rc_v4i{static_cast<int>(__builtin_amdgcn_alignbyte(d.y, d.x, sh)),
                  static_cast<int>(__builtin_amdgcn_alignbyte(d.z, d.y, sh)),
                  static_cast<int>(__builtin_amdgcn_alignbyte(d.w, d.z, sh)),
                  static_cast<int>(__builtin_amdgcn_alignbyte(e, d.w, sh))};
}

// (a0..3 + 2048) >> 12 clamped to 0..255 and packed (accumulators seeded with the
// rounding); v_ashr_pk_u8_i32 writes 16 bits, so the halves are joined by a perm
__device__ __forceinline__ uint32_t rc_round4(int a0, int a1, int a2, int a3) {
    uint32_t lo, hi;
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 12" : "=v"(lo) : "v"(a0), "v"(a1));
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 12" : "=v"(hi) : "v"(a2), "v"(a3));
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// Horizontal operand rows of one output byte o = B x + c (x's first tap sp, phase pp)
// for the 16 K bytes j0 .. j0 + 15 of the intermediate (staged pixel org + (j - c) / B),
// with libvips' COPY edge folded in: taps whose pixel clamps to the same edge pixel
// are summed onto it (the staged bytes outside the image are never weighted).  Used
// for the few lanes whose window crosses an image edge; the rest load the table.
__device__ __forceinline__ void rc_edge_frag(const float *tabf, int taps, int pp, int sp, int c, int j0, int org,
                                             int w, int B, rc_v4i *fh, rc_v4i *fl) {
    uint32_t hw[4] = {0u, 0u, 0u, 0u}, lw[4] = {0u, 0u, 0u, 0u};
    const float *cr = tabf + pp * taps;
    for (int e = 0; e < 16; ++e) {
        const int d = j0 + e - c;
        if (d < 0 || d % B != 0) continue;
        const int p = org + d / B;
        if (p < 0 || p > w - 1) continue;
        int v = 0;
        for (int k = 0; k < taps; ++k)
            if (clampi(sp + k, 0, w - 1) == p) v += static_cast<int>(cr[k]);
        hw[e >> 2] |= (static_cast<uint32_t>(v >> 6) & 0xffu) << (8 * (e & 3));
        lw[e >> 2] |= (static_cast<uint32_t>(v & 63)) << (8 * (e & 3));
    }
    *fh = rc_v4i{static_cast<int>(hw[0]), static_cast<int>(hw[1]), static_cast<int>(hw[2]), static_cast<int>(hw[3])};
    *fl = rc_v4i{static_cast<int>(lw[0]), static_cast<int>(lw[1]), static_cast<int>(lw[2]), static_cast<int>(lw[3])};
}

// LDS accesses of the step loop as inline asm.  The compiler cannot tell these from
// the direct-to-LDS loads in flight (the ring rows and taps of later steps, which go
// to slots nothing reads before their own counted wait) and would put vmcnt(0) before
// each one; as asm it does not, and the loop waits on lgkmcnt itself.
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
__device__ __forceinline__ rc_u2 lds_rd64(uint32_t a) {
    rc_u2 v;
    asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
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
__device__ __forceinline__ void lgkm_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// The wait must also be a data dependence of the values it waits for: an asm read's
// result is an ordinary register to the compiler, which could otherwise schedule its
// first use between the read and a separate wait (no hardware interlock on LDS returns)
template <typename T>
__device__ __forceinline__ void rc_pin(T &v) { asm volatile("" : "+v"(v)); }
template <int N, typename... T>
__device__ __forceinline__ void lgkm_wait_for(T &...v) {
    (rc_pin(v), ...);  // the values are live into the wait
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
    (rc_pin(v), ...);  // every later use reads the copy made after the wait
}

// 8 bytes of a kHmTabW tap row in LDS from byte o: the three dwords, then the shift.
// The rows are sliced [dword / 4][16 rows][dword % 4] (row = this lane's base, dword
// d at + (d >> 2) * 256 + (d & 3) * 4 bytes); dw0 = 0 for the hi row, 16 for the lo row.
struct RcTap8 { uint32_t a, b, c; int sh; };
__device__ __forceinline__ RcTap8 rc_taps8_issue(uint32_t row, int dw0, int o) {
    o = clampi(o, kHmTabPad - 8, kHmTabPad + 16);
    const int d = dw0 + (o >> 2);
    auto at = [&](int k) { return row + (((d + k) >> 2) << 8) + (((d + k) & 3) << 2); };
    return RcTap8{lds_rd32(at(0)), lds_rd32(at(1)), lds_rd32(at(2)), o & 3};
}
__device__ __forceinline__ rc_v2i rc_taps8_done(const RcTap8 &t) {
    return rc_v2i{static_cast<int>(__builtin_amdgcn_alignbyte(t.b, t.a, t.sh)),
                  static_cast<int>(__builtin_amdgcn_alignbyte(t.c, t.b, t.sh))};
}

__device__ __forceinline__ unsigned long long rc_now() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// s_waitcnt vmcnt(n) for a wave-uniform n (the instruction takes an immediate).
// Buffer loads, stores and LDS-DMA retire in issue order on the VM counter, so
// "all but the n youngest" is exact for them (MI355X_MICROARCH.md, vmcnt).
__device__ __forceinline__ void rc_wait_vm(int n) {
    switch (__builtin_amdgcn_readfirstlane(min(max(n, 0), 63))) {
#define RC_W(k) \
    case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
#define RC_W8(k) RC_W(k) RC_W(k + 1) RC_W(k + 2) RC_W(k + 3) RC_W(k + 4) RC_W(k + 5) RC_W(k + 6) RC_W(k + 7)
        RC_W8(0) RC_W8(8) RC_W8(16) RC_W8(24) RC_W8(32) RC_W8(40) RC_W8(48) RC_W8(56)
#undef RC_W8
#undef RC_W
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

constexpr int kRcD = 2;  // steps whose loads are in flight ahead of the step being computed

// WV waves per block, XW = 16 WV output pixels per strip: 3 (RGB) / 4 (RGBA) units per wave.
// A step's global traffic (its new ring rows, its 16 output rows' vertical tap rows and
// tap sums) is direct-to-LDS DMA issued kRcD steps ahead; the step waits for it with a
// counted vmcnt (every younger DMA of this wave stays in flight) and a barrier.
template <int B, int WV, int NKS>
__global__ void __launch_bounds__(512) k_rcol(RcArgs a) {
    constexpr int XW = 16 * WV;
    constexpr int NT = 64 * WV;       // threads
    constexpr int UPW = B;            // units per wave: XW B / 16 / WV
    constexpr int NSL = kRcD + 1;     // tap slots
    extern __shared__ __attribute__((aligned(16))) uint32_t rcs[];
    uint32_t *ring = rcs;                                                   // [ring][rs]
    u8 *inter = reinterpret_cast<u8 *>(ring + a.ring * a.rs);              // [16][iw] (pixel - 128)
    int *pbias = reinterpret_cast<int *>(inter + kRcRows * a.iw);          // [XW * B] 128 * tap sum + 2048
    uint32_t *vtap = reinterpret_cast<uint32_t *>(pbias + XW * B);         // [NSL][16 rows][hi 16 | lo 16 dwords]
    int *vsum = reinterpret_cast<int *>(vtap + NSL * kRcRows * 32);        // [NSL][16] tap sums

    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int strip = static_cast<int>(t % static_cast<uint32_t>(a.strips));
    const int rest = static_cast<int>(t / static_cast<uint32_t>(a.strips));
    const int seg = rest % a.segs;
    const int img = __builtin_amdgcn_readfirstlane(rest / a.segs);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n = lane & 15, kg = lane >> 4;
    const unsigned long long t_k0 = a.stamps ? rc_now() : 0;

    const int x0 = strip * XW, x_last = min(x0 + XW - 1, a.ow - 1);
    const int vbytes = B * (x_last - x0 + 1);  // output bytes of this strip row
    int lo, hi, ph;
    rc_pos(a.ox0 + x0, a.hs, a.hpad, &lo, &ph, a.centre);
    rc_pos(a.ox0 + x_last, a.hs, a.hpad, &hi, &ph, a.centre);
    hi += a.htaps - 1;
    const int org = lo & ~3;                 // first staged pixel (B org stays dword aligned)
    const int span = B * (hi - org + 1);     // staged bytes per row
    const int nt = (span + 15) >> 4;         // 16-byte column tiles
    const int ndw = (span + 3) >> 2;         // staged dwords per row
    const int cpr = (ndw + 63) >> 6;         // DMA instructions per row
    const int pitch = a.w * B;

    const int y_begin = seg * a.seg_steps * kRcRows;
    const int y_end = min(a.oh, y_begin + a.seg_steps * kRcRows);
    const int steps = (y_end - y_begin + kRcRows - 1) / kRcRows;

    const __amdgpu_buffer_rsrc_t src = image_rsrc(a.in + img * a.in_img, a.in_img);
    const __amdgpu_buffer_rsrc_t tsrc = image_rsrc(reinterpret_cast<const u8 *>(a.tabv),
                                                   (kTransformScale + 1) * (2 * kHmTabW + 4));
    u8 *ob = a.out + img * a.out_img;
    const __amdgpu_buffer_rsrc_t dst = __builtin_amdgcn_make_buffer_rsrc(ob, 0, static_cast<int>(a.out_img), 0x00020000);

    // step geometry: first ring row and end of the rows read (uniform)
    auto step_rows = [&](int st, int *r_lo, int *r_end) {
        const int y = y_begin + st * kRcRows, nr = min(kRcRows, y_end - y);
        int p;
        rc_pos(a.oy0 + y, a.vs, a.vpad, r_lo, &p, a.centre);
        rc_pos(a.oy0 + y + nr - 1, a.vs, a.vpad, r_end, &p, a.centre);
        *r_end += a.vtaps;
    };
    int r_lo0, r_end0;
    step_rows(0, &r_lo0, &r_end0);
    const int vbase = r_lo0;
    u8 *ringb = reinterpret_cast<u8 *>(ring);
    const int rsb = a.rs * 4;
    // DMA for step st: ring rows [v0, v1) and the step's vertical tap rows + sums, dealt to
    // the waves; returns this wave's instruction count.  Image row offsets ride in the
    // VGPR offset (range-checked per image); rows clamp (COPY edge).
    int slot_ld = 0;  // ring slot of row `loaded` ((loaded - vbase) mod ring, tracked without divisions)
    auto issue = [&](int st, int v0, int v1) -> int {
        // whole rows dealt to the waves (row l -> wave l mod WV), cpr instructions per row
        const int nrows = v1 - v0;
        int slot = slot_ld + wave;
        slot = slot >= a.ring ? slot - a.ring : slot;
        int cnt = 0;
        for (int l = wave; l < nrows; l += WV) {
            const int ro = clampi(v0 + l, 0, a.h - 1) * pitch + B * org + 4 * lane;
            u8 *drow = ringb + slot * rsb;
            for (int c = 0; c < cpr; ++c)
                if (64 * c + lane < ndw)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(src, (rc_lds_void *)(drow + 256 * c), 4, ro + 256 * c, 0, 0, 0);
            cnt += cpr;
            slot += WV;
            slot = slot >= a.ring ? slot - a.ring : slot;
        }
        slot_ld += nrows;
        slot_ld = slot_ld >= a.ring ? slot_ld - a.ring : slot_ld;
        const int sl = st % NSL;
        const int y = y_begin + st * kRcRows, nr = min(kRcRows, y_end - y);
        // 16 rows x 32 dwords (the hi and lo 64-byte tap rows of each output row's phase),
        // stored as 8 slices of [16 rows][4 dwords] so the 16 rows' reads of one dword
        // spread over 16 bank quads (instruction i, lane l: row l >> 2, dword 4 i + (l & 3))
        for (int i = wave; i < kRcRows * 32 / 64; i += WV) {
            const int r = lane >> 2, dw = 4 * i + (lane & 3);
            int sv, pv;
            rc_pos(a.oy0 + y + min(r, nr - 1), a.vs, a.vpad, &sv, &pv, a.centre);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(tsrc, (rc_lds_void *)(vtap + (sl * kRcRows * 32 + 64 * i)), 4,
                                                     (pv * 2 + (dw >> 4)) * kHmTabW + 4 * (dw & 15), 0, 0, 0);
            ++cnt;
        }
        if (wave == (kRcRows * 32 / 64) % WV) {  // the 16 tap sums (after the 129 x 2 rows)
            int sv, pv;
            rc_pos(a.oy0 + y + min(lane & 15, nr - 1), a.vs, a.vpad, &sv, &pv, a.centre);
            if (lane < kRcRows)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(tsrc, (rc_lds_void *)(vsum + sl * kRcRows), 4,
                                                         (kTransformScale + 1) * 2 * kHmTabW + 4 * pv, 0, 0, 0);
            ++cnt;
        }
        return cnt;
    };

    // ---- prime: steps 0 .. kRcD - 1 ----
    int loaded = vbase, cnt_next = 0;
    for (int st = 0; st < kRcD && st < steps; ++st) {
        int rl, re;
        step_rows(st, &rl, &re);
        const int c = issue(st, loaded, re);
        loaded = re;
        if (st == 1) cnt_next = c;
    }

    // ---- per-segment set-up: horizontal operands (registers, COPY edge folded) and biases ----
    for (int j = tid; j < XW * B; j += NT) {
        int sp, pp;
        rc_pos(a.ox0 + min(x0 + j / B, x_last), a.hs, a.hpad, &sp, &pp, a.centre);
        pbias[j] = 128 * a.sumh[pp] + 2048;
    }
    // every operand load issued before the first is used (one memory round trip)
    rc_v4i th[UPW][NKS], tl[UPW][NKS];
    uint4 qh[UPW][NKS], ql[UPW][NKS];
    uint32_t eh[UPW][NKS], el[UPW][NKS];
    int qsh[UPW][NKS];
    bool both[UPW];
    int kb[UPW];
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
        const int u = wave + WV * i;
        int sf, pf;
        rc_pos(a.ox0 + min(x0 + (16 * u) / B, x_last), a.hs, a.hpad, &sf, &pf, a.centre);
        kb[i] = __builtin_amdgcn_readfirstlane((B * (sf - org) + (16 * u) % B) & ~7);  // K origin (8-byte aligned)
        const int o = 16 * u + n, xl = o / B, c = o - B * xl;
        int sp, pp;
        rc_pos(a.ox0 + min(x0 + xl, x_last), a.hs, a.hpad, &sp, &pp, a.centre);
        const int lfold = -sp, rfold = sp + a.htaps - 1 - (a.w - 1);  // > 0: taps past that image edge
        const signed char *rh =
            lfold > 0 ? a.tabhf + ((static_cast<size_t>(lfold - 1) * (kTransformScale + 1) + pp) * 2) * kRsTabW
            : rfold > 0 ? a.tabhf + ((static_cast<size_t>(a.htaps - 1 + rfold - 1) * (kTransformScale + 1) + pp) * 2) * kRsTabW
                        : a.tabh + static_cast<size_t>(pp) * 2 * kRsTabW;
        both[i] = lfold > 0 && rfold > 0;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const int j0 = kb[i] + 64 * ks + 16 * kg;
            if (both[i]) {  // images narrower than the mask: fold both edges here
                rc_edge_frag(a.tabf, a.htaps, pp, sp, c, j0, org, a.w, B, &th[i][ks], &tl[i][ks]);
            } else {
                const int off = kRsTabPad + j0 - c - B * (sp - org);
                const uint32_t *ph = reinterpret_cast<const uint32_t *>(rh + (off & ~3));
                const uint32_t *pl = reinterpret_cast<const uint32_t *>(rh + kRsTabW + (off & ~3));
                qh[i][ks] = *reinterpret_cast<const uint4 *>(ph);
                eh[i][ks] = ph[4];
                ql[i][ks] = *reinterpret_cast<const uint4 *>(pl);
                el[i][ks] = pl[4];
                qsh[i][ks] = off & 3;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
        if (both[i]) continue;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const int sh = qsh[i][ks];
            const uint4 d = qh[i][ks], e = ql[i][ks];
            th[i][ks] = rc_v4i{static_cast<int>(__builtin_amdgcn_alignbyte(d.y, d.x, sh)),
                               static_cast<int>(__builtin_amdgcn_alignbyte(d.z, d.y, sh)),
                               static_cast<int>(__builtin_amdgcn_alignbyte(d.w, d.z, sh)),
                               static_cast<int>(__builtin_amdgcn_alignbyte(eh[i][ks], d.w, sh))};
            tl[i][ks] = rc_v4i{static_cast<int>(__builtin_amdgcn_alignbyte(e.y, e.x, sh)),
                               static_cast<int>(__builtin_amdgcn_alignbyte(e.z, e.y, sh)),
                               static_cast<int>(__builtin_amdgcn_alignbyte(e.w, e.z, sh)),
                               static_cast<int>(__builtin_amdgcn_alignbyte(el[i][ks], e.w, sh))};
        }
    }

    uint32_t res[UPW];
    int y_prev = 0, nr_prev = 0;
    int ring_lo = 0, r_lo_prev = vbase;
    const bool stamp = a.stamps != nullptr;  // uniform
    unsigned long long ph_t[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, t_prev = t_k0;
    auto mark = [&](int k) {
        if (stamp) {
            const unsigned long long t1 = rc_now();
            ph_t[k] += t1 - t_prev;
            t_prev = t1;
        }
    };
    mark(8); asm volatile(";@@MARK 8");  // prime + set-up
    for (int s = 0; s < steps; ++s) {
        const int y = y_begin + s * kRcRows;
        const int nr = min(kRcRows, y_end - y);
        int r_lo, r_end;
        step_rows(s, &r_lo, &r_end);
        // (C) this step's DMA has landed (this wave: all but the next step's loads; the
        // barrier: every wave), the intermediate is free (previous horizontal pass done)
        mark(0); asm volatile(";@@MARK 0");
        rc_wait_vm(s + 1 < steps ? cnt_next : 0);
        mark(1); asm volatile(";@@MARK 1");
        rc_barrier();
        mark(2); asm volatile(";@@MARK 2");
        // (D) the previous step's outputs
        if (s > 0) {
#pragma unroll
            for (int i = 0; i < UPW; ++i) {
                const int u = wave + WV * i;
                const int e = 16 * u + 4 * kg;  // strip byte of the lane's dword
                if (n >= nr_prev || e >= vbytes) continue;
                const int qo = (y_prev + n) * a.ow * B + B * x0 + e;
                if (a.out_aligned) {
                    __builtin_amdgcn_raw_buffer_store_b32(res[i], dst, qo, 0, 0);
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (e + k < vbytes)
                            __builtin_amdgcn_raw_buffer_store_b8(static_cast<u8>(res[i] >> (8 * k)), dst, qo + k, 0, 0);
                }
            }
        }
        // (B) step s + kRcD's loads: its new rows go to slots of rows below this step's
        // first (ring >= rows from this step's first to that step's last, host-checked)
        mark(3); asm volatile(";@@MARK 3");  // stores
        cnt_next = 0;
        if (s + kRcD < steps) {
            int rl, re;
            step_rows(s + kRcD, &rl, &re);
            cnt_next = issue(s + kRcD, loaded, re);
            loaded = re;
        }
        mark(4); asm volatile(";@@MARK 4");  // DMA issue
        // (E) vertical pass: 16-byte column tiles dealt to the waves.  K index 16 kg + e
        // holds relative row 8 kg + e (e < 8) or 32 + 8 kg + e - 8, so the 16 rows one
        // 32-lane half reads per transposed load sit in consecutive ring slots
        {
            const int sl = s % NSL;
            int sv, pv;
            rc_pos(a.oy0 + y + min(n, nr - 1), a.vs, a.vpad, &sv, &pv, a.centre);
            const uint32_t rv = rc_lds(vtap + sl * kRcRows * 32 + 4 * n);
            const int d = sv - r_lo - kHmTabPad;
            const RcTap8 qh0 = rc_taps8_issue(rv, 0, 8 * kg - d), qh1 = rc_taps8_issue(rv, 0, 32 + 8 * kg - d);
            const RcTap8 ql0 = rc_taps8_issue(rv, 16, 8 * kg - d), ql1 = rc_taps8_issue(rv, 16, 32 + 8 * kg - d);
            const uint32_t vsr = lds_rd32(rc_lds(vsum + sl * kRcRows + n));
            ring_lo += r_lo - r_lo_prev;  // ring slot of this step's first row
            ring_lo = ring_lo >= a.ring ? ring_lo - a.ring : ring_lo;
            r_lo_prev = r_lo;
            const int base = ring_lo;
            int s1 = base + 8 * kg + (n >> 1), s2 = s1 + 32;
            s1 = s1 >= a.ring ? s1 - a.ring : s1;
            s1 = s1 >= a.ring ? s1 - a.ring : s1;
            s2 = s2 >= a.ring ? s2 - a.ring : s2;
            s2 = s2 >= a.ring ? s2 - a.ring : s2;
            s2 = s2 >= a.ring ? s2 - a.ring : s2;
            const uint32_t a1 = rc_lds(ringb + s1 * rsb + 8 * (n & 1));
            const uint32_t a2 = rc_lds(ringb + s2 * rsb + 8 * (n & 1));
            const uint32_t iq = rc_lds(inter + n * a.iw + 4 * kg);
            RcTap8 th0 = qh0, th1 = qh1, tl0 = ql0, tl1 = ql1;
            uint32_t vsv = vsr;
            lgkm_wait_for<0>(th0.a, th0.b, th0.c, th1.a, th1.b, th1.c, tl0.a, tl0.b, tl0.c, tl1.a, tl1.b, tl1.c, vsv);
            const rc_v2i h0 = rc_taps8_done(th0), h1 = rc_taps8_done(th1);
            const rc_v2i l0 = rc_taps8_done(tl0), l1 = rc_taps8_done(tl1);
            const rc_v4i bh = rc_v4i{h0.x, h0.y, h1.x, h1.y};
            const rc_v4i bl = rc_v4i{l0.x, l0.y, l1.x, l1.y};
            const int vb = 128 * static_cast<int>(vsv) + 2048;
            auto tile = [&](int ct, rc_v2i t1, rc_v2i t2) {
                const rc_v4i av = rc_v4i{t1.x ^ static_cast<int>(0x80808080u), t1.y ^ static_cast<int>(0x80808080u),
                                         t2.x ^ static_cast<int>(0x80808080u), t2.y ^ static_cast<int>(0x80808080u)};
                rc_v4i dh = rc_v4i{0, 0, 0, 0}, dl = rc_v4i{vb, vb, vb, vb};
                dh = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bh, dh, 0, 0, 0);
                dl = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bl, dl, 0, 0, 0);
                const uint32_t wv = rc_round4((dh[0] << 6) + dl[0], (dh[1] << 6) + dl[1], (dh[2] << 6) + dl[2],
                                              (dh[3] << 6) + dl[3]);
                lds_wr32(iq + 16 * ct, wv ^ 0x80808080u);
            };
            // two tiles in flight per wait
            for (int ct = wave; ct < nt; ct += 2 * WV) {
                const bool two = ct + WV < nt;  // uniform
                rc_v2i t1a = lds_tr8(a1 + 16 * ct), t2a = lds_tr8(a2 + 16 * ct);
                rc_v2i t1b = t1a, t2b = t2a;
                if (two) {
                    t1b = lds_tr8(a1 + 16 * (ct + WV));
                    t2b = lds_tr8(a2 + 16 * (ct + WV));
                }
                lgkm_wait_for<0>(t1a, t2a, t1b, t2b);
                tile(ct, t1a, t2a);
                if (two) tile(ct + WV, t1b, t2b);
            }
        }
        mark(5); asm volatile(";@@MARK 5");  // vertical
        // (F) the intermediate is complete
        rc_barrier();
        mark(6); asm volatile(";@@MARK 6");
        // (H) horizontal pass: units wave + WV i, operands from registers; unit i + 1's
        // LDS reads are in flight while unit i computes
        {
            constexpr int RPU = 1 + 2 * NKS;  // LDS reads per unit
            rc_u4 bias[UPW];
            rc_u2 q[UPW][NKS][2];
            auto rd = [&](int i) {
                const int u = wave + WV * i;
                bias[i] = lds_rd128(rc_lds(pbias + 16 * u + 4 * kg));
                const uint32_t ir = rc_lds(inter + n * a.iw + kb[i] + 16 * kg);
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) {
                    q[i][ks][0] = lds_rd64(ir + 64 * ks);
                    q[i][ks][1] = lds_rd64(ir + 64 * ks + 8);
                }
            };
            // units past the strip's last output byte read in-range LDS and are not stored
            rd(0);
#pragma unroll
            for (int i = 0; i < UPW; ++i) {
                if (i + 1 < UPW) {
                    rd(i + 1);
                    if constexpr (NKS == 1) lgkm_wait_for<RPU>(bias[i], q[i][0][0], q[i][0][1]);
                    else lgkm_wait_for<RPU>(bias[i], q[i][0][0], q[i][0][1], q[i][NKS - 1][0], q[i][NKS - 1][1]);
                } else {
                    if constexpr (NKS == 1) lgkm_wait_for<0>(bias[i], q[i][0][0], q[i][0][1]);
                    else lgkm_wait_for<0>(bias[i], q[i][0][0], q[i][0][1], q[i][NKS - 1][0], q[i][NKS - 1][1]);
                }
                rc_v4i ah = rc_v4i{0, 0, 0, 0};
                rc_v4i al = rc_v4i{static_cast<int>(bias[i].x), static_cast<int>(bias[i].y), static_cast<int>(bias[i].z),
                                   static_cast<int>(bias[i].w)};
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) {
                    const rc_v4i bz = rc_v4i{static_cast<int>(q[i][ks][0].x), static_cast<int>(q[i][ks][0].y),
                                             static_cast<int>(q[i][ks][1].x), static_cast<int>(q[i][ks][1].y)};
                    ah = __builtin_amdgcn_mfma_i32_16x16x64_i8(th[i][ks], bz, ah, 0, 0, 0);
                    al = __builtin_amdgcn_mfma_i32_16x16x64_i8(tl[i][ks], bz, al, 0, 0, 0);
                }
                res[i] = rc_round4((ah[0] << 6) + al[0], (ah[1] << 6) + al[1], (ah[2] << 6) + al[2], (ah[3] << 6) + al[3]);
            }
        }
        mark(7); asm volatile(";@@MARK 7");  // horizontal
        y_prev = y;
        nr_prev = nr;
    }
    if (stamp && tid == 0) {
        for (int k = 0; k < 9; ++k) a.stamps[blockIdx.x * 10 + k] = ph_t[k];
        a.stamps[blockIdx.x * 10 + 9] = static_cast<unsigned long long>(steps);
    }
    // the last step's outputs
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
        const int u = wave + WV * i;
        const int e = 16 * u + 4 * kg;
        if (n >= nr_prev || e >= vbytes) continue;
        const int qo = (y_prev + n) * a.ow * B + B * x0 + e;
        if (a.out_aligned) {
            __builtin_amdgcn_raw_buffer_store_b32(res[i], dst, qo, 0, 0);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (e + k < vbytes)
                    __builtin_amdgcn_raw_buffer_store_b8(static_cast<u8>(res[i] >> (8 * k)), dst, qo + k, 0, 0);
        }
    }
}

int rc_start(int o, double s, int pad, bool centre) { return static_cast<int>(reduce_x_host(o, s, centre)) - pad; }

}  // namespace

// The column walker for both shrinks in (1, 2.75) on 3- / 4-band images whose
// input rows start on a dword; MIPX_EUNSUPPORTED otherwise (the caller runs
// another kernel).  Output window [ox0, ox0 + ow) x [oy0, oy0 + oh).
int reduce_col_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double hs, double vs, int ox0, int oy0,
                      int ow, int oh, hipStream_t st) {
    if ((b != 3 && b != 4) || !(hs > 1.0) || !(vs > 1.0)) return MIPX_EUNSUPPORTED;
    const long long in_img = img_bytes(w, h, b), out_img = img_bytes(ow, oh, b);
    if (in_img >= 0x7fffffffLL || out_img >= 0x7fffffffLL) return MIPX_EUNSUPPORTED;
    if ((w * b) % 4 != 0 || reinterpret_cast<uintptr_t>(in) % 4 != 0) return MIPX_EUNSUPPORTED;
    const int vtaps = reduce_points(vs), htaps = reduce_points(hs);
    if (vtaps > 16 || htaps > 16) return MIPX_EUNSUPPORTED;
    RcArgs a{};
    a.in = in;
    a.out = out;
    a.w = w;
    a.h = h;
    a.ox0 = ox0;
    a.oy0 = oy0;
    a.ow = ow;
    a.oh = oh;
    a.in_img = in_img;
    a.out_img = out_img;
    a.vtaps = vtaps;
    a.vpad = vtaps / 2 - 1;
    a.htaps = htaps;
    a.hpad = htaps / 2 - 1;
    a.vs = vs;
    a.hs = hs;
    a.out_aligned = (ow * b) % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 4 == 0;
    const bool centre = reduce_centre();
    a.centre = centre;
    // ring rows: from a step's first row to the last row of the step kRcD ahead (whose
    // loads are issued before the step's vertical pass), exact over the window's steps;
    // the MFMA K is 64 rows
    const int nsteps = (oh + kRcRows - 1) / kRcRows;
    int lmax = 0, ring = 0;
    auto first_row = [&](int st) { return rc_start(oy0 + st * kRcRows, vs, a.vpad, centre); };
    auto end_row = [&](int st) { return rc_start(oy0 + std::min(oh, (st + 1) * kRcRows) - 1, vs, a.vpad, centre) + vtaps; };
    for (int st = 0; st < nsteps; ++st) {
        lmax = std::max(lmax, end_row(st) - first_row(st));
        ring = std::max(ring, end_row(std::min(nsteps - 1, st + kRcD)) - first_row(st));
    }
    if (lmax > 64) return MIPX_EUNSUPPORTED;
    a.ring = (ring + 15) & ~15;
    int ntv = 0, nth = 0, ntf = 0;
    a.tabv = device_reduce_i8(vs, &ntv, &a.sumv);
    const int *sumh = nullptr;
    if (!device_reduce_i8(hs, &nth, &sumh)) return MIPX_EDEVICE;
    a.sumh = sumh;
    a.tabh = device_reduce_i8s(hs, b, &nth);
    a.tabf = device_reduce_table(hs, &ntf);
    int nfh = 0;
    a.tabhf = device_reduce_i8s_fold(hs, b, &nfh);
    if (!a.tabv || !a.tabh || !a.tabf || !a.tabhf || ntv != vtaps || nth != htaps || ntf != htaps || nfh != htaps)
        return MIPX_EDEVICE;

    // per strip width (16 output pixels per wave): staged bytes, K steps of the
    // horizontal units, LDS
    struct Geo { int wv, nt, nks, rs, iw; size_t lds; };
    auto geo_for = [&](int wv) {
        const int xw = 16 * wv;
        Geo g{wv, 0, 0, 0, 0, 0};
        int kbmax = 0;
        for (int x0 = 0; x0 < ow; x0 += xw) {
            const int xl = std::min(x0 + xw - 1, ow - 1);
            const int lo = rc_start(ox0 + x0, hs, a.hpad, centre), hi = rc_start(ox0 + xl, hs, a.hpad, centre) + htaps - 1;
            const int org = lo & ~3;
            g.nt = std::max(g.nt, (b * (hi - org + 1) + 15) >> 4);
            for (int u = 0; u < xw * b / 16; ++u) {
                const int o0 = 16 * u, o1 = 16 * u + 15;
                if (x0 + o0 / b > xl) break;
                const int xf = x0 + o0 / b, xe = std::min(x0 + o1 / b, xl);
                const int kbu = (b * (rc_start(ox0 + xf, hs, a.hpad, centre) - org) + o0 % b) & ~7;
                const int need = b * (rc_start(ox0 + xe, hs, a.hpad, centre) + htaps - 1 - org) + b;
                g.nks = std::max(g.nks, (need - kbu + 63) / 64);
                kbmax = std::max(kbmax, kbu);
            }
        }
        g.rs = 4 * g.nt;
        while (((g.rs & 63) >> 2) % 2 == 0) g.rs += 4;  // 16 consecutive rows on distinct bank quads
        g.iw = (std::max(16 * g.nt, kbmax + 64 * g.nks) + 16 + 15) & ~15;
        while ((g.iw / 4) % 8 != 4) g.iw += 16;  // 4 mod 8 dwords: the intermediate writes hit distinct banks
        g.lds = static_cast<size_t>(a.ring) * g.rs * 4 + static_cast<size_t>(kRcRows) * g.iw +
                static_cast<size_t>(xw) * b * 4 + static_cast<size_t>(kRcD + 1) * kRcRows * 33 * 4;
        return g;
    };
    Geo g = geo_for(8);  // 128-pixel strips, 512 threads: 2 workgroups per CU
    if (g.nks > 2 || g.lds > 72 * 1024) g = geo_for(4);
    if (g.nks > 2 || g.lds > 64 * 1024) return MIPX_EUNSUPPORTED;
    a.rs = g.rs;
    a.iw = g.iw;
    a.strips = (ow + 16 * g.wv - 1) / (16 * g.wv);
    // segments: enough blocks to fill the chip a few times over, >= 2 steps each
    const int steps = (oh + kRcRows - 1) / kRcRows;
    const long long cols = static_cast<long long>(a.strips) * n;
    // ~3 blocks per resident slot (LDS-limited workgroups per CU x 256 CUs): long segments
    // amortise the per-block set-up, several per slot keep the tail short
    const int wg_per_cu = std::max<int>(1, static_cast<int>((160 * 1024) / std::max<size_t>(g.lds, 1)));
    const long long target = 3LL * 256 * std::min(wg_per_cu, g.wv == 8 ? 2 : 8);
    int segs = static_cast<int>(std::min<long long>(steps, std::max<long long>(1, (target + cols - 1) / cols)));
    int seg_steps = (steps + segs - 1) / segs;
    if (seg_steps < 2 && steps >= 2) seg_steps = 2;
    segs = (steps + seg_steps - 1) / seg_steps;
    a.segs = segs;
    a.seg_steps = seg_steps;
    const long long blocks = cols * segs;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    const dim3 grid(static_cast<unsigned>(blocks)), blk(64 * g.wv);
    // diagnostic: MIPX_RCOL_STAMPS=1 records s_memtime cycles per step phase of every
    // block's first wave and prints the means to stderr (synchronises; timing runs only)
    const char *est = tune_env("MIPX_RCOL_STAMPS");
    unsigned long long *dstamps = nullptr;
    if (est && *est == '1' && hipMalloc(&dstamps, static_cast<size_t>(blocks) * 10 * 8) == hipSuccess) a.stamps = dstamps;
#define MIPX_RC(B_, WV_)                                                                                     \
    if (g.nks == 1) hipLaunchKernelGGL((k_rcol<B_, WV_, 1>), grid, blk, g.lds, st, a);                      \
    else hipLaunchKernelGGL((k_rcol<B_, WV_, 2>), grid, blk, g.lds, st, a);
    if (b == 3) {
        if (g.wv == 8) { MIPX_RC(3, 8) } else { MIPX_RC(3, 4) }
    } else {
        if (g.wv == 8) { MIPX_RC(4, 8) } else { MIPX_RC(4, 4) }
    }
#undef MIPX_RC
    if (dstamps) {
        std::vector<unsigned long long> h(static_cast<size_t>(blocks) * 10);
        if (hipStreamSynchronize(st) == hipSuccess &&
            hipMemcpy(h.data(), dstamps, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
            double tot[9] = {0}, nst = 0;
            for (long long bi = 0; bi < blocks; ++bi) {
                for (int k = 0; k < 9; ++k) tot[k] += static_cast<double>(h[bi * 10 + k]);
                nst += static_cast<double>(h[bi * 10 + 9]);
            }
            static const char *names[9] = {"top", "vm_wait", "barrier_c", "stores", "dma_issue", "vertical",
                                           "barrier_f", "horizontal", "setup_per_block"};
            std::fprintf(stderr, "{\"k_rcol_stamps\": {\"wv\": %d, \"blocks\": %lld, \"steps\": %.0f", g.wv, blocks, nst);
            for (int k = 0; k < 9; ++k)
                std::fprintf(stderr, ", \"%s\": %.1f", names[k], k == 8 ? tot[k] / blocks : tot[k] / nst);
            std::fprintf(stderr, "}}\n");
        }
        (void)hipFree(dstamps);
    }
    return launch_check("k_rcol");
}

}  // namespace mipx
