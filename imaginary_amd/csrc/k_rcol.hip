// k_rcol.hip — the generic Lanczos3 reduce (libvips vips_reduce: reducev then
// reduceh, both shrinks in (1, ~2.5], <= 16 taps each way) as a column walker on
// the i8 matrix cores.
//
// A block (4 waves) owns one strip of 64 output pixels of one image and walks a
// segment of its output rows down the image, 16 rows per step.  Steps sit on
// absolute 16-row groups of the op output (rows outside the window are computed and
// not stored), so every per-row quantity of the vertical pass comes from one
// per-shrink table (device_rcol_vplan): the step's first and end input rows, and per
// output row its vertical taps already placed at their K positions relative to the
// step's first row, split c = 64 hi + lo, plus the accumulator seed.  The loop does
// no position arithmetic.
//   * ring: the input rows a step reads live in an LDS ring of 32 / 64 rows (slot =
//     row & (ring - 1)).  Each input row is loaded once per segment: 16-byte chunks
//     dealt over the block's 256 lanes (the same lane -> (row, column) map every
//     step), loaded to registers two steps ahead (buffer loads, compiler-counted
//     vmcnt), flipped to pixel - 128 and written to the ring at the top of their step;
//   * vertical: per 16-byte column tile D[byte][row] = A[byte][ring row] x
//     B[ring row][row] on v_mfma_i32_16x16x64_i8, A from two ds_read_b64_tr_b8, B the
//     table's tap fragments (registers, loaded with the ring chunks); the result is
//     the uchar intermediate - 128 (v_ashr_pk_i8_i32), row-major in LDS;
//   * horizontal: on the interleaved bytes, a unit is 16 consecutive output bytes x
//     16 rows, output byte o = B x + c takes tap k at intermediate byte
//     B (start(x) + k - org) + c; those operands depend on the column only and are
//     held in registers for the whole segment (the COPY edge folded in at the image
//     edges), as are the per-byte seeds.  Two ds_read_b64 and two MFMAs per unit and
//     K step; a wave's units are consecutive, and its 16 rows x 16 B dwords go through a
//     wave-private LDS tile to 16-byte row pieces (r03: the 4-byte stores of 16 rows per
//     instruction had capped the kernel; the memory-only pattern, scripts/strip_probe.hip).
// Loads past the image read zeros (buffer range check); rows clamp at the load (COPY
// edge); columns past the image carry zero weight after the fold.
//
// Results are bit-identical to reducev -> reduceh (oracle/vips_ref.c): the same
// integer sums in int32, the same rounding (>> 12 with 2048 folded into the seed)
// and clamping, the same positions (sep_position / vips_ref.c reduce_position).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <utility>
#include <vector>

#include "device_common.h"
#include "lds_ops.h"
#include "r2front.h"

namespace mipx {
namespace {

using namespace dev;

typedef const __attribute__((address_space(4))) int rc_cint;

constexpr int kRcRows = 16;   // output rows per step (the MFMA N)
constexpr int kRcNT = 256;    // threads per block (4 waves, 64-pixel strips)

struct RcArgs {
    const u8 *in;
    u8 *out;
    int w, h;                 // input image
    int ox0, oy0, ow, oh;     // output window (op-output coordinates) and its size
    long long in_img, out_img;
    int strips, segs, seg_steps;
    int k0, ksteps;           // the window's first 16-row group (oy0 / 16) and group count
    int rmask;                // ring rows - 1 (31 or 63)
    int rcap;                 // ring chunks of rows rcap and below (in a load batch) idle
    int rs;                   // ring row stride in bytes ((rs / 4 mod 64) / 4 odd)
    int iw;                   // intermediate row stride in bytes
    int htaps, hpad;
    double hs;
    const u8 *plan;           // device_rcol_vplan(vs): [plan_rows][kRcolPlanRow], then [plan_rows / 16][2] ints
    int plan_rows;
    const signed char *tabh;  // device_reduce_i8s(hs, B): [129][hi, lo][kRsTabW]
    const int *sumh;          // device_reduce_i8(hs) per-phase tap sums
    const float *tabf;        // device_reduce_table(hs): [129][htaps] (edge operands, narrow images)
    const signed char *tabhf; // device_reduce_i8s_fold(hs, B): the COPY edge folded in
    int centre;               // centre sampling convention (mipx_set_reduce_sampling)
    int wst;                  // each wave's 16 rows x 16 UPW bytes go out as 16-byte row pieces
    int swz;                  // horizontal reads: odd K blocks read their second 8 bytes first
    int k4;                   // K origins 4-byte aligned (ds_read2_b32): one K step where 8-byte origins need two
    int allst;                // A/B: every strip issues the edge-piece dword stores (r05 before)
    int skipl;                // ring load batches no lane of the wave needs are not issued
};

// libvips reduce position (reducev.cpp / reduceh.cpp): X = reduce_x (o * shrink, or
// the centre convention), first tap floor(X) - pad, phase ((int)(X * 256) & 255 + 1) >> 1
__device__ __forceinline__ void rc_pos(int o, double s, int pad, int *start, int *phase, int centre) {
    const double X = reduce_x(o, s, centre);
    *start = static_cast<int>(X) - pad;
    *phase = ((static_cast<int>(X * 256.0) & 255) + 1) >> 1;
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

// KMAX ring chunks per lane per step (16 bytes each), NKS horizontal K steps (64 bytes
// each).  Output rows start on a dword (host-checked).
// WPE: the minimum waves per SIMD the register allocation must allow (1: the compiler's
// choice; 4 for the one build where that costs only two spilled registers)
// UNAL (r05): input rows off a dword (w B % 4 != 0, e.g. C5's 1333-pixel RGB rows): every
// 16-byte chunk is loaded from its dword-aligned-down offset with the next dword and
// realigned (v_alignbyte) when it is written to the ring
template <int B, int NKS, int KMAX, int WPE, bool UNAL = false>
__global__ void __launch_bounds__(kRcNT) __attribute__((amdgpu_waves_per_eu(WPE, 8))) k_rcol(RcArgs a) {
    constexpr int WV = kRcNT / 64, XW = 16 * WV;
    constexpr int UPW = B;  // horizontal units per wave: XW B / 16 / WV
    extern __shared__ __attribute__((aligned(16))) uint32_t rcs[];
    const uint32_t ring_l = rc_lds(rcs);                                            // [rmask + 1][rs]
    const uint32_t inter_l = ring_l + static_cast<uint32_t>((a.rmask + 1) * a.rs);  // [16][iw]

    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int strip = static_cast<int>(t % static_cast<uint32_t>(a.strips));
    const int rest = static_cast<int>(t / static_cast<uint32_t>(a.strips));
    const int seg = rest % a.segs;
    const int img = __builtin_amdgcn_readfirstlane(rest / a.segs);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n = lane & 15, kg = lane >> 4;

    const int x0 = strip * XW, x_last = min(x0 + XW - 1, a.ow - 1);
    const int vbytes = B * (x_last - x0 + 1);  // output bytes of this strip row
    int lo, hi, ph;
    rc_pos(a.ox0 + x0, a.hs, a.hpad, &lo, &ph, a.centre);
    rc_pos(a.ox0 + x_last, a.hs, a.hpad, &hi, &ph, a.centre);
    hi += a.htaps - 1;
    // first staged pixel: B org dword aligned; at the left edge (lo < 0) a multiple of 16
    // bytes, so no 16-byte chunk straddles the image start (a load at a negative offset
    // reads 0 whole, image bytes included)
    const int org = lo & (lo < 0 && B == 3 ? ~15 : ~3);
    const int span = B * (hi - org + 1);   // staged bytes per row
    const int cpr = (span + 15) >> 4;      // 16-byte chunks per row = vertical column tiles
    const int pitch = a.w * B;

    const int ka = a.k0 + seg * a.seg_steps;  // this segment's 16-row groups [ka, ka + steps)
    const int steps = min(a.k0 + a.ksteps, ka + a.seg_steps) - ka;

    int idelta = 0;  // UNAL: byte offset of the image in its dword-aligned-down descriptor
    const __amdgpu_buffer_rsrc_t src = UNAL ? image_rsrc_aligned(a.in + img * a.in_img, a.in_img, &idelta)
                                            : image_rsrc(a.in + img * a.in_img, a.in_img);
    const __amdgpu_buffer_rsrc_t prs = image_rsrc(a.plan, static_cast<long long>(a.plan_rows) * kRcolPlanRow);
    rc_cint *srow = (rc_cint *)(a.plan + static_cast<size_t>(a.plan_rows) * kRcolPlanRow);  // [group][first, end]
    const __amdgpu_buffer_rsrc_t dst = image_rsrc(a.out + img * a.out_img, a.out_img);

    // ---- per-segment set-up: horizontal operands (registers, COPY edge folded) ----
    // every operand load issued before the first is used (one memory round trip)
    rc_v4i th[UPW][NKS], tl[UPW][NKS];
    uint4 qh[UPW][NKS], ql[UPW][NKS];
    uint32_t eh[UPW][NKS], el[UPW][NKS];
    int qsh[UPW][NKS];
    bool both[UPW];
    int kb[UPW];
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
        const int u = a.wst ? UPW * wave + i : wave + WV * i;
        int sf, pf;
        rc_pos(a.ox0 + min(x0 + (16 * u) / B, x_last), a.hs, a.hpad, &sf, &pf, a.centre);
        // K origin: 8-byte aligned (ds_read_b64), 4-byte with k4
        kb[i] = __builtin_amdgcn_readfirstlane((B * (sf - org) + (16 * u) % B) & (a.k4 ? ~3 : ~7));
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
    // per output byte seeds of the horizontal pass (lane: bytes 16 u + 4 kg + j of row n)
    // and store offsets (past the strip's last byte: beyond any image, so dropped)
    rc_v4i hb[UPW];
    uint32_t sto[UPW];
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
        const int e = 16 * (a.wst ? UPW * wave + i : wave + WV * i) + 4 * kg;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            int sp, pp;
            rc_pos(a.ox0 + min(x0 + (e + j) / B, x_last), a.hs, a.hpad, &sp, &pp, a.centre);
            hb[i][j] = 128 * a.sumh[pp] + 2048;
        }
        sto[i] = e < vbytes ? static_cast<uint32_t>(B * x0 + e) : 0x20000000u;
    }

    // ring chunks: chunk c = tid + 256 j of a step's rows is (row rr, column col); the
    // same map every step.  A lane's chunks past the step's rows load rows below it:
    // harmless (host-checked: their slots hold rows no longer read).
    int rr[KMAX], cof[KMAX];
    uint32_t lcol[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        const int c = tid + kRcNT * j;
        rr[j] = c / cpr;
        const int col = c - rr[j] * cpr;
        cof[j] = B * org + 16 * col;
        lcol[j] = ring_l + static_cast<uint32_t>(16 * col);
    }
    const int lkf = (kRcNT * KMAX) / cpr;  // rows one load batch covers completely
    // skipl: batch j of this wave loads anything (uniform; the same every step)
    bool wl[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) wl[j] = !a.skipl || __builtin_amdgcn_ballot_w64(rr[j] < a.rcap) != 0;

    // ---- the step pipeline: register set P = (step - ka) & 1 holds step k + 2's ring
    // chunks and vertical operands from the middle of step k to the top of step k + 2.
    // Every step issues the same global loads and stores (out-of-range offsets where
    // there is nothing to do), so the compiler's vmcnt waits are the exact two-step
    // counts and never drain the loads of the next step.
    rc_u4 rv[2][KMAX];
    rc_v4i vh[2], vl[2];
    int vsd[2];
    const int toff = n * kRcolPlanRow + 16 * kg;  // this lane's tap fragment: output row n, K 16 kg ..
    auto issue_taps = [&](auto pc, int k) {
        constexpr int P = decltype(pc)::value;
        const int o = k * (kRcRows * kRcolPlanRow);
        vh[P] = __builtin_bit_cast(rc_v4i, __builtin_amdgcn_raw_buffer_load_b128(prs, toff + o, 0, 0));
        vl[P] = __builtin_bit_cast(rc_v4i, __builtin_amdgcn_raw_buffer_load_b128(prs, toff + o + 64, 0, 0));
        vsd[P] = __builtin_amdgcn_raw_buffer_load_b32(prs, n * kRcolPlanRow + 128 + o, 0, 0);
    };
    // chunks of rows rcap and below are idle: their loads take an offset past the image
    // (no memory access) and they write nothing, so a narrow strip's lanes do not reach
    // past a step's new rows into ring slots still in use (r03: admits narrow last
    // strips and shrinks to ~2.5)
    uint32_t re[2][UNAL ? KMAX : 1];  // UNAL: the dword after each chunk
    auto chunk_off = [&](int r, int j) { return clampi(r + rr[j], 0, a.h - 1) * pitch + cof[j] + idelta; };
    auto realign = [&](rc_u4 v, uint32_t e, int off) -> rc_u4 {
        if constexpr (!UNAL) return v;
        const uint32_t sh = static_cast<uint32_t>(off & 3);
        return rc_u4{__builtin_amdgcn_alignbyte(v.y, v.x, sh), __builtin_amdgcn_alignbyte(v.z, v.y, sh),
                     __builtin_amdgcn_alignbyte(v.w, v.z, sh), __builtin_amdgcn_alignbyte(e, v.w, sh)};
    };
    auto issue_ring = [&](auto pc, int r0) {
        constexpr int P = decltype(pc)::value;
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            if (!wl[j]) continue;
            const int off = rr[j] < a.rcap ? chunk_off(r0, j) : 0x7ffffff0;
            rv[P][j] = __builtin_bit_cast(rc_u4, __builtin_amdgcn_raw_buffer_load_b128(src, UNAL ? off & ~3 : off, 0, 0));
            if constexpr (UNAL)
                re[P][j] = static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(src, (off & ~3) + 16, 0, 0));
        }
    };
    auto write_ring = [&](auto pc, int r0) {
        constexpr int P = decltype(pc)::value;
#pragma unroll
        for (int j = 0; j < KMAX; ++j)
            if (rr[j] < a.rcap)
                lds_wr128(static_cast<uint32_t>(((r0 + rr[j]) & a.rmask) * a.rs) + lcol[j],
                          realign(rv[P][j], re[P][UNAL ? j : 0], chunk_off(r0, j)) ^ 0x80808080u);
    };
    // wst: the wave's units are consecutive (bytes 16 UPW wave ..), staged through a
    // wave-private LDS tile [16 rows][16 UPW (+ 16 for RGBA: bank spread) bytes] and
    // stored as 16-byte pieces: 16 UPW contiguous bytes per row instead of 16
    constexpr int WSR = 16 * UPW + (UPW == 4 ? 16 : 0);
    const uint32_t wst_l = inter_l + static_cast<uint32_t>(kRcRows * a.iw + wave * kRcRows * WSR);
    const int wrow = min(lane / UPW, kRcRows - 1), wch = lane - UPW * (lane / UPW);  // read-back: row, 16-byte chunk
    const int we = 16 * (UPW * wave + wch);                          // its first byte in the strip row
    auto store = [&](int k, bool live, const uint32_t *res) {
        if (a.wst) {
#pragma unroll
            for (int i = 0; i < UPW; ++i) lds_wr32(wst_l + static_cast<uint32_t>(n * WSR + 16 * i + 4 * kg), res[i]);
            rc_u4 q = lds_rd128(wst_l + static_cast<uint32_t>(wrow * WSR + 16 * wch));
            lgkm_wait_for<0>(q);
            const int o = k * kRcRows + wrow - a.oy0;
            const bool ok = live && lane < 16 * UPW && o >= 0 && o < a.oh;
            const int base = o * a.ow * B + B * x0 + we;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(rc_v4i, q), dst,
                                                   ok && we + 16 <= vbytes ? base : 0x7ffffff0, 0, 0);
            if (a.wst == 2 && (vbytes < 16 * UPW * WV || a.allst)) {
                // rows whose byte count is not a multiple of 16: the piece at the image edge in
                // dwords, in the last strip only (uniform: r05, the dword stores every other
                // strip issued with out-of-range offsets were 4 of every 5 store instructions)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    __builtin_amdgcn_raw_buffer_store_b32(
                        q[j], dst, ok && we + 16 > vbytes && we + 4 * j < vbytes ? base + 4 * j : 0x7ffffff0, 0, 0);
            } else if (a.wst == 3 && B * x0 + 16 * UPW * WV >= a.ow * B) {
                // rows not on a dword (the b128 pieces above went out unaligned): the last strip's
                // edge piece byte by byte
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    __builtin_amdgcn_raw_buffer_store_b8(static_cast<u8>(q[j >> 2] >> (8 * (j & 3))), dst,
                                                         ok && we + 16 > vbytes && we + j < vbytes ? base + j : 0x7ffffff0,
                                                         0, 0);
            }
            return;
        }
        const int o = k * kRcRows + n - a.oy0;  // window row of the lane's output row
        const uint32_t rb = live && o >= 0 && o < a.oh ? static_cast<uint32_t>(o * a.ow * B) : 0x80000000u;
#pragma unroll
        for (int i = 0; i < UPW; ++i) __builtin_amdgcn_raw_buffer_store_b32(res[i], dst, static_cast<int>(rb + sto[i]), 0, 0);
    };
    // vertical pass: 16-byte column tiles dealt to the waves, two in flight per wait.  K
    // index 16 kg + e holds relative row 8 kg + e (e < 8) or 32 + 8 kg + e - 8, so the 16
    // rows one 32-lane half reads per transposed load sit in consecutive ring slots
    auto vertical = [&](auto pc, int bk) {
        constexpr int P = decltype(pc)::value;
        const rc_v4i bh = vh[P], bl = vl[P];
        const int sd = vsd[P];
        const int r1 = bk + 8 * kg + (n >> 1);
        const uint32_t a1 = ring_l + static_cast<uint32_t>((r1 & a.rmask) * a.rs + 8 * (n & 1));
        const uint32_t a2 = ring_l + static_cast<uint32_t>(((r1 + 32) & a.rmask) * a.rs + 8 * (n & 1));
        const uint32_t iq = inter_l + static_cast<uint32_t>(n * a.iw + 4 * kg);
        auto tile = [&](int ct, rc_v2i t1, rc_v2i t2) {
            const rc_v4i av = rc_v4i{t1.x, t1.y, t2.x, t2.y};
            rc_v4i dh = rc_v4i{0, 0, 0, 0}, dl = rc_v4i{sd, sd, sd, sd};
            dh = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bh, dh, 0, 0, 0);
            dl = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bl, dl, 0, 0, 0);
            lds_wr32(iq + 16 * ct,
                     rc_round4s((dh[0] << 6) + dl[0], (dh[1] << 6) + dl[1], (dh[2] << 6) + dl[2], (dh[3] << 6) + dl[3]));
        };
            for (int ct = wave; ct < cpr; ct += 2 * WV) {
                const bool two = ct + WV < cpr;  // uniform
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
    };
    // horizontal pass: units wave + WV i, operands from registers, every unit's LDS
    // reads in flight together.  r05: a lane of an odd K block reads bytes 8..15 of its
    // 16 first (hsw = 8) and the operands' halves are swapped to match: with kg = 0 / 1
    // lanes in one 32-lane half on banks 0-1 / 2-3 (mod 4) each read is conflict-free
    // (both halves of one K block at once were 2-way); MIPX_RCOL_SWZ=0 keeps the old order
    const int hsw = a.swz && (kg & 1) ? 8 : 0, hsd = 8 - 2 * hsw;
    auto horizontal = [&](uint32_t *res) {
        rc_u2x2 q[UPW][NKS];
#pragma unroll
        for (int i = 0; i < UPW; ++i) {
            const uint32_t ir = inter_l + static_cast<uint32_t>(n * a.iw + kb[i] + 16 * kg + hsw);
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                // two ds_read_b64 (2 LDS cycles each) rather than one ds_read2_b64 (16): -0.3 to -2 %
                // (profiles/r04/small/rcol_rd64_ab.jsonl); lanes of odd K blocks read their
                // second half first (hsw), so each read's 32-lane half covers all 64 banks
                if (a.k4) {
                    q[i][ks].lo = lds_rd2x32(ir + 64 * ks);
                    q[i][ks].hi = lds_rd2x32(ir + 64 * ks + hsd);
                } else {
                    q[i][ks].lo = lds_rd64(ir + 64 * ks);
                    q[i][ks].hi = lds_rd64(ir + 64 * ks + hsd);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < UPW; ++i)
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) rc_pin(q[i][ks]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < UPW; ++i) {
            rc_v4i ah = rc_v4i{0, 0, 0, 0}, al = hb[i];
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                rc_pin(q[i][ks]);
                const rc_v4i bz = __builtin_bit_cast(rc_v4i, rc_join(q[i][ks]));
                ah = __builtin_amdgcn_mfma_i32_16x16x64_i8(th[i][ks], bz, ah, 0, 0, 0);
                al = __builtin_amdgcn_mfma_i32_16x16x64_i8(tl[i][ks], bz, al, 0, 0, 0);
            }
            res[i] = rc_round4((ah[0] << 6) + al[0], (ah[1] << 6) + al[1], (ah[2] << 6) + al[2], (ah[3] << 6) + al[3]);
        }
    };
    // one step (16-row group k): ring rows of k (loaded two steps ago) -> barrier ->
    // vertical -> loads of k + 2 -> barrier -> horizontal -> stores.  A phantom step
    // (live = false, the odd tail of a pair) issues the same loads and stores, all idle.
    auto body = [&](auto pc, int k, bool live, bool first) {
        uint32_t res[UPW];
#pragma unroll
        for (int i = 0; i < UPW; ++i) res[i] = 0u;
        if (live) {
            if (!first) write_ring(pc, srow[2 * (k - 1) + 1]);
            rc_barrier();
            vertical(pc, srow[2 * k]);
        }
        issue_ring(pc, srow[2 * (k + 1) + 1]);
        issue_taps(pc, k + 2);
        if (live) {
            rc_barrier();
            horizontal(res);
        }
        store(k, live, res);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    const uint32_t zero[UPW] = {};
    // ---- prime: group ka's rows straight into the ring (exact rows only), then the
    // pipeline's first loads (r05: issuing those before the prime's ring writes measured
    // within +-1 %, and the extra live registers spilled in the 4-wave build,
    // profiles/r05/prime_ab.jsonl) ----
    const int bka = srow[2 * ka], eka = srow[2 * ka + 1];
    for (int r = bka; r < eka; r += lkf) {
        rc_u4 tv[KMAX];
        uint32_t te[UNAL ? KMAX : 1];
#pragma unroll
        for (int j = 0; j < KMAX; ++j) {
            const int off = chunk_off(r, j);
            tv[j] = __builtin_bit_cast(rc_u4, __builtin_amdgcn_raw_buffer_load_b128(src, UNAL ? off & ~3 : off, 0, 0));
            if constexpr (UNAL) te[j] = static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(src, (off & ~3) + 16, 0, 0));
        }
#pragma unroll
        for (int j = 0; j < KMAX; ++j)
            if (rr[j] < lkf && r + rr[j] < eka)
                lds_wr128(static_cast<uint32_t>(((r + rr[j]) & a.rmask) * a.rs) + lcol[j],
                          realign(tv[j], te[UNAL ? j : 0], chunk_off(r, j)) ^ 0x80808080u);
    }
    issue_taps(I0{}, ka);
    store(ka, false, zero);  // idle: keeps the load / store sequence the loop's
    issue_ring(I1{}, eka);
    issue_taps(I1{}, ka + 1);
    store(ka, false, zero);
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
    if (hsw) {  // the K halves of odd blocks, in the order their data is read
#pragma unroll
        for (int i = 0; i < UPW; ++i)
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                th[i][ks] = rc_v4i{th[i][ks][2], th[i][ks][3], th[i][ks][0], th[i][ks][1]};
                tl[i][ks] = rc_v4i{tl[i][ks][2], tl[i][ks][3], tl[i][ks][0], tl[i][ks][1]};
            }
    }
    for (int s = 0; s < steps; s += 2) {
        body(I0{}, ka + s, true, s == 0);
        body(I1{}, ka + s + 1, s + 1 < steps, false);
    }
}

int rc_start(int o, double s, int pad, bool centre) { return static_cast<int>(reduce_x_host(o, s, centre)) - pad; }

// ===========================================================================
// k_rchain: vips_reduce 2 x 2 followed by a k_rcol reduce (and its extract window) in
// one launch — the /pipeline resize -> crop chain of C3 (reference image.go:379-410),
// without the 2 x 2 output in HBM.
//
// The block is k_rcol's (a strip of 64 output pixels, 16-row steps, the same vertical
// plan, horizontal operands, stores), but its LDS ring of 2 x 2-output rows is filled
// by a producer ("front") inside the block instead of by loads:
//   * front vertical, straight from HBM into the matrix cores (no input ring): a lane
//     (n, kg) loads dword column n of input rows 4 kg .. 4 kg + 3 of a 16-row block,
//     which is the B operand of v_mfma_i32_16x16x64_i8 with K = (row, byte); the A
//     operand holds the 2 x 2 taps at M = (output row r < 3, byte c), so D lane (n, kg)
//     is output row kg's dword n.  One group = 3 output rows (2r + 12 taps <= 16 rows),
//     one constant A operand for every group; 5 groups = 15 rows per front step;
//   * front horizontal = k_reduce2m's banded product: GP output pixels from a 64-byte
//     window of each of the 15 vertical-result rows, written to the ring (- 128 form);
//   * rows outside the 2 x 2 output (COPY edge) are copies of its first / last row.
// Per 16-row step: front steps until the ring holds the rows the step reads, then
// k_rcol's vertical and horizontal products.  The 2 x 2 sums are the ones k_reduce2x2
// / k_reduce2m compute (taps of the phase the sampling convention gives, same
// rounding), so the output is bit-identical to the two reduces run one after the other.
// ===========================================================================
constexpr int kChRing = 64;   // ring rows (power of two)
constexpr int kChFR = 15;     // 2 x 2-output rows per front step (5 groups of 3)
constexpr int kChFRows = 16;  // front intermediate rows allocated (the horizontal product reads 16)

struct RchArgs {
    const u8 *src;            // the original images (sw x sh x B); the 2 x 2 output is a.w x a.h
    int sw, sh;
    long long src_img;
    const rc_u4 *fops;        // [64 lanes][vh, vl, wh, wl]: the front's MFMA operands (rch_operands)
    int vseed, hseed;         // front seeds: 128 sum(T) + 2048 - (128 << 12) (results in - 128 form)
    int fis;                  // front intermediate row stride (bytes)
    float c0, c1, c3, c5, bias;  // FRONT 1: k_reduce2x2's corner taps / 4096 and its 2^-13 bias
};

// FRONT 0: the vertical pass straight from HBM into the matrix cores (r05 first build,
// 15-row steps); FRONT 1: the vertical pass on the VALU as k_reduce2x2 makes it (corner
// convention: every input row loaded once into a register ring of its odd rows, the next
// 12-row chunk prefetched while this one is consumed), the horizontal on the matrix cores
// W3: a build held to 3 waves per SIMD (168 VGPRs, a few spilled) instead of the
// compiler's 2 (FRONT 1 only; MIPX_CHAIN_W3, A/B)
template <int B, int NKS, int FRONT, int W3>
__global__ void __launch_bounds__(kRcNT) __attribute__((amdgpu_waves_per_eu(W3 ? 3 : 1, 8))) k_rchain(RcArgs a, RchArgs c) {
    using G = RCH<B>;
    constexpr int FR = FRONT ? 12 : kChFR;  // 2 x 2-output rows per front step
    constexpr int WV = kRcNT / 64, XW = 16 * WV, GP = G::GP;
    constexpr int UPW = B;
    extern __shared__ __attribute__((aligned(16))) uint32_t rcs[];
    const uint32_t ring_l = rc_lds(rcs);                                         // [64][rs]
    const uint32_t inter_l = ring_l + static_cast<uint32_t>(kChRing * a.rs);     // [16][iw] + wave tiles
    constexpr int WSR = 16 * UPW + (UPW == 4 ? 16 : 0);
    const uint32_t wst_l = inter_l + static_cast<uint32_t>(kRcRows * a.iw);
    const uint32_t fint_l = wst_l + static_cast<uint32_t>(WV * kRcRows * WSR);   // [FR][fis]
    u8 *fint = reinterpret_cast<u8 *>(rcs) + (fint_l - ring_l);
    u8 *ring = reinterpret_cast<u8 *>(rcs);

    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int strip = static_cast<int>(t % static_cast<uint32_t>(a.strips));
    const int rest = static_cast<int>(t / static_cast<uint32_t>(a.strips));
    const int seg = rest % a.segs;
    const int img = __builtin_amdgcn_readfirstlane(rest / a.segs);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n = lane & 15, kg = lane >> 4;

    const int x0 = strip * XW, x_last = min(x0 + XW - 1, a.ow - 1);
    const int vbytes = B * (x_last - x0 + 1);
    int lo, hi, ph;
    rc_pos(a.ox0 + x0, a.hs, a.hpad, &lo, &ph, a.centre);
    rc_pos(a.ox0 + x_last, a.hs, a.hpad, &hi, &ph, a.centre);
    hi += a.htaps - 1;
    const int org = lo & (lo < 0 && B == 3 ? ~15 : ~3);
    const int span = B * (hi - org + 1);
    const int cpr = (span + 15) >> 4;
    // front geometry: pixels org .. org + ni - 1 of the 2 x 2 output (covering the ring row)
    const int ni = (((16 * cpr + B - 1) / B + GP - 1) / GP) * GP;
    const int vst = 2 * org - 5;                // first front-intermediate pixel (input pixel index)
    const int vb0 = (B * vst) & ~63;            // 64-byte aligned byte of the first column tile
    const int ish = B * vst - vb0 + G::LOFF;    // LDS byte of front pixel 0 in a row; == SH (mod 8)
    const int ntile = (ish - G::LOFF + B * (2 * ni + 10) + 63) >> 6;
    const int ngr = ni / GP;
    const int spitch = c.sw * B;

    const int ka = a.k0 + seg * a.seg_steps;
    const int steps = min(a.k0 + a.ksteps, ka + a.seg_steps) - ka;

    const __amdgpu_buffer_rsrc_t src = image_rsrc(c.src + img * c.src_img, c.src_img);
    const __amdgpu_buffer_rsrc_t prs = image_rsrc(a.plan, static_cast<long long>(a.plan_rows) * kRcolPlanRow);
    rc_cint *srow = (rc_cint *)(a.plan + static_cast<size_t>(a.plan_rows) * kRcolPlanRow);
    const __amdgpu_buffer_rsrc_t dst = image_rsrc(a.out + img * a.out_img, a.out_img);

    // ---- back-end horizontal operands (k_rcol's, COPY edge folded) ----
    rc_v4i th[UPW][NKS], tl[UPW][NKS];
    int kb[UPW];
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
        const int u = UPW * wave + i;
        int sf, pf;
        rc_pos(a.ox0 + min(x0 + (16 * u) / B, x_last), a.hs, a.hpad, &sf, &pf, a.centre);
        kb[i] = __builtin_amdgcn_readfirstlane((B * (sf - org) + (16 * u) % B) & ~7);
        const int o = 16 * u + n, xl = o / B, cc = o - B * xl;
        int sp, pp;
        rc_pos(a.ox0 + min(x0 + xl, x_last), a.hs, a.hpad, &sp, &pp, a.centre);
        const int lfold = -sp, rfold = sp + a.htaps - 1 - (a.w - 1);
        const signed char *rh =
            lfold > 0 ? a.tabhf + ((static_cast<size_t>(lfold - 1) * (kTransformScale + 1) + pp) * 2) * kRsTabW
            : rfold > 0 ? a.tabhf + ((static_cast<size_t>(a.htaps - 1 + rfold - 1) * (kTransformScale + 1) + pp) * 2) * kRsTabW
                        : a.tabh + static_cast<size_t>(pp) * 2 * kRsTabW;
        const bool both = lfold > 0 && rfold > 0;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const int j0 = kb[i] + 64 * ks + 16 * kg;
            if (both) {
                rc_edge_frag(a.tabf, a.htaps, pp, sp, cc, j0, org, a.w, B, &th[i][ks], &tl[i][ks]);
            } else {
                const int off = kRsTabPad + j0 - cc - B * (sp - org);
                th[i][ks] = rc_frag16(rh, off);
                tl[i][ks] = rc_frag16(rh + kRsTabW, off);
            }
        }
    }
    rc_v4i hb[UPW];
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
        const int e = 16 * (UPW * wave + i) + 4 * kg;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            int sp, pp;
            rc_pos(a.ox0 + min(x0 + (e + j) / B, x_last), a.hs, a.hpad, &sp, &pp, a.centre);
            hb[i][j] = 128 * a.sumh[pp] + 2048;
        }
    }
    // ---- front operands ----
    const rc_u4 *fo = c.fops + 4 * lane;
    const rc_v4i fvh = __builtin_bit_cast(rc_v4i, fo[0]), fvl = __builtin_bit_cast(rc_v4i, fo[1]);
    const rc_v4i fwh = __builtin_bit_cast(rc_v4i, fo[2]), fwl = __builtin_bit_cast(rc_v4i, fo[3]);
    const int vsd = c.vseed, hsd = c.hseed;

    // COPY edge of the front's input columns: front pixels [0, nl) copy pixel nl, [fr, ...) pixel fr - 1
    const int nl = vst < 0 ? -vst : 0;
    const int fr = c.sw - vst;
    const int fr_end = 2 * ni + 9;
    const int nr = fr_end >= fr ? fr_end - fr + 1 : 0;
    const bool fedge = nl > 0 || nr > 0;

    // ---- front step: 2 x 2-output rows P .. P + 14 into the ring ----
    auto front = [&](int P) {
        const int hh = a.h;  // rows of the 2 x 2 output
        if constexpr (FRONT == 0) {
        if (P < hh) {
            // vertical: wave-dealt 64-byte column tiles; 5 groups of 3 rows, 20 loads per lane in flight
            for (int tl_ = wave; tl_ < ntile; tl_ += WV) {
                const int cb = vb0 + 64 * tl_ + 4 * n;
                const bool cin = cb >= 0 && cb < spitch;
                uint32_t v[5][4];
#pragma unroll
                for (int g = 0; g < 5; ++g)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int r = 2 * (P + 3 * g) - 5 + 4 * kg + j;
                        v[g][j] = static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(
                            src, cin ? clampi(r, 0, c.sh - 1) * spitch + cb : 0x7ffffff0, 0, 0));
                    }
                const uint32_t fw = fint_l + static_cast<uint32_t>(kg * c.fis + 64 * tl_ + 4 * n + G::LOFF);
#pragma unroll
                for (int g = 0; g < 5; ++g) {
                    const rc_v4i bv = rc_v4i{static_cast<int>(v[g][0] ^ 0x80808080u), static_cast<int>(v[g][1] ^ 0x80808080u),
                                             static_cast<int>(v[g][2] ^ 0x80808080u), static_cast<int>(v[g][3] ^ 0x80808080u)};
                    rc_v4i dh = rc_v4i{0, 0, 0, 0}, dl = rc_v4i{vsd, vsd, vsd, vsd};
                    dh = __builtin_amdgcn_mfma_i32_16x16x64_i8(fvh, bv, dh, 0, 0, 0);
                    dl = __builtin_amdgcn_mfma_i32_16x16x64_i8(fvl, bv, dl, 0, 0, 0);
                    if (kg < 3)
                        lds_wr32(fw + static_cast<uint32_t>(3 * g * c.fis),
                                 rc_round4s((dh[0] << 6) + dl[0], (dh[1] << 6) + dl[1], (dh[2] << 6) + dl[2],
                                            (dh[3] << 6) + dl[3]));
                }
            }
            rc_barrier();
            if (fedge) {  // EXTEND_COPY of the input columns, per byte
                const int nfill = nl + nr;
                for (int i = tid; i < FR * nfill * B; i += kRcNT) {
                    const int u = i / (nfill * B);
                    const int rem = i - u * nfill * B;
                    const int f = rem / B, ch = rem - f * B;
                    const int d = f < nl ? f : fr + (f - nl);
                    const int sp = f < nl ? nl : fr - 1;
                    fint[u * c.fis + ish + B * d + ch] = fint[u * c.fis + ish + B * sp + ch];
                }
                rc_barrier();
            }
            // horizontal: groups of GP pixels, 4 groups' windows under one wait
            const uint32_t fb = fint_l + static_cast<uint32_t>(n * c.fis + (ish & ~7) + 16 * kg);
            const bool wrow = n < FR && 4 * kg < B * GP;
            const uint32_t rrow = ring_l + static_cast<uint32_t>(((P + n) & (kChRing - 1)) * a.rs + 4 * kg);
            for (int q0 = wave; q0 < ngr; q0 += 4 * WV) {
                rc_u2x2 bq[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) bq[i] = lds_rd64x2(fb + static_cast<uint32_t>(2 * B * GP * min(q0 + WV * i, ngr - 1)));
                lgkm_wait_for<0>(bq[0], bq[1], bq[2], bq[3]);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int q = q0 + WV * i;
                    const rc_v4i bv = __builtin_bit_cast(rc_v4i, rc_join(bq[i]));
                    rc_v4i dh = rc_v4i{0, 0, 0, 0}, dl = rc_v4i{hsd, hsd, hsd, hsd};
                    dh = __builtin_amdgcn_mfma_i32_16x16x64_i8(fwh, bv, dh, 0, 0, 0);
                    dl = __builtin_amdgcn_mfma_i32_16x16x64_i8(fwl, bv, dl, 0, 0, 0);
                    if (wrow && q < ngr)
                        lds_wr32(rrow + static_cast<uint32_t>(B * GP * q),
                                 rc_round4s((dh[0] << 6) + dl[0], (dh[1] << 6) + dl[1], (dh[2] << 6) + dl[2],
                                            (dh[3] << 6) + dl[3]));
                }
            }
        }
        // rows outside the 2 x 2 output: copies of its first / last row (COPY edge of the
        // second reduce's vertical pass)
        if (P < 0 || P + FR > hh) {
            rc_barrier();
            const int rb = a.rs;  // bytes per ring row copied (>= 16 cpr)
            for (int i = tid; i < FR * (rb >> 2); i += kRcNT) {
                const int u = i / (rb >> 2), d = i - u * (rb >> 2);
                const int R = P + u;
                if (R >= 0 && R < hh) continue;
                const int S = R < 0 ? 0 : hh - 1;
                reinterpret_cast<uint32_t *>(ring + (R & (kChRing - 1)) * a.rs)[d] =
                    reinterpret_cast<const uint32_t *>(ring + (S & (kChRing - 1)) * a.rs)[d];
            }
        }
        }
    };

    // ---- FRONT 1: VALU vertical (k_reduce2x2's register ring), matrix-core horizontal ----
    typedef float f4v_ __attribute__((ext_vector_type(4)));
    auto cvt4 = [](uint32_t v) { return f4v_{ubyte_once<0>(v), ubyte_once<1>(v), ubyte_once<2>(v), ubyte_once<3>(v)}; };
    auto tap7 = [&](float e, float m1, float p1, float m3, float p3, float m5, float p5) {
        float acc = __builtin_fmaf(c.c0, e, c.bias);
        acc = __builtin_fmaf(c.c1, m1 + p1, acc);
        acc = __builtin_fmaf(c.c3, m3 + p3, acc);
        return __builtin_fmaf(c.c5, m5 + p5, acc);
    };
    auto pack4 = [](float x, float y, float z, float w) {
        uint32_t v = __builtin_amdgcn_cvt_pk_u8_f32(x, 0, 0u);
        v = __builtin_amdgcn_cvt_pk_u8_f32(y, 1, v);
        v = __builtin_amdgcn_cvt_pk_u8_f32(z, 2, v);
        return __builtin_amdgcn_cvt_pk_u8_f32(w, 3, v);
    };
    const int ib = vb0 + 4 * tid;  // the lane's input dword (front intermediate dword tid)
    const int nd = (ish - G::LOFF + B * (2 * ni + 10) + 3) >> 2;
    const bool vlane = tid < nd;
    const uint32_t voff = vlane && ib >= 0 && ib + 4 <= spitch ? static_cast<uint32_t>(ib) : 0x80000000u;
    auto load_row = [&](int r) -> uint32_t {
        return static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(
            src, voff, __builtin_amdgcn_readfirstlane(clampi(r, 0, c.sh - 1) * spitch), 0));
    };
    f4v_ vring[6];
    uint32_t podd[12], pevn[12];
    auto front2_init = [&](int Q) {  // Q: a multiple of 12
        if constexpr (FRONT == 1) {
            vring[3] = cvt4(load_row(2 * (Q - 3) + 1));
            vring[4] = cvt4(load_row(2 * (Q - 2) + 1));
            vring[5] = cvt4(load_row(2 * (Q - 1) + 1));
            vring[0] = cvt4(load_row(2 * Q + 1));
            vring[1] = cvt4(load_row(2 * (Q + 1) + 1));
            vring[2] = f4v_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int u = 0; u < 12; ++u) {
                podd[u] = load_row(2 * (Q + u + 2) + 1);
                pevn[u] = load_row(2 * (Q + u));
            }
        }
    };
    auto front2 = [&](int Q) {
        const int hh = a.h;
        if constexpr (FRONT == 1) {
            const uint32_t fw = fint_l + static_cast<uint32_t>(G::LOFF + 4 * tid);
#pragma unroll
            for (int u = 0; u < 12; ++u) {
                vring[(u + 2) % 6] = cvt4(podd[u]);
                const f4v_ e = cvt4(pevn[u]);
                podd[u] = load_row(2 * (Q + 12 + u + 2) + 1);  // the next chunk's rows, in flight from here
                pevn[u] = load_row(2 * (Q + 12 + u));
                const f4v_ m5 = vring[(u + 3) % 6], m3 = vring[(u + 4) % 6], m1 = vring[(u + 5) % 6];
                const f4v_ p1 = vring[u % 6], p3 = vring[(u + 1) % 6], p5 = vring[(u + 2) % 6];
                const uint32_t d = pack4(tap7(e.x, m1.x, p1.x, m3.x, p3.x, m5.x, p5.x),
                                         tap7(e.y, m1.y, p1.y, m3.y, p3.y, m5.y, p5.y),
                                         tap7(e.z, m1.z, p1.z, m3.z, p3.z, m5.z, p5.z),
                                         tap7(e.w, m1.w, p1.w, m3.w, p3.w, m5.w, p5.w));
                if (vlane) lds_wr32(fw + static_cast<uint32_t>(u * c.fis), d ^ 0x80808080u);
            }
            rc_barrier();
            if (fedge) {  // EXTEND_COPY of the input columns, per byte
                const int nfill = nl + nr;
                for (int i = tid; i < FR * nfill * B; i += kRcNT) {
                    const int u = i / (nfill * B);
                    const int rem = i - u * nfill * B;
                    const int f = rem / B, ch = rem - f * B;
                    const int d = f < nl ? f : fr + (f - nl);
                    const int sp = f < nl ? nl : fr - 1;
                    fint[u * c.fis + ish + B * d + ch] = fint[u * c.fis + ish + B * sp + ch];
                }
                rc_barrier();
            }
            const uint32_t fb = fint_l + static_cast<uint32_t>(n * c.fis + (ish & ~7) + 16 * kg);
            const bool wrow = n < FR && 4 * kg < B * GP;
            const uint32_t rrow = ring_l + static_cast<uint32_t>(((Q + n) & (kChRing - 1)) * a.rs + 4 * kg);
            for (int q0 = wave; q0 < ngr; q0 += 4 * WV) {
                rc_u2x2 bq[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) bq[i] = lds_rd64x2(fb + static_cast<uint32_t>(2 * B * GP * min(q0 + WV * i, ngr - 1)));
                lgkm_wait_for<0>(bq[0], bq[1], bq[2], bq[3]);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const rc_v4i bv = __builtin_bit_cast(rc_v4i, rc_join(bq[i]));
                    const rc_v4i dh = __builtin_amdgcn_mfma_i32_16x16x64_i8(fwh, bv, rc_v4i{0, 0, 0, 0}, 0, 0, 0);
                    const rc_v4i dl = __builtin_amdgcn_mfma_i32_16x16x64_i8(fwl, bv, rc_v4i{hsd, hsd, hsd, hsd}, 0, 0, 0);
                    if (wrow && q0 + WV * i < ngr)
                        lds_wr32(rrow + static_cast<uint32_t>(B * GP * (q0 + WV * i)),
                                 rc_round4s((dh[0] << 6) + dl[0], (dh[1] << 6) + dl[1], (dh[2] << 6) + dl[2], (dh[3] << 6) + dl[3]));
                }
            }
            // rows outside the 2 x 2 output: those past its last row in this chunk, and with
            // the first chunk (chunks start at row 0, never above it) the up to 11 rows above row 0
            if (Q == 0 || Q + FR > hh) {
                rc_barrier();
                const int rb = a.rs, u0 = Q == 0 ? -11 : 0;
                for (int i = tid; i < (FR - u0) * (rb >> 2); i += kRcNT) {
                    const int u = u0 + i / (rb >> 2), d = i - (u - u0) * (rb >> 2);
                    const int R = Q + u;
                    if (R >= 0 && R < hh) continue;
                    const int S = R < 0 ? 0 : hh - 1;
                    reinterpret_cast<uint32_t *>(ring + (R & (kChRing - 1)) * a.rs)[d] =
                        reinterpret_cast<const uint32_t *>(ring + (S & (kChRing - 1)) * a.rs)[d];
                }
            }
        }
    };

    // ---- back end: k_rcol's vertical / horizontal / stores ----
    const int toff = n * kRcolPlanRow + 16 * kg;
    const int wrow_ = min(lane / UPW, kRcRows - 1), wch = lane - UPW * (lane / UPW);
    const int we = 16 * (UPW * wave + wch);
    const uint32_t wst_w = wst_l + static_cast<uint32_t>(wave * kRcRows * WSR);
    int P = srow[2 * ka];  // next ring row to produce
    if constexpr (FRONT == 1) {  // chunks on multiples of 12 (the register ring's slot map)
        P = P >= 0 ? P / 12 * 12 : 0;  // rows above row 0 are copies of it, filled with chunk 0
        front2_init(P);
    }
    for (int k = ka; k < ka + steps; ++k) {
        const int o = k * (kRcRows * kRcolPlanRow);
        const rc_v4i bh = __builtin_bit_cast(rc_v4i, __builtin_amdgcn_raw_buffer_load_b128(prs, toff + o, 0, 0));
        const rc_v4i bl = __builtin_bit_cast(rc_v4i, __builtin_amdgcn_raw_buffer_load_b128(prs, toff + o + 64, 0, 0));
        const int sd = __builtin_amdgcn_raw_buffer_load_b32(prs, n * kRcolPlanRow + 128 + o, 0, 0);
        const int bk = srow[2 * k], ek = srow[2 * k + 1];
        bool first = true;
        while (P < ek) {
            if (!first) rc_barrier();  // the front intermediate is free again
            if (FRONT == 1) front2(P);
            else front(P);
            P += FR;
            first = false;
        }
        rc_barrier();  // ring rows of step k complete; the back intermediate free
        {
            const int r1 = bk + 8 * kg + (n >> 1);
            const uint32_t a1 = ring_l + static_cast<uint32_t>((r1 & (kChRing - 1)) * a.rs + 8 * (n & 1));
            const uint32_t a2 = ring_l + static_cast<uint32_t>(((r1 + 32) & (kChRing - 1)) * a.rs + 8 * (n & 1));
            const uint32_t iq = inter_l + static_cast<uint32_t>(n * a.iw + 4 * kg);
            for (int ct = wave; ct < cpr; ct += 2 * WV) {
                const bool two = ct + WV < cpr;
                rc_v2i t1a = lds_tr8(a1 + 16 * ct), t2a = lds_tr8(a2 + 16 * ct);
                rc_v2i t1b = t1a, t2b = t2a;
                if (two) {
                    t1b = lds_tr8(a1 + 16 * (ct + WV));
                    t2b = lds_tr8(a2 + 16 * (ct + WV));
                }
                lgkm_wait_for<0>(t1a, t2a, t1b, t2b);
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    if (hh == 1 && !two) break;
                    const rc_v4i av = hh ? rc_v4i{t1b.x, t1b.y, t2b.x, t2b.y} : rc_v4i{t1a.x, t1a.y, t2a.x, t2a.y};
                    rc_v4i dh = rc_v4i{0, 0, 0, 0}, dl = rc_v4i{sd, sd, sd, sd};
                    dh = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bh, dh, 0, 0, 0);
                    dl = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bl, dl, 0, 0, 0);
                    lds_wr32(iq + 16 * (ct + WV * hh), rc_round4s((dh[0] << 6) + dl[0], (dh[1] << 6) + dl[1],
                                                                  (dh[2] << 6) + dl[2], (dh[3] << 6) + dl[3]));
                }
            }
        }
        rc_barrier();  // the intermediate complete
        uint32_t res[UPW];
        {
            rc_u2x2 q[UPW][NKS];
#pragma unroll
            for (int i = 0; i < UPW; ++i) {
                const uint32_t ir = inter_l + static_cast<uint32_t>(n * a.iw + kb[i] + 16 * kg);
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) q[i][ks] = lds_rd64x2(ir + 64 * ks);
            }
#pragma unroll
            for (int i = 0; i < UPW; ++i)
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) rc_pin(q[i][ks]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < UPW; ++i) {
                rc_v4i ah = rc_v4i{0, 0, 0, 0}, al = hb[i];
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) {
                    rc_pin(q[i][ks]);
                    const rc_v4i bz = __builtin_bit_cast(rc_v4i, rc_join(q[i][ks]));
                    ah = __builtin_amdgcn_mfma_i32_16x16x64_i8(th[i][ks], bz, ah, 0, 0, 0);
                    al = __builtin_amdgcn_mfma_i32_16x16x64_i8(tl[i][ks], bz, al, 0, 0, 0);
                }
                res[i] = rc_round4((ah[0] << 6) + al[0], (ah[1] << 6) + al[1], (ah[2] << 6) + al[2], (ah[3] << 6) + al[3]);
            }
        }
        // stores: the wave's 16 rows x 16 UPW bytes through its LDS tile, 16-byte row pieces
#pragma unroll
        for (int i = 0; i < UPW; ++i) lds_wr32(wst_w + static_cast<uint32_t>(n * WSR + 16 * i + 4 * kg), res[i]);
        rc_u4 qv;
        {
            rc_u2x2 qq = lds_rd64x2(wst_w + static_cast<uint32_t>(wrow_ * WSR + 16 * wch));
            lgkm_wait_for<0>(qq);
            qv = rc_join(qq);
        }
        const int orow = k * kRcRows + wrow_ - a.oy0;
        const bool ok = lane < 16 * UPW && orow >= 0 && orow < a.oh;
        const int base = orow * a.ow * B + B * x0 + we;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(rc_v4i, qv), dst, ok && we + 16 <= vbytes ? base : 0x7ffffff0, 0, 0);
        if (a.wst == 2) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_raw_buffer_store_b32(qv[j], dst, ok && we + 16 > vbytes && we + 4 * j < vbytes ? base + 4 * j : 0x7ffffff0, 0, 0);
        } else if (a.wst == 3 && B * x0 + 16 * UPW * WV >= a.ow * B) {
#pragma unroll
            for (int j = 0; j < 16; ++j)
                __builtin_amdgcn_raw_buffer_store_b8(static_cast<u8>(qv[j >> 2] >> (8 * (j & 3))), dst,
                                                     ok && we + 16 > vbytes && we + j < vbytes ? base + j : 0x7ffffff0, 0, 0);
        }
    }
}

}  // namespace

// The column walker for both shrinks in (1, ~2.5] (<= 16 taps) on 3- / 4-band images
// whose input rows start on a dword; MIPX_EUNSUPPORTED otherwise (the caller runs
// another kernel).  Output window [ox0, ox0 + ow) x [oy0, oy0 + oh).
int reduce_col_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double hs, double vs, int ox0, int oy0,
                      int ow, int oh, hipStream_t st) {
    if ((b != 3 && b != 4) || !(hs > 1.0) || !(vs > 1.0)) return MIPX_EUNSUPPORTED;
    const long long in_img = img_bytes(w, h, b), out_img = img_bytes(ow, oh, b);
    // out-of-range store offsets are built from 2^29 and 2^31 (k_rcol store)
    if (in_img >= 0x7fffffffLL || out_img >= (1LL << 29)) return MIPX_EUNSUPPORTED;
    // input rows off a dword: the realigning build (RGB only; MIPX_RCOL_UNAL=0 keeps them
    // on k_rmf2, A/B)
    const bool unal = (w * b) % 4 != 0 || reinterpret_cast<uintptr_t>(in) % 4 != 0;
    const char *eun = tune_env("MIPX_RCOL_UNAL");
    if (unal && (b != 3 || (eun && *eun == '0') || in_img >= 0x7fffff00LL)) return MIPX_EUNSUPPORTED;
    // output rows off a dword go out as unaligned 16-byte pieces (wst 3); with the 4-byte
    // stores (MIPX_RCOL_WST=0) they stay on k_rmf2
    const bool out_al = (ow * b) % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 4 == 0;
    const char *ews0 = tune_env("MIPX_RCOL_WST");
    if (!out_al && ews0 && *ews0 == '0') return MIPX_EUNSUPPORTED;
    const int vtaps = reduce_points(vs), htaps = reduce_points(hs);
    if (vtaps > 16 || htaps > 16) return MIPX_EUNSUPPORTED;
    const bool centre = reduce_centre();
    const int vpad = vtaps / 2 - 1;
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
    a.htaps = htaps;
    a.hpad = htaps / 2 - 1;
    a.hs = hs;
    a.centre = centre;
    a.k0 = oy0 / kRcRows;
    const int k1 = (oy0 + oh - 1) / kRcRows;  // last group
    a.ksteps = k1 - a.k0 + 1;
    // the plan's group rows (host copy of the same formula)
    auto gb = [&](int k) { return rc_start(kRcRows * k, vs, vpad, centre); };
    auto ge = [&](int k) { return rc_start(kRcRows * k + kRcRows - 1, vs, vpad, centre) + vtaps; };
    int lmax = 0, maxnew = 0;
    for (int k = a.k0; k <= k1; ++k) {
        lmax = std::max(lmax, ge(k) - gb(k));
        if (k > a.k0) maxnew = std::max(maxnew, ge(k) - ge(k - 1));
    }
    if (lmax > 64) return MIPX_EUNSUPPORTED;  // the MFMA K

    // strip geometry: staged chunks per row, K steps of the horizontal units (8-byte K
    // origins, and 4-byte ones: k4 when that saves a K step, e.g. RGB / 1.667, C5's
    // 1333x1000 -> 800x600; MIPX_RCOL_K4=0 keeps 8, A/B)
    int cpr_min = 1 << 30, cpr_max = 0, nks = 0, kbmax = 0, nks4 = 0, kbmax4 = 0;
    for (int x0 = 0; x0 < ow; x0 += 64) {
        const int xl = std::min(x0 + 63, ow - 1);
        const int lo = rc_start(ox0 + x0, hs, a.hpad, centre), hi = rc_start(ox0 + xl, hs, a.hpad, centre) + htaps - 1;
        const int org = lo & (lo < 0 && b == 3 ? ~15 : ~3);  // as k_rcol
        const int cpr = (b * (hi - org + 1) + 15) >> 4;
        cpr_min = std::min(cpr_min, cpr);
        cpr_max = std::max(cpr_max, cpr);
        for (int u = 0; u < 64 * b / 16; ++u) {
            const int o0 = 16 * u, o1 = 16 * u + 15;
            if (x0 + o0 / b > xl) break;
            const int xf = x0 + o0 / b, xe = std::min(x0 + o1 / b, xl);
            const int kb0 = b * (rc_start(ox0 + xf, hs, a.hpad, centre) - org) + o0 % b;
            const int kbu = kb0 & ~7, kbu4 = kb0 & ~3;
            const int need = b * (rc_start(ox0 + xe, hs, a.hpad, centre) + htaps - 1 - org) + b;
            nks = std::max(nks, (need - kbu + 63) / 64);
            kbmax = std::max(kbmax, kbu);
            nks4 = std::max(nks4, (need - kbu4 + 63) / 64);
            kbmax4 = std::max(kbmax4, kbu4);
        }
    }
    const char *ek4 = tune_env("MIPX_RCOL_K4");
    a.k4 = nks4 < nks && !(ek4 && *ek4 == '0');
    const char *eas = tune_env("MIPX_RCOL_ALLST");
    a.allst = eas && *eas == '1';
    // r05: a wave issues no ring load batch whose lanes all idle (MIPX_RCOL_SKIPL=0: every
    // batch, out-of-range offsets; 500x375 +3 %, 1080p / 1.6 and / 2.4 +2 %,
    // profiles/r05/small/rcol_skipl_ab.jsonl)
    const char *esl = tune_env("MIPX_RCOL_SKIPL");
    a.skipl = !(esl && *esl == '0');
    if (a.k4) {
        nks = nks4;
        kbmax = kbmax4;
    }
    if (nks > 2) return MIPX_EUNSUPPORTED;
    // chunks per lane: the widest strip's rows of the largest step fit one batch; ring:
    // the rows of a step, and a batch's rows (at most the rows one step adds) must only
    // land on slots of rows above the step's first
    int kmax = 0, ring = 0;
    const int rcap = std::max(maxnew, 1);
    for (int km : {3, 6}) {
        if ((kRcNT * km) / cpr_max < rcap) continue;
        const int reach = std::min((kRcNT * km + cpr_min - 1) / cpr_min, rcap);
        for (int r : {32, 64}) {
            bool ok = lmax <= r;
            for (int k = a.k0 + 1; ok && k <= k1; ++k) ok = ge(k - 1) + reach <= gb(k) + r;
            if (ok) { ring = r; break; }
        }
        if (ring) { kmax = km; break; }
    }
    if (!kmax) return MIPX_EUNSUPPORTED;
    a.rmask = ring - 1;
    a.rcap = rcap;
    int rs = 4 * cpr_max;  // dwords
    while (((rs & 63) >> 2) % 2 == 0) rs += 4;  // 16 consecutive rows on distinct bank quads
    a.rs = 4 * rs;
    int iw = (std::max(16 * cpr_max, kbmax + 64 * nks) + 16 + 15) & ~15;
    while ((iw / 4) % 8 != 4) iw += 16;  // 4 mod 8 dwords: the intermediate writes hit distinct banks
    a.iw = iw;
    // + the wave store tiles (4 x 16 rows x (16 B + 16 for RGBA))
    const size_t lds = static_cast<size_t>(ring) * a.rs + static_cast<size_t>(kRcRows) * iw +
                       static_cast<size_t>(4 * kRcRows * (16 * b + (b == 4 ? 16 : 0)));
    if (lds > 64 * 1024) return MIPX_EUNSUPPORTED;

    int plan_rows = 0;
    a.plan = device_rcol_vplan(vs, centre, kRcRows * (k1 + 3), &plan_rows);
    a.plan_rows = plan_rows;
    int nth = 0, ntf = 0, nfh = 0;
    const int *sumh = nullptr;
    if (!a.plan || !device_reduce_i8(hs, &nth, &sumh)) return MIPX_EDEVICE;
    a.sumh = sumh;
    a.tabh = device_reduce_i8s(hs, b, &nth);
    a.tabf = device_reduce_table(hs, &ntf);
    a.tabhf = device_reduce_i8s_fold(hs, b, &nfh);
    if (!a.tabh || !a.tabf || !a.tabhf || nth != htaps || ntf != htaps || nfh != htaps) return MIPX_EDEVICE;

    // r03: 16-byte row pieces through a wave tile (1080p RGB / 1.6 -16 %, 1024^2 RGBA / 1.333
    // -31 %, profiles/r03/rcol_wst_ab.jsonl); MIPX_RCOL_WST=0 keeps the 4-byte stores (A/B)
    const char *ews = tune_env("MIPX_RCOL_WST");
    a.wst = !(ews && *ews == '0') ? (!out_al ? 3 : (ow * b) % 16 == 0 ? 1 : 2) : 0;
    const char *esz = tune_env("MIPX_RCOL_SWZ");
    a.swz = !(esz && *esz == '0');
    const void *fn = nullptr;
#define MIPX_RC_K(B_, NKS_, KM_)                                                                  \
    fn = unal ? reinterpret_cast<const void *>(&k_rcol<3, NKS_, KM_, 1, true>)                     \
              : reinterpret_cast<const void *>(&k_rcol<B_, NKS_, KM_, 1>);
#define MIPX_RC_KM(B_, NKS_) \
    if (kmax == 3) { MIPX_RC_K(B_, NKS_, 3) } else { MIPX_RC_K(B_, NKS_, 6) }
    if (b == 3) {
        if (nks == 1) { MIPX_RC_KM(3, 1) } else { MIPX_RC_KM(3, 2) }
    } else {
        if (nks == 1) { MIPX_RC_KM(4, 1) } else { MIPX_RC_KM(4, 2) }
    }
#undef MIPX_RC_KM
#undef MIPX_RC_K

    // segments: a block's set-up (operand loads, the first group's rows) costs about two
    // steps; pick the split that minimises (rounds of resident blocks) x (steps + 2)
    a.strips = (ow + 63) / 64;
    const long long cols = static_cast<long long>(a.strips) * n;
    auto plan = [&](const void *f, int *segs_out) {
        const long long slots = static_cast<long long>(device_cu_count()) * occupancy_per_cu(f, kRcNT, lds, 2);
        double best = 1e300;
        int rounds = 0;
        for (int segs = 1; segs <= a.ksteps; ++segs) {
            const int ss = (a.ksteps + segs - 1) / segs;
            if (segs > 1 && ss < 4) break;
            const long long blocks = cols * ((a.ksteps + ss - 1) / ss);
            const long long r = (blocks + slots - 1) / slots;
            const double cost = static_cast<double>(r) * (ss + 2);
            if (cost < best - 1e-9) {
                best = cost;
                *segs_out = segs;
                rounds = static_cast<int>(r);
            }
        }
        return std::make_pair(best, rounds);
    };
    int best_segs = 1;
    const double best = plan(fn, &best_segs).first;
    // <3, 1, 3> also has a 4-waves-per-SIMD build (128 VGPRs, 2 spilled): it wins only when
    // the whole launch then fits one round of resident blocks in fewer steps per block
    // (364x273 RGB x 128 -> 256^2: -18 %); with more rounds the spills cost 3-5 %
    // (480x270, 500x375, 1080p; profiles/r04/small/rcol_w4_ab.jsonl)
    // MIPX_RCOL_W4=1 (A/B): the 4-wave build whatever the plan says (RGBA too)
    const char *ew4 = tune_env("MIPX_RCOL_W4");
    const bool force4 = ew4 && *ew4 == '1';
    if (nks == 1 && kmax == 3 && !unal && (b == 3 || force4)) {
        const void *f4 = b == 3 ? reinterpret_cast<const void *>(&k_rcol<3, 1, 3, 4>)
                                : reinterpret_cast<const void *>(&k_rcol<4, 1, 3, 4>);
        int segs4 = 1;
        const auto p4 = plan(f4, &segs4);
        if (force4 || (p4.second == 1 && p4.first < best - 1e-9)) {
            fn = f4;
            best_segs = segs4;
        }
    }
    a.seg_steps = (a.ksteps + best_segs - 1) / best_segs;
    a.segs = (a.ksteps + a.seg_steps - 1) / a.seg_steps;
    const long long blocks = cols * a.segs;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    hipLaunchKernelGGL(reinterpret_cast<void (*)(RcArgs)>(const_cast<void *>(fn)), dim3(static_cast<unsigned>(blocks)),
                       dim3(kRcNT), lds, st, a);
    return launch_check("k_rcol");
}

// vips_reduce(2, 2) then vips_reduce(hs, vs) over output window [ox0, ox0 + ow) x [oy0,
// oy0 + oh) of the second, in one launch (k_rchain); MIPX_EUNSUPPORTED when the pair is
// outside the fused kernel's envelope (the caller runs the two reduces).  taps12: the 2 x 2
// reduce's 12 taps from 2x - 5 at the convention's phase (reduce2_front_taps).
int reduce2_chain_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double hs, double vs, int ox0, int oy0,
                         int ow, int oh, const int *taps12, hipStream_t st) {
    if ((b != 3 && b != 4) || !(hs > 1.0) || !(vs > 1.0)) return MIPX_EUNSUPPORTED;
    // MIPX_CHAIN=1 / 2 (tests: 2 = the chained kernel or an error); unset or 0: the two
    // reduces.  Off by default: on C3 the chain measures 3.90 ms per step against 2.43 ms
    // for k_reduce2x2 + k_rcol (profiles/r05/c3_chain_ab.jsonl)
    const char *ech = tune_env("MIPX_CHAIN");
    if (!(ech && (*ech == '1' || *ech == '2'))) return MIPX_EUNSUPPORTED;
    const int w2 = out_size_reduce(w, 2.0), h2 = out_size_reduce(h, 2.0);
    const long long src_img = img_bytes(w, h, b), out_img = img_bytes(ow, oh, b);
    if (src_img >= 0x7fffffffLL - 64 || out_img >= (1LL << 29)) return MIPX_EUNSUPPORTED;
    if ((w * b) % 4 != 0 || reinterpret_cast<uintptr_t>(in) % 4 != 0) return MIPX_EUNSUPPORTED;
    const bool out_al = (ow * b) % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 4 == 0;
    const int vtaps = reduce_points(vs), htaps = reduce_points(hs);
    if (vtaps > 16 || htaps > 16) return MIPX_EUNSUPPORTED;
    const bool centre = reduce_centre();
    const int vpad = vtaps / 2 - 1;
    RcArgs a{};
    a.in = nullptr;
    a.out = out;
    a.w = w2;
    a.h = h2;
    a.ox0 = ox0;
    a.oy0 = oy0;
    a.ow = ow;
    a.oh = oh;
    a.in_img = img_bytes(w2, h2, b);
    a.out_img = out_img;
    a.htaps = htaps;
    a.hpad = htaps / 2 - 1;
    a.hs = hs;
    a.centre = centre;
    a.k0 = oy0 / kRcRows;
    const int k1 = (oy0 + oh - 1) / kRcRows;
    a.ksteps = k1 - a.k0 + 1;
    auto gb = [&](int k) { return rc_start(kRcRows * k, vs, vpad, centre); };
    auto ge = [&](int k) { return rc_start(kRcRows * k + kRcRows - 1, vs, vpad, centre) + vtaps; };
    // the front: FRONT 1 (VALU vertical, corner convention only) unless forced
    // (MIPX_CHAIN_FRONT=0 / 1, A/B); FRONT 0 for the centre convention
    const char *efr = tune_env("MIPX_CHAIN_FRONT");
    int front = (efr && *efr) ? (*efr == '1' && !centre ? 1 : 0) : (centre ? 0 : 1);
    // FRONT 1 holds a strip's input row in one dword per lane: wider strips (shrinks past
    // ~1.55 on RGBA) take FRONT 0
    for (int x0 = 0; front && x0 < ow; x0 += 64) {
        const int xl = std::min(x0 + 63, ow - 1);
        const int lo = rc_start(ox0 + x0, hs, a.hpad, centre), hi = rc_start(ox0 + xl, hs, a.hpad, centre) + htaps - 1;
        const int org = lo & (lo < 0 && b == 3 ? ~15 : ~3);
        const int cpr = (b * (hi - org + 1) + 15) >> 4;
        const int gpf = b == 3 ? RCH<3>::GP : RCH<4>::GP;
        const int ni = (((16 * cpr + b - 1) / b + gpf - 1) / gpf) * gpf;
        const int vst = 2 * org - 5, ish = b * vst - ((b * vst) & ~63);  // (LOFF cancels)
        if ((ish + b * (2 * ni + 10) + 3) / 4 > kRcNT) front = 0;
    }
    const int fr = front ? 12 : kChFR, falign = front ? 11 : 0;
    for (int k = a.k0; k <= k1; ++k) {
        if (ge(k) - gb(k) > 64) return MIPX_EUNSUPPORTED;  // the MFMA K
        // the ring holds the step's rows plus one front step past its end (and, FRONT 1, the
        // rows a 12-aligned chunk makes above the step's first)
        if (ge(k) + fr - 1 + falign - gb(k) > kChRing) return MIPX_EUNSUPPORTED;
    }
    int cpr_max = 0, nks = 0, kbmax = 0, fbytes_max = 0, ni_max = 0;
    const int gp = b == 3 ? RCH<3>::GP : RCH<4>::GP;
    for (int x0 = 0; x0 < ow; x0 += 64) {
        const int xl = std::min(x0 + 63, ow - 1);
        const int lo = rc_start(ox0 + x0, hs, a.hpad, centre), hi = rc_start(ox0 + xl, hs, a.hpad, centre) + htaps - 1;
        const int org = lo & (lo < 0 && b == 3 ? ~15 : ~3);
        const int cpr = (b * (hi - org + 1) + 15) >> 4;
        cpr_max = std::max(cpr_max, cpr);
        const int ni = (((16 * cpr + b - 1) / b + gp - 1) / gp) * gp;
        ni_max = std::max(ni_max, ni);
        const int loff = b == 3 ? RCH<3>::LOFF : RCH<4>::LOFF;
        const int vst = 2 * org - 5, vb0 = (b * vst) & ~63, ish = b * vst - vb0 + loff;
        if ((ish & 7) != (b == 3 ? RCH<3>::SH : RCH<4>::SH)) return MIPX_EINVAL;  // the operand's window shift
        const int ntile = (ish - loff + b * (2 * ni + 10) + 63) >> 6;
        fbytes_max = std::max({fbytes_max, 64 * ntile + loff, (ish & ~7) + 2 * b * gp * (ni / gp - 1) + 64});
        for (int u = 0; u < 64 * b / 16; ++u) {
            const int o0 = 16 * u, o1 = 16 * u + 15;
            if (x0 + o0 / b > xl) break;
            const int xf = x0 + o0 / b, xe = std::min(x0 + o1 / b, xl);
            const int kbu = (b * (rc_start(ox0 + xf, hs, a.hpad, centre) - org) + o0 % b) & ~7;
            const int need = b * (rc_start(ox0 + xe, hs, a.hpad, centre) + htaps - 1 - org) + b;
            nks = std::max(nks, (need - kbu + 63) / 64);
            kbmax = std::max(kbmax, kbu);
        }
    }
    if (nks > 2) return MIPX_EUNSUPPORTED;
    // dwords, a multiple of 4 (the transposed reads need 8-byte rows; the vertical tiles are 16
    // bytes): the column tiles and every pixel the front writes
    int rs = 4 * std::max(cpr_max, (b * ni_max + 15) / 16);
    while (((rs & 63) >> 2) % 2 == 0) rs += 4;
    a.rs = 4 * rs;
    int iw = (std::max(16 * cpr_max, kbmax + 64 * nks) + 16 + 15) & ~15;
    while ((iw / 4) % 8 != 4) iw += 16;
    a.iw = iw;
    int fis = (fbytes_max + 15) & ~15;
    while ((fis / 4) % 32 % 4 != 2) fis += 8;  // 16 rows x 2 dwords of a half-wave's writes on distinct banks (k_reduce2m)
    RchArgs c{};
    c.src = in;
    c.sw = w;
    c.sh = h;
    c.src_img = src_img;
    c.fis = fis;
    const size_t lds = static_cast<size_t>(kChRing) * a.rs + static_cast<size_t>(kRcRows) * iw +
                       static_cast<size_t>(4 * kRcRows * (16 * b + (b == 4 ? 16 : 0))) +
                       static_cast<size_t>(kChFRows) * fis;
    if (lds > 64 * 1024) return MIPX_EUNSUPPORTED;

    int plan_rows = 0;
    a.plan = device_rcol_vplan(vs, centre, kRcRows * (k1 + 3), &plan_rows);
    a.plan_rows = plan_rows;
    int nth = 0, ntf = 0, nfh = 0;
    const int *sumh = nullptr;
    if (!a.plan || !device_reduce_i8(hs, &nth, &sumh)) return MIPX_EDEVICE;
    a.sumh = sumh;
    a.tabh = device_reduce_i8s(hs, b, &nth);
    a.tabf = device_reduce_table(hs, &ntf);
    a.tabhf = device_reduce_i8s_fold(hs, b, &nfh);
    if (!a.tabh || !a.tabf || !a.tabhf || nth != htaps || ntf != htaps || nfh != htaps) return MIPX_EDEVICE;
    a.wst = !out_al ? 3 : (ow * b) % 16 == 0 ? 1 : 2;
    int sum = 0;
    for (int i = 0; i < 12; ++i) {
        sum += taps12[i];
        if (taps12[i] < -128 * 64 || taps12[i] > 127 * 64 + 63) return MIPX_EUNSUPPORTED;
    }
    const std::vector<uint32_t> ops = b == 3 ? rch_operands<3>(taps12) : rch_operands<4>(taps12);
    c.fops = static_cast<const rc_u4 *>(device_blob(ops.data(), ops.size() * sizeof(uint32_t)));
    if (!c.fops) return MIPX_EDEVICE;
    c.vseed = c.hseed = 128 * sum + 2048 - (128 << 12);

    if (front) {
        float cc[4];
        if (!reduce2_taps(cc)) return MIPX_EUNSUPPORTED;
        c.c0 = cc[0] / 4096.0f, c.c1 = cc[1] / 4096.0f, c.c3 = cc[2] / 4096.0f, c.c5 = cc[3] / 4096.0f;
        c.bias = 1.0f / 8192.0f;
    }
    const void *fn = nullptr;
    const char *ew3 = tune_env("MIPX_CHAIN_W3");
    const bool w3 = !(ew3 && *ew3 == '0');
#define MIPX_RCH(B_, NKS_)                                                                                     \
    fn = front ? (w3 ? reinterpret_cast<const void *>(&k_rchain<B_, NKS_, 1, 1>)                              \
                     : reinterpret_cast<const void *>(&k_rchain<B_, NKS_, 1, 0>))                             \
               : reinterpret_cast<const void *>(&k_rchain<B_, NKS_, 0, 0>);
    if (b == 3) {
        if (nks == 1) { MIPX_RCH(3, 1) } else { MIPX_RCH(3, 2) }
    } else {
        if (nks == 1) { MIPX_RCH(4, 1) } else { MIPX_RCH(4, 2) }
    }
#undef MIPX_RCH
    // segments: one per strip unless the grid would not fill the device (a segment's first
    // front steps re-make the rows above its first step)
    a.strips = (ow + 63) / 64;
    const long long cols = static_cast<long long>(a.strips) * n;
    const long long slots = static_cast<long long>(device_cu_count()) * occupancy_per_cu(fn, kRcNT, lds, 2);
    const char *esg = tune_env("MIPX_CHAIN_SEGS");
    int segs = 1;
    if (esg && *esg) segs = std::max(1, std::atoi(esg));
    else
        while (cols * segs < 2 * slots && a.ksteps / (segs + 1) >= 8) ++segs;
    a.seg_steps = (a.ksteps + segs - 1) / segs;
    a.segs = (a.ksteps + a.seg_steps - 1) / a.seg_steps;
    const long long blocks = cols * a.segs;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    hipLaunchKernelGGL(reinterpret_cast<void (*)(RcArgs, RchArgs)>(const_cast<void *>(fn)),
                       dim3(static_cast<unsigned>(blocks)), dim3(kRcNT), lds, st, a, c);
    return launch_check("k_rchain");
}

}  // namespace mipx
