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
#include <type_traits>
#include <utility>
#include <vector>

#include "device_common.h"
#include "lds_ops.h"

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
    int trl;                  // RGBA store tile read back by tile_rd_lane (r06)
    int dbg;                  // MIPX_RCOL_DBG (PROBES builds only): 1 = set-up and prime, no steps; 2 = a third
                              // barrier + the horizontal pass twice, 3 = the vertical pass twice, 4 = both;
                              // 8 = per-step phase stamps (s_memtime) into stamps
    unsigned long long *stamps;  // PROBES, dbg 8: [block][8 + 8 seg_steps]
    const u8 *hops;           // r06, specialised builds: device_rcol_hops records [strip][unit][lane]
    const int *hkb;           // and the K origins [strip][unit]
};
#ifdef MIPX_PROBES
__device__ __forceinline__ int rc_dbg(const RcArgs &a) { return a.dbg; }
#else
__device__ __forceinline__ int rc_dbg(const RcArgs &) { return 0; }
#endif

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
// WSTC / K4C (r06): the store mode and the K-origin width fixed at compile time (0 / -1: read
// from the arguments), so the step carries only the one store path and operand read it runs
template <int B, int NKS, int KMAX, int WPE, bool UNAL = false, int WSTC = 0, int K4C = -1>
__global__ void __launch_bounds__(kRcNT) __attribute__((amdgpu_waves_per_eu(WPE, 8))) k_rcol(RcArgs a) {
    const int wst = WSTC ? WSTC : a.wst, k4 = K4C >= 0 ? K4C : a.k4;
    // the specialised builds run only with the default A/B switches (the launcher checks)
    constexpr bool SPEC = WSTC != 0;
    const bool skipl = SPEC || a.skipl, trl = SPEC || a.trl, swz = SPEC || a.swz, allst = !SPEC && a.allst;
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
    // PROBES, dbg 8: wave 0 lane 0 stamps the block's start / end and each step's phases
    unsigned long long *stp = nullptr;
    if (rc_dbg(a) == 8 && tid == 0) stp = a.stamps + static_cast<size_t>(blockIdx.x) * (8 + 8 * a.seg_steps);
    auto stamp = [&](int slot) {
        if (rc_dbg(a) == 8 && stp) stp[slot] = __builtin_amdgcn_s_memtime();
    };
    stamp(0);

    // ---- per-segment set-up: horizontal operands (registers, COPY edge folded) ----
    // every operand load issued before the first is used (one memory round trip)
    rc_v4i th[UPW][NKS], tl[UPW][NKS];
    uint4 qh[UPW][NKS], ql[UPW][NKS];
    uint32_t eh[UPW][NKS], el[UPW][NKS];
    int qsh[UPW][NKS];
    bool both[UPW];
    int kb[UPW];
    rc_v4i hb[UPW];
    // r06: the specialised builds load the host-built operands and seeds (device_rcol_hops):
    // three 16-byte loads per unit instead of the positions, table rows and edge folds
    constexpr bool HOPS = SPEC;
    if constexpr (HOPS) {
        typedef const __attribute__((address_space(4))) int rc_ckb;
#pragma unroll
        for (int i = 0; i < UPW; ++i) {
            const int u = UPW * wave + i;
            const u8 *rec = a.hops + (static_cast<size_t>(strip * 4 * UPW + u) * 64 + lane) * kRcolHopRec(NKS);
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                th[i][ks] = *reinterpret_cast<const rc_v4i *>(rec + 32 * ks);
                tl[i][ks] = *reinterpret_cast<const rc_v4i *>(rec + 32 * ks + 16);
            }
            hb[i] = *reinterpret_cast<const rc_v4i *>(rec + 32 * NKS);
            kb[i] = ((rc_ckb *)a.hkb)[strip * 4 * UPW + u];
            both[i] = true;  // (operands final: no realignment below)
        }
    }
#pragma unroll
    for (int i = 0; i < UPW && !HOPS; ++i) {
        const int u = wst ? UPW * wave + i : wave + WV * i;
        int sf, pf;
        rc_pos(a.ox0 + min(x0 + (16 * u) / B, x_last), a.hs, a.hpad, &sf, &pf, a.centre);
        // K origin: 8-byte aligned (ds_read_b64), 4-byte with k4
        kb[i] = __builtin_amdgcn_readfirstlane((B * (sf - org) + (16 * u) % B) & (k4 ? ~3 : ~7));
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
    stamp(2);
    // per output byte seeds of the horizontal pass (lane: bytes 16 u + 4 kg + j of row n)
    // and store offsets (past the strip's last byte: beyond any image, so dropped)
    uint32_t sto[UPW];
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
        const int e = 16 * (wst ? UPW * wave + i : wave + WV * i) + 4 * kg;
        if constexpr (!HOPS) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                int sp, pp;
                rc_pos(a.ox0 + min(x0 + (e + j) / B, x_last), a.hs, a.hpad, &sp, &pp, a.centre);
                hb[i][j] = 128 * a.sumh[pp] + 2048;
            }
        }
        sto[i] = e < vbytes ? static_cast<uint32_t>(B * x0 + e) : 0x20000000u;
    }

    stamp(3);
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
    for (int j = 0; j < KMAX; ++j) wl[j] = !skipl || __builtin_amdgcn_ballot_w64(rr[j] < a.rcap) != 0;

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
            // idle lanes: out of range for both loads, and (off & ~3) + 16 stays below 2^31
            const int off = rr[j] < a.rcap ? chunk_off(r0, j) : 0x7fffffe0;
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
    int wrow = min(lane / UPW, kRcRows - 1), wch = lane - UPW * (lane / UPW);  // read-back: row, 16-byte chunk
    // r06: RGBA (4 chunks a row, rows 80 bytes apart) reads back by tile_rd_lane: each
    // ds_read_b128 lane group on disjoint banks (MIPX_RCOL_TRL=0: lane / 4, A/B)
    if (UPW == 4 && trl) tile_rd_lane(lane, &wrow, &wch);
    const int we = 16 * (UPW * wave + wch);                          // its first byte in the strip row
    auto store = [&](int k, bool live, const uint32_t *res) {
        if (wst) {
#pragma unroll
            for (int i = 0; i < UPW; ++i) lds_wr32(wst_l + static_cast<uint32_t>(n * WSR + 16 * i + 4 * kg), res[i]);
            rc_u4 q = lds_rd128(wst_l + static_cast<uint32_t>(wrow * WSR + 16 * wch));
            lgkm_wait_for<0>(q);
            const int o = k * kRcRows + wrow - a.oy0;
            const bool ok = live && lane < 16 * UPW && o >= 0 && o < a.oh;
            const int base = o * a.ow * B + B * x0 + we;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(rc_v4i, q), dst,
                                                   ok && we + 16 <= vbytes ? base : 0x7ffffff0, 0, 0);
            if (wst == 2 && (vbytes < 16 * UPW * WV || allst)) {
                // rows whose byte count is not a multiple of 16: the piece at the image edge in
                // dwords, in the last strip only (uniform: r05, the dword stores every other
                // strip issued with out-of-range offsets were 4 of every 5 store instructions)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    __builtin_amdgcn_raw_buffer_store_b32(
                        q[j], dst, ok && we + 16 > vbytes && we + 4 * j < vbytes ? base + 4 * j : 0x7ffffff0, 0, 0);
            } else if (wst == 3 && B * x0 + 16 * UPW * WV >= a.ow * B) {
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
    const int hsw = swz && (kg & 1) ? 8 : 0, hsd = 8 - 2 * hsw;
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
                if (k4) {
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
        const int sb = 8 + 8 * (k - ka);  // stamp slots of this step (dbg 8)
#pragma unroll
        for (int i = 0; i < UPW; ++i) res[i] = 0u;
        if (live) {
            stamp(sb);
            if (!first) write_ring(pc, srow[2 * (k - 1) + 1]);
            stamp(sb + 1);
            rc_barrier();
            stamp(sb + 2);
            vertical(pc, srow[2 * k]);
            stamp(sb + 3);
            if (rc_dbg(a) == 3 || rc_dbg(a) == 4) vertical(pc, srow[2 * k]);  // probe: the vertical pass twice (same result)
        }
        issue_ring(pc, srow[2 * (k + 1) + 1]);
        issue_taps(pc, k + 2);
        if (live) {
            stamp(sb + 4);
            rc_barrier();
            stamp(sb + 5);
            horizontal(res);
            stamp(sb + 6);
            if (rc_dbg(a) == 2 || rc_dbg(a) == 4) {  // probe: a third barrier and the horizontal pass twice (wrong pixels)
                uint32_t r2[UPW];
                rc_barrier();
                horizontal(r2);
#pragma unroll
                for (int i = 0; i < UPW; ++i) res[i] += r2[i];
            }
        }
        store(k, live, res);
        if (live) stamp(sb + 7);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    const uint32_t zero[UPW] = {};
    // ---- prime: group ka's rows straight into the ring (exact rows only), then the
    // pipeline's first loads (r05: issuing those before the prime's ring writes measured
    // within +-1 %, and the extra live registers spilled in the 4-wave build,
    // profiles/r05/prime_ab.jsonl) ----
    stamp(4);
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
    stamp(5);
    issue_taps(I0{}, ka);
    store(ka, false, zero);  // idle: keeps the load / store sequence the loop's
    issue_ring(I1{}, eka);
    issue_taps(I1{}, ka + 1);
    store(ka, false, zero);
    stamp(6);
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
    if (hsw && !HOPS) {  // the K halves of odd blocks, in the order their data is read (the host did it for HOPS)
#pragma unroll
        for (int i = 0; i < UPW; ++i)
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                th[i][ks] = rc_v4i{th[i][ks][2], th[i][ks][3], th[i][ks][0], th[i][ks][1]};
                tl[i][ks] = rc_v4i{tl[i][ks][2], tl[i][ks][3], tl[i][ks][0], tl[i][ks][1]};
            }
    }
    if (rc_dbg(a) == 1) {  // timing probe: the set-up alone (kept live by a store no image reaches)
        if (a.ow < 0) {
            uint32_t v = 0;
#pragma unroll
            for (int i = 0; i < UPW; ++i)
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) v ^= th[i][ks][0] ^ tl[i][ks][3] ^ hb[i][1];
            __builtin_amdgcn_raw_buffer_store_b32(v ^ rv[0][0].x ^ rv[1][0].y ^ vh[0][0] ^ vl[1][1], dst, lane, 0, 0);
        }
        return;
    }
    stamp(7);
    for (int s = 0; s < steps; s += 2) {
        body(I0{}, ka + s, true, s == 0);
        body(I1{}, ka + s + 1, s + 1 < steps, false);
    }
    stamp(1);
}

int rc_start(int o, double s, int pad, bool centre) { return static_cast<int>(reduce_x_host(o, s, centre)) - pad; }

#ifdef MIPX_PROBES
// dbg 8 (scripts/ only): launch with per-step phase stamps, wait, and print one JSON line per
// 10th launch to stderr: block durations and start spread (the rounds of resident blocks),
// and each phase's mean cycles per live step (s_memtime ticks); the third launch only
int rcol_stamp_launch(const void *fn, RcArgs a, long long blocks, size_t lds, hipStream_t st, int ow, int oh, int n) {
    static int calls = 0;
    const size_t per = 8 + 8 * static_cast<size_t>(a.seg_steps), cnt = per * static_cast<size_t>(blocks);
    unsigned long long *d = nullptr;
    if (hipMalloc(&d, cnt * 8) != hipSuccess) return MIPX_EDEVICE;
    (void)hipMemsetAsync(d, 0, cnt * 8, st);
    a.stamps = d;
    hipLaunchKernelGGL(reinterpret_cast<void (*)(RcArgs)>(const_cast<void *>(fn)), dim3(static_cast<unsigned>(blocks)),
                       dim3(kRcNT), lds, st, a);
    int e = launch_check("k_rcol");
    std::vector<unsigned long long> h(cnt);
    if (!e && hipStreamSynchronize(st) == hipSuccess && hipMemcpy(h.data(), d, cnt * 8, hipMemcpyDeviceToHost) == hipSuccess &&
        ++calls == 3) {
        unsigned long long t0 = ~0ull, t1 = 0;
        double dur = 0, ph[7] = {0, 0, 0, 0, 0, 0, 0}, su[6] = {0, 0, 0, 0, 0, 0};
        long long nst = 0;
        std::vector<double> starts;
        for (long long b = 0; b < blocks; ++b) {
            const unsigned long long *p = h.data() + b * per;
            if (!p[0] || !p[1]) continue;
            t0 = std::min(t0, p[0]);
            t1 = std::max(t1, p[1]);
            dur += static_cast<double>(p[1] - p[0]);
            const int sl[7] = {0, 2, 3, 4, 5, 6, 7};  // set-up phase boundaries
            for (int i = 0; i < 6; ++i) su[i] += static_cast<double>(p[sl[i + 1]] - p[sl[i]]);
            starts.push_back(static_cast<double>(p[0]));
            for (int s = 0; s < a.seg_steps; ++s) {
                const unsigned long long *q = p + 8 + 8 * s;
                if (!q[0] || !q[7]) continue;
                for (int i = 0; i < 7; ++i) ph[i] += static_cast<double>(q[i + 1] - q[i]);
                ++nst;
            }
        }
        std::sort(starts.begin(), starts.end());
        const double nb = static_cast<double>(starts.size());
        auto pct = [&](double f) { return starts.empty() ? 0.0 : starts[static_cast<size_t>(f * (nb - 1))] - t0; };
        fprintf(stderr,
                "{\"rcol_stamps\": 1, \"ow\": %d, \"oh\": %d, \"n\": %d, \"blocks\": %lld, \"seg_steps\": %d, "
                "\"span\": %llu, \"block_mean\": %.0f, \"start_p25\": %.0f, \"start_p50\": %.0f, \"start_p75\": %.0f, "
                "\"start_max\": %.0f, \"steps\": %lld, \"ring_write\": %.1f, \"barrier1\": %.1f, \"vertical\": %.1f, "
                "\"issue\": %.1f, \"barrier2\": %.1f, \"horizontal\": %.1f, \"store\": %.1f, \"setup_operands\": %.0f, "
                "\"setup_seeds\": %.0f, \"setup_chunks\": %.0f, \"setup_prime\": %.0f, \"setup_issue\": %.0f, "
                "\"setup_realign\": %.0f}\n",
                ow, oh, n, blocks, a.seg_steps, t1 - t0, dur / std::max(1.0, nb), pct(0.25), pct(0.5), pct(0.75), pct(1.0), nst,
                ph[0] / std::max(1LL, nst), ph[1] / std::max(1LL, nst), ph[2] / std::max(1LL, nst), ph[3] / std::max(1LL, nst),
                ph[4] / std::max(1LL, nst), ph[5] / std::max(1LL, nst), ph[6] / std::max(1LL, nst), su[0] / std::max(1.0, nb),
                su[1] / std::max(1.0, nb), su[2] / std::max(1.0, nb), su[3] / std::max(1.0, nb), su[4] / std::max(1.0, nb),
                su[5] / std::max(1.0, nb));
    }
    (void)hipFree(d);
    return e;
}
#endif


}  // namespace

// The specialised k_rcol build of one geometry (r06): store mode wst (1..3; RGBA 1..2) and
// K-origin width k4 as template arguments, for every K-step count and chunk count
template <int B, int NKS, int KM, bool U>
const void *rc_spec_wk(int wst, int k4) {
    auto pk = [&](auto wc) -> const void * {
        constexpr int W = decltype(wc)::value;
        return k4 ? reinterpret_cast<const void *>(&k_rcol<B, NKS, KM, 1, U, W, 1>)
                  : reinterpret_cast<const void *>(&k_rcol<B, NKS, KM, 1, U, W, 0>);
    };
    if (wst == 1) return pk(std::integral_constant<int, 1>{});
    if (wst == 2) return pk(std::integral_constant<int, 2>{});
    if constexpr (B == 3) return pk(std::integral_constant<int, 3>{});
    return nullptr;
}
template <int B, bool U>
const void *rc_spec_pick(int nks, int kmax, int wst, int k4) {
    if (nks == 1) return kmax == 3 ? rc_spec_wk<B, 1, 3, U>(wst, k4) : rc_spec_wk<B, 1, 6, U>(wst, k4);
    return kmax == 3 ? rc_spec_wk<B, 2, 3, U>(wst, k4) : rc_spec_wk<B, 2, 6, U>(wst, k4);
}

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
#ifdef MIPX_PROBES
    const char *edb = tune_env("MIPX_RCOL_DBG");
    a.dbg = edb && *edb ? std::atoi(edb) : 0;
#endif
    const char *etr = tune_env("MIPX_RCOL_TRL");
    a.trl = !(etr && *etr == '0');
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
    // r06: builds with the store mode and K-origin width compiled in, loading the host-built
    // operands (device_rcol_hops) instead of computing them in the set-up
    // (profiles/r06/rcol_spec_ab.jsonl, rcol_hops_ab: 480x270 +12 %, 500x375 +8 %;
    // rcol_hops2_ab / rcol_hops2b_ab, two K steps: 1080p RGB / 2.4 +13 %, 4K / 2.4 +12 %,
    // 1333x1000 RGB / 2.4 +15 %, RGBA 1024^2 / 2.2 +11 %; rcol_spec3_ab: the rest);
    // MIPX_RCOL_SPEC=0: the argument-driven builds everywhere (A/B)
    const char *esp = tune_env("MIPX_RCOL_SPEC");
    bool spec = !(esp && *esp == '0') && a.wst >= 1 && a.wst <= (b == 3 ? 3 : 2) && a.skipl && a.trl && a.swz &&
                !a.allst;
    int hstrips = 0;
    const u8 *hops = spec ? device_rcol_hops(hs, b, centre, ox0, ow, w, a.k4, nks, &hstrips) : nullptr;
    spec = spec && hops;  // past the table cap: the builds that compute their operands
    if (spec) {
        a.hops = hops;
        a.hkb = reinterpret_cast<const int *>(hops + static_cast<size_t>(hstrips) * 4 * b * 64 * kRcolHopRec(nks));
        fn = b == 3 ? (unal ? rc_spec_pick<3, true>(nks, kmax, a.wst, a.k4) : rc_spec_pick<3, false>(nks, kmax, a.wst, a.k4))
                    : rc_spec_pick<4, false>(nks, kmax, a.wst, a.k4);
    }

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
        // r06: the specialised RGB build at 4 waves (5-6 spilled) where the specialised 3-wave
        // one was chosen: 364x273 x 128 -> 256^2 +10 % against the generic 4-wave build
        // (profiles/r06/rcol_sw4_ab.jsonl; forced on every shape it is 11-20 % slower)
        if (b == 3 && spec) {
#define MIPX_RC_S4(W_) f4 = a.k4 ? reinterpret_cast<const void *>(&k_rcol<3, 1, 3, 4, false, W_, 1>) \
                                 : reinterpret_cast<const void *>(&k_rcol<3, 1, 3, 4, false, W_, 0>);
            if (a.wst == 1) { MIPX_RC_S4(1) } else if (a.wst == 2) { MIPX_RC_S4(2) } else { MIPX_RC_S4(3) }
#undef MIPX_RC_S4
        }
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
#ifdef MIPX_PROBES
    if (a.dbg == 8) return rcol_stamp_launch(fn, a, blocks, lds, st, ow, oh, n);
#endif
    hipLaunchKernelGGL(reinterpret_cast<void (*)(RcArgs)>(const_cast<void *>(fn)), dim3(static_cast<unsigned>(blocks)),
                       dim3(kRcNT), lds, st, a);
    return launch_check("k_rcol");
}


}  // namespace mipx
