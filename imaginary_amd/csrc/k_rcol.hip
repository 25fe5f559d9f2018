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
    const float *tabf;        // device_reduce_table(hs): [129][htaps] (edge operands)
    int out_aligned;          // every output row starts on a dword
};

// libvips reduce position (reducev.cpp / reduceh.cpp, [U] corner convention):
// X = o * shrink, first tap floor(X) - pad, phase ((int)(X * 256) & 255 + 1) >> 1
__device__ __forceinline__ void rc_pos(int o, double s, int pad, int *start, int *phase) {
    const double X = o * s;
    *start = static_cast<int>(X) - pad;
    *phase = ((static_cast<int>(X * 256.0) & 255) + 1) >> 1;
}

__device__ __forceinline__ void rc_barrier() {  // LDS-only: stores and loads in flight survive it
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

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

// WV waves per block, XW = 16 WV output pixels per strip: 3 (RGB) / 4 (RGBA) units per wave
template <int B, int WV, int NKS>
__global__ void __launch_bounds__(512) k_rcol(RcArgs a) {
    constexpr int XW = 16 * WV;
    constexpr int NT = 64 * WV;       // threads
    constexpr int UPW = B;            // units per wave: XW B / 16 / WV
    extern __shared__ __attribute__((aligned(16))) uint32_t rcs[];
    uint32_t *ring = rcs;                                                   // [ring][rs]
    u8 *inter = reinterpret_cast<u8 *>(ring + a.ring * a.rs);              // [16][iw] (pixel - 128)
    int *pbias = reinterpret_cast<int *>(inter + kRcRows * a.iw);          // [XW * B] 128 * tap sum + 2048

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
    rc_pos(a.ox0 + x0, a.hs, a.hpad, &lo, &ph);
    rc_pos(a.ox0 + x_last, a.hs, a.hpad, &hi, &ph);
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
    u8 *ob = a.out + img * a.out_img;
    const __amdgpu_buffer_rsrc_t dst = __builtin_amdgcn_make_buffer_rsrc(ob, 0, static_cast<int>(a.out_img), 0x00020000);

    // ---- ring: image row v (COPY-clamped at the load) lives in slot (v - vbase) mod ring ----
    int r_lo0, r_end0;
    rc_pos(a.oy0 + y_begin, a.vs, a.vpad, &r_lo0, &ph);
    rc_pos(a.oy0 + min(y_begin + kRcRows, y_end) - 1, a.vs, a.vpad, &r_end0, &ph);
    r_end0 += a.vtaps;
    const int vbase = r_lo0;
    u8 *ringb = reinterpret_cast<u8 *>(ring);
    const int rsb = a.rs * 4;
    // rows [v0, v1) into the ring with direct-to-LDS dword loads, (row, chunk) pairs dealt
    // to the waves; the row offset rides in the VGPR offset (range-checked per image)
    auto stage = [&](int v0, int v1) {
        const int items = (v1 - v0) * cpr;
        for (int k = wave; k < items; k += WV) {
            const int l = k / cpr, c = k - l * cpr;
            const int v = v0 + l;
            const int slot = (v - vbase) % a.ring;
            if (64 * c + lane < ndw)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    src, (rc_lds_void *)(ringb + slot * rsb + 256 * c), 4,
                    clampi(v, 0, a.h - 1) * pitch + B * org + 4 * (64 * c + lane), 0, 0, 0);
        }
    };
    stage(r_lo0, r_end0);
    int loaded = r_end0;

    // ---- per-segment set-up: horizontal operands (registers, COPY edge folded) and biases ----
    for (int j = tid; j < XW * B; j += NT) {
        int sp, pp;
        rc_pos(a.ox0 + min(x0 + j / B, x_last), a.hs, a.hpad, &sp, &pp);
        pbias[j] = 128 * a.sumh[pp] + 2048;
    }
    rc_v4i th[UPW][NKS], tl[UPW][NKS];
    int kb[UPW];
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
        const int u = wave + WV * i;
        int sf, pf;
        rc_pos(a.ox0 + min(x0 + (16 * u) / B, x_last), a.hs, a.hpad, &sf, &pf);
        kb[i] = __builtin_amdgcn_readfirstlane((B * (sf - org) + (16 * u) % B) & ~7);  // K origin (8-byte aligned)
        const int o = 16 * u + n, xl = o / B, c = o - B * xl;
        int sp, pp;
        rc_pos(a.ox0 + min(x0 + xl, x_last), a.hs, a.hpad, &sp, &pp);
        const bool edge = sp < 0 || sp + a.htaps - 1 > a.w - 1;
        const signed char *rh = a.tabh + static_cast<size_t>(pp) * 2 * kRsTabW;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const int j0 = kb[i] + 64 * ks + 16 * kg;
            if (edge) {
                rc_edge_frag(a.tabf, a.htaps, pp, sp, c, j0, org, a.w, B, &th[i][ks], &tl[i][ks]);
            } else {
                const int off = kRsTabPad + j0 - c - B * (sp - org);
                th[i][ks] = rc_frag16(rh, off);
                tl[i][ks] = rc_frag16(rh + kRsTabW, off);
            }
        }
    }

    rc_v2i vt[4];  // the step's vertical tap operands (hi: 0, 1; lo: 2, 3); lane: output row n
    int vbn = 0;
    auto vtaps_for = [&](int y, int nr, int r_lo) {
        int sv, pv;
        rc_pos(a.oy0 + y + min(n, nr - 1), a.vs, a.vpad, &sv, &pv);
        const signed char *rv = a.tabv + static_cast<size_t>(pv) * 2 * kHmTabW;
        const int d = sv - r_lo - kHmTabPad;
        vt[0] = rc_taps8(rv, 8 * kg - d);
        vt[1] = rc_taps8(rv, 32 + 8 * kg - d);
        vt[2] = rc_taps8(rv + kHmTabW, 8 * kg - d);
        vt[3] = rc_taps8(rv + kHmTabW, 32 + 8 * kg - d);
        vbn = 128 * a.sumv[pv] + 2048;
    };
    vtaps_for(y_begin, min(kRcRows, y_end - y_begin), r_lo0);
    uint32_t res[UPW];
    int y_prev = 0, nr_prev = 0;

    for (int s = 0; s < steps; ++s) {
        const int y = y_begin + s * kRcRows;
        const int nr = min(kRcRows, y_end - y);
        int r_lo;
        rc_pos(a.oy0 + y, a.vs, a.vpad, &r_lo, &ph);
        const rc_v4i bh = rc_v4i{vt[0].x, vt[0].y, vt[1].x, vt[1].y};
        const rc_v4i bl = rc_v4i{vt[2].x, vt[2].y, vt[3].x, vt[3].y};
        const int vb = vbn;
        // (C) this step's rows are in the ring (every wave's loads landed); the
        // intermediate is free (every wave finished the previous horizontal pass)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        rc_barrier();
        // (B) the next step's new rows: their slots hold rows below this step's first
        // (ring >= this step's rows + the next step's new rows), and its vertical taps
        if (s + 1 < steps) {
            const int y1 = y + kRcRows, nr1 = min(kRcRows, y_end - y1);
            int r_lo1, r_end1;
            rc_pos(a.oy0 + y1, a.vs, a.vpad, &r_lo1, &ph);
            rc_pos(a.oy0 + y1 + nr1 - 1, a.vs, a.vpad, &r_end1, &ph);
            r_end1 += a.vtaps;
            stage(loaded, r_end1);
            loaded = r_end1;
            vtaps_for(y1, nr1, r_lo1);
        }
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
        // (E) vertical pass: 16-byte column tiles dealt to the waves.  K index 16 kg + e
        // holds relative row 8 kg + e (e < 8) or 32 + 8 kg + e - 8, so the 16 rows one
        // 32-lane half reads per transposed load sit in consecutive ring slots
        {
            const int base = (r_lo - vbase) % a.ring;
            int s1 = base + 8 * kg + (n >> 1), s2 = s1 + 32;
            s1 = s1 >= a.ring ? s1 - a.ring : s1;
            s1 = s1 >= a.ring ? s1 - a.ring : s1;
            s2 = s2 >= a.ring ? s2 - a.ring : s2;
            s2 = s2 >= a.ring ? s2 - a.ring : s2;
            s2 = s2 >= a.ring ? s2 - a.ring : s2;
            const u8 *p1 = ringb + s1 * rsb + 8 * (n & 1);
            const u8 *p2 = ringb + s2 * rsb + 8 * (n & 1);
            u8 *iq = inter + n * a.iw + 4 * kg;
            for (int ct = wave; ct < nt; ct += WV) {
                const rc_v2i t1 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
                    (__attribute__((address_space(3))) rc_v2i *)((rc_lds_void *)(const_cast<u8 *>(p1 + 16 * ct))));
                const rc_v2i t2 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
                    (__attribute__((address_space(3))) rc_v2i *)((rc_lds_void *)(const_cast<u8 *>(p2 + 16 * ct))));
                const rc_v4i av = rc_v4i{t1.x ^ static_cast<int>(0x80808080u), t1.y ^ static_cast<int>(0x80808080u),
                                         t2.x ^ static_cast<int>(0x80808080u), t2.y ^ static_cast<int>(0x80808080u)};
                rc_v4i dh = rc_v4i{0, 0, 0, 0}, dl = rc_v4i{vb, vb, vb, vb};
                dh = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bh, dh, 0, 0, 0);
                dl = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bl, dl, 0, 0, 0);
                const uint32_t wv = rc_round4((dh[0] << 6) + dl[0], (dh[1] << 6) + dl[1], (dh[2] << 6) + dl[2],
                                              (dh[3] << 6) + dl[3]);
                *reinterpret_cast<uint32_t *>(iq + 16 * ct) = wv ^ 0x80808080u;
            }
        }
        // (F) the intermediate is complete
        rc_barrier();
        // (H) horizontal pass: units wave + WV i, operands from registers
#pragma unroll
        for (int i = 0; i < UPW; ++i) {
            const int u = wave + WV * i;
            res[i] = 0u;
            if (16 * u >= vbytes) continue;
            const rc_v4i bias = *reinterpret_cast<const rc_v4i *>(pbias + 16 * u + 4 * kg);
            rc_v4i ah = rc_v4i{0, 0, 0, 0}, al = bias;
            const u8 *ir = inter + n * a.iw + kb[i] + 16 * kg;
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const uint2 q0 = *reinterpret_cast<const uint2 *>(ir + 64 * ks);
                const uint2 q1 = *reinterpret_cast<const uint2 *>(ir + 64 * ks + 8);
                const rc_v4i bz = rc_v4i{static_cast<int>(q0.x), static_cast<int>(q0.y), static_cast<int>(q1.x),
                                         static_cast<int>(q1.y)};
                ah = __builtin_amdgcn_mfma_i32_16x16x64_i8(th[i][ks], bz, ah, 0, 0, 0);
                al = __builtin_amdgcn_mfma_i32_16x16x64_i8(tl[i][ks], bz, al, 0, 0, 0);
            }
            res[i] = rc_round4((ah[0] << 6) + al[0], (ah[1] << 6) + al[1], (ah[2] << 6) + al[2], (ah[3] << 6) + al[3]);
        }
        y_prev = y;
        nr_prev = nr;
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

int rc_start(int o, double s, int pad) { return static_cast<int>(o * s) - pad; }

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
    // ring rows: a step's rows plus the next step's new ones (their loads are issued
    // before the step's vertical pass), exact over the window's steps; MFMA K = 64 rows
    int lmax = 0, ring = 0;
    for (int y = 0; y < oh; y += kRcRows) {
        const int y1 = std::min(oh, y + kRcRows) - 1;
        const int r0 = rc_start(oy0 + y, vs, a.vpad), r1 = rc_start(oy0 + y1, vs, a.vpad) + vtaps;
        lmax = std::max(lmax, r1 - r0);
        int need = r1 - r0;
        if (y + kRcRows < oh) need = rc_start(oy0 + std::min(oh, y + 2 * kRcRows) - 1, vs, a.vpad) + vtaps - r0;
        ring = std::max(ring, need);
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
    if (!a.tabv || !a.tabh || !a.tabf || ntv != vtaps || nth != htaps || ntf != htaps) return MIPX_EDEVICE;

    // per strip width (16 output pixels per wave): staged bytes, K steps of the
    // horizontal units, LDS
    struct Geo { int wv, nt, nks, rs, iw; size_t lds; };
    auto geo_for = [&](int wv) {
        const int xw = 16 * wv;
        Geo g{wv, 0, 0, 0, 0, 0};
        int kbmax = 0;
        for (int x0 = 0; x0 < ow; x0 += xw) {
            const int xl = std::min(x0 + xw - 1, ow - 1);
            const int lo = rc_start(ox0 + x0, hs, a.hpad), hi = rc_start(ox0 + xl, hs, a.hpad) + htaps - 1;
            const int org = lo & ~3;
            g.nt = std::max(g.nt, (b * (hi - org + 1) + 15) >> 4);
            for (int u = 0; u < xw * b / 16; ++u) {
                const int o0 = 16 * u, o1 = 16 * u + 15;
                if (x0 + o0 / b > xl) break;
                const int xf = x0 + o0 / b, xe = std::min(x0 + o1 / b, xl);
                const int kbu = (b * (rc_start(ox0 + xf, hs, a.hpad) - org) + o0 % b) & ~7;
                const int need = b * (rc_start(ox0 + xe, hs, a.hpad) + htaps - 1 - org) + b;
                g.nks = std::max(g.nks, (need - kbu + 63) / 64);
                kbmax = std::max(kbmax, kbu);
            }
        }
        g.rs = 4 * g.nt;
        while (((g.rs & 63) >> 2) % 2 == 0) g.rs += 4;  // 16 consecutive rows on distinct bank quads
        g.iw = (std::max(16 * g.nt, kbmax + 64 * g.nks) + 16 + 15) & ~15;
        while ((g.iw / 4) % 8 != 4) g.iw += 16;  // 4 mod 8 dwords: the intermediate writes hit distinct banks
        g.lds = static_cast<size_t>(a.ring) * g.rs * 4 + static_cast<size_t>(kRcRows) * g.iw +
                static_cast<size_t>(xw) * b * 4;
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
    const long long target = g.wv == 8 ? 2048 : 4096;
    int segs = static_cast<int>(std::min<long long>(steps, std::max<long long>(1, (target + cols - 1) / cols)));
    int seg_steps = (steps + segs - 1) / segs;
    if (seg_steps < 2 && steps >= 2) seg_steps = 2;
    segs = (steps + seg_steps - 1) / seg_steps;
    a.segs = segs;
    a.seg_steps = seg_steps;
    const long long blocks = cols * segs;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    const dim3 grid(static_cast<unsigned>(blocks)), blk(64 * g.wv);
#define MIPX_RC(B_, WV_)                                                                                     \
    if (g.nks == 1) hipLaunchKernelGGL((k_rcol<B_, WV_, 1>), grid, blk, g.lds, st, a);                      \
    else hipLaunchKernelGGL((k_rcol<B_, WV_, 2>), grid, blk, g.lds, st, a);
    if (b == 3) {
        if (g.wv == 8) { MIPX_RC(3, 8) } else { MIPX_RC(3, 4) }
    } else {
        if (g.wv == 8) { MIPX_RC(4, 8) } else { MIPX_RC(4, 4) }
    }
#undef MIPX_RC
    return launch_check("k_rcol");
}

}  // namespace mipx
