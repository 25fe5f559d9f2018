// k_bcol.hip — libvips vips_gaussblur (convsep.c: the horizontal 1 x n integer mask,
// then the vertical one, through convi.c: uchar intermediate, (sum + (scale + 1) / 2) /
// scale, clipped, EXTEND_COPY edges) as a column walker on the i8 matrix cores, r03.
//
// A block (4 waves) owns a strip of 64 output pixels of one image (or window) and walks
// a segment of its rows, 16 output rows per step:
//   * loads: the 16 input rows a step's horizontal pass needs (16 j + half ..) are
//     loaded as 16-byte chunks into registers two steps ahead, flipped to p - 128 and
//     written to one of two staging buffers in LDS (the step's parity), one barrier per
//     step.  Strips at the window edges repeat the edge pixel into the staged halo
//     (COPY) after a second barrier;
//   * horizontal: a wave owns UPW consecutive 16-byte output units of the strip; per
//     unit, D[output byte][row] = A[output byte][K] x B[K][row] on
//     v_mfma_i32_16x16x64_i8 with A = the banded taps (tap k at K = o + delta + B k,
//     the same for every unit: registers) and B = 16 staged rows' bytes; the rounded
//     uchar (as T - 128) goes to a ring of intermediate rows in LDS;
//   * vertical: per 16-byte column of the wave's own units, D[byte][output row] = A[byte]
//     [ring row] x B[ring row][output row], A from two ds_read_b64_tr_b8, B the banded
//     taps (registers).  A wave reads only the ring columns it wrote, so the vertical
//     pass needs no barrier;
//   * stores: 16 rows x 16 UPW bytes through a wave-private LDS tile as 16-byte row pieces.
// Every input row is loaded and filtered once per segment; the first steps of a segment
// filter the rows above it (taps - 1 of them).  Bit-identical to the two convi passes
// (oracle/vips_ref.c convi_pass): the same integer sums, the same rounding (magic
// multiply exact for sums below 2^32 / scale) and the same clamped edges.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "device_common.h"
#include "lds_ops.h"

namespace mipx {
namespace {

using namespace dev;

constexpr int kBcRows = 16;  // rows per step (the MFMA N)
constexpr int kBcNT = 256;   // threads per block
constexpr int kBcSB = 64;    // output bytes per strip and 16-byte unit per wave (strip = kBcSB * UPW bytes)

struct BcArgs {
    const u8 *in;
    u8 *out;
    long long in_base;  // byte offset of the window origin in an image
    int in_pitch;
    long long in_img, out_img;
    int w, h;           // window = output size (COPY clamp range)
    int strips, segs, seg_steps, ksteps;
    int half;           // taps / 2
    int sxb;            // staged rows start sxb bytes before the strip (a multiple of 16, >= B half)
    int spb;            // staged bytes per strip row
    int kb0;            // the H operand's first staged byte (e & ~3, e = sxb - B half)
    int cpr;            // 16-byte chunks per staged row
    int rsd;            // staging row stride (bytes)
    int rmask, tw;      // ring rows - 1, ring row stride (bytes)
    int pre;            // filter-only steps before a segment's first output step
    int kspan;          // horizontal K bytes the taps cover (16 + delta + B (taps - 1)): reads past it skipped
    uint32_t mag;       // floor(x / scale) == mulhi(x, mag) for the sums here
    int seed;           // 128 scale + (scale + 1) / 2
    int wst2;           // output rows not a multiple of 16 bytes: the edge piece as dwords
    int skipl;               // load batches no lane of the wave needs are not issued (r05)
    int a16;            // host: horizontal operands 16-byte aligned (k_bcol<.., A16 = true>)
    int sd;             // A16: staged rows start sd bytes into their LDS row (0 / 4 / 8 / 12)
    int vperm;          // r06: vertical K index 16 kg + e holds ring row 8 kg + e (e < 8) / 32 + 8 kg + e - 8
    int wsw;            // r06: the store tile's read-back lanes by tile_rd_lane (UPW 4)
    const signed char *ops;  // device_blur_ops: [NKS][64 lanes][16] horizontal, then [64][16] vertical
};

__device__ __forceinline__ uint32_t bc_pack(const rc_v4i &d, uint32_t mag) {
    const int t0 = __umulhi(static_cast<uint32_t>(d[0]), mag), t1 = __umulhi(static_cast<uint32_t>(d[1]), mag);
    const int t2 = __umulhi(static_cast<uint32_t>(d[2]), mag), t3 = __umulhi(static_cast<uint32_t>(d[3]), mag);
    uint32_t lo, hi;
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 0" : "=v"(lo) : "v"(t0), "v"(t1));
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 0" : "=v"(hi) : "v"(t2), "v"(t3));
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// 8 bytes at a 4-byte-aligned LDS address (two adjacent dwords, one instruction)
__device__ __forceinline__ rc_u2 lds_rd2x32(uint32_t a) {
    rc_u2 v;
    asm volatile("ds_read2_b32 %0, %1 offset1:1" : "=v"(v) : "v"(a));
    return v;
}

// B: bands, NKS: horizontal K steps of 64 bytes, KMAX: staging chunks per lane per step,
// UPW: 16-byte units per wave (strips of 64 UPW bytes; the passes are byte-column-wise and
// the taps of output byte X sit at X + B (k - half), so strips need not start on a pixel).
// 128-pixel strips (UPW 6 / 8, operands in chunks of half) measured 10-40 % slower at 2-3
// waves per SIMD (profiles/r03/bcol_px_chunk_ab.jsonl)
template <int B, int NKS, int KMAX, bool A16, int UPW>
__global__ void __launch_bounds__(kBcNT) k_bcol(BcArgs a) {
    constexpr int SB = kBcSB * UPW;  // strip bytes
    // store tile row stride: dwords = 4 mod 8 (the tile writes on distinct banks); with UPW 4
    // (wsw, r06) the read-back's lanes take rows by tile_rd_lane, so each ds_read_b128 lane
    // group reads 4 rows on disjoint banks (lane / 4 put rows 0 / 3 / 5 / 6 of one group on
    // shared banks)
    constexpr int WSR = 16 * UPW + (UPW % 2 == 0 ? 16 : 0);
    const bool wsw = UPW == 4 && a.wsw;
    constexpr int NPC = (16 * UPW + 63) / 64;                  // 16-byte row pieces per lane
    constexpr int UC = UPW;                                    // units per operand chunk
    extern __shared__ __attribute__((aligned(16))) uint32_t bcs[];
    const uint32_t stg_l = rc_lds(bcs);                                                  // [2][16][rsd]
    const uint32_t ring_l = stg_l + static_cast<uint32_t>(2 * kBcRows * a.rsd);          // [rmask + 1][tw]
    const uint32_t wst_l0 = ring_l + static_cast<uint32_t>((a.rmask + 1) * a.tw);        // [WV][16][WSR]
    u8 *stgb = reinterpret_cast<u8 *>(bcs);

    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int strip = static_cast<int>(t % static_cast<uint32_t>(a.strips));
    const int rest = static_cast<int>(t / static_cast<uint32_t>(a.strips));
    const int seg = rest % a.segs;
    const int img = __builtin_amdgcn_readfirstlane(rest / a.segs);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n = lane & 15, kg = lane >> 4;

    const int wb = a.w * B;                                 // window row bytes
    const int xb0 = strip * SB, vbytes = min(SB, wb - xb0);  // the strip's output bytes in a row
    const int sxb = xb0 - a.sxb;                            // window row byte of staged byte 0
    const bool edge = sxb < 0 || sxb + a.spb > wb;          // block-uniform
    const int ka = seg * a.seg_steps, kz = min(a.ksteps, ka + a.seg_steps);
    const int j0 = ka - a.pre;                              // first (filter-only) step

    const __amdgpu_buffer_rsrc_t src = image_rsrc(a.in + img * a.in_img, a.in_img);
    const __amdgpu_buffer_rsrc_t dst = image_rsrc(a.out + img * a.out_img, a.out_img);

    // operands: horizontal taps per K step and the vertical banded taps (registers)
    rc_v4i ta[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) ta[ks] = *reinterpret_cast<const rc_v4i *>(a.ops + (ks * 64 + lane) * 16);
    const rc_v4i tb = *reinterpret_cast<const rc_v4i *>(a.ops + (NKS * 64 + lane) * 16);

    // staging chunks: chunk c = tid + 256 k of a step is (row rr, column col)
    int rr[KMAX], cof[KMAX];
    uint32_t lsl[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int c = tid + kBcNT * k;
        rr[k] = c / a.cpr;
        const int col = c - rr[k] * a.cpr;
        cof[k] = static_cast<int>(a.in_base) + sxb + 16 * col;
        lsl[k] = static_cast<uint32_t>(rr[k] * a.rsd + 16 * col + (A16 ? a.sd : 0));
    }
    rc_u4 rv[2][KMAX];
    bool wl[KMAX];  // skipl: batch k of this wave loads anything (uniform, the same every step)
#pragma unroll
    for (int k = 0; k < KMAX; ++k) wl[k] = !a.skipl || __builtin_amdgcn_ballot_w64(rr[k] < kBcRows) != 0;
    auto issue = [&](auto pc, int j) {  // the input rows of step j: 16 j + half + rr
        constexpr int P = decltype(pc)::value;
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            if (!wl[k]) continue;
            const int r = clampi(kBcRows * j + a.half + rr[k], 0, a.h - 1);
            rv[P][k] = __builtin_bit_cast(
                rc_u4, __builtin_amdgcn_raw_buffer_load_b128(src, rr[k] < kBcRows ? r * a.in_pitch + cof[k] : 0x7ffffff0, 0, 0));
        }
    };
    auto stage = [&](auto pc) {
        constexpr int P = decltype(pc)::value;
#pragma unroll
        for (int k = 0; k < KMAX; ++k)
            if (rr[k] < kBcRows) {
                const uint32_t ad = stg_l + static_cast<uint32_t>(P * kBcRows * a.rsd) + lsl[k];
                if (A16 && a.sd) lds_wr4x32(ad, rv[P][k] ^ 0x80808080u);  // rows shifted onto the 16-byte operand grid
                else lds_wr128(ad, rv[P][k] ^ 0x80808080u);
            }
    };
    // COPY edge: staged bytes outside the window repeat its edge pixel's byte of their band
    // (only the nl bytes left of the window and the nr right of it are visited)
    const int nl = max(0, -sxb), nr = max(0, sxb + a.spb - wb), no = nl + nr;
    auto fixup = [&](auto pc) {
        constexpr int P = decltype(pc)::value;
        u8 *sb = stgb + P * kBcRows * a.rsd + (A16 ? a.sd : 0);
        for (int i = tid; i < kBcRows * no; i += kBcNT) {
            const int l = i / no, t = i - l * no;
            const int q = t < nl ? t : a.spb - nr + (t - nl), X = sxb + q;
            const int c = (X % B + B) % B;
            sb[l * a.rsd + q] = sb[l * a.rsd + (X < 0 ? c : wb - B + c) - sxb];
        }
    };
    // horizontal pass of step j: this wave's units, 16 staged rows -> ring rows 16 j + half + n
    auto horizontal = [&](auto pc, int j) {
        constexpr int P = decltype(pc)::value;
        const uint32_t sr = stg_l + static_cast<uint32_t>(P * kBcRows * a.rsd + n * a.rsd + a.kb0 + 16 * kg);
        const uint32_t rw = ring_l + static_cast<uint32_t>(((kBcRows * j + a.half + n) & a.rmask) * a.tw + 4 * kg);
        // units in chunks of UC (128-pixel strips: half the operand registers live at once)
#pragma unroll
        for (int c0 = 0; c0 < UPW; c0 += UC) {
            rc_u2 q[UC][NKS][2];
#pragma unroll
            for (int i = 0; i < UC; ++i)
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) {
                    const uint32_t ad = sr + static_cast<uint32_t>(16 * (UPW * wave + c0 + i) + 64 * ks);
                    if (64 * ks + 16 * kg < a.kspan) {  // lanes whose 16 K bytes lie past the taps read nothing
                        if (A16) {
                            const rc_u4 v = lds_rd128(ad);
                            q[i][ks][0] = rc_u2{v.x, v.y};
                            q[i][ks][1] = rc_u2{v.z, v.w};
                        } else {
                            q[i][ks][0] = lds_rd2x32(ad);
                            q[i][ks][1] = lds_rd2x32(ad + 8);
                        }
                    } else {
                        q[i][ks][0] = rc_u2{0u, 0u};
                        q[i][ks][1] = rc_u2{0u, 0u};
                    }
                }
#pragma unroll
            for (int i = 0; i < UC; ++i)
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) rc_pin(q[i][ks][0]), rc_pin(q[i][ks][1]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < UC; ++i) {
                rc_v4i acc = rc_v4i{a.seed, a.seed, a.seed, a.seed};
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) {
                    rc_pin(q[i][ks][0]);
                    rc_pin(q[i][ks][1]);
                    const rc_v4i bv = rc_v4i{static_cast<int>(q[i][ks][0].x), static_cast<int>(q[i][ks][0].y),
                                             static_cast<int>(q[i][ks][1].x), static_cast<int>(q[i][ks][1].y)};
                    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(ta[ks], bv, acc, 0, 0, 0);
                }
                lds_wr32(rw + static_cast<uint32_t>(16 * (UPW * wave + c0 + i)), bc_pack(acc, a.mag) ^ 0x80808080u);
            }
        }
    };
    // vertical pass of step j: ring rows 16 j - half + K, K = 16 kg + (0..7 | 8..15)
    const uint32_t wst_l = wst_l0 + static_cast<uint32_t>(wave * kBcRows * WSR);
    // (vperm: K 16 kg + e <-> row 8 kg + e / 32 + 8 kg + e - 8, so the 16 rows of one 32-lane
    // half's transposed read are consecutive ring slots on distinct banks; the identity
    // layout put rows r and r + 16 of one half on the same banks: 2-way on every read)
    auto vertical_store = [&](int j, bool live) {
        const int r1 = kBcRows * j - a.half + (a.vperm ? 8 : 16) * kg + (n >> 1);
        const uint32_t a1 = ring_l + static_cast<uint32_t>((r1 & a.rmask) * a.tw + 8 * (n & 1));
        const uint32_t a2 = ring_l + static_cast<uint32_t>(((r1 + (a.vperm ? 32 : 8)) & a.rmask) * a.tw + 8 * (n & 1));
#pragma unroll
        for (int c0 = 0; c0 < UPW; c0 += UC) {
            rc_v2i t1[UC], t2[UC];
#pragma unroll
            for (int i = 0; i < UC; ++i) {
                const uint32_t cb = static_cast<uint32_t>(16 * (UPW * wave + c0 + i));
                t1[i] = lds_tr8(a1 + cb);
                t2[i] = lds_tr8(a2 + cb);
            }
#pragma unroll
            for (int i = 0; i < UC; ++i) rc_pin(t1[i]), rc_pin(t2[i]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < UC; ++i) {
                rc_pin(t1[i]);
                rc_pin(t2[i]);
                const rc_v4i av = rc_v4i{t1[i].x, t1[i].y, t2[i].x, t2[i].y};
                lds_wr32(wst_l + static_cast<uint32_t>(n * WSR + 16 * (c0 + i) + 4 * kg),
                         bc_pack(__builtin_amdgcn_mfma_i32_16x16x64_i8(av, tb, rc_v4i{a.seed, a.seed, a.seed, a.seed}, 0, 0, 0),
                                 a.mag));
            }
        }
        rc_u4 qv[NPC];
#pragma unroll
        for (int r = 0; r < NPC; ++r) {  // piece lane + 64 r = (row, 16-byte chunk)
            const int pc = min(lane + 64 * r, 16 * UPW - 1);
            int wrow = pc / UPW, wch = pc - UPW * wrow;
            if (wsw) tile_rd_lane(lane, &wrow, &wch);
            qv[r] = lds_rd128(wst_l + static_cast<uint32_t>(wrow * WSR + 16 * wch));
        }
#pragma unroll
        for (int r = 0; r < NPC; ++r) rc_pin(qv[r]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int r = 0; r < NPC; ++r) {
            rc_pin(qv[r]);
            const int pc = lane + 64 * r;
            int wrow = pc / UPW, wch = pc - UPW * wrow;
            if (wsw) tile_rd_lane(lane, &wrow, &wch);  // (UPW 4: one piece per lane, r = 0)
            const int we = 16 * (UPW * wave + wch);  // the piece's first byte in the strip row
            const int y = kBcRows * j + wrow;
            const bool ok = live && pc < 16 * UPW && y < a.h;
            const int base = y * wb + xb0 + we;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(rc_v4i, qv[r]), dst,
                                                   ok && we + 16 <= vbytes ? base : 0x7ffffff0, 0, 0);
            if (a.wst2) {  // rows whose byte count is not a multiple of 16: the piece at the window edge in dwords
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    __builtin_amdgcn_raw_buffer_store_b32(
                        qv[r][k], dst, ok && we + 16 > vbytes && we + 4 * k < vbytes ? base + 4 * k : 0x7ffffff0, 0, 0);
            }
        }
    };
    // one step: stage rows of j (loaded two steps ago, set P) -> barrier [-> COPY fix-up ->
    // barrier] -> loads of j + 2 -> horizontal(j) -> vertical(j) + stores (idle before ka).
    // Two staging buffers: a wave writing step j + 1's rows has passed the barrier of step
    // j, so every wave is done with step j - 1's buffer.
    auto body = [&](auto pc, int j) {
        stage(pc);
        rc_barrier();
        if (edge) {
            fixup(pc);
            rc_barrier();
        }
        issue(pc, j + 2);
        horizontal(pc, j);
        vertical_store(j, j >= ka);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    issue(I0{}, j0);
    issue(I1{}, j0 + 1);
    for (int j = j0; j < kz; j += 2) {
        body(I0{}, j);
        if (j + 1 < kz) body(I1{}, j + 1);
    }
}

}  // namespace

// The column-walking blur of the (left, top, ow x oh) window: RGB / RGBA, dword-aligned
// rows, window start and output, masks of <= 33 non-negative taps below 128, scale below
// 4096; MIPX_EUNSUPPORTED otherwise (the caller runs k_bmf / k_blur2d).
int blur_col_launch(const u8 *in, u8 *out, int n, int w, int h, int b, int left, int top, int ow, int oh,
                    const std::vector<int> &mask, int scale, hipStream_t st) {
    const char *ec = tune_env("MIPX_BCOL");  // 0: k_bmf / k_blur2d (A/B)
    if (ec && *ec == '0') return MIPX_EUNSUPPORTED;
    const int taps = static_cast<int>(mask.size());
    if ((b != 3 && b != 4) || taps < 1 || taps > 33 || (taps & 1) == 0 || scale <= 0 || scale >= 4096)
        return MIPX_EUNSUPPORTED;
    for (int m : mask)
        if (m < 0 || m > 127) return MIPX_EUNSUPPORTED;
    if ((w * b) % 4 || (left * b) % 4 || reinterpret_cast<uintptr_t>(in) % 4 || (ow * b) % 4 ||
        reinterpret_cast<uintptr_t>(out) % 4)
        return MIPX_EUNSUPPORTED;
    BcArgs a{};
    a.in = in;
    a.out = out;
    a.in_pitch = w * b;
    a.in_base = (static_cast<long long>(top) * w + left) * b;
    a.in_img = img_bytes(w, h, b);
    a.out_img = img_bytes(ow, oh, b);
    if (a.in_img >= 0x7fffffffLL - 4096 || a.out_img >= 0x7fffffffLL - 4096) return MIPX_EUNSUPPORTED;
    a.w = ow;
    a.h = oh;
    a.half = taps / 2;
    // strips of 64 UPW bytes: RGBA 64 pixels (UPW 4); RGB 256 bytes (UPW 4, 85 1/3 pixels:
    // 1080p / 4K / 12 MP 7-12 % faster than 64-pixel strips, profiles/r03/bcol_rgb256_ab.jsonl;
    // MIPX_BCOL_RGB192=1 keeps those, A/B).  The staged origin sits sxb bytes before
    // the strip, on 16 bytes, so no chunk straddles a row start (a load at a negative offset
    // reads 0 whole)
    const char *e192 = tune_env("MIPX_BCOL_RGB192");
    const int upw = b == 4 || !(e192 && *e192 == '1') ? 4 : 3;
    const int sbytes = kBcSB * upw;
    a.sxb = (a.half * b + 15) / 16 * 16;
    a.spb = sbytes + a.sxb + a.half * b;
    // r03: the H operand starts on 16 bytes, so a unit's 16 K bytes are one ds_read_b128, and
    // staged rows 32 mod 64 bytes apart put the 16 rows x 4 K groups of every lane group on
    // distinct banks (two ds_read2_b32 on dword offsets hit 8 banks with 32 lanes: 4-way,
    // profiles/r03/pmc_bcol_*.txt).  The staged rows are written sd = 0 / 4 / 8 / 12 bytes
    // into their LDS rows (dword writes) so the operand's dword offset lands on 16 bytes and
    // the taps keep only the 0-3 byte offset (no extra K step); MIPX_BCOL_A16=0 keeps the
    // dword-aligned operand (A/B)
    const int e = a.sxb - b * a.half;
    const char *ea = tune_env("MIPX_BCOL_A16");
    a.a16 = !(ea && *ea == '0') || upw != b;  // the 256-byte RGB strips exist only with A16
    a.sd = a.a16 ? (16 - (e & 12)) & 12 : 0;
    const int delta = e & 3;
    a.kb0 = a.a16 ? (e + a.sd) & ~15 : e & ~3;
    a.kspan = 16 + delta + b * (taps - 1);
    const int nks = (a.kspan + 63) / 64;
    if (nks > 3) return MIPX_EUNSUPPORTED;
    a.cpr = (a.spb + 15) / 16;
    const int kmax = (kBcRows * a.cpr + kBcNT - 1) / kBcNT;
    if (kmax > 3) return MIPX_EUNSUPPORTED;
    // staging stride: every horizontal read in the row (+ 4 units of slack), dwords = 4 mod 8
    int rsd = std::max(16 * a.cpr + a.sd, a.kb0 + sbytes + 64 * nks) + 16;
    rsd = (rsd + 15) & ~15;
    if (a.a16) {
        while ((rsd / 16) % 4 != 2) rsd += 16;
    } else {
        while ((rsd / 4) % 8 != 4) rsd += 16;
    }
    a.rsd = rsd;
    const int ring = kBcRows + taps - 1 <= 32 ? 32 : 64;
    a.rmask = ring - 1;
    int twd = sbytes / 4;  // the transposed reads: (dwords mod 64) / 4 odd
    twd = (twd + 3) & ~3;
    while (((twd & 63) >> 2) % 2 == 0) twd += 4;
    a.tw = 4 * twd;
    a.pre = (2 * a.half + kBcRows - 1) / kBcRows;
    a.mag = static_cast<uint32_t>(((1ULL << 32) + scale - 1) / scale);
    a.seed = 128 * scale + (scale + 1) / 2;
    a.wst2 = (ow * b) % 16 != 0;
    // r05 (as k_rcol): MIPX_BCOL_SKIPL=0 issues every batch, idle lanes out of range; blur
    // +1-2.3 %, C3 +0.3 %, C5 +0.6 % (profiles/r05/bcol/bsl_ab.jsonl)
    const char *esl = tune_env("MIPX_BCOL_SKIPL");
    a.skipl = !(esl && *esl == '0');
    // r06: MIPX_BCOL_VPERM=0 / MIPX_BCOL_WSW=0 keep r05's vertical K
    // layout / padded store tile (A/B)
    const char *evp = tune_env("MIPX_BCOL_VPERM");
    a.vperm = !(evp && *evp == '0');
    const char *ews = tune_env("MIPX_BCOL_WSW");
    a.wsw = !(ews && *ews == '0');
    a.ops = device_blur_ops(mask, b, delta, nks, a.vperm);
    if (!a.ops) return MIPX_EDEVICE;
    const size_t lds = static_cast<size_t>(2 * kBcRows) * rsd + static_cast<size_t>(ring) * a.tw +
                       static_cast<size_t>(4 * kBcRows) * (16 * upw + (upw % 2 == 0 ? 16 : 0));
    if (lds > 64 * 1024) return MIPX_EUNSUPPORTED;

    const void *fn = nullptr;
#define MIPX_BC_K2(B_, NKS_, A_, U_)                                                               \
    fn = kmax == 1   ? reinterpret_cast<const void *>(&k_bcol<B_, NKS_, 1, A_, U_>)                \
         : kmax == 2 ? reinterpret_cast<const void *>(&k_bcol<B_, NKS_, 2, A_, U_>)                \
                     : reinterpret_cast<const void *>(&k_bcol<B_, NKS_, 3, A_, U_>);
#define MIPX_BC_K(B_, NKS_)                                                   \
    if (B_ == 3 && upw == 4) { MIPX_BC_K2(B_, NKS_, true, 4) }                \
    else if (a.a16) { MIPX_BC_K2(B_, NKS_, true, B_) }                        \
    else { MIPX_BC_K2(B_, NKS_, false, B_) }
    if (b == 3) {
        if (nks == 1) { MIPX_BC_K(3, 1) } else if (nks == 2) { MIPX_BC_K(3, 2) } else { MIPX_BC_K(3, 3) }
    } else {
        if (nks == 1) { MIPX_BC_K(4, 1) } else if (nks == 2) { MIPX_BC_K(4, 2) } else { MIPX_BC_K(4, 3) }
    }
#undef MIPX_BC_K
#undef MIPX_BC_K2

    // segments: a segment's first pre steps only filter.  About 6 rounds of resident blocks
    // (profiles/r03/bcol_segs_ab.jsonl, bcol_rgb256_ab.jsonl: 1080p RGB best at 7.5 rounds,
    // 12 MP at 8, 1080p RGBA at 3-6, C3's RGBA at 2 segments; one long segment per strip left
    // 1080p 30-40 % slower), segments of at least max(4, 4 pre) steps so the filter-only
    // steps stay <= 25 %
    a.strips = (ow * b + sbytes - 1) / sbytes;
    a.ksteps = (oh + kBcRows - 1) / kBcRows;
    const long long cols = static_cast<long long>(a.strips) * n;
    const int per_cu = occupancy_per_cu(fn, kBcNT, lds, 2);
    const long long slots = static_cast<long long>(device_cu_count()) * per_cu;
    const int ss_min = std::max(4, 4 * a.pre);
    int best_segs = static_cast<int>(std::max(1LL, (6 * slots + cols / 2) / cols));
    best_segs = std::min(best_segs, std::max(1, (a.ksteps + ss_min - 1) / ss_min));
    const char *esg = tune_env("MIPX_BCOL_SEGS");  // A/B: force the segment count
    if (esg && *esg) best_segs = std::max(1, std::min(a.ksteps, std::atoi(esg)));
    a.seg_steps = (a.ksteps + best_segs - 1) / best_segs;
    a.segs = (a.ksteps + a.seg_steps - 1) / a.seg_steps;
    const long long blocks = cols * a.segs;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
#ifdef MIPX_PROBES
    if (tune_env("MIPX_BCOL_DBG"))
        fprintf(stderr, "k_bcol b=%d upw=%d a16=%d nks=%d kmax=%d taps=%d sxb=%d spb=%d e=%d sd=%d kb0=%d rsd=%d tw=%d ring=%d lds=%zu per_cu=%d strips=%d segs=%d seg_steps=%d pre=%d blocks=%lld\n",
                b, upw, a.a16, nks, kmax, taps, a.sxb, a.spb, e, a.sd, a.kb0, a.rsd, a.tw, ring, lds, per_cu, a.strips, a.segs,
                a.seg_steps, a.pre, blocks);
#endif
    hipLaunchKernelGGL(reinterpret_cast<void (*)(BcArgs)>(const_cast<void *>(fn)), dim3(static_cast<unsigned>(blocks)),
                       dim3(kBcNT), lds, st, a);
    return launch_check("k_bcol");
}

}  // namespace mipx
