// k_rstrip.hip — libvips vips_reduce (reducev -> reduceh, Lanczos3) for ANY
// shrink pair in one launch, streaming: the uchar intermediate lives in LDS.
//
// libvips runs reducev, materialises the rounded uchar image, then reduceh
// (reduce.c; restated in oracle/vips_ref.c ref_reduce).  Two separate passes
// move in + 2 x intermediate + out bytes through HBM; for a 1.6 shrink that is
// 1.9x the compulsory traffic.  Here one workgroup owns a STRIP of TW output
// columns and walks DOWN a band of output rows, R rows per chunk:
//
//  * input rows: every lane prefetches 16 bytes of the next chunk's new rows
//    into registers while the current chunk computes (loads counted by the
//    compiler, so stores in between stay in flight), then writes them to an
//    LDS row ring once the vertical pass no longer reads the slots;
//  * vertical pass: lane = one unit of 4 pixels (B dwords), wave = two
//    adjacent output rows that share every tap pair: each byte pair of input
//    rows (2j, 2j+1) is packed once (v_perm) and dotted (int16 v_dot2, exact
//    integer sums) with each row's taps at that alignment; (sum + 2048) >> 12
//    clipped, written to LDS as one u32 slot per pixel;
//  * horizontal pass: lane = one output pixel, its tap pairs held in
//    registers, two slots per ds_read2, B dot2 per tap pair.
// Every output is the same integer sum over the same uchar intermediate as the
// two passes and the oracle: bit-exact.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "device_common.h"

namespace mipx {
namespace {

using namespace dev;

constexpr int kRsThreads = 256;
constexpr int kRsR = 8;          // output rows per chunk: two per wave in the vertical pass
constexpr int kRsPF = 6;         // prefetched rows per wave and chunk (chunk input rows <= 4 * kRsPF)
constexpr int kRsMaxTP = 12;     // tap pairs held per lane / row (taps <= 23)

typedef short short2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int dot2(uint32_t pr, uint32_t cw, int acc) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, pr), __builtin_bit_cast(short2v, cw), acc, false);
}
// byte z of lo / hi as an int16 pair [lo.z, hi.z]
__device__ __forceinline__ uint32_t pair_z(uint32_t lo, uint32_t hi, int z) {
    return __builtin_amdgcn_perm(hi, lo, 0x0C040C00u + 0x00010001u * static_cast<uint32_t>(z));
}
// (sum + 2048) >> 12 clipped; the asm barrier keeps the backend from fusing
// shift + clamp + packing into v_ashr_pk_u8_i32 (see k_sep.hip fixed_round_i)
__device__ __forceinline__ uint32_t rnd12(int sum) {
    int v = clampi((sum + 2048) >> 12, 0, 255);
    asm("" : "+v"(v));
    return static_cast<uint32_t>(v);
}
// libvips reduce geometry: output o samples X = o * shrink, taps from
// floor(X) - (n/2 - 1), phase ((int(X * 256) & 255) + 1) >> 1 (reduceh.cpp)
__device__ __forceinline__ void rs_position(double shrink, int pad, int o, int *start, int *phase, int centre) {
    const double X = reduce_x(o, shrink, centre);
    *start = static_cast<int>(X) - pad;
    *phase = ((static_cast<int>(X * 256.0) & 255) + 1) >> 1;
}

struct RsArgs {
    const u8 *in;
    u8 *out;
    int w, h, pitch;             // input image (pitch = w * B)
    long long in_img, out_img;
    int ox0, oy0, ow, oh;        // output window in reduce-output coordinates
    int band;                    // output rows per band (multiple of kRsR)
    int n_strips, n_bands;
    int rs;                      // ring row stride, dwords (multiple of 4)
    int ring;                    // ring rows
    int ns;                      // intermediate slots per row (u32 per pixel)
    int tv, th, padv, padh;
    int tpav, tpah;              // pair-table width (taps / 2 + 1)
    double vs, hs;
    int centre;                  // centre sampling convention (mipx_set_reduce_sampling)
    const uint32_t *vpairs, *hpairs;  // [129][2][tpa] int16 tap pairs
};

__device__ __forceinline__ int ring_slot(int p, int ring) {
    int s = p % ring;
    return s < 0 ? s + ring : s;
}

// Workgroup barrier for LDS hand-offs only: __syncthreads() would also make
// every wave wait for its outstanding global stores (vmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int B, bool SK, int TW>
__global__ void __launch_bounds__(kRsThreads) k_rstrip(RsArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t rsm[];
    uint32_t *ringb = rsm;                                   // ring x rs dwords
    uint32_t *mid = ringb + a.ring * a.rs;                   // kRsR x ns slots
    uint32_t *vtl = mid + kRsR * a.ns;                       // [129][2][tpav] vertical tap pairs
    int *skew = reinterpret_cast<int *>(vtl + (kTransformScale + 1) * 2 * a.tpav);  // ring entries (SK)
    const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
    const int strip = t % a.n_strips;
    const int rest = t / a.n_strips;
    const int bandi = rest % a.n_bands;
    const int img = rest / a.n_bands;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    // ---- column geometry of this strip ----
    const int x0 = strip * TW;
    const int nx = min(TW, a.ow - x0);
    int lo, hi, ph;
    rs_position(a.hs, a.padh, a.ox0 + x0, &lo, &ph, a.centre);
    rs_position(a.hs, a.padh, a.ox0 + x0 + nx - 1, &hi, &ph, a.centre);
    hi += a.th - 1;
    const int org = lo & ~3;                            // pixel of slot 0 (floor to 4)
    const int cl4 = max(lo, 0) & ~3;                     // first staged pixel
    const int ch = min(hi, a.w - 1);                     // last real pixel needed
    const int nu = (ch - cl4) / 4 + 1;                   // 4-pixel units staged
    const int slot0 = cl4 - org;                         // slot of the first staged pixel

    // ---- row geometry of this band ----
    const int yb0 = bandi * a.band;
    const int yb1 = min(yb0 + a.band, a.oh);
    const int tpv = (a.tv + 2) >> 1;                     // pairs a row can touch at either alignment
    auto first_pos = [&](int y) {
        int s, p;
        rs_position(a.vs, a.padv, a.oy0 + y, &s, &p, a.centre);
        return s;
    };
    auto end_pos = [&](int y0c) {  // exclusive end of the input positions chunk y0c reads
        const int last = min(y0c + kRsR, yb1) - 1;
        const int s = first_pos(last);
        return 2 * ((s >> 1) + tpv);                     // through the last aligned pair
    };

    int delta = 0;
    // img is block-uniform, but the compiler's divergence analysis lost that and wrapped every
    // staging load in a readfirstlane waterfall loop over the descriptor; say so explicitly
    const __amdgpu_buffer_rsrc_t rsrc =
        image_rsrc_aligned(a.in + static_cast<long long>(__builtin_amdgcn_readfirstlane(img)) * a.in_img, a.in_img, &delta);
    // ---- row staging: wave w fetches rows p0 + w, p0 + w + 4, ... (lane: 16 bytes) ----
    uint4 pf[kRsPF];
    auto row_off = [&](int p) {
        const int r = clampi(p, 0, a.h - 1);
        return delta + static_cast<long long>(r) * a.pitch + static_cast<long long>(B) * cl4;
    };
    auto fetch = [&](int p0, int p1) {
#pragma unroll
        for (int i = 0; i < kRsPF; ++i) {
            const int p = min(p0 + wave + 4 * i, p1 - 1);  // past the end: a duplicate row, never committed
            const int a4 = static_cast<int>(row_off(p) & ~3LL);
            pf[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, a4 + 16 * lane, 0, 0));
        }
    };
    auto commit = [&](int p0, int p1) {
#pragma unroll
        for (int i = 0; i < kRsPF; ++i) {
            const int p = p0 + wave + 4 * i;
            if (p < p1) {
                const int slot = ring_slot(p, a.ring);
                if (4 * lane < a.rs) *reinterpret_cast<uint4 *>(ringb + slot * a.rs + 4 * lane) = pf[i];
                if (SK && lane == 0) skew[slot] = static_cast<int>(row_off(p) & 3);
            }
        }
    };

    // this lane's horizontal taps (output column x0 + tid % TW), int16 pairs
    constexpr int HG = kRsThreads / TW;                  // output rows per horizontal pass
    const int xl = tid % TW;
    const int hrow0 = tid / TW;
    int hbase = 0;
    uint32_t hc[kRsMaxTP];
    {
        int s, p;
        rs_position(a.hs, a.padh, a.ox0 + x0 + min(xl, nx - 1), &s, &p, a.centre);
        hbase = s - org;
        const uint32_t *c = a.hpairs + static_cast<size_t>(p) * 2 * a.tpah;  // alignment 0
#pragma unroll
        for (int m = 0; m < kRsMaxTP; ++m) hc[m] = c[min(m, a.tpah - 1)];
#pragma unroll
        for (int m = 0; m < kRsMaxTP; ++m) hc[m] = m < a.tpah ? hc[m] : 0u;
    }
    const int tph = (a.th + 1) >> 1;
    const bool edge_l = lo < 0, edge_r = hi > a.w - 1;

    for (int i = tid; i < (kTransformScale + 1) * 2 * a.tpav; i += kRsThreads) vtl[i] = a.vpairs[i];
    // ---- prologue: the first chunk's rows (from an even position: pairs are
    // aligned), in rounds of 4 * kRsPF ----
    int loaded = first_pos(yb0) & ~1;
    {
        const int e0 = end_pos(yb0);
        for (int p = loaded; p < e0; p += 4 * kRsPF) {
            const int p1 = min(p + 4 * kRsPF, e0);
            fetch(p, p1);
            commit(p, p1);
        }
        loaded = e0;
    }
    lds_barrier();
    int nxt_end = loaded;
    if (yb0 + kRsR < yb1) {
        nxt_end = end_pos(yb0 + kRsR);
        fetch(loaded, nxt_end);
    }

    for (int yc = yb0; yc < yb1; yc += kRsR) {
        // ---- vertical pass: wave w -> intermediate rows yc + 2w, yc + 2w + 1 ----
        {  // vertical pass
            const int k0 = 2 * wave;
            const int y0r = yc + k0;
            if (y0r < yb1) {
                const bool two = y0r + 1 < yb1;
                int s0, p0, s1, p1;
                rs_position(a.vs, a.padv, a.oy0 + y0r, &s0, &p0, a.centre);
                rs_position(a.vs, a.padv, a.oy0 + y0r + (two ? 1 : 0), &s1, &p1, a.centre);
                const int j0 = s0 >> 1;                      // first aligned pair (2j0, 2j0 + 1)
                const int d1 = (s1 >> 1) - j0;               // row 1's first pair, relative (0..2)
                const int np = d1 + tpv;                     // pairs either row touches
                // tap pairs at each row's alignment (LDS table, wave-uniform broadcast reads)
                const uint32_t *c0 = vtl + (p0 * 2 + (s0 & 1)) * a.tpav;
                const uint32_t *c1 = vtl + (p1 * 2 + (s1 & 1)) * a.tpav - d1;
                const int sj = ring_slot(2 * j0, a.ring);
                const int u = lane;  // nu <= 64 (launcher)
                if (u < nu) {
                    int acc0[B][4], acc1[B][4];
#pragma unroll
                    for (int d = 0; d < B; ++d)
#pragma unroll
                        for (int z = 0; z < 4; ++z) acc0[d][z] = acc1[d][z] = 0;
                    int sa = sj;
#pragma unroll
                    for (int m = 0; m < kRsMaxTP + 2; ++m) {
                        if (m < np) {
                            int sb = sa + 1;
                            if (sb >= a.ring) sb -= a.ring;
                            const uint32_t *ra = ringb + sa * a.rs + B * u;
                            const uint32_t *rb = ringb + sb * a.rs + B * u;
                            uint32_t va[B], vb[B];
                            if (SK) {
                                const int ka = skew[sa], kb = skew[sb];
#pragma unroll
                                for (int d = 0; d < B; ++d) {
                                    va[d] = __builtin_amdgcn_alignbyte(ra[d + 1], ra[d], ka);
                                    vb[d] = __builtin_amdgcn_alignbyte(rb[d + 1], rb[d], kb);
                                }
                            } else if (B == 4) {
                                const uint4 qa = *reinterpret_cast<const uint4 *>(ra);
                                const uint4 qb = *reinterpret_cast<const uint4 *>(rb);
                                va[0] = qa.x, va[1 % B] = qa.y, va[2 % B] = qa.z, va[3 % B] = qa.w;
                                vb[0] = qb.x, vb[1 % B] = qb.y, vb[2 % B] = qb.z, vb[3 % B] = qb.w;
                            } else {
#pragma unroll
                                for (int d = 0; d < B; ++d) va[d] = ra[d], vb[d] = rb[d];
                            }
                            // taps outside a row's window are 0: every pair is dotted with
                            // both rows unconditionally (a predicated accumulate costs a
                            // v_cndmask + v_mov per dot2)
                            const bool r0 = m < tpv, r1 = two && m >= d1;
                            const uint32_t t0 = c0[min(m, tpv - 1)], t1 = c1[max(m, d1)];
                            const uint32_t cw0 = r0 ? t0 : 0u, cw1 = r1 ? t1 : 0u;
#pragma unroll
                            for (int d = 0; d < B; ++d)
#pragma unroll
                                for (int z = 0; z < 4; ++z) {
                                    const uint32_t pr = pair_z(va[d], vb[d], z);
                                    acc0[d][z] = dot2(pr, cw0, acc0[d][z]);
                                    acc1[d][z] = dot2(pr, cw1, acc1[d][z]);
                                }
                            sa = sb + 1;
                            if (sa >= a.ring) sa -= a.ring;
                        }
                    }
                    // rounded bytes -> 4 pixel slots per row
#pragma unroll
                    for (int rr = 0; rr < 2; ++rr) {
                        if (rr == 1 && !two) break;
                        uint32_t dw[B];
#pragma unroll
                        for (int d = 0; d < B; ++d) {
                            const int *ac = rr ? acc1[d] : acc0[d];
                            dw[d] = rnd12(ac[0]) | (rnd12(ac[1]) << 8) | (rnd12(ac[2]) << 16) | (rnd12(ac[3]) << 24);
                        }
                        uint4 px;
                        if (B == 4) {
                            px = uint4{dw[0], dw[1 % B], dw[2 % B], dw[3 % B]};
                        } else if (B == 3) {
                            px = uint4{__builtin_amdgcn_perm(dw[1 % B], dw[0], 0x0C020100u),
                                       __builtin_amdgcn_perm(dw[1 % B], dw[0], 0x0C050403u),
                                       __builtin_amdgcn_perm(dw[2 % B], dw[1 % B], 0x0C040302u),
                                       __builtin_amdgcn_perm(dw[2 % B], dw[2 % B], 0x0C030201u)};
                        } else if (B == 2) {
                            px = uint4{dw[0] & 0xffffu, dw[0] >> 16, dw[B - 1] & 0xffffu, dw[B - 1] >> 16};
                        } else {
                            px = uint4{dw[0] & 0xffu, (dw[0] >> 8) & 0xffu, (dw[0] >> 16) & 0xffu, dw[0] >> 24};
                        }
                        *reinterpret_cast<uint4 *>(mid + (k0 + rr) * a.ns + slot0 + 4 * u) = px;
                    }
                }
            }
        }
        lds_barrier();  // [A] intermediate rows ready; the ring slots are free for the next rows
        if (edge_l || edge_r) {  // EXTEND_COPY: slots outside [0, w) repeat the edge pixel
            const int nl = edge_l ? -org : 0;                       // slots [0, -org) -> slot of pixel 0
            const int nr = edge_r ? hi - (a.w - 1) : 0;             // pixels w .. hi -> pixel w - 1
            const int per = nl + nr;
            for (int i = tid; i < kRsR * per; i += kRsThreads) {
                const int k = i / per, f = i - k * per;
                uint32_t *row = mid + k * a.ns;
                if (f < nl) row[f] = row[-org];
                else row[a.w - org + (f - nl)] = row[a.w - 1 - org];
            }
            lds_barrier();
        }
        // ---- horizontal pass: lane = output pixel x0 + xl of rows yc + hrow0 + HG i ----
        {  // horizontal pass
#pragma unroll
            for (int i = 0; i < kRsR / HG; ++i) {
                const int k = hrow0 + HG * i;
                const int y = yc + k;
                if (y >= yb1) break;  // uniform per wave (a wave never straddles rows: TW >= 64)
                const uint32_t *sp = mid + k * a.ns + hbase;
                int acc[B];
#pragma unroll
                for (int c = 0; c < B; ++c) acc[c] = 0;
#pragma unroll
                for (int m = 0; m < kRsMaxTP; ++m) {
                    if (m < tph) {
                        const uint32_t v0 = sp[2 * m], v1 = sp[2 * m + 1];
#pragma unroll
                        for (int c = 0; c < B; ++c) acc[c] = dot2(pair_z(v0, v1, c), hc[m], acc[c]);
                    }
                }
                uint32_t o = 0;
#pragma unroll
                for (int c = 0; c < B; ++c) o |= rnd12(acc[c]) << (8 * c);
                const int x = x0 + xl;
                u8 *q = a.out + img * a.out_img + (static_cast<long long>(y) * a.ow + x) * B;
                if (B == 3) {
                    // 4 lanes' pixels as 3 dwords (one ds_bpermute), bytes at partial groups
                    const uint32_t nb = __shfl_down(o, 1, 64);
                    const int j = xl & 3;
                    u8 *qg = q - 3 * j;
                    const bool full = (x | 3) < x0 + nx;
                    if (xl < nx) {
                        if (full && (reinterpret_cast<uintptr_t>(qg) & 3u) == 0) {
                            if (j < 3) {
                                const uint32_t wv = j == 0 ? (o | (nb << 24)) : j == 1 ? ((o >> 8) | (nb << 16))
                                                                                     : ((o >> 16) | (nb << 8));
                                *reinterpret_cast<uint32_t *>(qg + 4 * j) = wv;
                            }
                        } else {
                            q[0] = static_cast<u8>(o);
                            q[1] = static_cast<u8>(o >> 8);
                            q[2] = static_cast<u8>(o >> 16);
                        }
                    }
                } else if (xl < nx) {
                    if (B == 4) {
                        *reinterpret_cast<uint32_t *>(q) = o;
                    } else {
#pragma unroll
                        for (int c = 0; c < B; ++c) q[c] = static_cast<u8>(o >> (8 * c));
                    }
                }
            }
        }
        // ---- the next chunk's new rows: registers (fetched a chunk ago) -> ring ----
        if (yc + kRsR < yb1) {
            commit(loaded, nxt_end);
            loaded = nxt_end;
        }
        lds_barrier();  // [B]
        if (yc + 2 * kRsR < yb1) {  // prefetch the rows of the chunk after next
            nxt_end = end_pos(yc + 2 * kRsR);
            fetch(loaded, nxt_end);
        }
    }
}

}  // namespace

// Fused reduce of the output window [ox0, ox0 + ow) x [oy0, oy0 + oh);
// MIPX_EUNSUPPORTED when the masks or a strip do not fit (the caller then runs
// the separable passes).  MIPX_RSTRIP=0 disables it (A/B).
int reduce_strip_launch(const u8 *in, u8 *out, int n, int w, int h, int b, double hs, double vs, int ox0, int oy0,
                        int ow, int oh, hipStream_t st) {
    // Measured (profiles/r02/rstrip_ab.jsonl, same-box A/B against the separable
    // passes): faster on small images (364x273 / 480x270 RGB: -16 / -21 %), even at
    // 500x375, slower on large ones (1080p RGB / 1.6: +9 %), where both are VALU-
    // issue bound and the two passes keep more waves busy.  MIPX_RSTRIP=0/1 forces.
    const char *ef = tune_env("MIPX_RSTRIP");
    if (ef && *ef) {
        if (*ef == '0') return MIPX_EUNSUPPORTED;
    } else if (img_bytes(w, h, b) > 512 * 1024) {
        return MIPX_EUNSUPPORTED;
    }
    if (!(hs > 1.0) || !(vs > 1.0)) return MIPX_EUNSUPPORTED;
    if (b == 4 && (reinterpret_cast<uintptr_t>(out) & 3u)) return MIPX_EUNSUPPORTED;
    RsArgs a{};
    a.vpairs = device_reduce_pairs(vs, &a.tv, &a.tpav);
    a.hpairs = device_reduce_pairs(hs, &a.th, &a.tpah);
    if (!a.vpairs || !a.hpairs) return MIPX_EDEVICE;
    if (a.tpah > kRsMaxTP || a.tpav > kRsMaxTP) return MIPX_EUNSUPPORTED;
    // a chunk's new input rows must fit the prefetch registers (4 waves x kRsPF)
    if (static_cast<int>(std::ceil(kRsR * vs)) + 3 > 4 * kRsPF) return MIPX_EUNSUPPORTED;
    a.in = in;
    a.out = out;
    a.w = w;
    a.h = h;
    a.pitch = w * b;
    a.in_img = img_bytes(w, h, b);
    a.out_img = img_bytes(ow, oh, b);
    if (a.in_img + 64 >= 0x7fffffffLL) return MIPX_EUNSUPPORTED;
    a.ox0 = ox0;
    a.oy0 = oy0;
    a.ow = ow;
    a.oh = oh;
    a.padv = a.tv / 2 - 1;
    a.padh = a.th / 2 - 1;
    a.vs = vs;
    a.hs = hs;
    a.centre = reduce_centre();
    // every row of every image starts dword aligned: no per-row byte skew
    const bool sk = (a.pitch % 4) != 0 || (a.in_img % 4) != 0 || (reinterpret_cast<uintptr_t>(in) % 4) != 0;
    // strip width: 128 output pixels when the staged span fits 64 lanes x 16
    // bytes, else 64
    auto units_for = [&](int tw) {
        const int span = static_cast<int>(std::ceil((tw - 1) * hs)) + a.th + 2;
        return (span + 3 + 3) / 4 + 1;
    };
    const char *etw = tune_env("MIPX_RSTRIP_TW");
    int tw = (etw && *etw && std::atoi(etw) == 64) ? 64
             : (units_for(128) <= 64 && units_for(128) * b + 1 <= 256 ? 128 : 64);
    if (ow <= 64) tw = 64;
    const int nu_max = units_for(tw);
    const int ndw = nu_max * b + (sk ? 1 : 0);
    if (ndw > 256 || nu_max > 64) return MIPX_EUNSUPPORTED;  // one unit per lane, 16 staged bytes per lane
    a.rs = ((ndw + 3) / 4) * 4;
    a.ns = 4 * nu_max + 8;
    const int tpv = (a.tv + 2) / 2;
    // rows one chunk reads (through its last aligned pair) + one
    a.ring = static_cast<int>(std::ceil((kRsR - 1) * vs)) + 2 * tpv + 4;
    const char *eb = tune_env("MIPX_RSTRIP_BAND");
    int band = (eb && *eb) ? std::max(kRsR, std::atoi(eb) / kRsR * kRsR) : 64;
    band = std::min(band, ((oh + kRsR - 1) / kRsR) * kRsR);
    a.band = band;
    a.n_strips = (ow + tw - 1) / tw;
    a.n_bands = (oh + band - 1) / band;
    const size_t lds = (static_cast<size_t>(a.ring) * a.rs + kRsR * static_cast<size_t>(a.ns) +
                        static_cast<size_t>(kTransformScale + 1) * 2 * a.tpav + a.ring) * 4;
    if (lds > 64 * 1024) return MIPX_EUNSUPPORTED;
    const long long blocks = static_cast<long long>(a.n_strips) * a.n_bands * n;
    if (!grid_ok(blocks)) return MIPX_EINVAL;
    const dim3 grid(static_cast<unsigned>(blocks)), blk(kRsThreads);
#define MIPX_RS(SK_, TW_) MIPX_DISPATCH_BANDS(b, hipLaunchKernelGGL((k_rstrip<B_, SK_, TW_>), grid, blk, lds, st, a))
    if (sk) {
        if (tw == 128) { MIPX_RS(true, 128) } else { MIPX_RS(true, 64) }
    } else {
        if (tw == 128) { MIPX_RS(false, 128) } else { MIPX_RS(false, 64) }
    }
#undef MIPX_RS
    return launch_check("k_rstrip");
}

}  // namespace mipx
