// mipx_internal.h — shared declarations between the planner, the runtime and
// the gfx950 kernels of libmipx.so.  Not part of the ABI (see include/mipx.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "mipx.h"

namespace mipx {

// ---- errors -------------------------------------------------------------
void set_error(const char *fmt, ...);
int hip_fail(hipError_t e, const char *what);  // records detail, returns MIPX_EDEVICE
#define MIPX_HIP(call)                                                    \
    do {                                                                  \
        hipError_t e_ = (call);                                           \
        if (e_ != hipSuccess) return ::mipx::hip_fail(e_, #call);         \
    } while (0)

// ---- kernel-selection knobs (mipx_tuning.cpp) -------------------------------
// The MIPX_* environment variables as snapshotted on first use (or by
// mipx_tuning_reload): nullptr when unset.  Launchers call this, never getenv.
const char *tune_env(const char *name);
void tune_reload();
// The Lanczos reduce sampling convention (PARITY_ASSUMPTIONS.md row 1): under
// MIPX_SAMPLE_CENTRE output o samples (o + 0.5) * shrink - 0.5 (libvips' centre
// convention) instead of o * shrink.  reduce_centre() is what every reduce launcher and
// the demand-region walk read: the innermost SamplingScope of this thread, else the
// process setting (mipx_set_reduce_sampling).  execute_plan opens a scope with the
// convention each reduce / smartcrop step recorded at mipx_plan_make time (step a[7]), and
// the per-op entry points snapshot the process setting once per call, so one launch never
// mixes conventions.
bool reduce_centre();
int reduce_sampling_now();  // the process setting (what mipx_plan_make records)
class SamplingScope {
   public:
    explicit SamplingScope(int convention);  // this convention until the scope ends
    SamplingScope();                          // snapshot: the enclosing scope's, else the process setting
    ~SamplingScope();
    SamplingScope(const SamplingScope &) = delete;
    SamplingScope &operator=(const SamplingScope &) = delete;

   private:
    int prev_;
};
// requests submitted through mipx_submit and not yet retired (mipx_runtime.cpp)
long long requests_in_flight();
inline double reduce_x_host(int o, double s, bool centre) { return centre ? (o + 0.5) * s - 0.5 : o * s; }

// ---- device properties, cached per device (mipx_tuning.cpp) --------------------
// compute units of the current device (256 on an MI355X in SPX mode; fewer per
// partition in CPX / DPX modes)
int device_cu_count();
// resident workgroups per CU for kernel fn at `threads` threads and `lds` dynamic LDS
// bytes on the current device (hipOccupancyMaxActiveBlocksPerMultiprocessor, queried
// once per (device, fn, threads, lds)); `fallback` when the query fails
int occupancy_per_cu(const void *fn, int threads, size_t lds, int fallback);

// ---- device capability probes (k_probe.hip), run once per device -------------
// Do direct-to-LDS dword buffer loads honour byte offsets that are not multiples of 4?
bool lds_dma_unaligned_ok();

// ---- libvips resample constants (resample/templates.h, [U]) ----------------
constexpr int kTransformScale = 128;  // VIPS_TRANSFORM_SCALE: 129 sub-pixel phases
constexpr int kInterpShift = 12;      // VIPS_INTERPOLATE_SHIFT
constexpr int kInterpScale = 1 << kInterpShift;

// Lanczos3 reduce geometry (libvips reduceh.cpp / reducev.cpp).
int reduce_points(double shrink);                      // 2 * rint(3 * shrink) + 1
void reduce_table(double shrink, std::vector<int> &t); // 129 x n truncated 12-bit taps
int out_size_reduce(int in, double shrink);            // VIPS_ROUND(in / shrink)
int out_size_shrink(int in, int shrink);               // VIPS_ROUND(in / shrink)

// Integer gaussmat (libvips create/gaussmat.c): returns width, fills mask/scale.
int gaussmat(double sigma, double min_ampl, std::vector<int> &mask, int &scale);

// Colour LUTs for the smartcrop scorer (libvips colour/*.c, [U]).
constexpr int kQuantElements = 100000;
const float *v2y8_table();    // 256 entries: sRGB 8-bit -> linear
const float *cbrt_table();    // kQuantElements entries: Lab f(t)
const float *y2v8_table();    // 257 entries: linear Y x 255 -> sRGB 8-bit (B_W)
void bicubic_table(int *t);   // 129 x 4 bicubic taps (vips_affine)

// vips_resize() downsize schedule used by the smartcrop scorer.
struct ResizeSchedule {
    int shrink_h = 1, shrink_v = 1;    // integer box shrink
    double reduce_h = 1.0, reduce_v = 1.0;  // residual Lanczos3 (1.0 = none)
    int w1 = 0, h1 = 0;                // after shrink
    int w2 = 0, h2 = 0;                // after reduce
};
int resize_schedule(int w, int h, double hscale, double vscale, ResizeSchedule &s);

// ---- device-side cached tables ----------------------------------------------
// float copy of reduce_table(shrink) resident on the current device.
const float *device_reduce_table(double shrink, int *n_taps);
// the same taps packed as int16 pairs: [129][2 alignments][*tpa] (k_rstrip)
const uint32_t *device_reduce_pairs(double shrink, int *n_taps, int *tpa);
constexpr int kHmTabW = 64;     // k_hmfma i8 tap rows: bytes per (phase, hi / lo) row (16.5 KB: L1-resident)
constexpr int kHmTabPad = 16;   // zero bytes in front of tap 0 (taps <= 16; windows clamped to [-16, 16])
constexpr int kRsTabPad = 128;  // k_rmf4 stride-B tap rows: zero bytes in front of tap 0
constexpr int kRsTabW = 272;    // bytes per (phase, hi / lo) row: pad + 2 K steps + a fragment (70 KB per table)
const signed char *device_reduce_i8(double shrink, int *n_taps, const int **sums);
const signed char *device_reduce_i8s(double shrink, int bands, int *n_taps);  // taps at a byte stride of bands
// the same with the COPY edge folded in: [2 sides][taps - 1][129][hi, lo][kRsTabW] (k_rcol)
const signed char *device_reduce_i8s_fold(double shrink, int bands, int *n_taps);
// k_rcol's vertical plan (per output row: K-placed split taps + seed; per 16-row group:
// first / end input rows) over at least `rows` op-output rows; *cap_rows = rows it holds
constexpr int kRcolPlanRow = 144;
const uint8_t *device_rcol_vplan(double shrink, bool centre, int rows, int *cap_rows);
// k_rcol's horizontal operands of one window geometry, built on the host (r06): per 64-pixel
// strip, per 16-byte output unit u < 4 bands, per lane: per K step the hi / lo tap fragments
// (COPY edge folded, odd K blocks' halves swapped), then the four per-byte seeds,
// kRcolHopRec(nks) bytes; then per (strip, unit) the K origin (int).  The specialised k_rcol
// builds load these instead of computing the positions in the block's set-up.
constexpr int kRcolHopRec(int nks) { return 32 * nks + 16; }
const uint8_t *device_rcol_hops(double hs, int bands, bool centre, int ox0, int ow, int w, int k4, int nks, int *strips);
// k_bmf's i8 MFMA operands for a blur mask (cached per device): [nks][64][16]
// horizontal taps at byte stride `bands` shifted by delta, then [64][16] vertical taps
const signed char *device_blur_ops(const std::vector<int> &mask, int bands, int delta, int nks, int vperm);
const float *device_colour_tables();  // [256 v2y | kQuantElements cbrt | 257 y2v]
const int *device_bicubic_table();     // 129 x 4
// float copy of the integer gaussmat mask; *scale = mask sum
const float *device_gauss_table(double sigma, double min_ampl, int *n_taps, int *scale);
// `bytes` of host data on the current device, cached by contents (small constant tables)
const void *device_blob(const void *data, size_t bytes);
void free_device_tables();
// bumped by free_device_tables: a launcher that caches a table pointer outside the maps
// above keeps the generation it was made in and refetches when it changed
unsigned device_tables_generation();
// free_device_tables also frees every table k_enlm keeps per (device, scale) (k_affine.hip)
void free_enlm_tables();

// ---- generic separable passes (k_sep.hip) -----------------------------------
enum { kSepReduce = 0, kSepConv = 1 };
struct SepSpec {            // one 1-D integer mask family
    const float *tab;       // device table: reduce 129 x taps phases, conv 1 x taps
    int taps;
    int mode;               // kSepReduce / kSepConv
    double shrink;          // reduce
    int scale;              // conv: divisor (mask sum)
};
struct SepWindow {          // geometry of one pass over a batch of n images
    int bands;
    int in_pitch;           // bytes between input rows
    long long in_base;      // byte offset of the local input origin inside an image
    long long in_img;       // bytes per input image
    int in_len;             // local input length along the pass axis (COPY clamp)
    int o0;                 // first output position along the pass axis (op-output coords)
    int out_w, out_h;       // packed output image of the pass
};
bool sep_spec_reduce(double shrink, SepSpec *s);
bool sep_spec_gauss(double sigma, double min_ampl, SepSpec *s);
int vpass_launch(const uint8_t *in, uint8_t *out, int n, const SepSpec &spec, const SepWindow &w, hipStream_t st);
int hpass_launch(const uint8_t *in, uint8_t *out, int n, const SepSpec &spec, const SepWindow &w, hipStream_t st);
int reduce_fused_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, double hs, double vs, int ox0,
                        int oy0, int ow, int oh, hipStream_t st);
// k_rstrip.hip: streaming fused reduce (LDS row ring + LDS intermediate), any shrink pair
// both shrinks > 1 in one launch (k_rcol, else k_rmf2, else the strip walker, else the
// small-image fused kernel); MIPX_EUNSUPPORTED = run the two separable passes
int reduce_one_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, double hs, double vs, int ox0,
                      int oy0, int ow, int oh, hipStream_t st);
// k_bcol.hip: the column-walking gaussblur (both convsep passes on the matrix cores)
int blur_col_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, int left, int top, int ow, int oh,
                    const std::vector<int> &mask, int scale, hipStream_t st);
// k_rcol.hip: the column walker (LDS row ring, both passes on the matrix cores)
int reduce_col_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, double hs, double vs, int ox0,
                      int oy0, int ow, int oh, hipStream_t st);
int reduce_mfma_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, double hs, double vs, int ox0,
                       int oy0, int ow, int oh, hipStream_t st);
int reduce_strip_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, double hs, double vs, int ox0,
                        int oy0, int ow, int oh, hipStream_t st);

// ---- kernel launchers (k_*.hip); batches of n images packed back to back -----
// k_reduce.hip
int reducev_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, double vshrink, hipStream_t st);
int reduceh_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, double hshrink, hipStream_t st);
int reduce_window_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, double hs, double vs, int left,
                         int top, int ow, int oh, void *ws, size_t ws_bytes, hipStream_t st);
bool reduce2_eligible(const uint8_t *in, int w, int h, int b, double hs, double vs);
int reduce2_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, hipStream_t st);
int reduce2_window_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, int x0, int y0, int x1,
                          int y1, hipStream_t st);
// k_reduce2m.hip: the centre-convention 2 x 2 reduce with its vertical pass on the matrix
// cores; taps12 = matrixi[64][0..11]
int reduce2m_window_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, int x0, int y0, int x1,
                           int y1, const int *taps12, hipStream_t st);
// the corner convention's 2 x 2 mask as k_reduce2x2 uses it: c0, c1, c3, c5 (k_reduce.hip)
bool reduce2_taps(float c[4]);
// k_shrink.hip
int shrink_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, int hs, int vs, hipStream_t st);
int shrink_window_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, int hs, int vs, int x0, int y0,
                         int x1, int y1, hipStream_t st);
// k_geometry.hip
int embed_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, int x, int y, int ow, int oh,
                 int extend, const int *bg, const int *d_origins, hipStream_t st);
int flip_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, int vertical, hipStream_t st);
int rot_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, int angle, hipStream_t st);
int device_copy(void *dst, const void *src, size_t bytes, hipStream_t st);  // a batch, device to device
int extract_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, int left, int top, int ow, int oh,
                   hipStream_t st);
// k_blur.hip (ws: n * w * h * b bytes for the uchar intermediate)
int blur_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, double sigma, double min_ampl,
                void *ws, size_t ws_bytes, hipStream_t st);
int blur_window_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, int left, int top, int ow,
                       int oh, double sigma, double min_ampl, void *ws, size_t ws_bytes, hipStream_t st);
// k_affine.hip
int affine_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, double xs, double ys, int extend,
                  hipStream_t st);
int zoom_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, int xf, int yf, hipStream_t st);
// k_colour.hip
int flatten_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, const int *bg, hipStream_t st);
int bw_launch(const uint8_t *in, uint8_t *out, int n, int w, int h, int b, hipStream_t st);
// k_composite.hip
int watermark_launch(const uint8_t *base, const uint8_t *wm, uint8_t *out, int n, int w, int h, int bands, int ww,
                     int wh, int wb, int left, int top, float opacity, hipStream_t st);
// k_smartcrop.hip
size_t smartcrop_workspace_bytes(int n, int w, int h, int bands);
int smartcrop_origins(const uint8_t *in, int *origins, int n, int w, int h, int b, int cw, int ch, void *ws,
                      size_t ws_bytes, hipStream_t st);
int smartcrop_extract(const uint8_t *in, uint8_t *out, int n, int w, int h, int bands, int cw, int ch, void *ws,
                      size_t ws_bytes, hipStream_t st);
// mipx_ops.cpp
size_t op_workspace_bytes(int op, int n, int w, int h, int bands, double p0, double p1);

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace mipx
