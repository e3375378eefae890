// vcf_dwt.hip -- 2D-DWT + deadzone encode and decode (src/2D-DWT.py) for
// gfx950, and the vcf_dwt_* entry points of the C ABI.
//
// What is computed (bit-exact to oracle/vcf_dwt_oracle.cpp, which is pinned
// to pywt 1.1.1 and the reference's own files):
//   encode 2D-DWT.py:57-78: int16 YCoCg (truncating store, A4), per channel
//     pywt.wavedec2(mode='per') in float64 (A6), deadzone (x/Q).astype(int32)
//     per subband (A5), LL + 128 -> u16, details + 128 -> u8 (wrap);
//   decode 2D-DWT.py:80-101: u16/u8 -> int16 - 128, Q*k in int16, waverec2
//     (float64), float64 to_RGB, clip, u8.
// The tap order of every output is pywt's (see the oracle's header): the
// forward tail outputs add their end-wrapped taps first in descending order,
// the inverse accumulates one product at a time, approximation then detail,
// and its first F/4 pair indices take the wrapped taps first, descending.
//
// Layout: a frame's coded subbands are packed back to back in
// the order the reference writes its files -- LL_L (u16, h_L x w_L x 3), then
// for r = L..1: LH_r, HL_r, HH_r (u8, h_r x w_r x 3) -- channels interleaved
// like the arrays the reference hands to its TIFF writer.  Intermediate
// planes (float64, one per frame and channel) live in a caller workspace.
//
// Kernels (one thread per output sample, HBM-bound at float64): per level a
// column pass (axis 0) writing the approximation/detail planes, then a row
// pass (axis 1) that quantizes the three detail subbands straight into the
// packed output and keeps LL in float64 for the next level; the inverse runs
// rows then columns per level and a final YCoCg->RGB kernel.
#include <hip/hip_runtime.h>

#include <atomic>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>

#include "vcf_amd.h"
#include "vcf_internal.h"
#include "vcf_pipeline.h"
#include "vcf_wavelets.h"

namespace vcf {
namespace {

constexpr int kMaxLevels = 30;

struct DwtGeom {
    int H, W, levels, F;
    int hs[kMaxLevels + 1], ws[kMaxLevels + 1];   // [0] = H, W; [l] = level-l subband shape
    long long sb_off[kMaxLevels + 1][3];           // packed byte offsets of LH/HL/HH of level l
    long long ll_off, packed_bytes;
};

void dwt_geom(int H, int W, int levels, int F, DwtGeom &g)
{
    g.H = H;
    g.W = W;
    g.levels = levels;
    g.F = F;
    g.hs[0] = H;
    g.ws[0] = W;
    for (int l = 1; l <= levels; ++l) {
        g.hs[l] = (g.hs[l - 1] + 1) / 2;
        g.ws[l] = (g.ws[l - 1] + 1) / 2;
    }
    g.ll_off = 0;
    long long off = 2LL * g.hs[levels] * g.ws[levels] * 3;
    for (int r = levels; r >= 1; --r)
        for (int s = 0; s < 3; ++s) {
            g.sb_off[r][s] = off;
            off += 3LL * g.hs[r] * g.ws[r];
        }
    g.packed_bytes = off;
}

// workspace per (frame, channel): two column-pass planes (ceil(h/2) x w) and
// two LL ping-pong planes (h_1 x w_1) -- enough for every level, both ways
long long plane_doubles(const DwtGeom &g)
{
    const long long col = (long long)g.hs[1] * g.ws[0];              // encode: A / D
    const long long inv = (long long)g.hs[1] * 2 * g.ws[1];          // decode: 'a' / 'd' rows
    const long long ll = (long long)2 * g.hs[1] * 2 * g.ws[1];       // reconstructed plane
    return 2 * std::max(col, inv) + 2 * ll;
}

// ---------------------------------------------------------------------------
// 1-D kernels of pywt's C code, one output at a time (device)
// ---------------------------------------------------------------------------
// forward 'per': output position i = F/2 + 2o of a line x[k*xs] of length N
template <typename Load>
__device__ __forceinline__ double dwt_tap_sum(const double *__restrict__ f, int F, int N, int i, Load &&load)
{
    const int Ne = N + (N & 1);
    auto at = [&](int p) -> double {
        p %= Ne;
        if (p < 0) p += Ne;
        return load(p < N ? p : N - 1);
    };
    double s = 0.0;
    if (i >= N) {
        for (int m = F - 1; m >= 0; --m)
            if (i - m >= N) s = s + f[m] * at(i - m);
        for (int m = 0; m < F; ++m)
            if (i - m < N) s = s + f[m] * at(i - m);
    } else {
        for (int m = 0; m < F; ++m) s = s + f[m] * at(i - m);
    }
    return s;
}

// pywt's order of the taps of input index i (0 <= i < N) in the inverse: the
// first T = F2/2 indices take taps top..0 descending, then top+1..F2-1; the
// others ascending.  top = the largest i + kN below T -- i itself unless the
// line is shorter than T (pywt's short-input branch wraps the input around
// more than once; checked against pywt 1.1.1 for every discrete wavelet and
// every N <= F2 + 3, tests/golden/make_golden_dwt_short.py)
__host__ __device__ __forceinline__ int idwt_top(int i, int N, int T)
{
    return i + N * ((T - 1 - i) / N);
}

// inverse 'per': output n (0 <= n < 2N) of idwt(a, d): the one input index i
// feeding it, then approximation taps and detail taps accumulated one product
// at a time (pywt: output zeroed, += per product, cA pass then cD pass)
template <typename LoadA, typename LoadD>
__device__ __forceinline__ double idwt_out(const double *__restrict__ lo, const double *__restrict__ hi, int F,
                                           int N, int n, LoadA &&la, LoadD &&ld)
{
    const int F2 = F / 2, shift = 1 - F2, T = F2 / 2;
    int q = n - shift;                     // = 2i + p (mod 2N)
    q %= 2 * N;
    if (q < 0) q += 2 * N;
    const int p = q & 1, i = q >> 1;
    const int top = i < T ? idwt_top(i, N, T) : 0;
    double s = 0.0;
    for (int pass = 0; pass < 2; ++pass) {
        const double *f = pass ? hi : lo;
        for (int t = 0; t < F2; ++t) {
            const int j = (i < T) ? (t <= top ? top - t : t) : t;
            int k = (i - j) % N;
            if (k < 0) k += N;
            const double c = pass ? ld(k) : la(k);
            s = s + f[2 * j + p] * c;
        }
    }
    return s;
}

// x / Q, correctly rounded as numpy divides.  For a power-of-two Q the
// quotient is an exact power-of-two scaling, which v_ldexp_f64 also rounds
// correctly: the same double without the ~12-instruction float64 division
// sequence (a sixth of the level-1 forward kernel's VALU instructions).
__device__ __forceinline__ double div_q(double x, int Q)
{
    return (Q & (Q - 1)) == 0 ? __builtin_ldexp(x, -__builtin_ctz((unsigned)Q)) : x / (double)Q;
}

__device__ __forceinline__ uint8_t quant_u8(double x, int Q)
{
    const int32_t k = (int32_t)div_q(x, Q);         // astype(int32): truncation toward zero
    return (uint8_t)(uint32_t)(k + 128);            // += 128, astype(uint8): wraps
}

__device__ __forceinline__ uint16_t quant_u16(double x, int Q)
{
    const int32_t k = (int32_t)div_q(x, Q);
    return (uint16_t)(uint32_t)(k + 128);
}

__device__ __forceinline__ double dequant(int16_t k, int Q)
{
    k = (int16_t)(k - 128);                                              // astype(int16) - 128
    return (double)(int16_t)(uint16_t)((uint32_t)Q * (uint32_t)(int32_t)k);  // Q * k in int16
}

struct Filters {
    const double *dec_lo, *dec_hi, *rec_lo, *rec_hi;
};

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
// Column pass of level l: plane (h x w) -> A, D (ceil(h/2) x w).  Level 1
// reads the RGB frame and forms the int16 YCoCg sample (A4) on the fly.
template <bool FIRST>
__global__ __launch_bounds__(256) void dwt_cols_kernel(const uint8_t *__restrict__ rgb, long long rgb_stride,
                                                       const double *__restrict__ in, long long plane_stride,
                                                       double *__restrict__ A, double *__restrict__ D,
                                                       long long ws_stride, int h, int w, int F, Filters flt)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    const int o = blockIdx.y;
    const int plane = blockIdx.z;             // frame * 3 + channel
    if (c >= w) return;
    const int ch = plane % 3;
    const long long frame = plane / 3;
    const int i = F / 2 + 2 * o;
    auto load = [&](int y) -> double {
        if (FIRST) {
            const uint8_t *px = rgb + frame * rgb_stride + ((long long)y * w + c) * 3;
            const double R = px[0], G = px[1], B = px[2];
            double v;
            if (ch == 0) v = R / 4 + G / 2 + B / 4;
            else if (ch == 1) v = R / 2 - B / 2;
            else v = -R / 4 + G / 2 - B / 4;
            return (double)(int16_t)v;        // empty_like(int16) store
        } else {
            return in[plane * plane_stride + (long long)y * w + c];
        }
    };
    const long long out = plane * ws_stride + (long long)o * w + c;
    A[out] = dwt_tap_sum(flt.dec_lo, F, h, i, load);
    D[out] = dwt_tap_sum(flt.dec_hi, F, h, i, load);
}

// Row pass of level l: A, D (hh x w) -> aa (kept, or quantized at the last
// level), da -> LH, ad -> HL, dd -> HH quantized into the packed output.
template <bool LAST>
__global__ __launch_bounds__(256) void dwt_rows_kernel(const double *__restrict__ A, const double *__restrict__ D,
                                                       long long ws_stride, double *__restrict__ LLout,
                                                       long long plane_stride, uint8_t *__restrict__ packed,
                                                       long long packed_stride, long long ll_off,
                                                       long long off_lh, long long off_hl, long long off_hh,
                                                       int hh, int w, int hw, int F, int Q, Filters flt)
{
    const int o = blockIdx.x * blockDim.x + threadIdx.x;
    const int r = blockIdx.y;
    const int plane = blockIdx.z;
    if (o >= hw) return;
    const int ch = plane % 3;
    const long long frame = plane / 3;
    const int i = F / 2 + 2 * o;
    const double *a = A + plane * ws_stride + (long long)r * w;
    const double *d = D + plane * ws_stride + (long long)r * w;
    auto la = [&](int k) -> double { return a[k]; };
    auto ld = [&](int k) -> double { return d[k]; };
    const double aa = dwt_tap_sum(flt.dec_lo, F, w, i, la);
    const double ad = dwt_tap_sum(flt.dec_hi, F, w, i, la);
    const double da = dwt_tap_sum(flt.dec_lo, F, w, i, ld);
    const double dd = dwt_tap_sum(flt.dec_hi, F, w, i, ld);
    uint8_t *pk = packed + frame * packed_stride;
    const long long e = ((long long)r * hw + o) * 3 + ch;
    pk[off_lh + e] = quant_u8(da, Q);   // cH ('da') -> LH
    pk[off_hl + e] = quant_u8(ad, Q);   // cV ('ad') -> HL
    pk[off_hh + e] = quant_u8(dd, Q);   // cD ('dd') -> HH
    if (LAST) {
        const uint16_t v = quant_u16(aa, Q);
        uint8_t *q = pk + ll_off + e * 2;
        q[0] = (uint8_t)v;
        q[1] = (uint8_t)(v >> 8);
    } else {
        LLout[plane * plane_stride + (long long)r * hw + o] = aa;
    }
}

// ---------------------------------------------------------------------------
// inverse
// ---------------------------------------------------------------------------
// Row pass of level r: aa (trimmed to h x w: level L from the packed LL,
// else the previous reconstruction with row stride lda), ad, da, dd from the
// packed file bytes -> 'a', 'd' rows (h x 2w).
template <bool FROM_PACKED_LL>
__global__ __launch_bounds__(256) void idwt_rows_kernel(const uint8_t *__restrict__ packed, long long packed_stride,
                                                        long long ll_off, long long off_lh, long long off_hl,
                                                        long long off_hh, const double *__restrict__ prev,
                                                        long long plane_stride, int lda, double *__restrict__ Aout,
                                                        double *__restrict__ Dout, long long ws_stride, int h,
                                                        int w, int F, int Q, Filters flt)
{
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    const int r = blockIdx.y;
    const int plane = blockIdx.z;
    if (n >= 2 * w) return;
    const int ch = plane % 3;
    const long long frame = plane / 3;
    const uint8_t *pk = packed + frame * packed_stride;
    const long long row = (long long)r * w;
    auto sb = [&](long long off, int k) -> double { return dequant((int16_t)pk[off + (row + k) * 3 + ch], Q); };
    auto laa = [&](int k) -> double {
        if (FROM_PACKED_LL) {
            const uint8_t *q = pk + ll_off + ((row + k) * 3 + ch) * 2;
            return dequant((int16_t)(uint16_t)(q[0] | (q[1] << 8)), Q);
        }
        return prev[plane * plane_stride + (long long)r * lda + k];
    };
    auto lad = [&](int k) -> double { return sb(off_hl, k); };   // 'ad' = cV = HL
    auto lda_ = [&](int k) -> double { return sb(off_lh, k); };  // 'da' = cH = LH
    auto ldd = [&](int k) -> double { return sb(off_hh, k); };   // 'dd' = cD = HH
    const long long out = plane * ws_stride + (long long)r * 2 * w + n;
    Aout[out] = idwt_out(flt.rec_lo, flt.rec_hi, F, w, n, laa, lad);
    Dout[out] = idwt_out(flt.rec_lo, flt.rec_hi, F, w, n, lda_, ldd);
}

// Column pass of level r: 'a', 'd' (h x w2) -> plane (2h x w2)
__global__ __launch_bounds__(256) void idwt_cols_kernel(const double *__restrict__ Ain, const double *__restrict__ Din,
                                                        long long ws_stride, double *__restrict__ out,
                                                        long long plane_stride, int h, int w2, int F, Filters flt)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = blockIdx.y;
    const int plane = blockIdx.z;
    if (c >= w2) return;
    const double *a = Ain + plane * ws_stride + c;
    const double *d = Din + plane * ws_stride + c;
    auto la = [&](int k) -> double { return a[(long long)k * w2]; };
    auto ld = [&](int k) -> double { return d[(long long)k * w2]; };
    out[plane * plane_stride + (long long)n * w2 + c] = idwt_out(flt.rec_lo, flt.rec_hi, F, h, n, la, ld);
}

// to_RGB (float64, A4) + clip + astype(uint8)
__global__ __launch_bounds__(256) void dwt_to_rgb_kernel(const double *__restrict__ planes, long long plane_stride,
                                                         uint8_t *__restrict__ rgb, long long npx, long long out_stride)
{
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long frame = blockIdx.y;
    if (p >= npx) return;
    const double Y = planes[(frame * 3 + 0) * plane_stride + p];
    const double Co = planes[(frame * 3 + 1) * plane_stride + p];
    const double Cg = planes[(frame * 3 + 2) * plane_stride + p];
    const double v[3] = {Y + Co - Cg, Y + Cg, Y - Co - Cg};
    uint8_t *o = rgb + frame * out_stride + p * 3;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double c = v[k] < 0.0 ? 0.0 : (v[k] > 255.0 ? 255.0 : v[k]);
        o[k] = (uint8_t)c;
    }
}

// ---------------------------------------------------------------------------
// fused level kernels (filters of at most kMaxFastF taps)
// ---------------------------------------------------------------------------
// One launch per level.  A workgroup owns a tile of a level's outputs, stages
// the input samples it needs (halo included, wrapped at load time) in LDS,
// runs both separable passes there and writes only the level's products:
// forward, the three quantized detail subbands (packed bytes) and LL (float64
// plane for the next level, or u16 at the last); inverse, the next level's
// float64 plane trimmed to what that level reads, or RGB at level 1.  The
// column-pass planes of the separable kernels never touch HBM.
//
// Every output sums its taps in exactly the order of dwt_tap_sum / idwt_out
// above: the tile holds samples at *logical* positions (before the periodic
// wrap), so only the index arithmetic differs.
constexpr int kFTH = 8;              // forward: output rows per tile
constexpr int kFIW = 128;            // forward: staged input columns, 2 (tw - 1) + F
constexpr int kITH = 16, kITW = 64;  // inverse: output tile (level samples)
constexpr int kG = 4;                // outputs per work item (register window)
constexpr int kMaxFastF = 18;        // longest filter with a compiled fast path

__host__ __device__ constexpr int fwd_tile_w(int F) { return (kFIW - F) / 2 + 1; }

// forward 'per' wrap of a logical sample position (odd N: extended by x[N-1])
__device__ __forceinline__ int per_wrap(int p, int N)
{
    const int Ne = N + (N & 1);
    p %= Ne;
    if (p < 0) p += Ne;
    return p < N ? p : N - 1;
}

__device__ __forceinline__ int mod_pos(int p, int N)
{
    p %= N;
    return p < 0 ? p + N : p;
}

// dwt_tap_sum with the load taking the logical position i - m
template <typename Load>
__device__ __forceinline__ double dwt_tap_sum_logical(const double *__restrict__ f, int F, int N, int i, Load &&load)
{
    double s = 0.0;
    if (i >= N) {
        for (int m = F - 1; m >= 0; --m)
            if (i - m >= N) s = s + f[m] * load(i - m);
        for (int m = 0; m < F; ++m)
            if (i - m < N) s = s + f[m] * load(i - m);
    } else {
        for (int m = 0; m < F; ++m) s = s + f[m] * load(i - m);
    }
    return s;
}

// idwt_out with the loads taking the logical input position ii - j
template <typename LoadA, typename LoadD>
__device__ __forceinline__ double idwt_out_logical(const double *__restrict__ lo, const double *__restrict__ hi,
                                                   int F, int N, int n, LoadA &&la, LoadD &&ld)
{
    const int F2 = F / 2, T = F2 / 2;
    const int qq = n + F2 - 1;            // n - shift, >= 0
    const int q = qq % (2 * N);
    const int p = q & 1, i = q >> 1, ii = qq >> 1;
    const int top = i < T ? idwt_top(i, N, T) : 0;
    double s = 0.0;
    for (int pass = 0; pass < 2; ++pass) {
        const double *f = pass ? hi : lo;
        for (int t = 0; t < F2; ++t) {
            const int j = (i < T) ? (t <= top ? top - t : t) : t;
            const double c = pass ? ld(ii - j) : la(ii - j);
            s = s + f[2 * j + p] * c;
        }
    }
    return s;
}

// filter taps by value: kernel arguments, i.e. scalar registers
template <int F>
struct Taps {
    double lo[F], hi[F];
};

__device__ __forceinline__ int pad_col(int e) { return e + (e >> 3); }

// Four consecutive outputs of both filters from a register window, pywt's
// natural tap order per output (0 + f[0] x[i] + f[1] x[i-1] + ...), the tap
// loop outermost so the eight sums are independent chains.
// ZLO / ZHI: compile-time masks of zero taps (bit m = tap m is 0.0), which
// are skipped.  With finite samples a zero tap adds a signed zero, which can
// change only the sign of a zero sum, and pywt's sums (started at +0.0) are
// never -0, so the outputs are bit-identical (tests/test_dwt_gpu.py).  A
// run-time branch per tap measured 15-20 % slower; the masks are template
// arguments for the filters that have zeros and matter (bior4.4 = CDF 9/7).
// Z0: each sum starts with its first nonzero product instead of 0.0 + that
// product -- the strip kernels' argument: only the sign of a zero sum can
// differ, a zero only ever contributes zero products downstream, and every
// output the codec keeps is truncated to an integer, so the bytes are equal.
__host__ __device__ constexpr int first_nonzero_tap(unsigned Z, int F)
{
    int m = 0;
    while (m < F && ((Z >> m) & 1u)) ++m;
    return m;
}

template <int F, unsigned ZLO = 0, unsigned ZHI = 0, bool Z0 = false>
__device__ __forceinline__ void fwd_group(const double (&flo)[F], const double (&fhi)[F],
                                          const double (&v)[2 * (kG - 1) + F], double (&lo)[kG], double (&hi)[kG])
{
    constexpr int m0lo = Z0 ? first_nonzero_tap(ZLO, F) : -1, m0hi = Z0 ? first_nonzero_tap(ZHI, F) : -1;
#pragma unroll
    for (int u = 0; u < kG; ++u) {
        lo[u] = 0.0;
        hi[u] = 0.0;
    }
#pragma unroll
    for (int m = 0; m < F; ++m) {
        const double fl = flo[m], fh = fhi[m];
#pragma unroll
        for (int u = 0; u < kG; ++u) {
            const double x = v[2 * u + F - 1 - m];
            if (!((ZLO >> m) & 1u)) lo[u] = m == m0lo ? fl * x : lo[u] + fl * x;
            if (!((ZHI >> m) & 1u)) hi[u] = m == m0hi ? fh * x : hi[u] + fh * x;
        }
    }
}

// quantize one row-pass result pair into the staged subband bytes / LL
template <bool LAST>
__device__ __forceinline__ void fwd_store(int src, double lo, double hi, int e, uint8_t *stage, uint8_t *stage16,
                                          int SB, int Q, double *ll_dst)
{
    if (src) {                                   // D rows: da -> LH, dd -> HH
        stage[0 * SB + e] = quant_u8(lo, Q);
        stage[2 * SB + e] = quant_u8(hi, Q);
    } else {                                     // A rows: ad -> HL, aa -> LL
        stage[1 * SB + e] = quant_u8(hi, Q);
        if (LAST) {
            const uint16_t q16 = quant_u16(lo, Q);
            stage16[2 * e] = (uint8_t)q16;
            stage16[2 * e + 1] = (uint8_t)(q16 >> 8);
        } else {
            *ll_dst = lo;
        }
    }
}

// Forward level: a tile of kFTH x tw subband samples of all three channels.
// Per channel: stage the (2 kFTH - 2 + F) x 128 input samples, column pass
// (work item = one staged column x 4 output rows, its 2*3+F input samples
// in registers), row pass (work item = one row of A or D x 4 outputs),
// quantize into a byte image of the three detail subbands; one copy-out of
// contiguous runs at the end.  Outputs whose taps wrap past the line end
// (i >= N) take pywt's order through the generic LDS sum.
// Decomposition taps as compile-time constants, bit for bit the table's
// (vcf_wavelets.h; the launcher checks): id 1 = bior4.4 (CDF 9/7, config
// C3), id 2 = db5 (the reference's default -w).
__host__ __device__ constexpr double ct_dec(int id, bool hi, int m)
{
    constexpr double b44lo[10] = {0x0.0p+0, 0x1.35e4056861677p-5, -0x1.86bfe8124f578p-6, -0x1.c51e1871dddccp-4,
                                  0x1.8275e4e918b25p-2, 0x1.b494ebd75f071p-1, 0x1.8275e4e918b25p-2,
                                  -0x1.c51e1871dddccp-4, -0x1.86bfe8124f578p-6, 0x1.35e4056861677p-5};
    constexpr double b44hi[10] = {-0x0.0p+0, -0x1.0859ec635ec44p-4, 0x1.4d53e4bd96b38p-5, 0x1.ac206180c9dfcp-2,
                                  -0x1.93b462ffa8216p-1, 0x1.ac206180c9dfcp-2, 0x1.4d53e4bd96b38p-5,
                                  -0x1.0859ec635ec44p-4, -0x0.0p+0, 0x0.0p+0};
    constexpr double db5lo[10] = {0x1.b5385e04e3c09p-9, -0x1.9c3eff3294128p-7, -0x1.990ad4579f2e8p-8,
                                  0x1.3dbb9b52515aap-4, -0x1.0826648a8dc74p-5, -0x1.f0384d3f81474p-3,
                                  0x1.1b80373befcc6p-3, 0x1.72d89143b54f5p-1, 0x1.35291c2c4b00cp-1,
                                  0x1.47e3c41a7b911p-3};
    constexpr double db5hi[10] = {-0x1.47e3c41a7b911p-3, 0x1.35291c2c4b00cp-1, -0x1.72d89143b54f5p-1,
                                  0x1.1b80373befcc6p-3, 0x1.f0384d3f81474p-3, -0x1.0826648a8dc74p-5,
                                  -0x1.3dbb9b52515aap-4, -0x1.990ad4579f2e8p-8, 0x1.9c3eff3294128p-7,
                                  0x1.b5385e04e3c09p-9};
    return id == 1 ? (hi ? b44hi[m] : b44lo[m]) : (hi ? db5hi[m] : db5lo[m]);
}

// CT: the taps are wavelet CT's (ct_dec) as compile-time constants,
// rematerialised instead of held in -- and spilled from -- scalar registers;
// 0 = taps from the kernel arguments.
// STG (level 1): 1 = the YCoCg samples staged as int16 (exact; 29 KB of LDS
// instead of 35 KB) with the registers held to 5 waves, so five workgroups
// fit a CU; 0 = staged as float, 4 waves.  Used for db5 (−7.5 %, ABBA); for
// bior4.4 the register cap spills (+2 %), so it keeps 0.
// Schedule: two barriers per channel -- channel c+1's samples are staged
// during channel c's row pass (the staging tile is free once the column pass
// has read it) -- and the LL outputs of a non-final level go straight from the
// row pass to HBM (4 consecutive doubles per work item, contiguous across a
// wave).  Wave priority 3 while a workgroup issues its loads and its
// copy-out (as the DCT encode).
template <int F, bool FIRST, bool LAST, unsigned ZLO = 0, unsigned ZHI = 0, int CT = 0, int STG = 0, bool Z0 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FIRST && STG ? 5 : 1)))
void dwt_level_kernel(const uint8_t *__restrict__ rgb, long long rgb_stride,
                                                        const double *__restrict__ in, long long plane_stride,
                                                        double *__restrict__ LLout, uint8_t *__restrict__ packed,
                                                        long long packed_stride, long long ll_off, long long off_lh,
                                                        long long off_hl, long long off_hh, int h, int w, int hh,
                                                        int hw, int Q, Taps<F> tp, Filters flt)
{
    constexpr int NT = 256, FTH = kFTH;
    constexpr int TW = fwd_tile_w(F), IH = 2 * (FTH - 1) + F, IW = kFIW;
    constexpr int NWIN = 2 * (kG - 1) + F;
    constexpr int NG = (TW + kG - 1) / kG;
    constexpr int SB = FTH * TW * 3;
    static_assert(NT % kFIW == 0 && 2 * (TW - 1) + F == IW, "tile geometry");
    constexpr int RS = IW + IW / 8;                  // A/D rows padded one double per 8 (bank spread)
    // level 1 stages int16-valued YCoCg samples (as int16, or exact in float)
    using Stage = typename std::conditional<FIRST, typename std::conditional<STG == 1, int16_t, float>::type,
                                            double>::type;
    __shared__ Stage tin[IH * IW];
    __shared__ double tA[FTH * RS + 8], tD[FTH * RS + 8];   // +8: the last row group's window overhang
    __shared__ __attribute__((aligned(16))) uint8_t stage[3 * SB];
    __shared__ uint8_t stage16[LAST ? 2 * SB : 1];
    const int o0 = blockIdx.y * FTH, c0 = blockIdx.x * TW;
    const long long frame = blockIdx.z;
    const int R0 = F / 2 + 2 * o0 - F + 1, C0 = F / 2 + 2 * c0 - F + 1;
    const int tid = threadIdx.x;
    const bool rows_in = R0 >= 0 && R0 + IH <= h, cols_in = C0 >= 0 && C0 + IW <= w;
    const bool col_tail = F / 2 + 2 * (o0 + FTH - 1) >= h, row_tail = F / 2 + 2 * (c0 + TW - 1) >= w;
    // taps into VGPRs through LDS (kernel-argument taps would sit in scalar
    // registers, which the pass loops exhaust)
    double flo[F], fhi[F];
#pragma unroll
    for (int m = 0; m < F; ++m) {
        flo[m] = CT ? ct_dec(CT, false, m) : tp.lo[m];
        fhi[m] = CT ? ct_dec(CT, true, m) : tp.hi[m];
    }
    // staged samples of this thread (PER per channel), fetched one channel
    // ahead into registers: level 1 reads its RGB bytes once for all three
    // channels, later levels prefetch the next channel's plane during the
    // current channel's passes
    constexpr int PER = IH * IW / NT;
    static_assert(PER * NT == IH * IW, "staging split");
    uint32_t pix[FIRST ? PER : 1];
    double nxt[FIRST ? 1 : PER];
    auto fetch = [&](int ch) {
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int t = tid + NT * j;
            const int r = t / IW, c = t % IW;
            const int y = rows_in ? R0 + r : per_wrap(R0 + r, h);
            const int x = cols_in ? C0 + c : per_wrap(C0 + c, w);
            if (FIRST) {
                const uint8_t *px = rgb + frame * rgb_stride + ((long long)y * w + x) * 3;
                pix[j] = (uint32_t)px[0] | ((uint32_t)px[1] << 8) | ((uint32_t)px[2] << 16);
            } else {
                nxt[FIRST ? 0 : j] = in[(frame * 3 + ch) * plane_stride + (long long)y * w + x];
            }
        }
    };
    // stage channel ch's samples into tin (level 1: YCoCg from the RGB bytes)
    auto stage_in = [&](int ch) {
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            double v;
            if (FIRST) {
                // (int16)(R/4 + G/2 + B/4) etc.: every float term is a multiple of 1/4
                // below 2^9, so the sums are exact and truncation is integer division
                const int R = pix[j] & 0xFF, G = (pix[j] >> 8) & 0xFF, B = pix[j] >> 16;
                int iv;
                if (ch == 0) iv = (R + 2 * G + B) >> 2;
                else if (ch == 1) iv = (R - B) / 2;
                else iv = (2 * G - R - B) / 4;
                tin[tid + NT * j] = (Stage)iv;
            } else {
                v = nxt[FIRST ? 0 : j];
                tin[tid + NT * j] = (Stage)v;
            }
        }
    };
    __builtin_amdgcn_s_setprio(3);
    fetch(0);
    __builtin_amdgcn_s_setprio(0);
    stage_in(0);
    if (!FIRST) fetch(1);
    for (int ch = 0; ch < 3; ++ch) {
        __syncthreads();
        {   // column pass (axis 0): 128 columns x 2 groups of 4 output rows
            const int c = tid % IW, g = tid / IW;
            double v[NWIN];
#pragma unroll
            for (int k = 0; k < NWIN; ++k) v[k] = (double)tin[(2 * kG * g + k) * IW + c];
            double a[kG], d[kG];
            fwd_group<F, ZLO, ZHI, Z0>(flo, fhi, v, a, d);
#pragma unroll
            for (int u = 0; u < kG; ++u) {
                tA[(kG * g + u) * RS + pad_col(c)] = a[u];
                tD[(kG * g + u) * RS + pad_col(c)] = d[u];
            }
        }
        if (col_tail) {   // tile-uniform: rows whose taps wrap past the end take pywt's order
            __syncthreads();
            const int first = max(0, (h - F / 2 + 1) / 2 - o0);   // first tile row with i >= h
            for (int t = tid; t < (FTH - first) * IW; t += NT) {
                const int o = first + t / IW, c = t % IW;
                const int i = F / 2 + 2 * (o0 + o);
                auto load = [&](int p) -> double { return (double)tin[(p - R0) * IW + c]; };
                tA[o * RS + pad_col(c)] = dwt_tap_sum_logical(flt.dec_lo, F, h, i, load);
                tD[o * RS + pad_col(c)] = dwt_tap_sum_logical(flt.dec_hi, F, h, i, load);
            }
        }
        __syncthreads();
        if (ch < 2) {   // tin is free: stage the next channel while this one's rows run
            stage_in(ch + 1);
            if (!FIRST && ch == 0) fetch(2);
        }
        // LL of a non-final level: straight to HBM
        double *const llp = LLout + (frame * 3 + ch) * plane_stride + (long long)o0 * hw + c0;
        auto ll_dst = [&](int o, int oc) -> double * { return llp + (long long)o * hw + oc; };
        // row pass (axis 1): (A or D) x FTH rows x NG groups of 4 outputs, 16 group
        // slots per row, so a lane's (src, o, gq) are bit fields and every half-wave
        // reads two whole rows -- conflict-free LDS banks -- with the slots past NG idle
        const int first_tail = row_tail ? max(0, (w - F / 2 + 1) / 2 - c0) : TW;   // first column with i >= w
        constexpr int NGP = 16;
        static_assert(NG <= NGP && 2 * FTH * NGP == NT, "row-pass slots");
        for (int t = tid; t < NT; t += NT) {
            const int src = t / (FTH * NGP), o = (t >> 4) & (FTH - 1), gq = t & (NGP - 1);
            if (gq >= NG) continue;
            const int oc0 = kG * gq;
            const double *row = (src ? tD : tA) + o * RS;
            double v[NWIN];
#pragma unroll
            for (int k = 0; k < NWIN; ++k) v[k] = row[9 * gq + k + (k >> 3)];   // pad_col(8 gq + k)
            double lo[kG], hi[kG];
            fwd_group<F, ZLO, ZHI, Z0>(flo, fhi, v, lo, hi);
            const bool rv = o0 + o < hh;
#pragma unroll
            for (int u = 0; u < kG; ++u) {
                const int oc = oc0 + u;
                if (rv && oc < min(TW, hw - c0) && oc < first_tail)
                    fwd_store<LAST>(src, lo[u], hi[u], (o * TW + oc) * 3 + ch, stage, stage16, SB, Q,
                                    ll_dst(o, oc));
            }
        }
        if (row_tail) {   // tile-uniform: outputs whose taps wrap past the line end
            const int n = min(TW, hw - c0) - first_tail;
            for (int t = tid; t < 2 * FTH * max(n, 0); t += NT) {
                const int src = t / (FTH * n), rest = t % (FTH * n);
                const int o = rest / n, oc = first_tail + rest % n;
                if (o0 + o >= hh) continue;
                const int i = F / 2 + 2 * (c0 + oc);
                const double *row = (src ? tD : tA) + o * RS;
                auto load = [&](int p) -> double { return row[pad_col(p - C0)]; };
                const double lo = dwt_tap_sum_logical(flt.dec_lo, F, w, i, load);
                const double hi = dwt_tap_sum_logical(flt.dec_hi, F, w, i, load);
                fwd_store<LAST>(src, lo, hi, (o * TW + oc) * 3 + ch, stage, stage16, SB, Q, ll_dst(o, oc));
            }
        }
    }
    __syncthreads();   // the byte image is complete
    __builtin_amdgcn_s_setprio(3);
    // copy-out: each subband row of the tile is one contiguous byte run, moved
    // as dwords when every run start is 4-byte aligned, else as bytes
    const int rows = min(FTH, hh - o0), nb = min(TW, hw - c0) * 3;
    uint8_t *pk = packed + frame * packed_stride;
    const long long offs[3] = {off_lh, off_hl, off_hh};
    constexpr int TWW = TW * 3 / 4;   // dwords per staged subband row
    const bool dw = (TW * 3) % 4 == 0 &&
                    ((reinterpret_cast<uintptr_t>(pk) | (uintptr_t)(off_lh | off_hl | off_hh | (long long)hw * 3 |
                                                                    (long long)c0 * 3 | nb)) & 3u) == 0;
    if (dw) {
        const int nw = nb >> 2;
        for (int t = tid; t < 3 * rows * TWW; t += NT) {
            const int sb = t / (rows * TWW), r = t - sb * (rows * TWW);
            const int o = r / TWW, b = r - o * TWW;
            if (b < nw)
                *reinterpret_cast<uint32_t *>(pk + offs[sb] + ((long long)(o0 + o) * hw + c0) * 3 + 4 * b) =
                    *reinterpret_cast<const uint32_t *>(stage + sb * SB + o * (TW * 3) + 4 * b);
        }
    } else {
        for (int sb = 0; sb < 3; ++sb)
            for (int t = tid; t < rows * TW * 3; t += NT) {
                const int o = t / (TW * 3), b = t - o * (TW * 3);
                if (b < nb) pk[offs[sb] + ((long long)(o0 + o) * hw + c0) * 3 + b] = stage[sb * SB + t];
            }
    }
    if (LAST)
        for (int t = tid; t < rows * TW * 6; t += NT) {
            const int o = t / (TW * 6), b = t - o * (TW * 6);
            if (b < 2 * nb) pk[ll_off + ((long long)(o0 + o) * hw + c0) * 6 + b] = stage16[t];
        }
}

// ---------------------------------------------------------------------------
// strip kernels (forward): one wave per column strip, no barriers
// ---------------------------------------------------------------------------
// A wave owns 64 consecutive input columns (one per lane) of a vertical
// segment of the level's output rows and slides down it: every step takes
// two new input rows into a circular register window of F samples per
// channel, forms that column's A and D (axis-0 pass, pywt's tap order) for
// all three channels, leaves them in a wave-private LDS row, and lanes
// (A|D, output column) run the axis-1 pass over that row straight into the
// quantized subband bytes / LL.  Consecutive input rows are loaded once, the
// window rotates by compile-time indices (the step loop is unrolled by F/2),
// and nothing waits on a workgroup barrier: a wave reads only what it wrote
// itself (LDS operations of one wave complete in order).
// Z0: the first product of a sum starts it instead of 0.0 + product.  That
// differs only in the sign of a zero sum, and every output is truncated to
// an integer (zeros of either sign give 0, and a zero sample only ever adds
// a zero product), so the subband bytes are identical.
constexpr int kSW = 64;   // input columns per strip (one per lane)
__host__ __device__ constexpr int strip_tw(int F) { return (kSW - F) / 2 + 1; }

template <int F, unsigned Z, bool Z0>
__device__ __forceinline__ double nat_sum(const double (&f)[F], const double (&v)[F])
{
    // v[k] = sample at logical position i - F + 1 + k, i.e. tap m = F - 1 - k
    double s = 0.0;
    bool first = true;
#pragma unroll
    for (int m = 0; m < F; ++m) {
        if ((Z >> m) & 1u) continue;
        const double p = f[m] * v[F - 1 - m];
        s = (Z0 && first) ? p : s + p;
        first = false;
    }
    return s;
}

// nat_sum's taps in pywt's order for an output whose taps wrap past the line
// end (i >= N: the wrapped taps first, descending, then the others; as
// dwt_tap_sum_logical), over the same window v; zero taps skipped as in nat_sum
template <int F, unsigned Z>
__device__ __forceinline__ double wrap_sum(const double (&f)[F], const double (&v)[F], int i, int N)
{
    double s = 0.0;
#pragma unroll
    for (int m = F - 1; m >= 0; --m)
        if (!((Z >> m) & 1u) && i - m >= N) s = s + f[m] * v[F - 1 - m];
#pragma unroll
    for (int m = 0; m < F; ++m)
        if (!((Z >> m) & 1u) && i - m < N) s = s + f[m] * v[F - 1 - m];
    return s;
}

__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// a register copy the compiler cannot see through (see the strip kernel's row prefetch)
__device__ __forceinline__ uint32_t opaque_mov(uint32_t x)
{
    uint32_t r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ double opaque_mov(double x)
{
    double r;
    asm volatile("v_mov_b64 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// level-1 YCoCg sample (int16 truncation, A4) of channel ch from packed RGB bytes
__device__ __forceinline__ double ycocg_sample(uint32_t pix, int ch)
{
    const int R = pix & 0xFF, G = (pix >> 8) & 0xFF, B = (pix >> 16) & 0xFF;
    const int iv = ch == 0 ? (R + 2 * G + B) >> 2 : ch == 1 ? (R - B) / 2 : (2 * G - R - B) / 4;
    return (double)iv;
}

// the axis-1 pass of a strip's last wave, whose last outputs' taps wrap past
// the line end (pywt's order through the generic sum); out of line, rare
template <int F>
__device__ __forceinline__ void strip_row_generic(const double *row, Filters flt, int w, int ic, int C0,
                                                            double &lo, double &hi)
{
    auto load = [&](int p) -> double { return row[p - C0]; };
    lo = dwt_tap_sum_logical(flt.dec_lo, F, w, ic, load);
    hi = dwt_tap_sum_logical(flt.dec_hi, F, w, ic, load);
}

// The strip holding the outputs whose taps wrap past the line end slides like
// the others (its wrapping lanes reorder their row-pass taps from the same
// window, wrap_sum) instead of running every row through the generic sums with
// per-tap global loads -- the slowest wave of a small level
template <int F, bool FIRST, bool LAST, unsigned ZLO = 0, unsigned ZHI = 0, int CT = 0, bool Z0 = true,
          bool QP2 = true>
__global__ __launch_bounds__(192) void dwt_strip_kernel(const uint8_t *__restrict__ rgb, long long rgb_stride,
                                                        const double *__restrict__ in, long long plane_stride,
                                                        double *__restrict__ LLout, uint8_t *__restrict__ packed,
                                                        long long packed_stride, long long ll_off, long long off_lh,
                                                        long long off_hl, long long off_hh, int h, int w, int hh,
                                                        int hw, int Q, int n_strips, int seg_rows, Taps<F> tp,
                                                        Filters flt)
{
    constexpr int TWS = strip_tw(F), P = F / 2;
    // [channel wave][step of the group][A | D][column]: a buffer per unrolled step, so
    // one step's axis-1 reads and the next step's writes are independent
    // (the D row starts 2 doubles further on, so A and D lanes' reads fall in different banks)
    __shared__ __attribute__((aligned(16))) double rowbuf[3][P][2][kSW + 2];
    const int lane = threadIdx.x & 63;
    const int ch = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // one wave per channel (wave-uniform)
    // 1-D grid over (strip, segment, frame), the last strip -- whose last
    // outputs take the slow wrapped-tap path -- dispatched first
    const int n_segs = (hh + seg_rows - 1) / seg_rows;
    const int per_s = (int)gridDim.x / n_strips;                   // segments x frames
    const int strip = n_strips - 1 - (int)blockIdx.x / per_s;
    const int seg = (int)blockIdx.x % per_s % n_segs;
    const long long frame = (long long)blockIdx.x % per_s / n_segs;
    const int oc0 = strip * TWS;
    const int C0 = F / 2 + 2 * oc0 - F + 1;                          // logical column of lane 0
    const int x = per_wrap(C0 + lane, w);
    const int o0 = seg * seg_rows, o1 = min(hh, o0 + seg_rows);
    if (o0 >= o1) return;
    const int o_tail = min(o1, max(o0, (h - F / 2 + 1) / 2));   // first output row whose taps wrap past h
    double flo[F], fhi[F];
#pragma unroll
    for (int m = 0; m < F; ++m) {
        flo[m] = CT ? ct_dec(CT, false, m) : tp.lo[m];
        fhi[m] = CT ? ct_dec(CT, true, m) : tp.hi[m];
    }
    const int qsh = __builtin_ctz((unsigned)Q);
    auto q8 = [&](double v) -> uint8_t {   // (x / Q).astype(int32) + 128, astype(uint8)
        return (uint8_t)(uint32_t)((int32_t)(QP2 ? __builtin_ldexp(v, -qsh) : v / (double)Q) + 128);
    };
    auto q16 = [&](double v) -> uint16_t {
        return (uint16_t)(uint32_t)((int32_t)(QP2 ? __builtin_ldexp(v, -qsh) : v / (double)Q) + 128);
    };
    // axis-1 roles: lanes [0, TWS) take the A row, [TWS, 2 TWS) the D row
    const int src = lane >= TWS ? 1 : 0, oc = lane - src * TWS, ocg = oc0 + oc;
    const int nw = min(TWS, hw - oc0);                             // this strip's output columns
    const bool col_ok = lane < 2 * TWS && oc < nw;
    const int ic = F / 2 + 2 * ocg;                                  // its centre position on the line
    // wave-uniform: does this strip hold outputs whose taps wrap past the line end?
    const bool strip_tail = F / 2 + 2 * (oc0 + nw - 1) >= w;
    uint8_t *const pk = packed + frame * packed_stride;
    const uint8_t *const frgb = rgb + frame * rgb_stride;
    const double *const fin = in + (frame * 3 + ch) * plane_stride;
    const long long off_r1 = src ? off_lh : off_hl;   // this lane's first run: LH (D) / HL (A)
    // level 1: this lane's RGB bytes as one (unaligned) dword that starts a byte
    // early -- or, at x = 0, at the pixel -- so it never leaves the frame
    const int x3 = 3 * x, xl = x > 0 ? x3 - 1 : x3, xs = x > 0 ? 8 : 0;

    // per_wrap without a division or a branch: the launcher runs strips only on
    // planes of at least 2F rows and columns, so every row index here lies in
    // (-Ne, 2 Ne)
    const int Ne = h + (h & 1);
    auto row_of = [&](int r) -> long long {
        int y = r < 0 ? r + Ne : r;
        y = y >= Ne ? y - Ne : y;
        return y < h ? y : h - 1;
    };
    using Raw = typename std::conditional<FIRST, uint32_t, double>::type;   // a sample before conversion
    auto load_raw = [&](int r) -> Raw {
        const long long y = row_of(r);
        if constexpr (FIRST) {
            const uint8_t *rowp = frgb + y * w * 3;
            uint32_t d;
            __builtin_memcpy(&d, rowp + xl, 4);
            return d;   // the pixel is (d >> xs) & 0xFFFFFF (convert)
        } else {
            return (fin + y * w)[x];
        }
    };
    auto convert = [&](Raw v) -> double {
        if constexpr (FIRST) return ycocg_sample((v >> xs) & 0xFFFFFFu, ch);
        else return v;
    };
    // the same with the channel a compile-time constant (no branch per sample)
    auto convert_c = [&](Raw v, auto chc) -> double {
        if constexpr (FIRST) return ycocg_sample((v >> xs) & 0xFFFFFFu, decltype(chc)::value);
        else return v;
    };
    auto load_sample = [&](int r) -> double { return convert(load_raw(r)); };

    // Stores through buffer resources: a lane without an output (col_ok false,
    // or the other half's subband) stores at an offset past the buffer, which
    // the hardware drops.  So every store instruction issues unconditionally and
    // the compiler's vmcnt bookkeeping counts them: the waits for the input rows
    // loaded P steps ahead are then exact (with stores under an exec branch it
    // can only count the loads, and waits for far more recent operations).
    constexpr uint32_t kDrop = 0x80000000u;
    typedef unsigned int U32x2 __attribute__((__vector_size__(8)));
    const __amdgpu_buffer_rsrc_t rs_pk = __builtin_amdgcn_make_buffer_rsrc(pk, 0, (int)packed_stride, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_ll = __builtin_amdgcn_make_buffer_rsrc(
        LLout + (frame * 3 + ch) * plane_stride, 0, (int)((long long)hh * hw * 8), 0x00020000);
    const int ocr = min(oc, TWS - 1);                                // axis-1 reads stay inside the row
    const uint32_t e_lane = (uint32_t)(3 * oc + ch);
    // per-lane drop bits (loop-invariant data, not control flow): OR-ed into an offset
    const uint32_t drop1 = col_ok ? 0u : kDrop, drop_d = col_ok && src ? 0u : kDrop,
                   drop_a = col_ok && !src ? 0u : kDrop;
    // axis-1 pass of output row o over the wave's LDS row, quantize, store
    // (GENERIC: the strip holding the outputs whose taps wrap past the line end)
    auto row_pass = [&](int o, int bi, auto generic) {
        if (decltype(generic)::value) wave_lds_sync();
        const uint32_t rb = (uint32_t)(((long long)o * hw + oc0) * 3);   // the strip's first byte in a subband row
        const double *row = rowbuf[ch][bi][src];
        double lo, hi;
        if (!decltype(generic)::value) {
            double v[F];
#pragma unroll
            for (int k = 0; k < F; k += 2) {
                const double2 p = *(const double2 *)(row + 2 * ocr + k);
                v[k] = p.x;
                if (k + 1 < F) v[k + 1] = p.y;
            }
            lo = nat_sum<F, ZLO, Z0>(flo, v);
            hi = nat_sum<F, ZHI, Z0>(fhi, v);
            if (strip_tail && ic >= w) {   // this lane's taps wrap past the line end
                lo = wrap_sum<F, ZLO>(flo, v, ic, w);
                hi = wrap_sum<F, ZHI>(fhi, v, ic, w);
            }
        } else {
            lo = hi = 0.0;
            if (col_ok) strip_row_generic<F>(row, flt, w, ic, C0, lo, hi);
        }
        // A lanes: ad -> HL, aa -> LL; D lanes: da -> LH, dd -> HH
        const uint32_t e = rb + e_lane;
        __builtin_amdgcn_raw_buffer_store_b8(q8(src ? lo : hi), rs_pk, ((uint32_t)off_r1 + e) | drop1, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b8(q8(hi), rs_pk, ((uint32_t)off_hh + e) | drop_d, 0, 0);
        if (LAST)
            __builtin_amdgcn_raw_buffer_store_b16(q16(lo), rs_pk, ((uint32_t)ll_off + 2 * e) | drop_a, 0, 0);
        else
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(U32x2, lo), rs_ll,
                                                  (uint32_t)(((long long)o * hw + ocg) * 8) | drop_a, 0, 0);
        if (decltype(generic)::value) wave_lds_sync();
    };

    // rows from direct loads, the axis-0 taps in pywt's order (the rows whose
    // taps wrap past the bottom; every row of the tail strip)
    auto direct_rows = [&](int from, auto generic) {
        for (int o = from; o < o1; ++o) {
            const int i = F / 2 + 2 * o;
            wave_lds_sync();
            rowbuf[ch][0][0][lane] = dwt_tap_sum_logical(flt.dec_lo, F, h, i, load_sample);
            rowbuf[ch][0][1][lane] = dwt_tap_sum_logical(flt.dec_hi, F, h, i, load_sample);
            wave_lds_sync();
            row_pass(o, 0, generic);
        }
    };
    // sliding rows: groups of P steps; window slot (2u + k) % F of step u of a
    // group holds logical input row 2o - F/2 + 1 + k.  Rows are loaded P
    // steps ahead.  Level 1 runs one copy of the loop per channel (the YCoCg
    // formula a constant in each).
    int o = o0;
    auto slide = [&](auto chc) {
        double win[F];
#pragma unroll
        for (int k = 0; k < F - 2; ++k) win[k] = convert_c(load_raw(2 * o0 - F / 2 + 1 + k), chc);
        const int o_main = o0 + (o_tail - o0) / P * P;
        if (o >= o_main) return;
        // The next group's 2P input rows are loaded at the top of each group
        // and handed to the following group through register copies the
        // compiler cannot fold (opaque_mov): its wait for them then sits at the
        // end of this group, in straight-line code, and counts exactly the
        // stores issued since (values loaded in one iteration and first read
        // in the next make it wait for everything at the loop head).
        Raw cur[P][2];
#pragma unroll
        for (int u = 0; u < P; ++u) {
            cur[u][0] = load_raw(2 * (o + u) + F / 2 - 1);
            cur[u][1] = load_raw(2 * (o + u) + F / 2);
        }
        for (; o < o_main; o += P) {
            Raw nxt[P][2];
#pragma unroll
            for (int u = 0; u < P; ++u) {   // past the segment: wrapped rows, unused
                nxt[u][0] = load_raw(2 * (o + u + P) + F / 2 - 1);
                nxt[u][1] = load_raw(2 * (o + u + P) + F / 2);
            }
#pragma unroll
            for (int u = 0; u < P; ++u) {
                win[(2 * u + F - 2) % F] = convert_c(cur[u][0], chc);
                win[(2 * u + F - 1) % F] = convert_c(cur[u][1], chc);
                double v[F];
#pragma unroll
                for (int k = 0; k < F; ++k) v[k] = win[(2 * u + k) % F];
                // LDS operations of a wave complete in order, and the compiler keeps
                // this lane's write before the reads of the others (same array, no
                // proof of distinct addresses): no barrier needed
                rowbuf[ch][u][0][lane] = nat_sum<F, ZLO, Z0>(flo, v);
                rowbuf[ch][u][1][lane] = nat_sum<F, ZHI, Z0>(fhi, v);
                row_pass(o + u, u, std::false_type());
            }
#pragma unroll
            for (int u = 0; u < P; ++u) {
                cur[u][0] = opaque_mov(nxt[u][0]);
                cur[u][1] = opaque_mov(nxt[u][1]);
            }
        }
    };
    if (FIRST && ch == 0) slide(std::integral_constant<int, 0>());
    else if (FIRST && ch == 1) slide(std::integral_constant<int, 1>());
    else slide(std::integral_constant<int, 2>());
    wave_lds_sync();
    direct_rows(o, std::false_type());   // fewer than P rows, and the bottom rows' wrapped taps
}

// fused forward levels 1 + 2 (the default for 10-tap filters on planes of even
// sizes at both levels)
#include "vcf_dwt_band.h"

// Four consecutive outputs of the inverse from the register windows of the
// approximation (xa) and detail (xd) inputs: pywt's order for a pair index
// i >= F/4 (approximation taps j = 0.., then detail taps), tap loop outermost.
template <int F, unsigned ZLO = 0, unsigned ZHI = 0>   // zero-tap masks as in fwd_group
__device__ __forceinline__ void inv_group(const double (&flo)[F], const double (&fhi)[F],
                                          const double (&xa)[F / 2 + (((F / 2 - 1) & 1) + kG - 1) / 2],
                                          const double (&xd)[F / 2 + (((F / 2 - 1) & 1) + kG - 1) / 2],
                                          double (&s)[kG])
{
    constexpr int F2 = F / 2, P0 = (F2 - 1) & 1;
#pragma unroll
    for (int u = 0; u < kG; ++u) s[u] = 0.0;
#pragma unroll
    for (int j = 0; j < F2; ++j)
#pragma unroll
        for (int u = 0; u < kG; ++u)
            if (!((ZLO >> (2 * j + ((P0 + u) & 1))) & 1u))
                s[u] = s[u] + flo[2 * j + ((P0 + u) & 1)] * xa[F2 - 1 + ((P0 + u) >> 1) - j];
#pragma unroll
    for (int j = 0; j < F2; ++j)
#pragma unroll
        for (int u = 0; u < kG; ++u)
            if (!((ZHI >> (2 * j + ((P0 + u) & 1))) & 1u))
                s[u] = s[u] + fhi[2 * j + ((P0 + u) & 1)] * xd[F2 - 1 + ((P0 + u) >> 1) - j];
}

// the column pass's reordered outputs (rare: first / last rows of a plane)
__device__ __attribute__((noinline)) double inv_col_generic(Filters flt, int F, int h, int n, const double *ta,
                                                            const double *td, int K0r, int nc, int itw)
{
    auto la = [&](int k) -> double { return ta[(k - K0r) * itw + nc]; };
    auto ld = [&](int k) -> double { return td[(k - K0r) * itw + nc]; };
    return idwt_out_logical(flt.rec_lo, flt.rec_hi, F, h, n, la, ld);
}

// Inverse level r: subbands h x w (aa from the packed LL or from the previous
// level's plane with row stride lda) -> outputs [0, oh) x [0, ow) of the
// 2h x 2w reconstruction (only what the next level reads).  Row pass work
// item = one staged input row x 4 outputs of 'a' or 'd'; column pass = one
// column x 4 outputs.  TO_RGB (level 1): all three channels per tile, kept
// in registers, then to_RGB + clip + u8.  Outputs whose wrapped pair index
// is below F/4 take pywt's reordered taps through the generic LDS sum.
// reconstruction taps as compile-time constants (ids as ct_dec)
__host__ __device__ constexpr double ct_rec(int id, bool hi, int m)
{
    constexpr double b44lo[10] = {0x0.0p+0, -0x1.0859ec635ec44p-4, -0x1.4d53e4bd96b38p-5, 0x1.ac206180c9dfcp-2,
                                  0x1.93b462ffa8216p-1, 0x1.ac206180c9dfcp-2, -0x1.4d53e4bd96b38p-5,
                                  -0x1.0859ec635ec44p-4, 0x0.0p+0, 0x0.0p+0};
    constexpr double b44hi[10] = {0x0.0p+0, -0x1.35e4056861677p-5, -0x1.86bfe8124f578p-6, 0x1.c51e1871dddccp-4,
                                  0x1.8275e4e918b25p-2, -0x1.b494ebd75f071p-1, 0x1.8275e4e918b25p-2,
                                  0x1.c51e1871dddccp-4, -0x1.86bfe8124f578p-6, -0x1.35e4056861677p-5};
    constexpr double db5lo[10] = {0x1.47e3c41a7b911p-3, 0x1.35291c2c4b00cp-1, 0x1.72d89143b54f5p-1,
                                  0x1.1b80373befcc6p-3, -0x1.f0384d3f81474p-3, -0x1.0826648a8dc74p-5,
                                  0x1.3dbb9b52515aap-4, -0x1.990ad4579f2e8p-8, -0x1.9c3eff3294128p-7,
                                  0x1.b5385e04e3c09p-9};
    constexpr double db5hi[10] = {0x1.b5385e04e3c09p-9, 0x1.9c3eff3294128p-7, -0x1.990ad4579f2e8p-8,
                                  -0x1.3dbb9b52515aap-4, -0x1.0826648a8dc74p-5, 0x1.f0384d3f81474p-3,
                                  0x1.1b80373befcc6p-3, -0x1.72d89143b54f5p-1, 0x1.35291c2c4b00cp-1,
                                  -0x1.47e3c41a7b911p-3};
    return id == 1 ? (hi ? b44hi[m] : b44lo[m]) : (hi ? db5hi[m] : db5lo[m]);
}

// CT: reconstruction taps of wavelet CT (ct_rec) as compile-time constants
// (no tap registers: 40 fewer VGPRs than taps staged through LDS).  Output
// tiles of 64 x 16 (32 x 32 / 128 x 8 measured +3 % / +21 % on C3,
// profiles/r02_dwt_decode_ab_tiles.log); wave priority 3 while the subbands
// are staged.
template <int F, bool FROM_PACKED_LL, bool TO_RGB, unsigned ZLO = 0, unsigned ZHI = 0, int CT = 0>
__global__ __launch_bounds__(256) void idwt_level_kernel(const uint8_t *__restrict__ packed, long long packed_stride,
                                                         long long ll_off, long long off_lh, long long off_hl,
                                                         long long off_hh, const double *__restrict__ prev,
                                                         long long plane_stride, int lda, double *__restrict__ out,
                                                         int h, int w, int oh, int ow, int Q, Taps<F> tp,
                                                         Filters flt, uint8_t *__restrict__ rgb, long long rgb_stride)
{
    constexpr int ITW = kITW, ITH = 1024 / ITW;
    constexpr int F2 = F / 2, T = F2 / 2;
    constexpr int KHm = ITH / 2 + F2, KWm = ITW / 2 + F2;
    constexpr int P0 = (F2 - 1) & 1;                 // parity of n + F2 - 1 for even n
    constexpr int NW = F2 + ((P0 + kG - 1) >> 1);    // window of a 4-output group
    constexpr int NGC = ITW / kG, NGR = ITH / kG;
    static_assert(NGC * NGR * kG * kG == ITH * ITW && ITW * NGR == 256, "tile geometry");
    constexpr int S = (KHm * KWm + 1) & ~1;          // even, so the offsets below are odd apart (bank spread)
    __shared__ double sub[4 * S + 4];
    __shared__ double ta[KHm * ITW], td[KHm * ITW];
    double *sAA = sub, *sDA = sub + S + 1, *sAD = sub + 2 * S + 2, *sDD = sub + 3 * S + 3;
    const int n0r = blockIdx.y * ITH, n0c = blockIdx.x * ITW;
    const int K0r = ((n0r + F2 - 1) >> 1) - F2 + 1, K0c = ((n0c + F2 - 1) >> 1) - F2 + 1;
    const int KH = ((n0r + ITH - 1 + F2 - 1) >> 1) - K0r + 1;
    const int KW = ((n0c + ITW - 1 + F2 - 1) >> 1) - K0c + 1;
    const bool rows_in = K0r >= 0 && K0r + KH <= h, cols_in = K0c >= 0 && K0c + KW <= w;
    const bool row_tail = n0c == 0 || n0c + ITW + F2 - 2 >= 2 * w;
    const bool col_tail = n0r == 0 || n0r + ITH + F2 - 2 >= 2 * h;
    const int tid = threadIdx.x;
    const long long frame = TO_RGB ? blockIdx.z : blockIdx.z / 3;
    const uint8_t *pk = packed + frame * packed_stride;
    double acc[TO_RGB ? 3 : 1][kG];
    const int ch_lo = TO_RGB ? 0 : (int)(blockIdx.z % 3), ch_hi = TO_RGB ? 3 : ch_lo + 1;
    const int nc = tid % ITW, gr = tid / ITW;      // column-pass item
    __shared__ double taps[CT ? 1 : 2 * F];
    if (!CT) {
        if (tid < F) {
            taps[tid] = tp.lo[tid];
            taps[F + tid] = tp.hi[tid];
        }
        __syncthreads();
    }
    double flo[F], fhi[F];
#pragma unroll
    for (int m = 0; m < F; ++m) {
        flo[m] = CT ? ct_rec(CT, false, m) : taps[m];
        fhi[m] = CT ? ct_rec(CT, true, m) : taps[F + m];
    }
    for (int ch = ch_lo; ch < ch_hi; ++ch) {
        __builtin_amdgcn_s_setprio(3);
        for (int t = tid; t < KH * KW; t += 256) {
            const int r = t / KW, c = t - r * KW;
            const int y = rows_in ? K0r + r : mod_pos(K0r + r, h);
            const int x = cols_in ? K0c + c : mod_pos(K0c + c, w);
            const long long e = ((long long)y * w + x) * 3 + ch;
            double vaa;
            if (FROM_PACKED_LL) {
                const uint8_t *q = pk + ll_off + e * 2;
                vaa = dequant((int16_t)(uint16_t)(q[0] | (q[1] << 8)), Q);
            } else {
                vaa = prev[(frame * 3 + ch) * plane_stride + (long long)y * lda + x];
            }
            const int l = r * KWm + c;
            sAA[l] = vaa;
            sAD[l] = dequant((int16_t)pk[off_hl + e], Q);   // 'ad' = cV = HL
            sDA[l] = dequant((int16_t)pk[off_lh + e], Q);   // 'da' = cH = LH
            sDD[l] = dequant((int16_t)pk[off_hh + e], Q);   // 'dd' = cD = HH
        }
        __builtin_amdgcn_s_setprio(0);
        __syncthreads();
        // row pass (axis 1): 'a' = idwt(aa, ad), 'd' = idwt(da, dd)
        for (int t = tid; t < KH * NGC * 2; t += 256) {
            const int src = t & 1, r = (t >> 1) / NGC, g = (t >> 1) % NGC;
            const int n0 = n0c + kG * g;
            const int base = r * KWm + ((n0 + F2 - 1) >> 1) - F2 + 1 - K0c;
            const double *X = src ? sDA : sAA, *Y = src ? sDD : sAD;
            double xa[NW], xd[NW];
#pragma unroll
            for (int k = 0; k < NW; ++k) {
                xa[k] = X[base + k];
                xd[k] = Y[base + k];
            }
            double sum[kG];
            inv_group<F, ZLO, ZHI>(flo, fhi, xa, xd, sum);
            double *dst = (src ? td : ta) + r * ITW + kG * g;
#pragma unroll
            for (int u = 0; u < kG; ++u) dst[u] = sum[u];
        }
        if (row_tail) {   // tile-uniform: outputs whose wrapped pair index is below F/4
            __syncthreads();
            for (int t = tid; t < KH * ITW * 2; t += 256) {
                const int src = t & 1, r = (t >> 1) / ITW, nc2 = (t >> 1) % ITW;
                const int n = n0c + nc2, q = n + F2 - 1;
                if (n >= ow || ((q % (2 * w)) >> 1) >= T) continue;
                const double *Xr = (src ? sDA : sAA) + r * KWm - K0c, *Yr = (src ? sDD : sAD) + r * KWm - K0c;
                auto la = [&](int k) -> double { return Xr[k]; };
                auto ld = [&](int k) -> double { return Yr[k]; };
                (src ? td : ta)[r * ITW + nc2] = idwt_out_logical(flt.rec_lo, flt.rec_hi, F, w, n, la, ld);
            }
        }
        __syncthreads();
        {   // column pass (axis 0): 64 columns x 4 groups of 4 output rows
            const int n0 = n0r + kG * gr;
            const int base = ((n0 + F2 - 1) >> 1) - F2 + 1 - K0r;
            double xa[NW], xd[NW];
#pragma unroll
            for (int k = 0; k < NW; ++k) {
                xa[k] = ta[(base + k) * ITW + nc];
                xd[k] = td[(base + k) * ITW + nc];
            }
            double sum[kG];
            inv_group<F, ZLO, ZHI>(flo, fhi, xa, xd, sum);
            if (col_tail) {
#pragma unroll
                for (int u = 0; u < kG; ++u) {
                    const int n = n0 + u, q = n + F2 - 1;
                    if (((q % (2 * h)) >> 1) < T) sum[u] = inv_col_generic(flt, F, h, n, ta, td, K0r, nc, ITW);
                }
            }
#pragma unroll
            for (int u = 0; u < kG; ++u) acc[TO_RGB ? ch : 0][u] = sum[u];
        }
        __syncthreads();
    }
    const int m = n0c + nc;
#pragma unroll
    for (int u = 0; u < kG; ++u) {
        const int n = n0r + kG * gr + u;
        if (n >= oh || m >= ow) continue;
        if (TO_RGB) {
            const double Y = acc[0][u], Co = acc[TO_RGB ? 1 : 0][u], Cg = acc[TO_RGB ? 2 : 0][u];
            const double v[3] = {Y + Co - Cg, Y + Cg, Y - Co - Cg};
            uint8_t *o = rgb + frame * rgb_stride + ((long long)n * ow + m) * 3;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double c = v[k] < 0.0 ? 0.0 : (v[k] > 255.0 ? 255.0 : v[k]);
                o[k] = (uint8_t)c;
            }
        } else {
            out[(frame * 3 + ch_lo) * plane_stride + (long long)n * ow + m] = acc[0][u];
        }
    }
}

// line-based inverse level (the default for 10-tap filters)
#include "vcf_idwt_line.h"
// inverse levels 2 + 1 in one launch (the default where the planes halve evenly)
#include "vcf_idwt_band21.h"
// the opt-in lifting form of bior4.4 (not bit-exact)
#include "vcf_dwt_lift.h"

#ifndef VCF_DWT_KERNELS_ONLY   // (micro-experiments compile the kernels alone)
// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// filter banks uploaded once per (device, wavelet)
std::mutex g_filt_mu;
double *g_filt[64][kNumWavelets] = {};

int device_filters(int wavelet, Filters &flt)
{
    int dev = 0;
    int rc = hip_check(hipGetDevice(&dev), "hipGetDevice");
    if (rc != VCF_OK) return rc;
    if (dev < 0 || dev >= 64) return set_error(VCF_ERR_INVALID, "device %d", dev);
    const WaveletDef &wd = kWavelets[wavelet];
    std::lock_guard<std::mutex> lk(g_filt_mu);
    double *&p = g_filt[dev][wavelet];
    if (!p) {
        double host[4 * 128];
        const int F = wd.len;
        memcpy(host, wd.dec_lo, sizeof(double) * F);
        memcpy(host + F, wd.dec_hi, sizeof(double) * F);
        memcpy(host + 2 * F, wd.rec_lo, sizeof(double) * F);
        memcpy(host + 3 * F, wd.rec_hi, sizeof(double) * F);
        rc = hip_check(hipMalloc((void **)&p, sizeof(double) * 4 * F), "hipMalloc(filters)");
        if (rc != VCF_OK) return rc;
        rc = hip_check(hipMemcpy(p, host, sizeof(double) * 4 * F, hipMemcpyHostToDevice), "filters upload");
        if (rc != VCF_OK) {
            (void)hipFree(p);
            p = nullptr;
            return rc;
        }
    }
    const int F = wd.len;
    flt = Filters{p, p + F, p + 2 * F, p + 3 * F};
    return VCF_OK;
}

int check_dwt(const void *a, const void *b, int64_t n_frames, int32_t H, int32_t W, int32_t wavelet,
              int32_t levels, int32_t Q, bool decode)
{
    if (n_frames < 0) return set_error(VCF_ERR_INVALID, "n_frames < 0");
    if (H <= 0 || W <= 0) return set_error(VCF_ERR_INVALID, "bad frame shape %d x %d", H, W);
    if (wavelet < 0 || wavelet >= kNumWavelets) return set_error(VCF_ERR_INVALID, "unknown wavelet %d", wavelet);
    if (levels < 1 || levels > kMaxLevels) return set_error(VCF_ERR_INVALID, "levels %d out of range", levels);
    if (Q < 1 || (decode && Q > 32767)) return set_error(VCF_ERR_INVALID, "quantization step %d out of range", Q);
    if ((long long)H * W * 3 >= (1LL << 31)) return set_error(VCF_ERR_INVALID, "frame too large");
    if (n_frames > 0 && (!a || !b)) return set_error(VCF_ERR_INVALID, "null buffer");
    return VCF_OK;
}

unsigned gx(int n) { return (unsigned)((n + 255) / 256); }

bool fast_filter(int F) { return F >= 2 && F <= kMaxFastF && (F & 1) == 0; }

template <int F>
Taps<F> taps_of(const double *lo, const double *hi)
{
    Taps<F> t;
    for (int m = 0; m < F; ++m) {
        t.lo[m] = lo[m];
        t.hi[m] = hi[m];
    }
    return t;
}

struct LevelArgs {
    const uint8_t *rgb;
    long long rgb_stride;
    const double *in;
    long long plane_stride;
    double *LLout;
    uint8_t *packed;
    long long packed_stride, ll_off, off_lh, off_hl, off_hh;
    int h, w, hh, hw, Q, lda;
    unsigned n_frames;
    Filters flt;
    const WaveletDef *wd;
    hipStream_t s;
};

// bit m set = tap m is exactly 0.0
unsigned zero_mask(const double *t, int F)
{
    unsigned m = 0;
    for (int k = 0; k < F && k < 32; ++k)
        if (t[k] == 0.0) m |= 1u << k;
    return m;
}

// the zero-tap masks of bior4.4 (CDF 9/7, config C3): decomposition lo / hi,
// reconstruction lo / hi
constexpr unsigned kB44DecLo = 0x001u, kB44DecHi = 0x301u, kB44RecLo = 0x301u, kB44RecHi = 0x001u;

template <int F, unsigned ZLO, unsigned ZHI>
void launch_fwd_kernel(const LevelArgs &a, const Taps<F> &tp, const dim3 &grid, bool first, bool last)
{
    auto kern = first ? (last ? dwt_level_kernel<F, true, true, ZLO, ZHI> : dwt_level_kernel<F, true, false, ZLO, ZHI>)
                      : (last ? dwt_level_kernel<F, false, true, ZLO, ZHI> : dwt_level_kernel<F, false, false, ZLO, ZHI>);
    if constexpr (F == 10) {   // bior4.4 / db5: compile-time taps, sums started by their first product
        constexpr int id = ZLO != 0 ? 1 : 2;
        constexpr int stg = id == 2 ? 1 : 0;
        bool ct = true;
        for (int m = 0; m < F; ++m) {
            const double l = ct_dec(id, false, m), h = ct_dec(id, true, m);
            ct = ct && std::memcmp(&l, &tp.lo[m], 8) == 0 && std::memcmp(&h, &tp.hi[m], 8) == 0;
        }
        if (ct)
            kern = first ? (last ? dwt_level_kernel<F, true, true, ZLO, ZHI, id, stg, true>
                                 : dwt_level_kernel<F, true, false, ZLO, ZHI, id, stg, true>)
                         : (last ? dwt_level_kernel<F, false, true, ZLO, ZHI, id, 0, true>
                                 : dwt_level_kernel<F, false, false, ZLO, ZHI, id, 0, true>);
    }
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, a.s, a.rgb, a.rgb_stride, a.in, a.plane_stride, a.LLout, a.packed,
                       a.packed_stride, a.ll_off, a.off_lh, a.off_hl, a.off_hh, a.h, a.w, a.hh, a.hw, a.Q, tp, a.flt);
}

template <int F>
void launch_fwd_level(const LevelArgs &a, bool first, bool last)
{
    const Taps<F> tp = taps_of<F>(a.wd->dec_lo, a.wd->dec_hi);
    constexpr int TW = fwd_tile_w(F);
    const dim3 grid((a.hw + TW - 1) / TW, (a.hh + kFTH - 1) / kFTH, a.n_frames);
    if (F == 10 && zero_mask(a.wd->dec_lo, F) == kB44DecLo && zero_mask(a.wd->dec_hi, F) == kB44DecHi)
        launch_fwd_kernel<F, (F == 10 ? kB44DecLo : 0u), (F == 10 ? kB44DecHi : 0u)>(a, tp, grid, first, last);
    else
        launch_fwd_kernel<F, 0u, 0u>(a, tp, grid, first, last);
}

// strip kernels
constexpr int kMaxStripF = 10;   // longest filter with a strip kernel (F samples of window in VGPRs)

template <int F>
using StripKern = void (*)(const uint8_t *, long long, const double *, long long, double *, uint8_t *, long long,
                           long long, long long, long long, long long, int, int, int, int, int, int, int, Taps<F>,
                           Filters);

template <int F, unsigned ZL, unsigned ZH, int CT, bool QP2>
StripKern<F> strip_kern(bool first, bool last)
{
    return first ? (last ? dwt_strip_kernel<F, true, true, ZL, ZH, CT, true, QP2>
                         : dwt_strip_kernel<F, true, false, ZL, ZH, CT, true, QP2>)
                 : (last ? dwt_strip_kernel<F, false, true, ZL, ZH, CT, true, QP2>
                         : dwt_strip_kernel<F, false, false, ZL, ZH, CT, true, QP2>);
}

template <int F>
void launch_strip_level(const LevelArgs &a, bool first, bool last)
{
    if constexpr (F > kMaxStripF) {
        return;
    } else {
        const Taps<F> tp = taps_of<F>(a.wd->dec_lo, a.wd->dec_hi);
        constexpr int TWS = strip_tw(F), P = F / 2;
        const int n_strips = (a.hw + TWS - 1) / TWS;
        // segments: ~16 waves per SIMD over the chip (three per strip-segment),
        // at least 2F rows, whole groups of F/2 sliding steps
        const long long cols = (long long)n_strips * a.n_frames * 3;
        int seg = (int)std::max<long long>(2 * F, (a.hh * cols + 16383) / 16384);
        seg = std::min((seg + P - 1) / P * P, a.hh);
        const long long nblk = (long long)n_strips * ((a.hh + seg - 1) / seg) * a.n_frames;
        const bool qp2 = (a.Q & (a.Q - 1)) == 0;
        StripKern<F> kern = qp2 ? strip_kern<F, 0u, 0u, 0, true>(first, last) : strip_kern<F, 0u, 0u, 0, false>(first, last);
        if constexpr (F == 10) {   // bior4.4 (zero taps skipped) / db5: compile-time taps
            const bool b44 = zero_mask(a.wd->dec_lo, F) == kB44DecLo && zero_mask(a.wd->dec_hi, F) == kB44DecHi;
            const int id = b44 ? 1 : 2;
            bool ct = true;
            for (int m = 0; ct && m < F; ++m) {
                const double l = ct_dec(id, false, m), h = ct_dec(id, true, m);
                ct = std::memcmp(&l, &tp.lo[m], 8) == 0 && std::memcmp(&h, &tp.hi[m], 8) == 0;
            }
            if (ct && b44)
                kern = qp2 ? strip_kern<F, kB44DecLo, kB44DecHi, 1, true>(first, last)
                           : strip_kern<F, kB44DecLo, kB44DecHi, 1, false>(first, last);
            else if (ct)
                kern = qp2 ? strip_kern<F, 0u, 0u, 2, true>(first, last) : strip_kern<F, 0u, 0u, 2, false>(first, last);
        }
        hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(192), 0, a.s, a.rgb, a.rgb_stride, a.in,
                           a.plane_stride, a.LLout, a.packed, a.packed_stride, a.ll_off, a.off_lh, a.off_hl,
                           a.off_hh, a.h, a.w, a.hh, a.hw, a.Q, n_strips, seg, tp, a.flt);
    }
}

// level r of the inverse: subbands a.h x a.w -> outputs a.hh x a.hw (= oh x ow)
template <int F, unsigned ZLO, unsigned ZHI>
void launch_inv_kernel(const LevelArgs &a, const Taps<F> &tp, dim3 grid, bool from_packed, bool to_rgb,
                       uint8_t *rgb_out)
{
    auto kern = from_packed
                    ? (to_rgb ? idwt_level_kernel<F, true, true, ZLO, ZHI> : idwt_level_kernel<F, true, false, ZLO, ZHI>)
                    : (to_rgb ? idwt_level_kernel<F, false, true, ZLO, ZHI> : idwt_level_kernel<F, false, false, ZLO, ZHI>);
    if constexpr (F == 10) {   // bior4.4 / db5: compile-time taps
        constexpr int id = ZLO != 0 ? 1 : 2;
        bool ct = true;
        for (int m = 0; m < F; ++m) {
            const double l = ct_rec(id, false, m), h = ct_rec(id, true, m);
            ct = ct && std::memcmp(&l, &tp.lo[m], 8) == 0 && std::memcmp(&h, &tp.hi[m], 8) == 0;
        }
        if (ct)
            kern = from_packed ? (to_rgb ? idwt_level_kernel<F, true, true, ZLO, ZHI, id>
                                         : idwt_level_kernel<F, true, false, ZLO, ZHI, id>)
                               : (to_rgb ? idwt_level_kernel<F, false, true, ZLO, ZHI, id>
                                         : idwt_level_kernel<F, false, false, ZLO, ZHI, id>);
    }
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, a.s, a.packed, a.packed_stride, a.ll_off, a.off_lh, a.off_hl,
                       a.off_hh, a.in, a.plane_stride, a.lda, a.LLout, a.h, a.w, a.hh, a.hw, a.Q, tp, a.flt, rgb_out,
                       (long long)a.hh * a.hw * 3);
}

template <int F>
void launch_inv_level(const LevelArgs &a, bool from_packed, bool to_rgb, uint8_t *rgb_out)
{
    const Taps<F> tp = taps_of<F>(a.wd->rec_lo, a.wd->rec_hi);
    const dim3 grid((a.hw + kITW - 1) / kITW, (a.hh + kITH - 1) / kITH, to_rgb ? a.n_frames : 3 * a.n_frames);
    if (F == 10 && zero_mask(a.wd->rec_lo, F) == kB44RecLo && zero_mask(a.wd->rec_hi, F) == kB44RecHi)
        launch_inv_kernel<F, (F == 10 ? kB44RecLo : 0u), (F == 10 ? kB44RecHi : 0u)>(a, tp, grid, from_packed,
                                                                                        to_rgb, rgb_out);
    else
        launch_inv_kernel<F, 0u, 0u>(a, tp, grid, from_packed, to_rgb, rgb_out);
}

// Levels 1 and 2 in one launch (dwt_band12_kernel): 10-tap filters with
// compile-time taps (bior4.4, db5), planes with h % 4 == 0 and w % 4 == 0 and
// at least 64 x 512 (the windows wrap at most once), levels >= 2.
bool band12_ok(const DwtGeom &g, const WaveletDef &wd, int &id)
{
    if (g.F != 10 || g.levels < 2 || g.H % 4 || g.W % 4 || g.H < 64 || g.W < 512) return false;
    const bool b44 = zero_mask(wd.dec_lo, 10) == kB44DecLo && zero_mask(wd.dec_hi, 10) == kB44DecHi;
    id = b44 ? 1 : 2;
    for (int m = 0; m < 10; ++m) {
        const double l = ct_dec(id, false, m), h = ct_dec(id, true, m);
        if (std::memcmp(&l, &wd.dec_lo[m], 8) || std::memcmp(&h, &wd.dec_hi[m], 8)) return false;
    }
    return true;
}

template <unsigned ZL, unsigned ZH, int CT>
void launch_band12_t(const DwtGeom &g, const uint8_t *rgb, long long n_frames, double *LL2, long long plane_stride,
                     uint8_t *packed, int Q, hipStream_t s, long long rule_frames)
{
    const int h2 = g.hs[2], w2 = g.ws[2];
    const int n_tiles = (w2 + kBT2 - 1) / kBT2;
    // bands: the time is about (rounds of resident workgroups) x (steps per band,
    // 2 rows + the F - 2 halo rows + 3 of pipeline per level-2 row pair); two
    // 512-thread workgroups fit a CU (VGPRs)
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0, v = 0;
        n_cu = hipGetDevice(&dev) == hipSuccess &&
                       hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0
                   ? v
                   : 256;
    }
    // (rule_frames: the frames of the whole call -- a pipelined call's chunks run side by side)
    const long long slots = 2LL * n_cu, per_band = 3LL * rule_frames * n_tiles;
    int n_bands = 1;
    long long best = -1;
    for (int nb = 1; nb <= std::max(1, h2 / 2); ++nb) {
        const int br = (h2 + nb - 1) / nb;
        if (nb > 1 && (h2 + br - 1) / br != nb) continue;
        const long long rounds = (per_band * nb + slots - 1) / slots;
        const long long cost = rounds * (2LL * br + 10 + 3);
        if (best < 0 || cost < best) {
            best = cost;
            n_bands = nb;
        }
    }
    if (const char *e = getenv("VCF_DWT_BANDS"))   // tuning knob (A/B of the band cut)
        n_bands = std::max(1, std::min(atoi(e), std::max(1, h2 / 2)));
    const int brows = (h2 + n_bands - 1) / n_bands;
    n_bands = (h2 + brows - 1) / brows;
    const long long units = n_frames * n_tiles * n_bands;
    const unsigned grid = (unsigned)(24 * ((units + 7) / 8));
    const bool last2 = g.levels == 2, qp2 = (Q & (Q - 1)) == 0;
    auto kern = last2 ? (qp2 ? dwt_band12_kernel<10, ZL, ZH, CT, true, true> : dwt_band12_kernel<10, ZL, ZH, CT, true, false>)
                      : (qp2 ? dwt_band12_kernel<10, ZL, ZH, CT, false, true>
                             : dwt_band12_kernel<10, ZL, ZH, CT, false, false>);
    const Taps<10> tp{};
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBNT), 0, s, rgb, (long long)g.H * g.W * 3, LL2, plane_stride, packed,
                       g.packed_bytes, g.ll_off, g.sb_off[1][0], g.sb_off[1][1], g.sb_off[1][2], g.sb_off[2][0],
                       g.sb_off[2][1], g.sb_off[2][2], g.H, g.W, Q, n_tiles, n_bands, brows, (int)units, tp);
}

void launch_band12(int id, const DwtGeom &g, const uint8_t *rgb, long long n_frames, double *LL2,
                   long long plane_stride, uint8_t *packed, int Q, hipStream_t s, long long rule_frames)
{
    if (id == 1) launch_band12_t<kB44DecLo, kB44DecHi, 1>(g, rgb, n_frames, LL2, plane_stride, packed, Q, s, rule_frames);
    else launch_band12_t<0u, 0u, 2>(g, rgb, n_frames, LL2, plane_stride, packed, Q, s, rule_frames);
}

// Line-based inverse level (idwt_line_kernel): 10-tap reconstruction filters
// with compile-time taps (bior4.4, db5) on subbands of at least 5 x 5.
bool line_ok(const WaveletDef &wd, int h, int w, int &id)
{
    if (wd.len != 10 || h < 5 || w < 5) return false;
    const bool b44 = zero_mask(wd.rec_lo, 10) == kB44RecLo && zero_mask(wd.rec_hi, 10) == kB44RecHi;
    id = b44 ? 1 : 2;
    for (int m = 0; m < 10; ++m) {
        const double l = ct_rec(id, false, m), hv = ct_rec(id, true, m);
        if (std::memcmp(&l, &wd.rec_lo[m], 8) || std::memcmp(&hv, &wd.rec_hi[m], 8)) return false;
    }
    return true;
}

template <bool FP, bool RGB, unsigned ZL, unsigned ZH, int CT>
void launch_line_t(const LevelArgs &a, uint8_t *rgb_out)
{
    // Q <= 256: the detail dequant never wraps in int16 (the fma form)
    auto kern = a.Q <= 256 ? idwt_line_kernel<FP, RGB, ZL, ZH, CT, true> : idwt_line_kernel<FP, RGB, ZL, ZH, CT, false>;
    static int slots = 0;   // resident workgroups on the device (per instantiation)
    if (!slots) {
        int dev = 0, n_cu = 0, per_cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
            n_cu = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kINT, 0) != hipSuccess || per_cu <= 0)
            per_cu = 2;
        slots = n_cu * per_cu;
    }
    const int n_tiles = (a.w + kILC - 1) / kILC, ohp = (a.hh + 1) / 2;
    // bands: time ~ (rounds of resident workgroups) x (steps per band: rows + 4 halo + 1)
    const long long per_band = (long long)n_tiles * a.n_frames;
    int n_bands = 1;
    long long best = -1;
    for (int nb = 1; nb <= ohp; ++nb) {
        const int br = (ohp + nb - 1) / nb;
        if (nb > 1 && (ohp + br - 1) / br != nb) continue;
        const long long rounds = (per_band * nb + slots - 1) / slots;
        const long long cost = rounds * (br + 5);
        if (best < 0 || cost < best) {
            best = cost;
            n_bands = nb;
        }
    }
    if (const char *e = getenv("VCF_IDWT_BANDS"))   // tuning knob (A/B of the band cut)
        n_bands = std::max(1, std::min(atoi(e), ohp));
    const int brows = (ohp + n_bands - 1) / n_bands;
    n_bands = (ohp + brows - 1) / brows;
    const long long grid = per_band * n_bands;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kINT), 0, a.s, a.packed, a.packed_stride, a.ll_off, a.off_lh,
                       a.off_hl, a.off_hh, a.in, a.plane_stride, a.lda, a.LLout, rgb_out, a.h, a.w, a.hh, a.hw, a.Q,
                       n_tiles, n_bands, brows);
}

template <unsigned ZL, unsigned ZH, int CT>
void launch_line_id(const LevelArgs &a, bool from_packed, bool to_rgb, uint8_t *rgb_out)
{
    if (from_packed) {
        if (to_rgb) launch_line_t<true, true, ZL, ZH, CT>(a, rgb_out);
        else launch_line_t<true, false, ZL, ZH, CT>(a, rgb_out);
    } else {
        if (to_rgb) launch_line_t<false, true, ZL, ZH, CT>(a, rgb_out);
        else launch_line_t<false, false, ZL, ZH, CT>(a, rgb_out);
    }
}

void launch_line(int id, const LevelArgs &a, bool from_packed, bool to_rgb, uint8_t *rgb_out)
{
    if (id == 1) launch_line_id<kB44RecLo, kB44RecHi, 1>(a, from_packed, to_rgb, rgb_out);
    else launch_line_id<0u, 0u, 2>(a, from_packed, to_rgb, rgb_out);
}

// Inverse levels 2 + 1 in one launch (idwt_band21_kernel): line_ok filters on
// planes that halve evenly from level 2 to level 1 (h1 = 2 h2, w1 = 2 w2).
std::atomic<int> g_band21{1};   // vcf_dwt_set_inverse_band21 (A/B and tests)
bool band21_ok(const DwtGeom &g, const WaveletDef &wd, int &id)
{
    if (!g_band21.load(std::memory_order_relaxed) || g.levels < 2) return false;
    const int h2 = g.hs[2], w2 = g.ws[2], h1 = g.hs[1], w1 = g.ws[1];
    return h1 == 2 * h2 && w1 == 2 * w2 && line_ok(wd, h2, w2, id) && line_ok(wd, h1, w1, id);
}

template <bool FP, unsigned ZL, unsigned ZH, int CT>
void launch_band21_t(const DwtGeom &g, const uint8_t *packed, long long n_frames, const double *prev,
                     long long plane_stride, int lda, uint8_t *rgb, int Q, hipStream_t s, long long rule_frames)
{
    auto kern = Q <= 256 ? idwt_band21_kernel<FP, ZL, ZH, CT, true> : idwt_band21_kernel<FP, ZL, ZH, CT, false>;
    static int slots = 0;   // resident workgroups on the device (per instantiation)
    if (!slots) {
        int dev = 0, n_cu = 0, per_cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
            n_cu = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kB21NT, 0) != hipSuccess || per_cu <= 0)
            per_cu = 2;
        slots = n_cu * per_cu;
    }
    const int h1 = g.hs[1], w1 = g.ws[1];
    const int n_tiles = (w1 + kB21C - 1) / kB21C;
    // bands of an even number of level-1 rows: the shortest bands (each re-reads a 7-row
    // halo) that still leave at most three workgroups per resident slot -- measured
    // (scripts/dwt_bands_scan.py, profiles/r06_dwt_band_cuts_decode.json): C3 decode 0.546 ms
    // with one round of 216-row bands (the previous rounds x (rows + 7) model's pick), 0.529
    // with 60-108 rows, 0.655 with 360: a few rounds of shorter bands balance better
    // (rule_frames: the frames of the whole call -- a pipelined call's chunks run side by side)
    const long long per_band = (long long)n_tiles * rule_frames;
    int brows = (h1 + 1) / 2 * 2;
    for (int br = 16; br <= (h1 + 1) / 2 * 2; br += 2)
        if (per_band * ((h1 + br - 1) / br) <= 3 * slots) {
            brows = br;
            break;
        }
    if (const char *e = getenv("VCF_IDWT21_BROWS"))   // tuning knob (A/B of the band cut): level-1 rows per band
        brows = std::max(2, std::min(atoi(e) / 2 * 2, (h1 + 1) / 2 * 2));
    const int n_bands = (h1 + brows - 1) / brows;
    const long long grid = (long long)n_tiles * n_frames * n_bands;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kB21NT), 0, s, packed, g.packed_bytes, g.ll_off,
                       g.sb_off[2][0], g.sb_off[2][1], g.sb_off[2][2], g.sb_off[1][0], g.sb_off[1][1], g.sb_off[1][2],
                       prev, plane_stride, lda, rgb, g.hs[2], g.ws[2], h1, w1, Q, n_tiles, n_bands, brows);
}

void launch_band21(int id, const DwtGeom &g, const uint8_t *packed, long long n_frames, const double *prev,
                   long long plane_stride, int lda, uint8_t *rgb, int Q, hipStream_t s, long long rule_frames)
{
    const bool fp = g.levels == 2;   // LL2 from the packed u16 subband, else the level-3 plane
    const long long rf = rule_frames;
    if (id == 1) {
        if (fp) launch_band21_t<true, kB44RecLo, kB44RecHi, 1>(g, packed, n_frames, prev, plane_stride, lda, rgb, Q, s, rf);
        else launch_band21_t<false, kB44RecLo, kB44RecHi, 1>(g, packed, n_frames, prev, plane_stride, lda, rgb, Q, s, rf);
    } else {
        if (fp) launch_band21_t<true, 0u, 0u, 2>(g, packed, n_frames, prev, plane_stride, lda, rgb, Q, s, rf);
        else launch_band21_t<false, 0u, 0u, 2>(g, packed, n_frames, prev, plane_stride, lda, rgb, Q, s, rf);
    }
}

#define VCF_DWT_FOR_EACH_F(X) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(18)

void fwd_level(int F, const LevelArgs &a, bool first, bool last)
{
    switch (F) {
#define X(n)                                                                                                       \
    case n:                                                                                                        \
        launch_fwd_level<n>(a, first, last);                                                                       \
        break;
        VCF_DWT_FOR_EACH_F(X)
#undef X
    default:
        break;
    }
}

void strip_level(int F, const LevelArgs &a, bool first, bool last)
{
    switch (F) {
#define X(n)                                                                                                       \
    case n:                                                                                                        \
        launch_strip_level<n>(a, first, last);                                                                     \
        break;
        VCF_DWT_FOR_EACH_F(X)
#undef X
    default:
        break;
    }
}

void inv_level(int F, const LevelArgs &a, bool from_packed, bool to_rgb, uint8_t *rgb_out)
{
    switch (F) {
#define X(n)                                                                                                       \
    case n:                                                                                                        \
        launch_inv_level<n>(a, from_packed, to_rgb, rgb_out);                                                      \
        break;
        VCF_DWT_FOR_EACH_F(X)
#undef X
    default:
        break;
    }
}

// ---------------------------------------------------------------------------
// Frame pipeline over library streams (the encode's level-by-level chain)
// ---------------------------------------------------------------------------
// A 4K level 1 fills the chip; levels 3 .. l hold a few thousand waves or a
// few hundred workgroups each, whose serial chains leave most SIMDs idle
// (C3: levels 4 and 5 take 0.09 ms for 1/300 of level 1's samples).  Frames
// are independent, so a batch is cut into chunks of frames whose level
// chains run on several streams: one chunk's small levels overlap another's
// large ones.  The caller's stream forks to the library's streams through an
// event and joins them again, so the call keeps its stream semantics; each
// chunk touches only its own frames' input, output and workspace planes.
// (helpers in vcf_pipeline.h)
// the default: batches of at least two frames of at least 2^20 pixels
// (smaller frames stay on the caller's stream)
bool pipeline_default(long long n_frames, int H, int W) { return n_frames >= 2 && (long long)H * W >= (1LL << 20); }
// (measured on C3, ABBA: encode two unstaggered chunks -7.8 %; staggering, more chunks or
// streams, and every decode pipeline were slower -- DESIGN.md §6)
constexpr PipeShape kEncodePipe{2, 2, false};

// ---------------------------------------------------------------------------
// lifting path (vcf_dwt_lift.h): launches
// ---------------------------------------------------------------------------
// resident workgroups of one kernel on the device
template <typename K>
int resident_slots(K kern, int threads)
{
    int dev = 0, n_cu = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
        n_cu = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, 0) != hipSuccess || per_cu <= 0)
        per_cu = 4;
    return n_cu * per_cu;
}

// band rows of a lifting launch: time ~ (rounds of resident workgroups) x
// (row pairs per band + the 4 of the pipeline's warm-up)
int lift_brows(long long per_band, int rows, int slots, int steps_per_row = 1, int warmup = 4)
{
    int n_bands = 1;
    long long best = -1;
    for (int nb = 1; nb <= rows; ++nb) {
        const int br = (rows + nb - 1) / nb;
        if (nb > 1 && (rows + br - 1) / br != nb) continue;
        const long long rounds = (per_band * nb + slots - 1) / slots;
        const long long cost = rounds * ((long long)steps_per_row * br + warmup);
        if (best < 0 || cost < best) {
            best = cost;
            n_bands = nb;
        }
    }
    return (rows + n_bands - 1) / n_bands;
}

int lift_check(int wavelet)
{
    if (strcmp(kWavelets[wavelet].name, "bior4.4") != 0)
        return set_error(VCF_ERR_INVALID, "lifting path: bior4.4 (CDF 9/7) only, not %s", kWavelets[wavelet].name);
    return VCF_OK;
}

#endif  // VCF_DWT_KERNELS_ONLY
// A/B knob of the opt-in lifting path (tests/test_dwt_lift_gpu.py compares the two
// forms): vcf_dwt_lift_set_fused(0) selects one launch per level instead of the
// fused level pairs, for the whole process.
std::atomic<int> g_lift_fused{1};
inline bool lift_nofuse() { return g_lift_fused.load(std::memory_order_relaxed) == 0; }
}  // namespace
}  // namespace vcf

#ifndef VCF_DWT_KERNELS_ONLY
using namespace vcf;

extern "C" {

int vcf_wavelet_index(const char *name, int32_t *index)
{
    if (!name || !index) return set_error(VCF_ERR_INVALID, "null pointer");
    for (int i = 0; i < kNumWavelets; ++i)
        if (strcmp(kWavelets[i].name, name) == 0) {
            *index = i;
            return VCF_OK;
        }
    return set_error(VCF_ERR_INVALID, "unknown wavelet '%s'", name);
}

int vcf_dwt_layout(int32_t H, int32_t W, int32_t levels, int32_t *sub_h, int32_t *sub_w, int64_t *packed_bytes,
                   int64_t *workspace_bytes_per_frame)
{
    if (H <= 0 || W <= 0 || levels < 1 || levels > kMaxLevels) return set_error(VCF_ERR_INVALID, "bad layout args");
    DwtGeom g;
    dwt_geom(H, W, levels, 2, g);
    for (int l = 1; l <= levels; ++l) {
        if (sub_h) sub_h[l - 1] = g.hs[l];
        if (sub_w) sub_w[l - 1] = g.ws[l];
    }
    if (packed_bytes) *packed_bytes = g.packed_bytes;
    if (workspace_bytes_per_frame) *workspace_bytes_per_frame = 3 * plane_doubles(g) * (int64_t)sizeof(double);
    return VCF_OK;
}

// one stream's level chain of the encode (the frame pipeline calls it per
// chunk of frames with its hook).  Levels: 1 and 2 in one band launch when
// band12_ok (10-tap filters with compile-time taps, C3), else fused level
// kernels; levels between the first and the last on the strip kernels
// (F <= kMaxStripF and planes of at least 2F); levels after the first whose
// input planes have at most kSepArea samples on the separable kernels -- one
// thread per output beats the fused tile's three serial channels there (-2.2 %
// on C3, ABBA); filters longer than kMaxFastF on the separable kernels alone.
constexpr long long kSepArea = 40000;

static int encode_chain(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t wavelet,
                        int32_t levels, int32_t Q, uint8_t *packed_dev, void *workspace_dev, hipStream_t s,
                        const PipeHook *hook, long long rule_frames)
{
    int rc = VCF_OK;
    Filters flt;
    if ((rc = device_filters(wavelet, flt)) != VCF_OK) return rc;
    DwtGeom g;
    dwt_geom(H, W, levels, kWavelets[wavelet].len, g);
    const int F = g.F;
    const long long pd = plane_doubles(g);
    double *base = (double *)workspace_dev;
    const long long ws_stride = pd;                          // per plane
    double *A = base, *D = base + std::max<long long>((long long)g.hs[1] * g.ws[0], (long long)g.hs[1] * 2 * g.ws[1]);
    double *LL0 = D + (D - A), *LL1 = LL0 + 4LL * g.hs[1] * g.ws[1];
    const unsigned planes = (unsigned)(n_frames * 3);
    const double *in = nullptr;
    const bool fused = fast_filter(F);
    // one level on the separable kernels (column pass, then the row pass into the subbands / LL)
    auto sep_level = [&](int l) {
        const int h = g.hs[l - 1], w = g.ws[l - 1], hh = g.hs[l], hw = g.ws[l];
        if (l == 1)
            hipLaunchKernelGGL(dwt_cols_kernel<true>, dim3(gx(w), hh, planes), dim3(256), 0, s, rgb_dev,
                               (long long)H * W * 3, nullptr, 0LL, A, D, ws_stride, h, w, F, flt);
        else
            hipLaunchKernelGGL(dwt_cols_kernel<false>, dim3(gx(w), hh, planes), dim3(256), 0, s, nullptr, 0LL, in,
                               ws_stride, A, D, ws_stride, h, w, F, flt);
        double *LLout = (l & 1) ? LL0 : LL1;
        if (l == levels)
            hipLaunchKernelGGL(dwt_rows_kernel<true>, dim3(gx(hw), hh, planes), dim3(256), 0, s, A, D, ws_stride,
                               LLout, ws_stride, packed_dev, g.packed_bytes, g.ll_off, g.sb_off[l][0],
                               g.sb_off[l][1], g.sb_off[l][2], hh, w, hw, F, Q, flt);
        else
            hipLaunchKernelGGL(dwt_rows_kernel<false>, dim3(gx(hw), hh, planes), dim3(256), 0, s, A, D, ws_stride,
                               LLout, ws_stride, packed_dev, g.packed_bytes, g.ll_off, g.sb_off[l][0],
                               g.sb_off[l][1], g.sb_off[l][2], hh, w, hw, F, Q, flt);
    };
    int l_start = 1;
    int band_id = 0;
    if (fused && band12_ok(g, kWavelets[wavelet], band_id)) {
        // levels 1 and 2 in one launch: LL1 never leaves the chip; LL2 lands where level 2's would
        if ((rc = hook_wait(hook, s)) != VCF_OK) return rc;
        launch_band12(band_id, g, rgb_dev, n_frames, LL1, ws_stride, packed_dev, Q, s, rule_frames);
        if ((rc = hip_check(hipGetLastError(), "dwt_band12_kernel launch")) != VCF_OK) return rc;
        if ((rc = hook_rec(hook, s)) != VCF_OK) return rc;
        in = LL1;
        l_start = 3;
    }
    for (int l = l_start; l <= levels; ++l) {
        double *LLout = (l & 1) ? LL0 : LL1;
        if (l == 1 && (rc = hook_wait(hook, s)) != VCF_OK) return rc;
        if (!fused || (l > 1 && (long long)g.hs[l - 1] * g.ws[l - 1] <= kSepArea)) {
            sep_level(l);
        } else {
            const LevelArgs a{rgb_dev, (long long)H * W * 3, in, ws_stride, LLout, packed_dev, g.packed_bytes, g.ll_off,
                              g.sb_off[l][0], g.sb_off[l][1], g.sb_off[l][2], g.hs[l - 1], g.ws[l - 1], g.hs[l],
                              g.ws[l], Q, 0, (unsigned)n_frames, flt, &kWavelets[wavelet], s};
            // strips need planes of at least 2F rows and columns (their row wrap)
            const bool strip = F <= kMaxStripF && g.hs[l - 1] >= 2 * F && g.ws[l - 1] >= 2 * F && l > 1 && l < levels;
            if (strip) strip_level(F, a, false, false);
            else fwd_level(F, a, l == 1, l == levels);
        }
        in = LLout;
        if ((rc = hip_check(hipGetLastError(), "dwt level launch")) != VCF_OK) return rc;
        if (l == 1 && (rc = hook_rec(hook, s)) != VCF_OK) return rc;
    }
    return VCF_OK;
}

int vcf_dwt_dz_encode(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t wavelet,
                      int32_t levels, int32_t Q, uint8_t *packed_dev, void *workspace_dev, void *stream)
{
    int rc = check_dwt(rgb_dev, packed_dev, n_frames, H, W, wavelet, levels, Q, false);
    if (rc != VCF_OK) return rc;
    if (n_frames == 0) return VCF_OK;
    if (!workspace_dev) return set_error(VCF_ERR_INVALID, "null workspace");
    if (n_frames * 3 > 65535) return set_error(VCF_ERR_INVALID, "at most 21845 frames per call");
    hipStream_t s = (hipStream_t)stream;
    DwtGeom g;
    dwt_geom(H, W, levels, kWavelets[wavelet].len, g);
    int id = 0;
    // the frame pipeline pays only for the level-by-level chain: with the fused
    // level-1+2 band kernel one launch fills the chip (C3: 0.594 ms on one
    // stream vs 0.635 ms pipelined, ABBA)
    const bool band = fast_filter(g.F) && band12_ok(g, kWavelets[wavelet], id);
    bool pipe = !band && fast_filter(g.F) && pipeline_default(n_frames, H, W);
    // (A/B: VCF_DWT_ENC_PIPE=0/1, read per call; with the band kernel the chunks keep the call's band cut)
    if (const char *e = getenv("VCF_DWT_ENC_PIPE")) pipe = atoi(e) != 0 && fast_filter(g.F) && pipeline_default(n_frames, H, W);
    if (pipe) {
        const long long fpx = (long long)H * W * 3, wsf = 3 * plane_doubles(g);
        return run_pipelined(n_frames, kEncodePipe, s, [&](long long f0, long long n, hipStream_t cs, const PipeHook *hook) {
            return encode_chain(rgb_dev + f0 * fpx, n, H, W, wavelet, levels, Q, packed_dev + f0 * g.packed_bytes,
                                (double *)workspace_dev + f0 * wsf, cs, hook, n_frames);
        });
    }
    return encode_chain(rgb_dev, n_frames, H, W, wavelet, levels, Q, packed_dev, workspace_dev, s, nullptr, n_frames);
}

// one stream's level chain of the decode: coarsest level first; the line
// kernel (idwt_line_kernel) where line_ok, else the fused level kernels;
// subbands shorter than F/2 (pywt's short-input branch: the coefficients wrap
// around more than once) and filters longer than kMaxFastF on the separable
// kernels, whose loads take any index modulo the line length
// the fast decode's level chain over n_frames frames on stream s (the frame pipeline
// calls it per chunk); rule_frames: the call's frames, for the band cut of levels 2 + 1
static int decode_chain_fast(const uint8_t *packed_dev, int64_t n_frames, int32_t H, int32_t W, int32_t wavelet,
                             int32_t levels, int32_t Q, uint8_t *rgb_dev, void *workspace_dev, hipStream_t s,
                             long long rule_frames)
{
    int rc = VCF_OK;
    Filters flt;
    if ((rc = device_filters(wavelet, flt)) != VCF_OK) return rc;
    DwtGeom g;
    dwt_geom(H, W, levels, kWavelets[wavelet].len, g);
    const int F = g.F;
    const long long pd = plane_doubles(g);
    double *base = (double *)workspace_dev;
    const long long ws_stride = pd;
    double *A = base, *D = base + std::max<long long>((long long)g.hs[1] * g.ws[0], (long long)g.hs[1] * 2 * g.ws[1]);
    double *P0 = D + (D - A), *P1 = P0 + 4LL * g.hs[1] * g.ws[1];
    const double *prev = nullptr;
    int lda = 0;
    int id21 = 0;
    const bool b21 = band21_ok(g, kWavelets[wavelet], id21);
    for (int r = levels; r >= 1; --r) {
        if (b21 && r == 2) {   // levels 2 and 1 in one launch, LL1 on chip
            launch_band21(id21, g, packed_dev, n_frames, prev, ws_stride, lda, rgb_dev, Q, s, rule_frames);
            return hip_check(hipGetLastError(), "idwt_band21_kernel launch");
        }
        const int h = g.hs[r], w = g.ws[r];
        const int oh = r > 1 ? g.hs[r - 1] : 2 * h, ow = r > 1 ? g.ws[r - 1] : 2 * w;
        double *out = (r & 1) ? P0 : P1;
        const LevelArgs a{nullptr, 0, prev, ws_stride, out, const_cast<uint8_t *>(packed_dev), g.packed_bytes,
                          g.ll_off, g.sb_off[r][0], g.sb_off[r][1], g.sb_off[r][2], h, w, oh, ow, Q, lda,
                          (unsigned)n_frames, flt, &kWavelets[wavelet], s};
        int id = 0;
        if (line_ok(kWavelets[wavelet], h, w, id)) launch_line(id, a, r == levels, r == 1, rgb_dev);
        else inv_level(F, a, r == levels, r == 1, rgb_dev);
        prev = out;
        lda = ow;
        if ((rc = hip_check(hipGetLastError(), "idwt level launch")) != VCF_OK) return rc;
    }
    return VCF_OK;
}

// The decode as a frame pipeline (two chunks on two library streams, one chunk's small
// coarse levels beside the other chunk's levels 2 + 1 band, the band cut kept at the
// whole call's): off -- measured slower in every form, round 6's with the fused band
// included (C3 0.591 vs 0.528 ms, profiles/r06_dwt_decode_pipeline_not_kept.json).
// VCF_DWT_DEC_PIPE=1 (read per call) selects it for A/B.
constexpr PipeShape kDecodePipe{2, 2, false};
#ifndef VCF_DWT_DEC_PIPE_DEFAULT
#define VCF_DWT_DEC_PIPE_DEFAULT 0
#endif

int vcf_dwt_dz_decode(const uint8_t *packed_dev, int64_t n_frames, int32_t H, int32_t W, int32_t wavelet,
                      int32_t levels, int32_t Q, uint8_t *rgb_dev, void *workspace_dev, void *stream)
{
    int rc = check_dwt(packed_dev, rgb_dev, n_frames, H, W, wavelet, levels, Q, true);
    if (rc != VCF_OK) return rc;
    if (n_frames == 0) return VCF_OK;
    if (!workspace_dev) return set_error(VCF_ERR_INVALID, "null workspace");
    if (n_frames * 3 > 65535) return set_error(VCF_ERR_INVALID, "at most 21845 frames per call");
    hipStream_t s = (hipStream_t)stream;
    Filters flt;
    if ((rc = device_filters(wavelet, flt)) != VCF_OK) return rc;
    DwtGeom g;
    dwt_geom(H, W, levels, kWavelets[wavelet].len, g);
    const int F = g.F;
    const long long pd = plane_doubles(g);
    double *base = (double *)workspace_dev;
    const long long ws_stride = pd;
    double *A = base, *D = base + std::max<long long>((long long)g.hs[1] * g.ws[0], (long long)g.hs[1] * 2 * g.ws[1]);
    double *P0 = D + (D - A), *P1 = P0 + 4LL * g.hs[1] * g.ws[1];
    const unsigned planes = (unsigned)(n_frames * 3);
    const double *prev = nullptr;
    int lda = 0;
    const bool short_lines = g.hs[levels] < F / 2 || g.ws[levels] < F / 2;
    if (fast_filter(F) && !short_lines) {
        int id21 = 0;
        bool pipe = VCF_DWT_DEC_PIPE_DEFAULT && band21_ok(g, kWavelets[wavelet], id21) && levels > 2 &&
                    pipeline_default(n_frames, H, W);
        if (const char *e = getenv("VCF_DWT_DEC_PIPE")) pipe = atoi(e) != 0 && pipeline_default(n_frames, H, W);
        if (pipe) {
            const long long fpx = (long long)H * W * 3, wsf = 3 * pd;
            return run_pipelined(n_frames, kDecodePipe, s, [&](long long f0, long long n, hipStream_t cs, const PipeHook *) {
                return decode_chain_fast(packed_dev + f0 * g.packed_bytes, n, H, W, wavelet, levels, Q,
                                         rgb_dev + f0 * fpx, (double *)workspace_dev + f0 * wsf, cs, n_frames);
            });
        }
        return decode_chain_fast(packed_dev, n_frames, H, W, wavelet, levels, Q, rgb_dev, workspace_dev, s, n_frames);
    }
    for (int r = levels; r >= 1; --r) {
        const int h = g.hs[r], w = g.ws[r];
        if (r == levels)
            hipLaunchKernelGGL(idwt_rows_kernel<true>, dim3(gx(2 * w), h, planes), dim3(256), 0, s, packed_dev,
                               g.packed_bytes, g.ll_off, g.sb_off[r][0], g.sb_off[r][1], g.sb_off[r][2], nullptr,
                               0LL, 0, A, D, ws_stride, h, w, F, Q, flt);
        else
            hipLaunchKernelGGL(idwt_rows_kernel<false>, dim3(gx(2 * w), h, planes), dim3(256), 0, s, packed_dev,
                               g.packed_bytes, g.ll_off, g.sb_off[r][0], g.sb_off[r][1], g.sb_off[r][2], prev,
                               ws_stride, lda, A, D, ws_stride, h, w, F, Q, flt);
        double *out = (r & 1) ? P0 : P1;
        hipLaunchKernelGGL(idwt_cols_kernel, dim3(gx(2 * w), 2 * h, planes), dim3(256), 0, s, A, D, ws_stride, out,
                           ws_stride, h, 2 * w, F, flt);
        prev = out;
        lda = 2 * w;   // the next level trims rows/cols by indexing only h' x w'
        if ((rc = hip_check(hipGetLastError(), "dwt decode launch")) != VCF_OK) return rc;
    }
    const int Ho = 2 * g.hs[1], Wo = 2 * g.ws[1];
    const long long npx = (long long)Ho * Wo;
    hipLaunchKernelGGL(dwt_to_rgb_kernel, dim3((unsigned)((npx + 255) / 256), (unsigned)n_frames), dim3(256), 0, s,
                       prev, ws_stride, rgb_dev, npx, npx * 3);
    return hip_check(hipGetLastError(), "dwt to_rgb launch");
}

// The lifting path (vcf_dwt_lift.h): bior4.4 only, same buffers, layout and
// workspace as vcf_dwt_dz_encode / _decode; results within +-1 of theirs.
int vcf_dwt_set_inverse_band21(int32_t on)
{
    g_band21.store(on ? 1 : 0, std::memory_order_relaxed);
    return VCF_OK;
}

int vcf_dwt_lift_set_fused(int32_t fused)
{
    g_lift_fused.store(fused ? 1 : 0, std::memory_order_relaxed);
    return VCF_OK;
}

int vcf_dwt_dz_encode_lift(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t wavelet,
                           int32_t levels, int32_t Q, uint8_t *packed_dev, void *workspace_dev, void *stream)
{
    int rc = check_dwt(rgb_dev, packed_dev, n_frames, H, W, wavelet, levels, Q, false);
    if (rc != VCF_OK || (rc = lift_check(wavelet)) != VCF_OK) return rc;
    if (n_frames == 0) return VCF_OK;
    if (!workspace_dev) return set_error(VCF_ERR_INVALID, "null workspace");
    hipStream_t s = (hipStream_t)stream;
    DwtGeom g;
    dwt_geom(H, W, levels, 10, g);
    const long long pd = plane_doubles(g);
    // (the second plane starts 16-byte aligned: the kernels' double2 loads)
    double *P[2] = {(double *)workspace_dev, (double *)workspace_dev + ((long long)g.hs[1] * g.ws[1] + 1) / 2 * 2};
    const bool qp2 = (Q & (Q - 1)) == 0;
    // explicit ping-pong: a launch reads `in` (level l - 1's LL) and writes the other plane
    const double *in = nullptr;
    int nb = 0;
    const bool nofuse = lift_nofuse();
    for (int l = 1; l <= levels;) {
        const int h = g.hs[l - 1], w = g.ws[l - 1], hh = g.hs[l], hw = g.ws[l];
        const bool first = l == 1;
        double *out = P[nb];
        // levels l and l + 1 in one launch (lift_fwd12_kernel) on planes that halve evenly
        // twice with dword-aligned level-l subband rows (C3: levels 1 + 2 and 3 + 4)
        if (!nofuse && l + 1 <= levels && w % 4 == 0 && h % 4 == 0 && hw % 8 == 0 && w == 2 * hw &&
            g.packed_bytes % 4 == 0 && g.sb_off[l][0] % 4 == 0 && (g.sb_off[l][1] - g.sb_off[l][0]) % 4 == 0) {
            const int hh2 = g.hs[l + 1], hw2 = g.ws[l + 1];
            const bool last2 = l + 1 == levels;
            auto pick = [&](auto fc) {
                constexpr bool F1 = decltype(fc)::value;
                return qp2 ? (last2 ? lift::lift_fwd12_kernel<true, true, F1> : lift::lift_fwd12_kernel<true, false, F1>)
                           : (last2 ? lift::lift_fwd12_kernel<false, true, F1> : lift::lift_fwd12_kernel<false, false, F1>);
            };
            auto kern = first ? pick(std::true_type{}) : pick(std::false_type{});
            const int n_strips = (hw2 + lift::kV2 - 1) / lift::kV2;
            const long long per_band = n_frames * n_strips;
            const int brows = lift_brows(per_band, hh2, resident_slots(kern, lift::kNT), 2, 12);
            const int n_bands = (hh2 + brows - 1) / brows;
            const long long grid = per_band * n_bands;
            if (grid > 0x7fffffffLL) return set_error(VCF_ERR_INVALID, "too many frames per call");
            hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(lift::kNT), 0, s, rgb_dev, (long long)H * W * 3, in,
                               out, pd, packed_dev, g.packed_bytes, g.ll_off, g.sb_off[l][0], g.sb_off[l][1],
                               g.sb_off[l + 1][0], g.sb_off[l + 1][1], g.sb_off[l + 1][2], h, w, hh, hw, hh2, hw2, Q,
                               n_strips, n_bands, brows);
            if ((rc = hip_check(hipGetLastError(), "lift_fwd12_kernel launch")) != VCF_OK) return rc;
            in = out;
            nb ^= 1;
            l += 2;
            continue;
        }
        const bool last = l == levels;
        const int n_strips = (hw + lift::kValid - 1) / lift::kValid;
        // the branch-free body for even planes with dword-aligned subband rows, else the general one
        const bool aligned = w == 2 * hw && hw % 4 == 0 && g.packed_bytes % 4 == 0 && g.sb_off[l][0] % 4 == 0 &&
                             (g.sb_off[l][1] - g.sb_off[l][0]) % 4 == 0;
        const int n_int = aligned ? n_strips : 0;
        const long long per_band = n_frames * n_strips;
        auto kern = qp2 ? (first ? (last ? lift::lift_fwd_kernel<true, true, true> : lift::lift_fwd_kernel<true, false, true>)
                                 : (last ? lift::lift_fwd_kernel<false, true, true>
                                         : lift::lift_fwd_kernel<false, false, true>))
                        : (first ? (last ? lift::lift_fwd_kernel<true, true, false>
                                         : lift::lift_fwd_kernel<true, false, false>)
                                 : (last ? lift::lift_fwd_kernel<false, true, false>
                                         : lift::lift_fwd_kernel<false, false, false>));
        const int brows = lift_brows(per_band, hh, resident_slots(kern, lift::kNT));
        const int n_bands = (hh + brows - 1) / brows, n_edge = n_strips - n_int;
        const int brows_e = brows, n_bands_e = n_bands;
        const long long edge_blocks = n_frames * n_edge * n_bands_e;
        const long long grid = n_frames * n_int * n_bands + edge_blocks;
        if (grid > 0x7fffffffLL) return set_error(VCF_ERR_INVALID, "too many frames per call");
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(lift::kNT), 0, s, rgb_dev, (long long)H * W * 3, in, pd,
                           out, packed_dev, g.packed_bytes, g.ll_off, g.sb_off[l][0], g.sb_off[l][1], g.sb_off[l][2], h,
                           w, hh, hw, Q, n_int, n_edge, n_bands, brows, n_bands_e, brows_e, (int)edge_blocks);
        if ((rc = hip_check(hipGetLastError(), "lift_fwd_kernel launch")) != VCF_OK) return rc;
        in = out;
        nb ^= 1;
        ++l;
    }
    return VCF_OK;
}

// The lifting path's float64 coefficients before quantization, for one frame (the
// tolerance measurement of tests/test_dwt_lift_gpu.py): one general-body launch per
// level; coef_dev receives, per level l = 1..levels, the details [LH, HL, HH][Y, Co,
// Cg][hs[l] x ws[l]], then LL_levels [Y, Co, Cg][hs x ws]; packed_dev (the packed
// layout's bytes) receives Q = 1 indices as scratch.
int vcf_dwt_lift_analyze_f64(const uint8_t *rgb_dev, int32_t H, int32_t W, int32_t levels, double *coef_dev,
                             uint8_t *packed_dev, void *workspace_dev, void *stream)
{
    int32_t wavelet = 0;
    int rc = vcf_wavelet_index("bior4.4", &wavelet);
    if (rc != VCF_OK) return rc;
    rc = check_dwt(rgb_dev, packed_dev, 1, H, W, wavelet, levels, 1, false);
    if (rc != VCF_OK) return rc;
    if (!coef_dev || !workspace_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    hipStream_t s = (hipStream_t)stream;
    DwtGeom g;
    dwt_geom(H, W, levels, 10, g);
    const long long pd = plane_doubles(g);
    double *P[2] = {(double *)workspace_dev, (double *)workspace_dev + ((long long)g.hs[1] * g.ws[1] + 1) / 2 * 2};
    const double *in = nullptr;
    int nb = 0;
    double *raw = coef_dev;
    for (int l = 1; l <= levels; ++l) {
        const int h = g.hs[l - 1], w = g.ws[l - 1], hh = g.hs[l], hw = g.ws[l];
        double *out = P[nb];
        const int n_strips = (hw + lift::kValid - 1) / lift::kValid, brows = 16;
        const int n_bands = (hh + brows - 1) / brows;
        auto kern = l == 1 ? lift::lift_fwd_raw_kernel<true> : lift::lift_fwd_raw_kernel<false>;
        hipLaunchKernelGGL(kern, dim3((unsigned)(n_strips * n_bands)), dim3(lift::kNT), 0, s, rgb_dev, in, pd, out,
                           packed_dev, g.packed_bytes, g.sb_off[l][0], g.sb_off[l][1], g.sb_off[l][2], h, w, hh, hw,
                           n_strips, n_bands, brows, raw);
        if ((rc = hip_check(hipGetLastError(), "lift_fwd_raw_kernel launch")) != VCF_OK) return rc;
        raw += 9LL * hh * hw;
        in = out;
        nb ^= 1;
    }
    const int hh = g.hs[levels], hw = g.ws[levels];
    for (int ch = 0; ch < 3; ++ch)
        if ((rc = hip_check(hipMemcpyAsync(raw + (long long)ch * hh * hw, in + ch * pd, sizeof(double) * hh * hw,
                                           hipMemcpyDeviceToDevice, s), "hipMemcpyAsync")) != VCF_OK)
            return rc;
    return VCF_OK;
}

int vcf_dwt_dz_decode_lift(const uint8_t *packed_dev, int64_t n_frames, int32_t H, int32_t W, int32_t wavelet,
                           int32_t levels, int32_t Q, uint8_t *rgb_dev, void *workspace_dev, void *stream)
{
    int rc = check_dwt(packed_dev, rgb_dev, n_frames, H, W, wavelet, levels, Q, true);
    if (rc != VCF_OK || (rc = lift_check(wavelet)) != VCF_OK) return rc;
    if (n_frames == 0) return VCF_OK;
    if (!workspace_dev) return set_error(VCF_ERR_INVALID, "null workspace");
    hipStream_t s = (hipStream_t)stream;
    DwtGeom g;
    dwt_geom(H, W, levels, 10, g);
    const long long pd = plane_doubles(g);
    double *P[2] = {(double *)workspace_dev, (double *)workspace_dev + ((long long)g.hs[1] * g.ws[1] + 1) / 2 * 2};
    // explicit ping-pong: a launch reads `in` (the LL of the level above) and writes the other plane
    const double *in = nullptr;
    int nb = 0;
    const bool nofuse = lift_nofuse();
    for (int r = levels; r >= 1;) {
        const int h = g.hs[r], w = g.ws[r];
        const bool coarsest = r == levels;
        double *out = P[nb];
        // levels r and r - 1 in one launch (lift_inv21_kernel) when each LL is exactly twice
        // the one above both ways (C3: levels 4 + 3 and 2 + 1)
        const int hl = r >= 2 ? g.hs[r - 1] : 0, wl = r >= 2 ? g.ws[r - 1] : 0;
        if (!nofuse && r >= 2 && hl == 2 * h && wl == 2 * w && w % 2 == 0 &&
            (r - 1 == 1 || (g.hs[r - 2] == 2 * hl && g.ws[r - 2] == 2 * wl))) {
            const bool rgb = r - 1 == 1;
            auto kern = coarsest ? (rgb ? lift::lift_inv21_kernel<true, true> : lift::lift_inv21_kernel<true, false>)
                                 : (rgb ? lift::lift_inv21_kernel<false, true> : lift::lift_inv21_kernel<false, false>);
            const int n_strips = (w + lift::kV2 - 1) / lift::kV2;
            const long long per_band = n_frames * n_strips;
            // a band of B upper-level rows: B + 6 of its steps, 2 B + 4 lower-level ones
            const int brows = lift_brows(per_band, h, resident_slots(kern, lift::kNT), 2, 12);
            const int n_bands = (h + brows - 1) / brows;
            const long long grid = per_band * n_bands;
            if (grid > 0x7fffffffLL) return set_error(VCF_ERR_INVALID, "too many frames per call");
            hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(lift::kNT), 0, s, packed_dev, g.packed_bytes, g.ll_off,
                               g.sb_off[r][0], g.sb_off[r][1], g.sb_off[r][2], g.sb_off[r - 1][0],
                               g.sb_off[r - 1][1], g.sb_off[r - 1][2], in, pd, out, rgb_dev,
                               (long long)(2 * g.hs[1]) * (2 * g.ws[1]) * 3, h, w, hl, wl, Q, n_strips, n_bands,
                               brows);
            if ((rc = hip_check(hipGetLastError(), "lift_inv21_kernel launch")) != VCF_OK) return rc;
            in = out;
            nb ^= 1;
            r -= 2;
            continue;
        }
        const int oh = r > 1 ? g.hs[r - 1] : 2 * h, ow = r > 1 ? g.ws[r - 1] : 2 * w;
        const bool rgb = r == 1;
        const int n_strips = (w + lift::kValid - 1) / lift::kValid;
        // the branch-free body for even planes (and even trimmed outputs), else the general one
        const bool aligned = w % 2 == 0 && ow % 2 == 0;
        const int n_int = aligned ? n_strips : 0;
        const long long per_band = n_frames * n_strips;
        auto kern = coarsest ? (rgb ? lift::lift_inv_kernel<true, true> : lift::lift_inv_kernel<true, false>)
                             : (rgb ? lift::lift_inv_kernel<false, true> : lift::lift_inv_kernel<false, false>);
        const int brows = lift_brows(per_band, h, resident_slots(kern, lift::kNT));
        const int n_bands = (h + brows - 1) / brows, n_edge = n_strips - n_int;
        const int brows_e = brows, n_bands_e = n_bands;
        const long long edge_blocks = n_frames * n_edge * n_bands_e;
        const long long grid = n_frames * n_int * n_bands + edge_blocks;
        if (grid > 0x7fffffffLL) return set_error(VCF_ERR_INVALID, "too many frames per call");
        // level r reads the plane the level above wrote (h x w, row stride w) and writes the other
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(lift::kNT), 0, s, packed_dev, g.packed_bytes, g.ll_off,
                           g.sb_off[r][0], g.sb_off[r][1], g.sb_off[r][2], in, pd, w, out, rgb_dev,
                           (long long)(2 * g.hs[1]) * (2 * g.ws[1]) * 3, h, w, oh, ow, Q, n_int, n_edge, n_bands,
                           brows, n_bands_e, brows_e, (int)edge_blocks);
        if ((rc = hip_check(hipGetLastError(), "lift_inv_kernel launch")) != VCF_OK) return rc;
        in = out;
        nb ^= 1;
        --r;
    }
    return VCF_OK;
}

}  // extern "C"
#endif  // VCF_DWT_KERNELS_ONLY
