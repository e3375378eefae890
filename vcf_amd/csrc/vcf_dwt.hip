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

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>

#include "vcf_amd.h"
#include "vcf_internal.h"
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
    const int top = i < F2 - 1 ? i : F2 - 1;
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

__device__ __forceinline__ uint8_t quant_u8(double x, int Q)
{
    const int32_t k = (int32_t)(x / (double)Q);     // astype(int32): truncation toward zero
    return (uint8_t)(uint32_t)(k + 128);            // += 128, astype(uint8): wraps
}

__device__ __forceinline__ uint16_t quant_u16(double x, int Q)
{
    const int32_t k = (int32_t)(x / (double)Q);
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
    // pywt takes a different code path for lines shorter than F/2 (not restated)
    DwtGeom g;
    dwt_geom(H, W, levels, kWavelets[wavelet].len, g);
    const int F2 = kWavelets[wavelet].len / 2;
    if (decode && (g.hs[levels] < F2 || g.ws[levels] < F2))
        return set_error(VCF_ERR_UNSUPPORTED,
                         "level-%d subbands of %d x %d are shorter than the %s filter half-length %d",
                         levels, g.hs[levels], g.ws[levels], kWavelets[wavelet].name, F2);
    return VCF_OK;
}

unsigned gx(int n) { return (unsigned)((n + 255) / 256); }

}  // namespace
}  // namespace vcf

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

int vcf_dwt_dz_encode(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t wavelet,
                      int32_t levels, int32_t Q, uint8_t *packed_dev, void *workspace_dev, void *stream)
{
    int rc = check_dwt(rgb_dev, packed_dev, n_frames, H, W, wavelet, levels, Q, false);
    if (rc != VCF_OK) return rc;
    if (n_frames == 0) return VCF_OK;
    if (!workspace_dev) return set_error(VCF_ERR_INVALID, "null workspace");
    if (n_frames * 3 > 65535) return set_error(VCF_ERR_INVALID, "at most 21845 frames per call");
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
    hipStream_t s = (hipStream_t)stream;
    const unsigned planes = (unsigned)(n_frames * 3);
    const double *in = nullptr;
    for (int l = 1; l <= levels; ++l) {
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
        in = LLout;
        rc = hip_check(hipGetLastError(), "dwt encode launch");
        if (rc != VCF_OK) return rc;
    }
    return VCF_OK;
}

int vcf_dwt_dz_decode(const uint8_t *packed_dev, int64_t n_frames, int32_t H, int32_t W, int32_t wavelet,
                      int32_t levels, int32_t Q, uint8_t *rgb_dev, void *workspace_dev, void *stream)
{
    int rc = check_dwt(packed_dev, rgb_dev, n_frames, H, W, wavelet, levels, Q, true);
    if (rc != VCF_OK) return rc;
    if (n_frames == 0) return VCF_OK;
    if (!workspace_dev) return set_error(VCF_ERR_INVALID, "null workspace");
    if (n_frames * 3 > 65535) return set_error(VCF_ERR_INVALID, "at most 21845 frames per call");
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
    hipStream_t s = (hipStream_t)stream;
    const unsigned planes = (unsigned)(n_frames * 3);
    const double *prev = nullptr;
    int lda = 0;
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
        rc = hip_check(hipGetLastError(), "dwt decode launch");
        if (rc != VCF_OK) return rc;
    }
    const int Ho = 2 * g.hs[1], Wo = 2 * g.ws[1];
    const long long npx = (long long)Ho * Wo;
    hipLaunchKernelGGL(dwt_to_rgb_kernel, dim3((unsigned)((npx + 255) / 256), (unsigned)n_frames), dim3(256), 0, s,
                       prev, ws_stride, rgb_dev, npx, npx * 3);
    return hip_check(hipGetLastError(), "dwt to_rgb launch");
}

}  // extern "C"
