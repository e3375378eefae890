// vcf_plugins.hip -- the alternative colour and quantizer plug-ins of the hot
// path:
//
// * YCrCb (src/YCrCb.py:25-72), the stand-alone pixel codec: RGB -> YCrCb,
//   int16, deadzone quantizer, uint16 indices (and back).  The transform is
//   color_transforms.YCrCb, which the reference does not vendor; it is taken
//   to be OpenCV's integer RGB<->YCrCb (assumption A12: yuv_shift 14,
//   CV_DESCALE rounding, saturate_cast; parity unpinned).
// * LloydMax (src/LloydMax.py:75-143), the quantizer plug-in of 2D-DCT.py,
//   YCrCb.py and the stand-alone LloydMax.py: per channel
//   numpy.histogram(x, bins=max_val-min_val+1, range=(min_val, max_val))
//   (numpy 1.26's uniform-bin arithmetic, pinned by tests/golden/
//   plug_histograms.npz), +1, scalar_quantization's LloydMax_Quantizer
//   (un-vendored; assumption A13: the textbook Lloyd-Max design, restated in
//   oracle/plugins.py), encode = searchsorted(thresholds, x, 'right'),
//   decode = centroids[k].
//
// The per-sample work -- colour conversion, quantization, the histograms,
// the threshold search and the centroid lookup -- runs here; the Lloyd-Max
// design itself (a few iterations over <= 65536 histogram bins) is a host
// function on the downloaded counts.  All kernels are elementwise and
// HBM-bound: grid-stride loops, channels interleaved (H x W x C).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <mutex>
#include <type_traits>
#include <vector>

#include "vcf_amd.h"
#include "vcf_internal.h"

namespace vcf {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxBins = 65536;

unsigned grid_for(int64_t n, int64_t per_thread = 4)
{
    const int64_t g = (n + kThreads * per_thread - 1) / (kThreads * per_thread);
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, 256 * 32));
}

// ---- A12: OpenCV's RGB2YCrCb_i / YCrCb2RGB_i for uint8 ---------------------
__device__ __forceinline__ int sat8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

__device__ __forceinline__ void rgb_to_ycrcb(int r, int g, int b, int &y, int &cr, int &cb)
{
    y = (r * 4899 + g * 9617 + b * 1868 + (1 << 13)) >> 14;
    cr = sat8(((r - y) * 11682 + (128 << 14) + (1 << 13)) >> 14);
    cb = sat8(((b - y) * 9241 + (128 << 14) + (1 << 13)) >> 14);
    y = sat8(y);
}

__device__ __forceinline__ void ycrcb_to_rgb(int y, int cr, int cb, int &r, int &g, int &b)
{
    cr -= 128;
    cb -= 128;
    r = sat8(y + ((cr * 22987 + (1 << 13)) >> 14));
    g = sat8(y + ((cb * -5636 + cr * -11698 + (1 << 13)) >> 14));
    b = sat8(y + ((cb * 29049 + (1 << 13)) >> 14));
}

__global__ __launch_bounds__(kThreads) void ycrcb_from_rgb_kernel(const uint8_t *__restrict__ rgb, int64_t n_px,
                                                                  uint8_t *__restrict__ out)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_px; p += stride) {
        int y, cr, cb;
        rgb_to_ycrcb(rgb[3 * p], rgb[3 * p + 1], rgb[3 * p + 2], y, cr, cb);
        out[3 * p] = (uint8_t)y;
        out[3 * p + 1] = (uint8_t)cr;
        out[3 * p + 2] = (uint8_t)cb;
    }
}

__global__ __launch_bounds__(kThreads) void ycrcb_to_rgb_kernel(const uint8_t *__restrict__ ycc, int64_t n_px,
                                                                uint8_t *__restrict__ out)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_px; p += stride) {
        int r, g, b;
        ycrcb_to_rgb(ycc[3 * p], ycc[3 * p + 1], ycc[3 * p + 2], r, g, b);
        out[3 * p] = (uint8_t)r;
        out[3 * p + 1] = (uint8_t)g;
        out[3 * p + 2] = (uint8_t)b;
    }
}

// YCrCb.encode (:33-51) with the deadzone quantizer: from_RGB, astype(int16),
// += [0, 0, 0] (:29-30), (x / Q).astype(int32) (A5, float64 true division),
// astype(uint16)
__global__ __launch_bounds__(kThreads) void ycrcb_dz_encode_kernel(const uint8_t *__restrict__ rgb, int64_t n_px,
                                                                   int Q, uint16_t *__restrict__ k)
{
    const double q = (double)Q;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_px; p += stride) {
        int c3[3];
        rgb_to_ycrcb(rgb[3 * p], rgb[3 * p + 1], rgb[3 * p + 2], c3[0], c3[1], c3[2]);
#pragma unroll
        for (int c = 0; c < 3; ++c) k[3 * p + c] = (uint16_t)(int32_t)((double)c3[c] / q);
    }
}

// YCrCb.decode (:53-72): Q * k in uint16 (A5), astype(int16), -= 0,
// astype(uint8), to_RGB, clip -- the low byte of Q * k goes to to_RGB
__global__ __launch_bounds__(kThreads) void ycrcb_dz_decode_kernel(const uint16_t *__restrict__ k, int64_t n_px,
                                                                   int Q, uint8_t *__restrict__ rgb)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_px; p += stride) {
        int v[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c] = (uint8_t)(int16_t)(uint16_t)((uint32_t)Q * k[3 * p + c]);
        int r, g, b;
        ycrcb_to_rgb(v[0], v[1], v[2], r, g, b);
        rgb[3 * p] = (uint8_t)r;
        rgb[3 * p + 1] = (uint8_t)g;
        rgb[3 * p + 2] = (uint8_t)b;
    }
}

// ---- YCoCg.py and deadzone.py, the stand-alone pixel codecs ----------------
// YCoCg.encode (src/YCoCg.py:33-56) with -a deadzone: img.astype(int16),
// from_RGB into an int16 array (A4: Y = R/4 + G/2 + B/4, Co = R/2 - B/2,
// Cg = -R/4 + G/2 - B/4 in float64 -- exact quarter multiples -- stored with
// the C cast, i.e. truncated toward zero), += offset [0, 0, 0] (:27-28),
// deadzone (x / Q).astype(int32) (A5: float64 true division of small
// integers, which truncates exactly like integer division), astype(uint16)
// (negative indices wrap).  Four pixels per thread: 12 bytes in, 24 out.
__device__ __forceinline__ void ycocg_i16(int r, int g, int b, int &y, int &co, int &cg)
{
    y = (r + 2 * g + b) / 4;     // C division truncates toward zero, as the int16 store does
    co = (r - b) / 2;
    cg = (-r + 2 * g - b) / 4;
}

__global__ __launch_bounds__(kThreads) void ycocg_dz_encode_kernel(const uint8_t *__restrict__ rgb, int64_t n_px,
                                                                   int Q, uint16_t *__restrict__ k)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; 4 * p < n_px; p += stride) {
        const int64_t p0 = 4 * p;
        const int np = (int)min((int64_t)4, n_px - p0);
        uint8_t px[12];
        if (np == 4 && (((uintptr_t)(rgb + 3 * p0)) & 3) == 0) {
            const uint32_t *s = reinterpret_cast<const uint32_t *>(rgb + 3 * p0);
#pragma unroll
            for (int w = 0; w < 3; ++w) {
                const uint32_t v = s[w];
#pragma unroll
                for (int j = 0; j < 4; ++j) px[4 * w + j] = (uint8_t)(v >> (8 * j));
            }
        } else {
#pragma unroll
            for (int j = 0; j < 12; ++j) px[j] = j < 3 * np ? rgb[3 * p0 + j] : 0;
        }
        uint16_t o[12];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int c[3];
            ycocg_i16(px[3 * i], px[3 * i + 1], px[3 * i + 2], c[0], c[1], c[2]);
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) o[3 * i + ch] = (uint16_t)(int32_t)(c[ch] / Q);
        }
        if (np == 4 && (((uintptr_t)(k + 3 * p0)) & 7) == 0) {
            uint2 *d = reinterpret_cast<uint2 *>(k + 3 * p0);
#pragma unroll
            for (int w = 0; w < 3; ++w)
                d[w] = make_uint2((uint32_t)o[4 * w] | (uint32_t)o[4 * w + 1] << 16,
                                  (uint32_t)o[4 * w + 2] | (uint32_t)o[4 * w + 3] << 16);
        } else {
            for (int j = 0; j < 3 * np; ++j) k[3 * p0 + j] = o[j];
        }
    }
}

// YCoCg.decode (:58-85): k.astype(int16), deadzone Q * k (int16 x Python int
// stays int16 under numpy 1.26's value-based casting: wraps), -= offset 0,
// to_RGB in int16 (A4: R = Y + Co - Cg, G = Y + Cg, B = Y - Co - Cg, each
// wrapping), clip(0, 255), astype(uint8).
__global__ __launch_bounds__(kThreads) void ycocg_dz_decode_kernel(const uint16_t *__restrict__ k, int64_t n_px,
                                                                   int Q, uint8_t *__restrict__ rgb)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_px; p += stride) {
        int v[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c] = (int16_t)(uint16_t)((uint32_t)Q * k[3 * p + c]);
        const int r = (int16_t)(v[0] + v[1] - v[2]), g = (int16_t)(v[0] + v[2]), b = (int16_t)(v[0] - v[1] - v[2]);
        rgb[3 * p] = (uint8_t)sat8(r);
        rgb[3 * p + 1] = (uint8_t)sat8(g);
        rgb[3 * p + 2] = (uint8_t)sat8(b);
    }
}

// YCoCg.py with -a LloydMax: the int16 YCoCg image + offset [-128, 0, 0]
// (:29-30) for the quantizer plug-in, and back (the dequantized int16 image
// - offset, to_RGB in int16, clip, uint8).
__global__ __launch_bounds__(kThreads) void ycocg_i16_from_rgb_kernel(const uint8_t *__restrict__ rgb, int64_t n_px,
                                                                      int off0, int16_t *__restrict__ out)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_px; p += stride) {
        int y, co, cg;
        ycocg_i16(rgb[3 * p], rgb[3 * p + 1], rgb[3 * p + 2], y, co, cg);
        out[3 * p] = (int16_t)(y + off0);
        out[3 * p + 1] = (int16_t)co;
        out[3 * p + 2] = (int16_t)cg;
    }
}

__global__ __launch_bounds__(kThreads) void ycocg_i16_to_rgb_kernel(const int16_t *__restrict__ in, int64_t n_px,
                                                                    int off0, uint8_t *__restrict__ rgb)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_px; p += stride) {
        const int y = (int16_t)(in[3 * p] - off0), co = in[3 * p + 1], cg = in[3 * p + 2];
        rgb[3 * p] = (uint8_t)sat8((int16_t)(y + co - cg));
        rgb[3 * p + 1] = (uint8_t)sat8((int16_t)(y + cg));
        rgb[3 * p + 2] = (uint8_t)sat8((int16_t)(y - co - cg));
    }
}

// deadzone.encode (src/deadzone.py:67-79): img.astype(int16), (x / Q).astype(int32)
// (A5), astype(uint8); decode (:81-93): Q * k in uint8 (value-based casting of
// a Python int Q <= 255 against uint8 keeps uint8: wraps).  Elementwise over
// n bytes, 16 per thread.
template <bool ENC>
__global__ __launch_bounds__(kThreads) void dz_u8_kernel(const uint8_t *__restrict__ x, int64_t n, int Q,
                                                         uint8_t *__restrict__ y)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; 16 * p < n; p += stride) {
        const int64_t b0 = 16 * p;
        auto f = [&](uint32_t v) -> uint32_t { return ENC ? (uint32_t)((int)v / Q) & 0xffu : ((uint32_t)Q * v) & 0xffu; };
        if (b0 + 16 <= n && (((uintptr_t)(x + b0) | (uintptr_t)(y + b0)) & 15) == 0) {
            const uint4 in = *reinterpret_cast<const uint4 *>(x + b0);
            uint32_t w[4] = {in.x, in.y, in.z, in.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t o = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) o |= f((w[i] >> (8 * j)) & 0xffu) << (8 * j);
                w[i] = o;
            }
            *reinterpret_cast<uint4 *>(y + b0) = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
            for (int64_t q = b0; q < min(n, b0 + 16); ++q) y[q] = (uint8_t)f(x[q]);
        }
    }
}

// ---- numpy.histogram(x[..., c], bins=n, range=(lo, hi)), numpy 1.26 --------
// bin_type BT = result_type(lo, hi, x): float32 for float32 x, float64 for
// integer x.  keep = lo <= x <= hi; f = ((x - lo) / (hi - lo)) * n in BT;
// i = int(f); i == n -> n-1; one correction step against the BT edges
// linspace(lo, hi, n+1) (lib/histograms.py, uniform-bin fast path).
template <typename T, typename BT, bool LDS>
__global__ __launch_bounds__(kThreads) void lm_hist_kernel(const T *__restrict__ x, int64_t n, int C, int lo, int hi,
                                                           const BT *__restrict__ edges,
                                                           unsigned long long *__restrict__ counts)
{
    extern __shared__ unsigned int hist[];
    const int nb = hi - lo + 1;
    if constexpr (LDS) {
        for (int i = threadIdx.x; i < C * nb; i += blockDim.x) hist[i] = 0u;
        __syncthreads();
    }
    const BT blo = (BT)lo, span = (BT)(hi - lo), bn = (BT)nb;
    const double dlo = (double)lo, dhi = (double)hi;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const T v = x[i];
        const double dv = (double)v;
        if (!(dv >= dlo && dv <= dhi)) continue;
        const int c = (int)(i % C);
        const BT a = (BT)v;
        const BT f = ((a - blo) / span) * bn;
        int idx = (int)f;
        if (idx == nb) idx -= 1;
        if (a < edges[idx]) idx -= 1;
        if (a >= edges[idx + 1] && idx != nb - 1) idx += 1;
        if constexpr (LDS) atomicAdd(&hist[c * nb + idx], 1u);
        else atomicAdd(&counts[(int64_t)c * nb + idx], 1ull);
    }
    if constexpr (LDS) {
        __syncthreads();
        for (int i = threadIdx.x; i < C * nb; i += blockDim.x)
            if (hist[i]) atomicAdd(&counts[i], (unsigned long long)hist[i]);
    }
}

// ---- encode: k = searchsorted((c[:-1] + c[1:]) / 2, x, 'right') -------------
template <typename TI, typename TO, bool LDS>
__global__ __launch_bounds__(kThreads) void lm_encode_kernel(const TI *__restrict__ x, int64_t n, int C,
                                                             const double *__restrict__ cent, int N,
                                                             TO *__restrict__ k)
{
    extern __shared__ double thr_lds[];
    const int nt = N - 1;
    if constexpr (LDS) {
        for (int i = threadIdx.x; i < C * nt; i += blockDim.x) {
            const int c = i / nt, j = i % nt;
            thr_lds[i] = (cent[c * N + j] + cent[c * N + j + 1]) / 2;
        }
        __syncthreads();
    }
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int c = (int)(i % C);
        const double v = (double)x[i];
        int a = 0, b = nt;   // first threshold > v
        if (v != v) a = nt;  // NaN sorts last
        while (a < b) {
            const int m = (a + b) >> 1;
            double t;
            if constexpr (LDS) t = thr_lds[c * nt + m];
            else t = (cent[c * N + m] + cent[c * N + m + 1]) / 2;
            if (t <= v) a = m + 1;
            else b = m;
        }
        k[i] = (TO)a;   // stored into the caller's array type (C cast, as numpy's setitem)
    }
}

// ---- decode: y = centroids[k] stored into y's integer type ------------------
template <typename TI, typename TO>
__global__ __launch_bounds__(kThreads) void lm_decode_kernel(const TI *__restrict__ k, int64_t n, int C,
                                                             const double *__restrict__ cent, int N,
                                                             TO *__restrict__ y, int32_t *__restrict__ bad)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int c = (int)(i % C);
        int64_t kk = (int64_t)k[i];
        if (kk < 0) kk += N;   // numpy's negative indices
        if (kk < 0 || kk >= N) {
            bad[0] = 1;       // numpy raises IndexError; the host reports it
            y[i] = (TO)0;
            continue;
        }
        y[i] = (TO)(int64_t)cent[(int64_t)c * N + kk];   // float64 -> integer: truncation
    }
}

template <typename F>
int dispatch_dtype(int dt, F &&f)
{
    switch (dt) {
    case VCF_DTYPE_U8: return f((uint8_t *)nullptr);
    case VCF_DTYPE_I16: return f((int16_t *)nullptr);
    case VCF_DTYPE_U16: return f((uint16_t *)nullptr);
    case VCF_DTYPE_F32: return f((float *)nullptr);
    default: return set_error(VCF_ERR_INVALID, "dtype %d not supported here", dt);
    }
}

int check_range(int lo, int hi)
{
    if (hi < lo) return set_error(VCF_ERR_INVALID, "max must be larger than min in range parameter.");
    if ((int64_t)hi - lo + 1 > kMaxBins)
        return set_error(VCF_ERR_UNSUPPORTED, "histogram of %lld bins (at most %d)", (long long)hi - lo + 1, kMaxBins);
    return VCF_OK;
}

// linspace(lo, hi, n + 1) in float64 (arange * step + start, last = stop), cast to BT
template <typename BT>
std::vector<BT> hist_edges(int lo, int hi)
{
    const int nb = hi - lo + 1;
    const double step = (double)(hi - lo) / (double)nb;
    std::vector<BT> e((size_t)nb + 1);
    for (int i = 0; i <= nb; ++i) e[(size_t)i] = (BT)((double)i * step + (double)lo);
    e[(size_t)nb] = (BT)hi;
    return e;
}

// device copies of the edge tables, one per (device, type, range)
template <typename BT>
int edges_dev(int lo, int hi, const BT *&out)
{
    struct Key { int dev, lo, hi; };
    static std::vector<std::pair<Key, BT *>> cache;
    static std::mutex mu;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    std::lock_guard<std::mutex> lock(mu);
    for (auto &kv : cache)
        if (kv.first.dev == dev && kv.first.lo == lo && kv.first.hi == hi) { out = kv.second; return VCF_OK; }
    const std::vector<BT> e = hist_edges<BT>(lo, hi);
    BT *d = nullptr;
    int rc = hip_check(hipMalloc(&d, e.size() * sizeof(BT)), "hipMalloc(histogram edges)");
    if (rc != VCF_OK) return rc;
    rc = hip_check(hipMemcpy(d, e.data(), e.size() * sizeof(BT), hipMemcpyHostToDevice), "hipMemcpy(edges)");
    if (rc != VCF_OK) { (void)hipFree(d); return rc; }
    cache.push_back({Key{dev, lo, hi}, d});
    out = d;
    return VCF_OK;
}

template <typename T>
int launch_hist(const void *x, int64_t n, int C, int lo, int hi, int64_t *counts, hipStream_t s)
{
    using BT = typename std::conditional<std::is_same<T, float>::value, float, double>::type;
    const BT *e = nullptr;
    int rc = edges_dev<BT>(lo, hi, e);
    if (rc != VCF_OK) return rc;
    const int nb = hi - lo + 1;
    const size_t lds = (size_t)C * nb * sizeof(unsigned int);
    unsigned long long *cnt = (unsigned long long *)counts;
    if (lds <= 48 * 1024) {
        const unsigned grid = std::min<unsigned>(grid_for(n, 16), 1024);
        hipLaunchKernelGGL((lm_hist_kernel<T, BT, true>), dim3(grid), dim3(kThreads), lds, s, (const T *)x, n, C, lo,
                           hi, e, cnt);
    } else {
        hipLaunchKernelGGL((lm_hist_kernel<T, BT, false>), dim3(grid_for(n)), dim3(kThreads), 0, s, (const T *)x, n,
                           C, lo, hi, e, cnt);
    }
    return hip_check(hipGetLastError(), "lm_hist_kernel launch");
}

template <typename TI, typename TO>
int launch_encode(const void *x, int64_t n, int C, const double *cent, int N, void *k, hipStream_t s)
{
    const size_t lds = (size_t)C * (N - 1) * sizeof(double);
    if (lds <= 48 * 1024)
        hipLaunchKernelGGL((lm_encode_kernel<TI, TO, true>), dim3(grid_for(n)), dim3(kThreads), lds, s,
                           (const TI *)x, n, C, cent, N, (TO *)k);
    else
        hipLaunchKernelGGL((lm_encode_kernel<TI, TO, false>), dim3(grid_for(n)), dim3(kThreads), 0, s,
                           (const TI *)x, n, C, cent, N, (TO *)k);
    return hip_check(hipGetLastError(), "lm_encode_kernel launch");
}

}  // namespace
}  // namespace vcf

using namespace vcf;

extern "C" {

int vcf_ycrcb_from_rgb(const uint8_t *rgb_dev, int64_t n_px, uint8_t *ycrcb_dev, void *stream)
{
    if (n_px < 0) return set_error(VCF_ERR_INVALID, "n_px < 0");
    if (n_px == 0) return VCF_OK;
    if (!rgb_dev || !ycrcb_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    hipLaunchKernelGGL(ycrcb_from_rgb_kernel, dim3(grid_for(n_px)), dim3(kThreads), 0, (hipStream_t)stream, rgb_dev,
                       n_px, ycrcb_dev);
    return hip_check(hipGetLastError(), "ycrcb_from_rgb_kernel launch");
}

int vcf_ycrcb_to_rgb(const uint8_t *ycrcb_dev, int64_t n_px, uint8_t *rgb_dev, void *stream)
{
    if (n_px < 0) return set_error(VCF_ERR_INVALID, "n_px < 0");
    if (n_px == 0) return VCF_OK;
    if (!rgb_dev || !ycrcb_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    hipLaunchKernelGGL(ycrcb_to_rgb_kernel, dim3(grid_for(n_px)), dim3(kThreads), 0, (hipStream_t)stream, ycrcb_dev,
                       n_px, rgb_dev);
    return hip_check(hipGetLastError(), "ycrcb_to_rgb_kernel launch");
}

int vcf_ycrcb_dz_encode(const uint8_t *rgb_dev, int64_t n_px, int32_t Q, uint16_t *k_dev, void *stream)
{
    if (n_px < 0) return set_error(VCF_ERR_INVALID, "n_px < 0");
    if (Q < 1) return set_error(VCF_ERR_INVALID, "quantization step %d out of range", Q);
    if (n_px == 0) return VCF_OK;
    if (!rgb_dev || !k_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    hipLaunchKernelGGL(ycrcb_dz_encode_kernel, dim3(grid_for(n_px)), dim3(kThreads), 0, (hipStream_t)stream, rgb_dev,
                       n_px, Q, k_dev);
    return hip_check(hipGetLastError(), "ycrcb_dz_encode_kernel launch");
}

int vcf_ycrcb_dz_decode(const uint16_t *k_dev, int64_t n_px, int32_t Q, uint8_t *rgb_dev, void *stream)
{
    if (n_px < 0) return set_error(VCF_ERR_INVALID, "n_px < 0");
    if (Q < 1) return set_error(VCF_ERR_INVALID, "quantization step %d out of range", Q);
    if (n_px == 0) return VCF_OK;
    if (!rgb_dev || !k_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    hipLaunchKernelGGL(ycrcb_dz_decode_kernel, dim3(grid_for(n_px)), dim3(kThreads), 0, (hipStream_t)stream, k_dev,
                       n_px, Q, rgb_dev);
    return hip_check(hipGetLastError(), "ycrcb_dz_decode_kernel launch");
}

int vcf_ycocg_dz_encode(const uint8_t *rgb_dev, int64_t n_px, int32_t Q, uint16_t *k_dev, void *stream)
{
    if (n_px < 0) return set_error(VCF_ERR_INVALID, "n_px < 0");
    if (Q < 1) return set_error(VCF_ERR_INVALID, "quantization step %d out of range", Q);
    if (n_px == 0) return VCF_OK;
    if (!rgb_dev || !k_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    hipLaunchKernelGGL(ycocg_dz_encode_kernel, dim3(grid_for(n_px, 16)), dim3(kThreads), 0, (hipStream_t)stream,
                       rgb_dev, n_px, Q, k_dev);
    return hip_check(hipGetLastError(), "ycocg_dz_encode_kernel launch");
}

int vcf_ycocg_dz_decode(const uint16_t *k_dev, int64_t n_px, int32_t Q, uint8_t *rgb_dev, void *stream)
{
    if (n_px < 0) return set_error(VCF_ERR_INVALID, "n_px < 0");
    if (Q < 1 || Q > 32767)
        return set_error(VCF_ERR_UNSUPPORTED, "quantization step %d: int16 dequantization needs 1 <= Q <= 32767", Q);
    if (n_px == 0) return VCF_OK;
    if (!rgb_dev || !k_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    hipLaunchKernelGGL(ycocg_dz_decode_kernel, dim3(grid_for(n_px)), dim3(kThreads), 0, (hipStream_t)stream, k_dev,
                       n_px, Q, rgb_dev);
    return hip_check(hipGetLastError(), "ycocg_dz_decode_kernel launch");
}

int vcf_ycocg_i16_from_rgb(const uint8_t *rgb_dev, int64_t n_px, int32_t offset0, int16_t *out_dev, void *stream)
{
    if (n_px < 0) return set_error(VCF_ERR_INVALID, "n_px < 0");
    if (n_px == 0) return VCF_OK;
    if (!rgb_dev || !out_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    hipLaunchKernelGGL(ycocg_i16_from_rgb_kernel, dim3(grid_for(n_px)), dim3(kThreads), 0, (hipStream_t)stream,
                       rgb_dev, n_px, offset0, out_dev);
    return hip_check(hipGetLastError(), "ycocg_i16_from_rgb_kernel launch");
}

int vcf_ycocg_i16_to_rgb(const int16_t *in_dev, int64_t n_px, int32_t offset0, uint8_t *rgb_dev, void *stream)
{
    if (n_px < 0) return set_error(VCF_ERR_INVALID, "n_px < 0");
    if (n_px == 0) return VCF_OK;
    if (!rgb_dev || !in_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    hipLaunchKernelGGL(ycocg_i16_to_rgb_kernel, dim3(grid_for(n_px)), dim3(kThreads), 0, (hipStream_t)stream, in_dev,
                       n_px, offset0, rgb_dev);
    return hip_check(hipGetLastError(), "ycocg_i16_to_rgb_kernel launch");
}

int vcf_dz_u8_encode(const uint8_t *x_dev, int64_t n, int32_t Q, uint8_t *k_dev, void *stream)
{
    if (n < 0) return set_error(VCF_ERR_INVALID, "n < 0");
    if (Q < 1) return set_error(VCF_ERR_INVALID, "quantization step %d out of range", Q);
    if (n == 0) return VCF_OK;
    if (!x_dev || !k_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    hipLaunchKernelGGL(dz_u8_kernel<true>, dim3(grid_for(n, 64)), dim3(kThreads), 0, (hipStream_t)stream, x_dev, n,
                       Q, k_dev);
    return hip_check(hipGetLastError(), "dz_u8_kernel launch");
}

int vcf_dz_u8_decode(const uint8_t *k_dev, int64_t n, int32_t Q, uint8_t *y_dev, void *stream)
{
    if (n < 0) return set_error(VCF_ERR_INVALID, "n < 0");
    if (Q < 1 || Q > 255)
        return set_error(VCF_ERR_UNSUPPORTED, "quantization step %d: uint8 dequantization needs 1 <= Q <= 255", Q);
    if (n == 0) return VCF_OK;
    if (!k_dev || !y_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    hipLaunchKernelGGL(dz_u8_kernel<false>, dim3(grid_for(n, 64)), dim3(kThreads), 0, (hipStream_t)stream, k_dev, n,
                       Q, y_dev);
    return hip_check(hipGetLastError(), "dz_u8_kernel launch");
}

int vcf_lm_levels(int32_t Q_step, int32_t min_val, int32_t max_val)
{
    if (Q_step < 1) return set_error(VCF_ERR_INVALID, "quantization step %d out of range", Q_step);
    const int rc = check_range(min_val, max_val);
    if (rc != VCF_OK) return rc;
    const int64_t L = (int64_t)max_val - min_val + 1;
    return (int)((L + Q_step - 1) / Q_step);
}

int vcf_lm_histogram(const void *x_dev, int32_t x_dtype, int64_t n_px, int32_t channels, int32_t min_val,
                     int32_t max_val, int64_t *counts_dev, void *stream)
{
    int rc = check_range(min_val, max_val);
    if (rc != VCF_OK) return rc;
    if (n_px < 0 || channels < 1) return set_error(VCF_ERR_INVALID, "bad shape");
    if (!counts_dev || (n_px && !x_dev)) return set_error(VCF_ERR_INVALID, "null buffer");
    const hipStream_t s = (hipStream_t)stream;
    const int64_t nb = (int64_t)max_val - min_val + 1;
    rc = hip_check(hipMemsetAsync(counts_dev, 0, (size_t)(channels * nb) * sizeof(int64_t), s), "hipMemsetAsync");
    if (rc != VCF_OK || n_px == 0) return rc;
    const int64_t n = n_px * channels;
    return dispatch_dtype(x_dtype, [&](auto *tag) -> int {
        using T = typename std::remove_pointer<decltype(tag)>::type;
        return launch_hist<T>(x_dev, n, channels, min_val, max_val, counts_dev, s);
    });
}

int vcf_lm_design(const int64_t *counts, int32_t n_bins, int32_t Q_step, int32_t min_val, double *centroids)
{
    if (!counts || !centroids) return set_error(VCF_ERR_INVALID, "null buffer");
    if (n_bins < 1 || n_bins > kMaxBins || Q_step < 1) return set_error(VCF_ERR_INVALID, "bad design arguments");
    for (int i = 0; i < n_bins; ++i)
        if (counts[i] < 1) return set_error(VCF_ERR_INVALID, "histogram bin %d is empty (the glue adds 1)", i);
    const int N = (n_bins + Q_step - 1) / Q_step;
    // exact prefix sums of n_v and v * n_v
    std::vector<int64_t> S0((size_t)n_bins + 1, 0), S1((size_t)n_bins + 1, 0);
    for (int i = 0; i < n_bins; ++i) {
        S0[(size_t)i + 1] = S0[(size_t)i] + counts[i];
        S1[(size_t)i + 1] = S1[(size_t)i] + counts[i] * (int64_t)(min_val + i);
    }
    std::vector<int> lo((size_t)N + 1), nl((size_t)N + 1);
    for (int j = 0; j < N; ++j) lo[(size_t)j] = j * Q_step;
    lo[(size_t)N] = n_bins;
    auto cent = [&](const std::vector<int> &b) {
        for (int j = 0; j < N; ++j)
            centroids[j] = (double)(S1[(size_t)b[(size_t)j + 1]] - S1[(size_t)b[(size_t)j]]) /
                           (double)(S0[(size_t)b[(size_t)j + 1]] - S0[(size_t)b[(size_t)j]]);
    };
    for (int it = 0; it < 100; ++it) {
        cent(lo);
        nl[0] = 0;
        nl[(size_t)N] = n_bins;
        for (int j = 1; j < N; ++j) nl[(size_t)j] = (int)std::ceil((centroids[j - 1] + centroids[j]) / 2) - min_val;
        if (nl == lo) break;
        lo.swap(nl);
    }
    cent(lo);
    return N;
}

int vcf_lm_encode(const void *x_dev, int32_t x_dtype, int64_t n_px, int32_t channels, const double *centroids_dev,
                  int32_t n_levels, void *k_dev, int32_t k_dtype, void *stream)
{
    if (n_px < 0 || channels < 1 || n_levels < 1) return set_error(VCF_ERR_INVALID, "bad shape");
    if (n_px == 0) return VCF_OK;
    if (!x_dev || !k_dev || !centroids_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    const int64_t n = n_px * channels;
    const hipStream_t s = (hipStream_t)stream;
    return dispatch_dtype(x_dtype, [&](auto *ti) -> int {
        using TI = typename std::remove_pointer<decltype(ti)>::type;
        return dispatch_dtype(k_dtype, [&](auto *to) -> int {
            using TO = typename std::remove_pointer<decltype(to)>::type;
            return launch_encode<TI, TO>(x_dev, n, channels, centroids_dev, n_levels, k_dev, s);
        });
    });
}

int vcf_lm_decode(const void *k_dev, int32_t k_dtype, int64_t n_px, int32_t channels, const double *centroids_dev,
                  int32_t n_levels, void *y_dev, int32_t y_dtype, int32_t *bad_dev, void *stream)
{
    if (n_px < 0 || channels < 1 || n_levels < 1) return set_error(VCF_ERR_INVALID, "bad shape");
    if (k_dtype == VCF_DTYPE_F32 || y_dtype == VCF_DTYPE_F32)
        return set_error(VCF_ERR_INVALID, "indices and levels are stored in integer arrays");
    if (n_px == 0) return VCF_OK;
    if (!k_dev || !y_dev || !centroids_dev || !bad_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    const int64_t n = n_px * channels;
    const hipStream_t s = (hipStream_t)stream;
    return dispatch_dtype(k_dtype, [&](auto *ti) -> int {
        using TI = typename std::remove_pointer<decltype(ti)>::type;
        return dispatch_dtype(y_dtype, [&](auto *to) -> int {
            using TO = typename std::remove_pointer<decltype(to)>::type;
            if constexpr (std::is_same<TI, float>::value || std::is_same<TO, float>::value) {
                return set_error(VCF_ERR_INVALID, "integer arrays only");
            } else {
                hipLaunchKernelGGL((lm_decode_kernel<TI, TO>), dim3(grid_for(n)), dim3(kThreads), 0, s,
                                   (const TI *)k_dev, n, channels, centroids_dev, n_levels, (TO *)y_dev, bad_dev);
                return hip_check(hipGetLastError(), "lm_decode_kernel launch");
            }
        });
    });
}

}  // extern "C"
