// vcf_dct_any.hip -- DCT + deadzone encode/decode for block sizes other than
// the 8x8 fast path: the -B option of src/2D-DCT.py (:29) and the 2..128
// sweep of the -L rate-distortion search (optimize_block_size, :533-579).
//
// What is computed is the same frame pipeline as vcf_dct_dz.hip
// (src/2D-DCT.py:276-361 encode, :399-466 decode; assumptions A1-A5), with the
// length-B pocketfft transforms of vcf_pocketfft.h (compiled in for the 38
// lengths pocketfft factors into 4, 2, 3 and 5 up to 128: 1, 2, 3, 4, 5, 6, 8,
// 9, 10, 12, 15, 16, ..., 120, 125, 128) or of vcf_pocketfft_rt.h (any other
// B <= 4096 that pocketfft plans with rfftp, prime factors above 5 through its
// generic radfg/radbg passes, and the lengths pocketfft_r plans with
// Bluestein -- the first is 191 -- through vcf_pocketfft_blue.h).
//
// Mapping.  A "unit" is one channel of one BxB block.  A workgroup holds
// U = 256/B units (encode, fp32) or 128/B units (decode, fp64), B lanes per
// unit, and one padded LDS tile per unit:
//   encode: lane x builds column x of its unit's YCoCg channel straight from
//     the RGB bytes, runs the column DCT-II in registers and parks it in the
//     tile; after one barrier lane y takes row y, runs the row DCT-II,
//     quantizes and writes its indices to their subband (or -x) positions;
//   decode: lane x gathers column x of the indices from the subband layout,
//     dequantizes, runs the column DCT-III in fp64 and parks it; lane y then
//     runs row y and stores the truncated integers into a padded-frame
//     workspace (stream-ordered allocation); a second, elementwise kernel
//     crops, converts YCoCg->RGB, adds 128 and clips.
// Two index types cover the two places the reference runs this pipeline:
//   u8 / int16 (encode_fn/decode_fn: k + 128 wrapped to uint8 :348,361;
//     astype(int16) - 128, Q*k in int16, the IDCT stored into int16 :399-440);
//   int32 (optimize_block_size :533-579: the int32 k of quantize_decom, Q*k in
//     int32, the IDCT stored into int32, to_RGB in int32).  The search runs
//     from CoDec.__init__ (:99-103) before the deadzone offset of 128 is set
//     (:106-109), so self.offset is still YCoCg's [0, 0, 0] (YCoCg.py:28-29):
//     no -128 before the colour transform and no +128 on k or the pixels;
//   float32 / int16 coefficients ("raw": encode_fn/decode_fn with a quantizer
//     other than deadzone, e.g. -a LloydMax: offset 0 (:106-109), the float32
//     coefficients handed to quantize_decom (:340) and the int16 ones its
//     dequantize_decom returns (:410); the quantizer runs in vcf_plugins.hip).
// These are not the headline kernels (the 8x8 path is); they favour a small,
// uniform implementation over peak bandwidth.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <map>
#include <mutex>
#include <vector>

#include "vcf_amd.h"
#include "vcf_internal.h"
#include "vcf_pocketfft.h"
#include "vcf_pocketfft_rt.h"
#include "vcf_pocketfft_tables.h"

namespace vcf {
namespace {

// Per-device workspace of the two-pass decode.  One buffer per device,
// reused across calls; an event recorded after each use orders the next user
// (any stream) behind the previous one, and growing waits for it first.
struct Scratch {
    std::mutex mu;
    void *ptr = nullptr;
    size_t bytes = 0;
    hipEvent_t done = nullptr;

    int acquire(size_t need, hipStream_t s)
    {
        int rc = VCF_OK;
        if (!done) {
            rc = hip_check(hipEventCreateWithFlags(&done, hipEventDisableTiming), "hipEventCreate");
            if (rc != VCF_OK) return rc;
            rc = hip_check(hipEventRecord(done, s), "hipEventRecord");
            if (rc != VCF_OK) return rc;
        }
        if (need > bytes) {
            rc = hip_check(hipEventSynchronize(done), "hipEventSynchronize");
            if (rc != VCF_OK) return rc;
            if (ptr) (void)hipFree(ptr);
            ptr = nullptr;
            bytes = 0;
            rc = hip_check(hipMalloc(&ptr, need), "hipMalloc(decode workspace)");
            if (rc != VCF_OK) return rc;
            bytes = need;
        }
        return hip_check(hipStreamWaitEvent(s, done, 0), "hipStreamWaitEvent");
    }
    int release(hipStream_t s) { return hip_check(hipEventRecord(done, s), "hipEventRecord"); }
};

Scratch &scratch_for_current_device()
{
    static Scratch per_dev[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    return per_dev[dev];
}

struct GeomB {
    int H, W, Hp, Wp, top, left, nbx, nby;
    long long in_stride, out_stride;   // elements per frame (RGB bytes, coefficient samples)
    long long units;                   // n_frames * nby * nbx * 3
    int sub;                           // subband layout (not -x)
};



// Offset (in samples) of coefficient (i, j) of block (by, bx) inside a
// coefficient frame: get_subbands (A3) puts it in subband (i, j) at
// (by, bx); -x leaves it in place.
template <int B>
__device__ __forceinline__ long long coef_offset(const GeomB &g, int by, int bx, int i, int j)
{
    const long long row = g.sub ? (long long)i * g.nby + by : (long long)by * B + i;
    const long long col = g.sub ? (long long)j * g.nbx + bx : (long long)bx * B + j;
    return (row * g.Wp + col) * 3;
}

// unit -> (frame, block row, block column, channel); channel fastest, so the
// three units of a block share their RGB loads in the cache
__device__ __forceinline__ void unit_coords(const GeomB &g, long long u, long long &f, int &by, int &bx, int &c)
{
    c = (int)(u % 3);
    long long b = u / 3;
    bx = (int)(b % g.nbx);
    b /= g.nbx;
    by = (int)(b % g.nby);
    f = b / g.nby;
}

template <int B> constexpr int enc_units() { return B >= 256 ? 1 : 256 / B; }

// index type of a launch: encode_fn's u8 (k + 128), the -L search's int32, or raw coefficients
enum Mode : int { kU8 = 0, kK32 = 1, kRaw = 2 };
template <int B> constexpr int dec_units() { return B >= 128 ? 1 : 128 / B; }

// ---- encode: RGB u8 -> k (u8 = k + 128 wrapped, int32 k, or float32 coefficients) --
template <int B, int M>
__global__ __launch_bounds__(256) void dct_any_encode_kernel(const uint8_t *__restrict__ rgb,
                                                            void *__restrict__ out, GeomB g, int Q,
                                                            const double *__restrict__ pw)
{
    constexpr int U = enc_units<B>();
    constexpr int LD = B + 1;   // padded row: row-pass reads stride LD words (no bank conflicts)
    __shared__ float tile[U * B * LD];
    const float *tw = c_tw_f32 + slot_off(B);

    const int t = threadIdx.x;
    const int lu = t / B, x = t % B;
    const long long u = (long long)blockIdx.x * U + lu;
    const bool active = lu < U && u < g.units;
    long long f = 0;
    int by = 0, bx = 0, c = 0;
    float *T = tile + (lu < U ? lu : 0) * B * LD;
    if (active) {
        unit_coords(g, u, f, by, bx, c);
        const uint8_t *img = rgb + f * g.in_stride;
        // :276 float32, :282 centred zero padding, :292 -= 128, :298 from_RGB (A4)
        float v[B];
        const int sx = bx * B + x - g.left;
#pragma unroll
        for (int y = 0; y < B; ++y) {
            const int sy = by * B + y - g.top;
            float R = 0.f, G = 0.f, Bl = 0.f;
            if (sy >= 0 && sy < g.H && sx >= 0 && sx < g.W) {
                const uint8_t *p = img + ((long long)sy * g.W + sx) * 3;
                R = (float)p[0]; G = (float)p[1]; Bl = (float)p[2];
            }
            if constexpr (M == kU8) { R = R - 128.f; G = G - 128.f; Bl = Bl - 128.f; }
            float o;
            if (c == 0) o = (R / 4.f + G / 2.f) + Bl / 4.f;
            else if (c == 1) o = R / 2.f - Bl / 2.f;
            else o = ((-R) / 4.f + G / 2.f) - Bl / 4.f;
            v[y] = o;
        }
        // :303 analyze_image (A1): axis 0 (columns) first
        pfft::dct2<float, B>(v, tw);
#pragma unroll
        for (int y = 0; y < B; ++y) T[y * LD + x] = v[y];
    }
    __syncthreads();
    if (active) {
        const int y = x;   // this lane's row
        float v[B];
#pragma unroll
        for (int j = 0; j < B; ++j) v[j] = T[y * LD + j];
        pfft::dct2<float, B>(v, tw);
        if (pw) {   // :313-327 -p: block[..., c] *= QSSs / 121 (or 99), float64 product into float32
            const double *wr = pw + (c ? B * B : 0) + y * B;
#pragma unroll
            for (int j = 0; j < B; ++j) v[j] = (float)((double)v[j] * wr[j]);
        }
        const float q = (float)Q;
        // :343 quantize (A5: (x / Q).astype(int32)), :348 += 128, :361 uint8
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const long long o = f * g.out_stride + coef_offset<B>(g, by, bx, y, j) + c;
            if constexpr (M == kRaw) {
                ((float *)out)[o] = v[j];
            } else {
                const int k = (int)__fdiv_rn(v[j], q);
                if constexpr (M == kK32) ((int32_t *)out)[o] = k;
                else ((uint8_t *)out)[o] = (uint8_t)(k + 128);
            }
        }
    }
}

// ---- decode, pass 1: k -> IDCT'd integers in a padded-frame workspace ------
template <int B, int M>
__global__ __launch_bounds__(128) void dct_any_decode_kernel(const void *__restrict__ kin,
                                                            void *__restrict__ ws, GeomB g, int Q,
                                                            const double *__restrict__ pw)
{
    constexpr int U = dec_units<B>();
    constexpr int LD = B + 1;
    __shared__ double tile[U * B * LD];
    const double *tw = c_tw_f64 + slot_off(B);

    const int t = threadIdx.x;
    const int lu = t / B, x = t % B;
    const long long u = (long long)blockIdx.x * U + lu;
    const bool active = lu < U && u < g.units;
    long long f = 0;
    int by = 0, bx = 0, c = 0;
    double *T = tile + (lu < U ? lu : 0) * B * LD;
    if (active) {
        unit_coords(g, u, f, by, bx, c);
        double v[B];
#pragma unroll
        for (int i = 0; i < B; ++i) {
            const long long o = f * g.out_stride + coef_offset<B>(g, by, bx, i, x) + c;
            if constexpr (M == kK32) {
                // :560-562 decom_k (int32) -> dequantize Q*k in int32
                v[i] = (double)(int32_t)((uint32_t)Q * (uint32_t)((const int32_t *)kin)[o]);
            } else {
                int16_t y16;
                if constexpr (M == kRaw) {
                    y16 = ((const int16_t *)kin)[o];   // :410 the other quantizer's int16 output
                } else {
                    // :399-411 astype(int16) - 128, Q*k in int16 (A5)
                    const int16_t k = (int16_t)((int)((const uint8_t *)kin)[o] - 128);
                    y16 = (int16_t)(Q * (int)k);
                }
                if (pw) {   // :421-435 -p: float32 block /= QSSs / 121 (or 99), stored back into int16
                    const float f = (float)((double)(float)y16 / pw[(c ? B * B : 0) + i * B + x]);
                    y16 = (int16_t)(int)f;
                }
                v[i] = (double)y16;
            }
        }
        // :440 synthesize_image (A2): idct over the integer block -> float64
        pfft::dct3<double, B>(v, tw);
#pragma unroll
        for (int i = 0; i < B; ++i) T[i * LD + x] = v[i];
    }
    __syncthreads();
    if (active) {
        const int y = x;
        double v[B];
#pragma unroll
        for (int j = 0; j < B; ++j) v[j] = T[y * LD + j];
        pfft::dct3<double, B>(v, tw);
        // stored back into the integer array (truncation toward zero)
        const long long row = (long long)by * B + y;
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const long long o = f * ((long long)g.Hp * g.Wp * 3) + (row * g.Wp + (long long)bx * B + j) * 3 + c;
            if constexpr (M == kK32) ((int32_t *)ws)[o] = (int32_t)v[j];
            else ((int16_t *)ws)[o] = (int16_t)(int32_t)v[j];
        }
    }
}

// ---- decode, pass 2: crop, to_RGB, += 128 (0 in raw mode), clip, uint8 -----
template <int M>
__global__ __launch_bounds__(256) void dct_any_to_rgb_kernel(const void *__restrict__ ws, uint8_t *__restrict__ rgb,
                                                             GeomB g, long long n_px)
{
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_px) return;
    const long long per = (long long)g.H * g.W;
    const long long f = p / per;
    const long long r = p % per;
    const int y = (int)(r / g.W), x = (int)(r % g.W);
    const long long o = f * ((long long)g.Hp * g.Wp * 3) + ((long long)(y + g.top) * g.Wp + x + g.left) * 3;
    int o3[3];
    if constexpr (M == kK32) {
        // int32 arithmetic, offset 0 (optimize_block_size: to_RGB of the int32 array, :567-568)
        const int32_t *s = (const int32_t *)ws + o;
        const uint32_t Y = (uint32_t)s[0], Co = (uint32_t)s[1], Cg = (uint32_t)s[2];
        o3[0] = (int32_t)(Y + Co - Cg);
        o3[1] = (int32_t)(Y + Cg);
        o3[2] = (int32_t)(Y - Co - Cg);
    } else {
        // :449 to_RGB in int16 (wrapping), :454 += self.offset in int16 (128; 0 for other quantizers)
        const int16_t *s = (const int16_t *)ws + o;
        const int Y = s[0], Co = s[1], Cg = s[2];
        constexpr int off = M == kRaw ? 0 : 128;
        o3[0] = (int16_t)((int16_t)(Y + Co - Cg) + off);
        o3[1] = (int16_t)((int16_t)(Y + Cg) + off);
        o3[2] = (int16_t)((int16_t)(Y - Co - Cg) + off);
    }
    uint8_t *d = rgb + p * 3;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) d[ch] = (uint8_t)std::min(255, std::max(0, o3[ch]));   // :466 clip, uint8
}

// ---- run-time-length path: block sizes without a compiled kernel ----------
// A workgroup runs one unit at a time (grid-stride): threads take the columns
// (then the rows) of the unit's block, each on its own scratch line, and the
// block sits in a scratch tile between the passes.  Same arithmetic as the
// compiled kernels above, through pfft::RtFft.
constexpr int kRtThreads = 256;
constexpr int kRtMaxB = 4096;

__device__ __forceinline__ long long coef_offset_rt(const GeomB &g, int B, int by, int bx, int i, int j)
{
    const long long row = g.sub ? (long long)i * g.nby + by : (long long)by * B + i;
    const long long col = g.sub ? (long long)j * g.nbx + bx : (long long)bx * B + j;
    return (row * g.Wp + col) * 3;
}

// scratch per workgroup: the B x B tile, then the threads' lines (two of B,
// plus Bluestein's complex arrays), interleaved thread-fastest
__host__ __device__ inline long long rt_ws_per_wg(const pfft::RtPlan &P)
{
    return (long long)P.n * P.n + pfft::rt_line_reals(P) * kRtThreads;
}

template <int M>
__global__ __launch_bounds__(256) void dct_rt_encode_kernel(const uint8_t *__restrict__ rgb, void *__restrict__ out,
                                                           GeomB g, int Q, pfft::RtPlan P,
                                                           const float *__restrict__ mem, float *__restrict__ ws,
                                                           const double *__restrict__ pw)
{
    const int B = P.n, tid = threadIdx.x;
    float *tile = ws + (long long)blockIdx.x * rt_ws_per_wg(P);
    float *lines = tile + (long long)B * B;
    const pfft::Line<float> c{lines + tid, kRtThreads}, ch{lines + (long long)B * kRtThreads + tid, kRtThreads};
    const pfft::RtFft<float> F{mem, lines + 2LL * B * kRtThreads + tid, kRtThreads};
    for (long long u = blockIdx.x; u < g.units; u += gridDim.x) {
        long long f = 0;
        int by = 0, bx = 0, cc = 0;
        unit_coords(g, u, f, by, bx, cc);
        const uint8_t *img = rgb + f * g.in_stride;
        for (int x = tid; x < B; x += kRtThreads) {
            // :276 float32, :282 centred zero padding, :292 -= 128, :298 from_RGB (A4)
            const int sx = bx * B + x - g.left;
            for (int y = 0; y < B; ++y) {
                const int sy = by * B + y - g.top;
                float R = 0.f, G = 0.f, Bl = 0.f;
                if (sy >= 0 && sy < g.H && sx >= 0 && sx < g.W) {
                    const uint8_t *p = img + ((long long)sy * g.W + sx) * 3;
                    R = (float)p[0]; G = (float)p[1]; Bl = (float)p[2];
                }
                if constexpr (M == kU8) { R = R - 128.f; G = G - 128.f; Bl = Bl - 128.f; }
                float o;
                if (cc == 0) o = (R / 4.f + G / 2.f) + Bl / 4.f;
                else if (cc == 1) o = R / 2.f - Bl / 2.f;
                else o = ((-R) / 4.f + G / 2.f) - Bl / 4.f;
                c[y] = o;
            }
            F.dct2(c, ch, P);   // :303 analyze_image (A1): axis 0 first
            for (int y = 0; y < B; ++y) tile[(long long)y * B + x] = c[y];
        }
        __syncthreads();
        const float q = (float)Q;
        for (int y = tid; y < B; y += kRtThreads) {
            for (int j = 0; j < B; ++j) c[j] = tile[(long long)y * B + j];
            F.dct2(c, ch, P);
            const double *wr = pw ? pw + (cc ? B * B : 0) + (long long)y * B : nullptr;
            // :313-327 -p, :343 quantize (A5), :348 += 128, :361 uint8
            for (int j = 0; j < B; ++j) {
                const float t = wr ? (float)((double)c[j] * wr[j]) : c[j];
                const long long o = f * g.out_stride + coef_offset_rt(g, B, by, bx, y, j) + cc;
                if constexpr (M == kRaw) {
                    ((float *)out)[o] = t;
                } else {
                    const int k = (int)__fdiv_rn(t, q);
                    if constexpr (M == kK32) ((int32_t *)out)[o] = k;
                    else ((uint8_t *)out)[o] = (uint8_t)(k + 128);
                }
            }
        }
        __syncthreads();
    }
}

template <int M>
__global__ __launch_bounds__(256) void dct_rt_decode_kernel(const void *__restrict__ kin, void *__restrict__ wsout,
                                                           GeomB g, int Q, pfft::RtPlan P,
                                                           const double *__restrict__ mem, double *__restrict__ ws,
                                                           const double *__restrict__ pw)
{
    const int B = P.n, tid = threadIdx.x;
    double *tile = ws + (long long)blockIdx.x * rt_ws_per_wg(P);
    double *lines = tile + (long long)B * B;
    const pfft::Line<double> c{lines + tid, kRtThreads}, ch{lines + (long long)B * kRtThreads + tid, kRtThreads};
    const pfft::RtFft<double> F{mem, lines + 2LL * B * kRtThreads + tid, kRtThreads};
    for (long long u = blockIdx.x; u < g.units; u += gridDim.x) {
        long long f = 0;
        int by = 0, bx = 0, cc = 0;
        unit_coords(g, u, f, by, bx, cc);
        for (int x = tid; x < B; x += kRtThreads) {
            for (int i = 0; i < B; ++i) {
                const long long o = f * g.out_stride + coef_offset_rt(g, B, by, bx, i, x) + cc;
                if constexpr (M == kK32) {
                    c[i] = (double)(int32_t)((uint32_t)Q * (uint32_t)((const int32_t *)kin)[o]);
                } else {
                    int16_t y16;
                    if constexpr (M == kRaw) {
                        y16 = ((const int16_t *)kin)[o];
                    } else {
                        const int16_t k = (int16_t)((int)((const uint8_t *)kin)[o] - 128);
                        y16 = (int16_t)(Q * (int)k);
                    }
                    if (pw) {   // :421-435 -p
                        const float f = (float)((double)(float)y16 / pw[(cc ? B * B : 0) + (long long)i * B + x]);
                        y16 = (int16_t)(int)f;
                    }
                    c[i] = (double)y16;
                }
            }
            F.dct3(c, ch, P);   // :440 synthesize_image (A2)
            for (int i = 0; i < B; ++i) tile[(long long)i * B + x] = c[i];
        }
        __syncthreads();
        for (int y = tid; y < B; y += kRtThreads) {
            for (int j = 0; j < B; ++j) c[j] = tile[(long long)y * B + j];
            F.dct3(c, ch, P);
            const long long row = (long long)by * B + y;
            for (int j = 0; j < B; ++j) {
                const long long o = f * ((long long)g.Hp * g.Wp * 3) + (row * g.Wp + (long long)bx * B + j) * 3 + cc;
                if constexpr (M == kK32) ((int32_t *)wsout)[o] = (int32_t)c[j];
                else ((int16_t *)wsout)[o] = (int16_t)(int32_t)c[j];
            }
        }
        __syncthreads();
    }
}

// lengths the run-time path covers (plans: pfft::rt_fill, vcf_pocketfft_rt.h)
bool rt_covered(int B) { return B >= 1 && B <= kRtMaxB; }

// cv2.resize of an 8x8 uint8 table to B x B, as src/2D-DCT.py:85-90 calls it
// (INTER_AREA for B < 8, INTER_LINEAR otherwise), restating OpenCV's scalar
// code paths (imgproc/src/resize.cpp): for INTER_LINEAR on 8U the
// fixed-point generic resize (coefficients (1 - f, f) * 2048 rounded to short,
// horizontal int sums, vertical (s0 b0 + s1 b1 + 2^21) >> 22); for INTER_AREA
// with an integer scale resizeAreaFast_ (cvRound(sum * (1.f / area))), with a
// fractional scale resizeArea_ (computeResizeAreaTab float weights,
// row-then-column float accumulation, cvRound).  cv2 is not installed here,
// so this is unpinned (OpenCV's SIMD kernels round some ties differently
// from its scalar code).
inline int cv_round(double v) { return (int)std::nearbyint(v); }   // cvRound: round half to even
inline int cv_floor(double v) { int i = (int)v; return i - (i > v); }
inline int cv_ceil(double v) { int i = (int)v; return i + (i < v); }
inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

void cv_resize_8x8(const uint8_t *src, int B, uint8_t *dst)
{
    const int S = 8;
    if (B == S) { for (int i = 0; i < S * S; ++i) dst[i] = src[i]; return; }
    if (B > S) {   // INTER_LINEAR, 8U, fixed point
        const double inv_scale = (double)B / S, scale = 1. / inv_scale;
        int ofs[4096];
        short alpha[2 * 4096];
        for (int d = 0; d < B; ++d) {
            float f = (float)((d + 0.5) * scale - 0.5);
            int s = cv_floor(f);
            f -= s;
            if (s < 0) { f = 0.f; s = 0; }
            if (s >= S - 1) { f = 0.f; s = S - 1; }
            ofs[d] = s;
            alpha[2 * d] = (short)cv_round((1.f - f) * 2048);
            alpha[2 * d + 1] = (short)cv_round(f * 2048);
        }
        std::vector<int> rows((size_t)S * B);
        for (int y = 0; y < S; ++y)
            for (int d = 0; d < B; ++d) {
                const int s = ofs[d];
                rows[(size_t)y * B + d] = s + 1 < S ? src[y * S + s] * alpha[2 * d] + src[y * S + s + 1] * alpha[2 * d + 1]
                                                    : src[y * S + s] * 2048;
            }
        for (int dy = 0; dy < B; ++dy) {
            const int sy = ofs[dy], sy1 = sy + 1 < S ? sy + 1 : sy;
            const int b0 = alpha[2 * dy], b1 = alpha[2 * dy + 1];
            for (int d = 0; d < B; ++d) {
                const int v = rows[(size_t)sy * B + d] * b0 + rows[(size_t)sy1 * B + d] * b1;
                dst[dy * B + d] = sat_u8((v + (1 << 21)) >> 22);
            }
        }
        return;
    }
    if (S % B == 0) {   // INTER_AREA, integer scale: resizeAreaFast_
        const int k = S / B, area = k * k;
        const float sc = 1.f / area;
        for (int dy = 0; dy < B; ++dy)
            for (int dx = 0; dx < B; ++dx) {
                int sum = 0;
                for (int y = 0; y < k; ++y)
                    for (int x = 0; x < k; ++x) sum += src[(dy * k + y) * S + dx * k + x];
                dst[dy * B + dx] = sat_u8(cv_round(sum * sc));
            }
        return;
    }
    // INTER_AREA, fractional scale: resizeArea_
    struct Tab { int di, si; float alpha; };
    auto area_tab = [&](std::vector<Tab> &tab) {
        const double scale = (double)S / B;
        for (int dx = 0; dx < B; ++dx) {
            const double fsx1 = dx * scale, fsx2 = fsx1 + scale;
            const double cell = std::min(scale, S - fsx1);
            int sx1 = cv_ceil(fsx1), sx2 = cv_floor(fsx2);
            sx2 = std::min(sx2, S - 1);
            sx1 = std::min(sx1, sx2);
            if (sx1 - fsx1 > 1e-3) tab.push_back({dx, sx1 - 1, (float)((sx1 - fsx1) / cell)});
            for (int sx = sx1; sx < sx2; ++sx) tab.push_back({dx, sx, (float)(1.0 / cell)});
            if (fsx2 - sx2 > 1e-3) tab.push_back({dx, sx2, (float)(std::min(std::min(fsx2 - sx2, 1.), cell) / cell)});
        }
    };
    std::vector<Tab> xt, yt;
    area_tab(xt);
    area_tab(yt);
    std::vector<float> buf(B), sum(B, 0.f);
    int prev = yt[0].di;
    for (size_t j = 0; j < yt.size(); ++j) {
        const float beta = yt[j].alpha;
        const int dy = yt[j].di, sy = yt[j].si;
        for (int dx = 0; dx < B; ++dx) buf[dx] = 0.f;
        for (const Tab &t : xt) buf[t.di] += src[sy * S + t.si] * t.alpha;
        if (dy != prev) {
            for (int dx = 0; dx < B; ++dx) {
                dst[prev * B + dx] = sat_u8(cv_round(sum[dx]));
                sum[dx] = beta * buf[dx];
            }
            prev = dy;
        } else {
            for (int dx = 0; dx < B; ++dx) sum[dx] += beta * buf[dx];
        }
    }
    for (int dx = 0; dx < B; ++dx) dst[prev * B + dx] = sat_u8(cv_round(sum[dx]));
}

// the JPEG tables of -p (2D-DCT.py:66-84), uint8
constexpr uint8_t kJpegY[64] = {16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
                                14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
                                18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
                                49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
constexpr uint8_t kJpegC[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                                24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                                99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                                99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

// -p weights of block size B in HBM: Y_QSSs / 121 then C_QSSs / 99 (float64,
// numpy's uint8 / int), B*B each, row-major within the block; per device, kept
int perceptual_weights(int B, const double *&out)
{
    static std::mutex mu;
    static std::map<std::pair<int, int>, double *> cache;
    int dev = 0;
    int rc = hip_check(hipGetDevice(&dev), "hipGetDevice");
    if (rc != VCF_OK) return rc;
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find({dev, B});
    if (it != cache.end()) { out = it->second; return VCF_OK; }
    std::vector<uint8_t> ty((size_t)B * B), tc((size_t)B * B);
    cv_resize_8x8(kJpegY, B, ty.data());
    cv_resize_8x8(kJpegC, B, tc.data());
    std::vector<double> w(2 * (size_t)B * B);
    for (size_t i = 0; i < (size_t)B * B; ++i) {
        w[i] = (double)ty[i] / 121.0;
        w[(size_t)B * B + i] = (double)tc[i] / 99.0;
    }
    double *d = nullptr;
    if ((rc = hip_check(hipMalloc(&d, w.size() * sizeof(double)), "hipMalloc(-p weights)")) != VCF_OK) return rc;
    if ((rc = hip_check(hipMemcpy(d, w.data(), w.size() * sizeof(double), hipMemcpyHostToDevice), "-p weights")) !=
        VCF_OK)
        return rc;
    cache[{dev, B}] = d;
    out = d;
    return VCF_OK;
}

struct RtPlanDev {
    pfft::RtPlan P;
    float *f32 = nullptr;
    double *f64 = nullptr;
};

// plans per (device, length), uploaded once and kept
int rt_plan(int n, RtPlanDev &out)
{
    static std::mutex mu;
    static std::map<std::pair<int, int>, RtPlanDev> cache;
    int dev = 0;
    int rc = hip_check(hipGetDevice(&dev), "hipGetDevice");
    if (rc != VCF_OK) return rc;
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find({dev, n});
    if (it != cache.end()) { out = it->second; return VCF_OK; }
    RtPlanDev d;
    std::vector<float> mf;
    std::vector<double> md;
    pfft::rt_fill<float>(n, d.P, mf);
    pfft::RtPlan P2;
    pfft::rt_fill<double>(n, P2, md);   // same offsets
    if ((rc = hip_check(hipMalloc(&d.f32, mf.size() * sizeof(float)), "hipMalloc(rt plan)")) != VCF_OK) return rc;
    if ((rc = hip_check(hipMalloc(&d.f64, md.size() * sizeof(double)), "hipMalloc(rt plan)")) != VCF_OK) return rc;
    if ((rc = hip_check(hipMemcpy(d.f32, mf.data(), mf.size() * sizeof(float), hipMemcpyHostToDevice),
                        "rt plan upload")) != VCF_OK)
        return rc;
    if ((rc = hip_check(hipMemcpy(d.f64, md.data(), md.size() * sizeof(double), hipMemcpyHostToDevice),
                        "rt plan upload")) != VCF_OK)
        return rc;
    cache[{dev, n}] = d;
    out = d;
    return VCF_OK;
}

Scratch &rt_scratch_for_current_device()
{
    static Scratch per_dev[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    return per_dev[dev];
}

// workgroups of a run-time-path launch: enough to fill the chip, scratch <= ~1 GiB
unsigned rt_grid(long long units, const pfft::RtPlan &P, size_t esz)
{
    const long long per = rt_ws_per_wg(P) * (long long)esz;
    long long wgs = std::min<long long>(units, 4096);
    wgs = std::min<long long>(wgs, std::max<long long>(1, (1LL << 30) / per));
    return (unsigned)std::max<long long>(wgs, 1);
}

int rt_launch_encode(const uint8_t *rgb, void *out, int mode, const GeomB &g, int B, int Q, const double *pw,
                     hipStream_t s)
{
    RtPlanDev pl;
    int rc = rt_plan(B, pl);
    if (rc != VCF_OK) return rc;
    const unsigned grid = rt_grid(g.units, pl.P, sizeof(float));
    Scratch &scr = rt_scratch_for_current_device();
    std::lock_guard<std::mutex> lock(scr.mu);
    rc = scr.acquire((size_t)grid * rt_ws_per_wg(pl.P) * sizeof(float), s);
    if (rc != VCF_OK) return rc;
    float *ws = (float *)scr.ptr;
    if (mode == kK32) hipLaunchKernelGGL((dct_rt_encode_kernel<kK32>), dim3(grid), dim3(kRtThreads), 0, s, rgb, out, g, Q, pl.P, pl.f32, ws, pw);
    else if (mode == kRaw) hipLaunchKernelGGL((dct_rt_encode_kernel<kRaw>), dim3(grid), dim3(kRtThreads), 0, s, rgb, out, g, Q, pl.P, pl.f32, ws, pw);
    else hipLaunchKernelGGL((dct_rt_encode_kernel<kU8>), dim3(grid), dim3(kRtThreads), 0, s, rgb, out, g, Q, pl.P, pl.f32, ws, pw);
    rc = hip_check(hipGetLastError(), "dct_rt_encode_kernel launch");
    const int rc2 = scr.release(s);
    return rc != VCF_OK ? rc : rc2;
}

int rt_launch_decode(const void *kin, void *wsout, int mode, const GeomB &g, int B, int Q, const double *pw,
                     hipStream_t s)
{
    RtPlanDev pl;
    int rc = rt_plan(B, pl);
    if (rc != VCF_OK) return rc;
    const unsigned grid = rt_grid(g.units, pl.P, sizeof(double));
    Scratch &scr = rt_scratch_for_current_device();
    std::lock_guard<std::mutex> lock(scr.mu);
    rc = scr.acquire((size_t)grid * rt_ws_per_wg(pl.P) * sizeof(double), s);
    if (rc != VCF_OK) return rc;
    double *ws = (double *)scr.ptr;
    if (mode == kK32) hipLaunchKernelGGL((dct_rt_decode_kernel<kK32>), dim3(grid), dim3(kRtThreads), 0, s, kin, wsout, g, Q, pl.P, pl.f64, ws, pw);
    else if (mode == kRaw) hipLaunchKernelGGL((dct_rt_decode_kernel<kRaw>), dim3(grid), dim3(kRtThreads), 0, s, kin, wsout, g, Q, pl.P, pl.f64, ws, pw);
    else hipLaunchKernelGGL((dct_rt_decode_kernel<kU8>), dim3(grid), dim3(kRtThreads), 0, s, kin, wsout, g, Q, pl.P, pl.f64, ws, pw);
    rc = hip_check(hipGetLastError(), "dct_rt_decode_kernel launch");
    const int rc2 = scr.release(s);
    return rc != VCF_OK ? rc : rc2;
}

int make_geom_b(int H, int W, int B, uint32_t flags, int64_t n_frames, GeomB &g)
{
    g.H = H; g.W = W;
    g.Hp = (H + B - 1) / B * B;
    g.Wp = (W + B - 1) / B * B;
    g.top = (g.Hp - H) / 2;     // 2D-DCT.py:208-222: centred, extra row/col bottom/right
    g.left = (g.Wp - W) / 2;
    g.nby = g.Hp / B;
    g.nbx = g.Wp / B;
    g.in_stride = (long long)H * W * 3;
    g.out_stride = (long long)g.Hp * g.Wp * 3;
    g.units = (long long)n_frames * g.nby * g.nbx * 3;
    g.sub = (flags & VCF_DCT_NO_SUBBANDS) ? 0 : 1;
    return VCF_OK;
}

template <int B>
int launch_encode(const uint8_t *rgb, void *out, int mode, const GeomB &g, int Q, const double *pw, hipStream_t s)
{
    constexpr int U = enc_units<B>();
    const long long wgs = (g.units + U - 1) / U;
    if (wgs > 0x7fffffffLL) return set_error(VCF_ERR_INVALID, "batch too large");
    if (mode == kK32) hipLaunchKernelGGL((dct_any_encode_kernel<B, kK32>), dim3((unsigned)wgs), dim3(256), 0, s, rgb, out, g, Q, pw);
    else if (mode == kRaw) hipLaunchKernelGGL((dct_any_encode_kernel<B, kRaw>), dim3((unsigned)wgs), dim3(256), 0, s, rgb, out, g, Q, pw);
    else hipLaunchKernelGGL((dct_any_encode_kernel<B, kU8>), dim3((unsigned)wgs), dim3(256), 0, s, rgb, out, g, Q, pw);
    return hip_check(hipGetLastError(), "dct_any_encode_kernel launch");
}

template <int B>
int launch_decode(const void *kin, void *ws, int mode, const GeomB &g, int Q, const double *pw, hipStream_t s)
{
    constexpr int U = dec_units<B>();
    const long long wgs = (g.units + U - 1) / U;
    if (wgs > 0x7fffffffLL) return set_error(VCF_ERR_INVALID, "batch too large");
    if (mode == kK32) hipLaunchKernelGGL((dct_any_decode_kernel<B, kK32>), dim3((unsigned)wgs), dim3(128), 0, s, kin, ws, g, Q, pw);
    else if (mode == kRaw) hipLaunchKernelGGL((dct_any_decode_kernel<B, kRaw>), dim3((unsigned)wgs), dim3(128), 0, s, kin, ws, g, Q, pw);
    else hipLaunchKernelGGL((dct_any_decode_kernel<B, kU8>), dim3((unsigned)wgs), dim3(128), 0, s, kin, ws, g, Q, pw);
    return hip_check(hipGetLastError(), "dct_any_decode_kernel launch");
}

// the 5-smooth block sizes <= 128 (kLens)
#define VCF_ANY_SWITCH(B, CALL)                                                                  \
    switch (B) {                                                                                 \
    case 1: return CALL(1); case 2: return CALL(2); case 3: return CALL(3); case 4: return CALL(4); \
    case 5: return CALL(5); case 6: return CALL(6); case 8: return CALL(8); case 9: return CALL(9); \
    case 10: return CALL(10); case 12: return CALL(12); case 15: return CALL(15);                \
    case 16: return CALL(16); case 18: return CALL(18); case 20: return CALL(20);                \
    case 24: return CALL(24); case 25: return CALL(25); case 27: return CALL(27);                \
    case 30: return CALL(30); case 32: return CALL(32); case 36: return CALL(36);                \
    case 40: return CALL(40); case 45: return CALL(45); case 48: return CALL(48);                \
    case 50: return CALL(50); case 54: return CALL(54); case 60: return CALL(60);                \
    case 64: return CALL(64); case 72: return CALL(72); case 75: return CALL(75);                \
    case 80: return CALL(80); case 81: return CALL(81); case 90: return CALL(90);                \
    case 96: return CALL(96); case 100: return CALL(100); case 108: return CALL(108);            \
    case 120: return CALL(120); case 125: return CALL(125); case 128: return CALL(128);          \
    default: break;                                                                              \
    }

int check_any(const void *a, const void *b, int64_t n_frames, int H, int W, int B, int Q, uint32_t flags,
              bool decode, int mode)
{
    const bool k32 = mode == kK32;
    if (!a || !b) return set_error(VCF_ERR_INVALID, "null buffer");
    if (n_frames < 0) return set_error(VCF_ERR_INVALID, "n_frames < 0");
    if (H <= 0 || W <= 0)
        return set_error(VCF_ERR_INVALID, "Input image must be a 3D array (height, width, channels).");
    if (B < 1) return set_error(VCF_ERR_INVALID, "block size %d", B);
    if (slot_of(B) < 0 && !rt_covered(B))
        return set_error(VCF_ERR_UNSUPPORTED, "block size %d: the HIP path covers B <= 4096", B);
    if (Q < 1 || (decode && mode == kU8 && Q > 32767))
        return set_error(VCF_ERR_INVALID, "quantization step %d out of range", Q);
    if ((flags & VCF_DCT_PERCEPTUAL) && k32)
        return set_error(VCF_ERR_UNSUPPORTED,
                         "the -L search runs without perceptual quantization (2D-DCT.py:100-105)");
    if (flags & ~(VCF_DCT_NO_SUBBANDS | VCF_DCT_PERCEPTUAL))
        return set_error(VCF_ERR_INVALID, "unknown flags 0x%x", flags);
    const long long Hp = (H + B - 1) / B * (long long)B, Wp = (W + B - 1) / B * (long long)B;
    if (Hp * Wp * 3 >= (1LL << 31)) return set_error(VCF_ERR_INVALID, "frame too large");
    return VCF_OK;
}

int any_encode(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t B, int32_t Q,
               uint32_t flags, void *k_dev, int mode, void *stream)
{
    int rc = check_any(rgb_dev, k_dev, n_frames, H, W, B, Q, flags, false, mode);
    if (rc != VCF_OK || n_frames == 0) return rc;
    rc = ensure_tables();
    if (rc != VCF_OK) return rc;
    GeomB g;
    make_geom_b(H, W, B, flags, n_frames, g);
    const hipStream_t s = (hipStream_t)stream;
    const double *pw = nullptr;
    if ((flags & VCF_DCT_PERCEPTUAL) && (rc = perceptual_weights(B, pw)) != VCF_OK) return rc;
#define VCF_ENC_ANY(b) launch_encode<b>(rgb_dev, k_dev, mode, g, Q, pw, s)
    VCF_ANY_SWITCH(B, VCF_ENC_ANY)
#undef VCF_ENC_ANY
    return rt_launch_encode(rgb_dev, k_dev, mode, g, B, Q, pw, s);
}

int any_decode(const void *k_dev, int64_t n_frames, int32_t H, int32_t W, int32_t B, int32_t Q, uint32_t flags,
               uint8_t *rgb_dev, int mode, void *stream)
{
    int rc = check_any(k_dev, rgb_dev, n_frames, H, W, B, Q, flags, true, mode);
    if (rc != VCF_OK || n_frames == 0) return rc;
    rc = ensure_tables();
    if (rc != VCF_OK) return rc;
    const hipStream_t s = (hipStream_t)stream;
    const double *pw = nullptr;
    if ((flags & VCF_DCT_PERCEPTUAL) && (rc = perceptual_weights(B, pw)) != VCF_OK) return rc;
    GeomB g0;
    make_geom_b(H, W, B, flags, 1, g0);
    const size_t esz = mode == kK32 ? 4 : 2;
    const size_t frame_ws = (size_t)g0.Hp * g0.Wp * 3 * esz;
    // workspace in chunks of frames, at most ~1 GiB at a time
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(n_frames, (int64_t)((1ull << 30) / frame_ws)));
    Scratch &scr = scratch_for_current_device();
    std::lock_guard<std::mutex> lock(scr.mu);
    rc = scr.acquire(frame_ws * chunk, s);
    if (rc != VCF_OK) return rc;
    void *ws = scr.ptr;
    const size_t kesz = mode == kK32 ? 4 : (mode == kRaw ? 2 : 1);
    for (int64_t f0 = 0; f0 < n_frames && rc == VCF_OK; f0 += chunk) {
        const int64_t n = std::min(chunk, n_frames - f0);
        GeomB g;
        make_geom_b(H, W, B, flags, n, g);
        const void *kin = (const uint8_t *)k_dev + (size_t)f0 * g.out_stride * kesz;
        auto pass1 = [&]() -> int {
#define VCF_DEC_ANY(b) launch_decode<b>(kin, ws, mode, g, Q, pw, s)
            VCF_ANY_SWITCH(B, VCF_DEC_ANY)
#undef VCF_DEC_ANY
            return rt_launch_decode(kin, ws, mode, g, B, Q, pw, s);
        };
        rc = pass1();
        if (rc != VCF_OK) break;
        const long long npx = (long long)n * H * W;
        const unsigned grid = (unsigned)((npx + 255) / 256);
        uint8_t *out = rgb_dev + (size_t)f0 * g.in_stride;
        if (mode == kK32) hipLaunchKernelGGL((dct_any_to_rgb_kernel<kK32>), dim3(grid), dim3(256), 0, s, ws, out, g, npx);
        else if (mode == kRaw) hipLaunchKernelGGL((dct_any_to_rgb_kernel<kRaw>), dim3(grid), dim3(256), 0, s, ws, out, g, npx);
        else hipLaunchKernelGGL((dct_any_to_rgb_kernel<kU8>), dim3(grid), dim3(256), 0, s, ws, out, g, npx);
        rc = hip_check(hipGetLastError(), "dct_any_to_rgb_kernel launch");
    }
    const int rc2 = scr.release(s);
    return rc != VCF_OK ? rc : rc2;
}

}  // namespace

// entry used by vcf_dct_dz_encode/decode for block_size != 8
int dct_any_encode_u8(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t B, int32_t Q,
                      uint32_t flags, uint8_t *k_dev, void *stream)
{
    return any_encode(rgb_dev, n_frames, H, W, B, Q, flags, k_dev, kU8, stream);
}

int dct_any_decode_u8(const uint8_t *k_dev, int64_t n_frames, int32_t H, int32_t W, int32_t B, int32_t Q,
                      uint32_t flags, uint8_t *rgb_dev, void *stream)
{
    return any_decode(k_dev, n_frames, H, W, B, Q, flags, rgb_dev, kU8, stream);
}

}  // namespace vcf

extern "C" {

int vcf_dct_block_size_supported(int32_t block_size)
{
    return vcf::slot_of(block_size) >= 0 || vcf::rt_covered(block_size) ? 1 : 0;
}

int vcf_dct_perceptual_tables(int32_t block_size, uint8_t *y_qss, uint8_t *c_qss)
{
    if (!y_qss || !c_qss) return vcf::set_error(VCF_ERR_INVALID, "null buffer");
    if (block_size < 1 || block_size > vcf::kRtMaxB) return vcf::set_error(VCF_ERR_INVALID, "block size %d", block_size);
    vcf::cv_resize_8x8(vcf::kJpegY, block_size, y_qss);
    vcf::cv_resize_8x8(vcf::kJpegC, block_size, c_qss);
    return VCF_OK;
}

int vcf_dct_dz_encode_k32(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                          int32_t Q, uint32_t flags, int32_t *k_dev, void *stream)
{
    return vcf::any_encode(rgb_dev, n_frames, H, W, block_size, Q, flags, k_dev, vcf::kK32, stream);
}

int vcf_dct_dz_decode_k32(const int32_t *k_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                          int32_t Q, uint32_t flags, uint8_t *rgb_dev, void *stream)
{
    return vcf::any_decode(k_dev, n_frames, H, W, block_size, Q, flags, rgb_dev, vcf::kK32, stream);
}

int vcf_dct_dz_encode_any(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                          int32_t Q, uint32_t flags, uint8_t *k_dev, void *stream)
{
    return vcf::any_encode(rgb_dev, n_frames, H, W, block_size, Q, flags, k_dev, vcf::kU8, stream);
}

int vcf_dct_dz_decode_any(const uint8_t *k_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                          int32_t Q, uint32_t flags, uint8_t *rgb_dev, void *stream)
{
    return vcf::any_decode(k_dev, n_frames, H, W, block_size, Q, flags, rgb_dev, vcf::kU8, stream);
}

int vcf_dct_raw_encode(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                       uint32_t flags, float *coef_dev, void *stream)
{
    return vcf::any_encode(rgb_dev, n_frames, H, W, block_size, 1, flags, coef_dev, vcf::kRaw, stream);
}

int vcf_dct_raw_decode(const int16_t *coef_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                       uint32_t flags, uint8_t *rgb_dev, void *stream)
{
    return vcf::any_decode(coef_dev, n_frames, H, W, block_size, 1, flags, rgb_dev, vcf::kRaw, stream);
}

}  // extern "C"
