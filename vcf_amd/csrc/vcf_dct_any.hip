// vcf_dct_any.hip -- DCT + deadzone encode/decode for block sizes other than
// the 8x8 fast path: the -B option of src/2D-DCT.py (:29) and the 2..128
// sweep of the -L rate-distortion search (optimize_block_size, :533-579).
//
// What is computed is the same frame pipeline as vcf_dct_dz.hip
// (src/2D-DCT.py:276-361 encode, :399-466 decode; assumptions A1-A5), with the
// length-B pocketfft transforms of vcf_pocketfft.h.  Supported B: the
// lengths pocketfft factors into 4, 2, 3 and 5 up to 128 (1, 2, 3, 4, 5, 6,
// 8, 9, 10, 12, 15, 16, ..., 120, 125, 128: 38 sizes); larger B or a prime
// factor above 5 (pocketfft's generic radfg/radbg) return VCF_ERR_UNSUPPORTED.
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
//     no -128 before the colour transform and no +128 on k or the pixels.
// These are not the headline kernels (the 8x8 path is); they favour a small,
// uniform implementation over peak bandwidth.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <mutex>

#include "vcf_amd.h"
#include "vcf_internal.h"
#include "vcf_pocketfft.h"
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
template <int B> constexpr int dec_units() { return B >= 128 ? 1 : 128 / B; }

// ---- encode: RGB u8 -> k (u8 = k + 128 wrapped, or int32 k) --------------
template <int B, bool K32>
__global__ __launch_bounds__(256) void dct_any_encode_kernel(const uint8_t *__restrict__ rgb,
                                                            void *__restrict__ out, GeomB g, int Q)
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
            if constexpr (!K32) { R = R - 128.f; G = G - 128.f; Bl = Bl - 128.f; }
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
        const float q = (float)Q;
        // :343 quantize (A5: (x / Q).astype(int32)), :348 += 128, :361 uint8
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const int k = (int)__fdiv_rn(v[j], q);
            const long long o = f * g.out_stride + coef_offset<B>(g, by, bx, y, j) + c;
            if constexpr (K32) ((int32_t *)out)[o] = k;
            else ((uint8_t *)out)[o] = (uint8_t)(k + 128);
        }
    }
}

// ---- decode, pass 1: k -> IDCT'd integers in a padded-frame workspace ------
template <int B, bool K32>
__global__ __launch_bounds__(128) void dct_any_decode_kernel(const void *__restrict__ kin,
                                                            void *__restrict__ ws, GeomB g, int Q)
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
            if constexpr (K32) {
                // :560-562 decom_k (int32) -> dequantize Q*k in int32
                v[i] = (double)(int32_t)((uint32_t)Q * (uint32_t)((const int32_t *)kin)[o]);
            } else {
                // :399-411 astype(int16) - 128, Q*k in int16 (A5)
                const int16_t k = (int16_t)((int)((const uint8_t *)kin)[o] - 128);
                v[i] = (double)(int16_t)(Q * (int)k);
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
            if constexpr (K32) ((int32_t *)ws)[o] = (int32_t)v[j];
            else ((int16_t *)ws)[o] = (int16_t)(int32_t)v[j];
        }
    }
}

// ---- decode, pass 2: crop, to_RGB, += 128, clip, uint8 ---------------------
template <bool K32>
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
    if constexpr (K32) {
        // int32 arithmetic, offset 0 (optimize_block_size: to_RGB of the int32 array, :567-568)
        const int32_t *s = (const int32_t *)ws + o;
        const uint32_t Y = (uint32_t)s[0], Co = (uint32_t)s[1], Cg = (uint32_t)s[2];
        o3[0] = (int32_t)(Y + Co - Cg);
        o3[1] = (int32_t)(Y + Cg);
        o3[2] = (int32_t)(Y - Co - Cg);
    } else {
        // :449 to_RGB in int16 (wrapping), :454 += 128 in int16
        const int16_t *s = (const int16_t *)ws + o;
        const int Y = s[0], Co = s[1], Cg = s[2];
        o3[0] = (int16_t)((int16_t)(Y + Co - Cg) + 128);
        o3[1] = (int16_t)((int16_t)(Y + Cg) + 128);
        o3[2] = (int16_t)((int16_t)(Y - Co - Cg) + 128);
    }
    uint8_t *d = rgb + p * 3;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) d[ch] = (uint8_t)std::min(255, std::max(0, o3[ch]));   // :466 clip, uint8
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
int launch_encode(const uint8_t *rgb, void *out, bool k32, const GeomB &g, int Q, hipStream_t s)
{
    constexpr int U = enc_units<B>();
    const long long wgs = (g.units + U - 1) / U;
    if (wgs > 0x7fffffffLL) return set_error(VCF_ERR_INVALID, "batch too large");
    if (k32) hipLaunchKernelGGL((dct_any_encode_kernel<B, true>), dim3((unsigned)wgs), dim3(256), 0, s, rgb, out, g, Q);
    else hipLaunchKernelGGL((dct_any_encode_kernel<B, false>), dim3((unsigned)wgs), dim3(256), 0, s, rgb, out, g, Q);
    return hip_check(hipGetLastError(), "dct_any_encode_kernel launch");
}

template <int B>
int launch_decode(const void *kin, void *ws, bool k32, const GeomB &g, int Q, hipStream_t s)
{
    constexpr int U = dec_units<B>();
    const long long wgs = (g.units + U - 1) / U;
    if (wgs > 0x7fffffffLL) return set_error(VCF_ERR_INVALID, "batch too large");
    if (k32) hipLaunchKernelGGL((dct_any_decode_kernel<B, true>), dim3((unsigned)wgs), dim3(128), 0, s, kin, ws, g, Q);
    else hipLaunchKernelGGL((dct_any_decode_kernel<B, false>), dim3((unsigned)wgs), dim3(128), 0, s, kin, ws, g, Q);
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
    default: return set_error(VCF_ERR_UNSUPPORTED, "block size %d is not supported", B);         \
    }

int check_any(const void *a, const void *b, int64_t n_frames, int H, int W, int B, int Q, uint32_t flags,
              bool decode, bool k32)
{
    if (!a || !b) return set_error(VCF_ERR_INVALID, "null buffer");
    if (n_frames < 0) return set_error(VCF_ERR_INVALID, "n_frames < 0");
    if (H <= 0 || W <= 0)
        return set_error(VCF_ERR_INVALID, "Input image must be a 3D array (height, width, channels).");
    if (B < 1) return set_error(VCF_ERR_INVALID, "block size %d", B);
    if (slot_of(B) < 0)
        return set_error(VCF_ERR_UNSUPPORTED,
                         "block size %d: the HIP path covers the 5-smooth B <= 128 (pocketfft radix 2/3/4/5)", B);
    if (Q < 1 || (decode && !k32 && Q > 32767))
        return set_error(VCF_ERR_INVALID, "quantization step %d out of range", Q);
    if (flags & VCF_DCT_PERCEPTUAL)
        return set_error(VCF_ERR_UNSUPPORTED,
                         "perceptual quantization is only available for block_size=8 (2D-DCT.py:100-105)");
    if (flags & ~(VCF_DCT_NO_SUBBANDS | VCF_DCT_PERCEPTUAL))
        return set_error(VCF_ERR_INVALID, "unknown flags 0x%x", flags);
    const long long Hp = (H + B - 1) / B * (long long)B, Wp = (W + B - 1) / B * (long long)B;
    if (Hp * Wp * 3 >= (1LL << 31)) return set_error(VCF_ERR_INVALID, "frame too large");
    return VCF_OK;
}

int any_encode(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t B, int32_t Q,
               uint32_t flags, void *k_dev, bool k32, void *stream)
{
    int rc = check_any(rgb_dev, k_dev, n_frames, H, W, B, Q, flags, false, k32);
    if (rc != VCF_OK || n_frames == 0) return rc;
    rc = ensure_tables();
    if (rc != VCF_OK) return rc;
    GeomB g;
    make_geom_b(H, W, B, flags, n_frames, g);
    const hipStream_t s = (hipStream_t)stream;
#define VCF_ENC_ANY(b) launch_encode<b>(rgb_dev, k_dev, k32, g, Q, s)
    VCF_ANY_SWITCH(B, VCF_ENC_ANY)
#undef VCF_ENC_ANY
}

int any_decode(const void *k_dev, int64_t n_frames, int32_t H, int32_t W, int32_t B, int32_t Q, uint32_t flags,
               uint8_t *rgb_dev, bool k32, void *stream)
{
    int rc = check_any(k_dev, rgb_dev, n_frames, H, W, B, Q, flags, true, k32);
    if (rc != VCF_OK || n_frames == 0) return rc;
    rc = ensure_tables();
    if (rc != VCF_OK) return rc;
    const hipStream_t s = (hipStream_t)stream;
    GeomB g0;
    make_geom_b(H, W, B, flags, 1, g0);
    const size_t esz = k32 ? 4 : 2;
    const size_t frame_ws = (size_t)g0.Hp * g0.Wp * 3 * esz;
    // workspace in chunks of frames, at most ~1 GiB at a time
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(n_frames, (int64_t)((1ull << 30) / frame_ws)));
    Scratch &scr = scratch_for_current_device();
    std::lock_guard<std::mutex> lock(scr.mu);
    rc = scr.acquire(frame_ws * chunk, s);
    if (rc != VCF_OK) return rc;
    void *ws = scr.ptr;
    const size_t kesz = k32 ? 4 : 1;
    for (int64_t f0 = 0; f0 < n_frames && rc == VCF_OK; f0 += chunk) {
        const int64_t n = std::min(chunk, n_frames - f0);
        GeomB g;
        make_geom_b(H, W, B, flags, n, g);
        const void *kin = (const uint8_t *)k_dev + (size_t)f0 * g.out_stride * kesz;
        auto pass1 = [&]() -> int {
#define VCF_DEC_ANY(b) launch_decode<b>(kin, ws, k32, g, Q, s)
            VCF_ANY_SWITCH(B, VCF_DEC_ANY)
#undef VCF_DEC_ANY
        };
        rc = pass1();
        if (rc != VCF_OK) break;
        const long long npx = (long long)n * H * W;
        const unsigned grid = (unsigned)((npx + 255) / 256);
        uint8_t *out = rgb_dev + (size_t)f0 * g.in_stride;
        if (k32) hipLaunchKernelGGL((dct_any_to_rgb_kernel<true>), dim3(grid), dim3(256), 0, s, ws, out, g, npx);
        else hipLaunchKernelGGL((dct_any_to_rgb_kernel<false>), dim3(grid), dim3(256), 0, s, ws, out, g, npx);
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
    return any_encode(rgb_dev, n_frames, H, W, B, Q, flags, k_dev, false, stream);
}

int dct_any_decode_u8(const uint8_t *k_dev, int64_t n_frames, int32_t H, int32_t W, int32_t B, int32_t Q,
                      uint32_t flags, uint8_t *rgb_dev, void *stream)
{
    return any_decode(k_dev, n_frames, H, W, B, Q, flags, rgb_dev, false, stream);
}

}  // namespace vcf

extern "C" {

int vcf_dct_block_size_supported(int32_t block_size)
{
    return vcf::slot_of(block_size) >= 0 ? 1 : 0;
}

int vcf_dct_dz_encode_k32(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                          int32_t Q, uint32_t flags, int32_t *k_dev, void *stream)
{
    return vcf::any_encode(rgb_dev, n_frames, H, W, block_size, Q, flags, k_dev, true, stream);
}

int vcf_dct_dz_decode_k32(const int32_t *k_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                          int32_t Q, uint32_t flags, uint8_t *rgb_dev, void *stream)
{
    return vcf::any_decode(k_dev, n_frames, H, W, block_size, Q, flags, rgb_dev, true, stream);
}

int vcf_dct_dz_encode_any(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                          int32_t Q, uint32_t flags, uint8_t *k_dev, void *stream)
{
    return vcf::any_encode(rgb_dev, n_frames, H, W, block_size, Q, flags, k_dev, false, stream);
}

int vcf_dct_dz_decode_any(const uint8_t *k_dev, int64_t n_frames, int32_t H, int32_t W, int32_t block_size,
                          int32_t Q, uint32_t flags, uint8_t *rgb_dev, void *stream)
{
    return vcf::any_decode(k_dev, n_frames, H, W, block_size, Q, flags, rgb_dev, false, stream);
}

}  // extern "C"
