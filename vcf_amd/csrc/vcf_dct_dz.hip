// vcf_dct_dz.hip -- fused DCT(B=8) + deadzone encode and decode kernels for
// gfx950, and the vcf_dct_dz_* entry points of the C ABI.
//
// What the kernels compute is src/2D-DCT.py encode_fn :276-361 and decode_fn
// :399-466 of the reference (see include/vcf_amd.h for the line map), with
// the upstream-package semantics A1-A5 of SURVEY.md Appendix A, bit-exact to
// oracle/vcf_oracle.c.
//
// Layout and mapping:
//   * a workgroup of 256 lanes owns one block row (8 pixel rows) x 256
//     consecutive 8x8 blocks; lane = block.  The 192 input bytes of a block
//     sit in 48 VGPRs; each YCoCg channel is built, transformed (column pass,
//     then row pass, dct2_8r), quantized and dropped as bytes into an LDS
//     image laid out exactly like the output (64 subband runs of 768 B);
//   * the LDS image leaves with 16-byte coalesced stores: for a full tile
//     every (i, j) subband run is 768 contiguous bytes of the output frame;
//   * decode mirrors it: coalesced 16-byte loads of the 64 runs into LDS,
//     lane-per-block fp64 inverse transform (dct3_8r), int16 YCoCg->RGB,
//     RGB rows written straight from registers.
// No MFMA: the transforms must follow pocketfft's rounding sequence exactly.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "vcf_amd.h"
#include "vcf_dct8.h"
#include "vcf_dct_block.h"
#include "vcf_internal.h"

namespace vcf {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kTile = 256;                 // blocks (= lanes) per workgroup
constexpr int kSegBytes = kTile * 3;       // one (i, j) subband run of a full tile
constexpr int kStageBytes = 64 * kSegBytes;  // 48 KiB LDS image

struct Geom {
    int H, W, Hp, Wp, top, left, nbx, nby, tiles_per_row;
    long long in_stride, out_stride;   // bytes per frame (input, output)
    int vec;                           // 16-B path valid for the coefficient frames
};

__device__ __forceinline__ long long seg_offset_sub(const Geom &g, int by, int bx0, int seg)
{
    const int i = seg >> 3, j = seg & 7;
    return ((long long)(i * g.nby + by) * g.Wp + (long long)j * g.nbx + bx0) * 3;
}

__device__ __forceinline__ long long seg_offset_nosub(const Geom &g, int by, int bx0, int i)
{
    return ((long long)(by * 8 + i) * g.Wp + (long long)bx0 * 8) * 3;
}

// Copy the LDS image <-> the coefficient frame.  TO_GLOBAL selects direction.
template <bool SUB, bool TO_GLOBAL>
__device__ __forceinline__ void move_runs(const Geom &g, uint8_t *stage, uint8_t *frame, int by,
                                          int bx0, int nvalid)
{
    const int nseg = SUB ? 64 : 8;
    const int seg_len = SUB ? 3 * nvalid : 24 * nvalid;
    const int lds_stride = SUB ? kSegBytes : kTile * 24;
    const int tid = threadIdx.x;
    if (g.vec) {
        const int cps = seg_len >> 4;
        const int total = nseg * cps;
        for (int q = tid; q < total; q += kTile) {
            const int seg = q / cps;
            const int off = (q - seg * cps) << 4;
            const long long go = (SUB ? seg_offset_sub(g, by, bx0, seg) : seg_offset_nosub(g, by, bx0, seg)) + off;
            u32x4 *lp = reinterpret_cast<u32x4 *>(stage + seg * lds_stride + off);
            u32x4 *gp = reinterpret_cast<u32x4 *>(frame + go);
            if (TO_GLOBAL) __builtin_nontemporal_store(*lp, gp);
            else *lp = __builtin_nontemporal_load(gp);
        }
    } else {
        const int total = nseg * seg_len;
        for (int q = tid; q < total; q += kTile) {
            const int seg = q / seg_len;
            const int off = q - seg * seg_len;
            const long long go = (SUB ? seg_offset_sub(g, by, bx0, seg) : seg_offset_nosub(g, by, bx0, seg)) + off;
            if (TO_GLOBAL) frame[go] = stage[seg * lds_stride + off];
            else stage[seg * lds_stride + off] = frame[go];
        }
    }
}

__device__ __forceinline__ void opaque(uint32_t (&raw)[8][6])
{
#pragma unroll
    for (int y = 0; y < 8; ++y)
#pragma unroll
        for (int w = 0; w < 6; ++w) VCF_OPAQUE(raw[y][w]);
}

template <int C, bool POW2, bool SUB, bool PERC>
__device__ __forceinline__ void encode_channel(const uint32_t (&raw)[8][6], const float (&qd)[4],
                                               uint8_t *stage, int tid)
{
    uint8_t kb[64];
    encode_block_channel<C, POW2, PERC>(raw, qd, kb);
#pragma unroll
    for (int n = 0; n < 64; ++n) {
        const int i = n >> 3, j = n & 7;
        if (SUB) stage[n * kSegBytes + tid * 3 + C] = kb[n];
        else stage[i * (kTile * 24) + tid * 24 + j * 3 + C] = kb[n];
    }
}

template <bool POW2, bool SUB, bool PERC, bool PAD>
__global__ __launch_bounds__(kTile, 2) void dct_dz_encode_kernel(const uint8_t *__restrict__ rgb,
                                                                 uint8_t *__restrict__ kout, Geom g,
                                                                 float4 qd4)
{
    __shared__ __attribute__((aligned(16))) uint8_t stage[kStageBytes];
    const int tid = threadIdx.x;
    const long long frame = blockIdx.y;
    const int by = blockIdx.x / g.tiles_per_row;
    const int bx0 = (blockIdx.x - by * g.tiles_per_row) * kTile;
    const int nvalid = min(kTile, g.nbx - bx0);
    const int bx = bx0 + tid;
    const uint8_t *src = rgb + frame * g.in_stride;
    const float qd[4] = {qd4.x, qd4.y, qd4.z, qd4.w};

    if (tid < nvalid) {
        uint32_t raw[8][6];
        if (!PAD) {
#pragma unroll
            for (int y = 0; y < 8; ++y) {
                const u32x2 *p = reinterpret_cast<const u32x2 *>(
                    src + ((long long)(by * 8 + y) * g.W + bx * 8) * 3);
                const u32x2 a = __builtin_nontemporal_load(p);
                const u32x2 b = __builtin_nontemporal_load(p + 1);
                const u32x2 c = __builtin_nontemporal_load(p + 2);
                raw[y][0] = a.x; raw[y][1] = a.y; raw[y][2] = b.x;
                raw[y][3] = b.y; raw[y][4] = c.x; raw[y][5] = c.y;
            }
        } else {
            // zero padding, centred (2D-DCT.py:187-229)
#pragma unroll
            for (int y = 0; y < 8; ++y) {
                const int sy = by * 8 + y - g.top;
#pragma unroll
                for (int w = 0; w < 6; ++w) raw[y][w] = 0;
#pragma unroll
                for (int n = 0; n < 24; ++n) {
                    const int sx = bx * 8 + n / 3 - g.left;
                    uint32_t b = 0;
                    if (sy >= 0 && sy < g.H && sx >= 0 && sx < g.W)
                        b = src[((long long)sy * g.W + sx) * 3 + n % 3];
                    raw[y][n >> 2] |= b << ((n & 3) * 8);
                }
            }
        }
        // Keep the three channels' live ranges apart: the empty asm makes raw[]
        // look redefined, so the 192 byte extractions are not CSE'd across
        // channels (that alone kept 192 values live and spilled).
        encode_channel<0, POW2, SUB, PERC>(raw, qd, stage, tid);
        opaque(raw);
        encode_channel<1, POW2, SUB, PERC>(raw, qd, stage, tid);
        opaque(raw);
        encode_channel<2, POW2, SUB, PERC>(raw, qd, stage, tid);
    }
    __syncthreads();
    move_runs<SUB, true>(g, stage, kout + frame * g.out_stride, by, bx0, nvalid);
}

template <int C, bool SUB, bool PERC>
__device__ __forceinline__ void decode_channel(const uint8_t *stage, int tid, int Q,
                                               uint32_t (&res)[32])
{
    uint8_t kb[64];
#pragma unroll
    for (int n = 0; n < 64; ++n) {
        const int i = n >> 3, j = n & 7;
        kb[n] = SUB ? stage[n * kSegBytes + tid * 3 + C] : stage[i * (kTile * 24) + tid * 24 + j * 3 + C];
    }
    decode_block_channel<C, PERC>(kb, Q, res);
}

template <bool SUB, bool PERC, bool PAD>
__global__ __launch_bounds__(kTile, 2) void dct_dz_decode_kernel(const uint8_t *__restrict__ kin,
                                                                 uint8_t *__restrict__ rgb, Geom g,
                                                                 int Q)
{
    __shared__ __attribute__((aligned(16))) uint8_t stage[kStageBytes];
    const int tid = threadIdx.x;
    const long long frame = blockIdx.y;
    const int by = blockIdx.x / g.tiles_per_row;
    const int bx0 = (blockIdx.x - by * g.tiles_per_row) * kTile;
    const int nvalid = min(kTile, g.nbx - bx0);
    const int bx = bx0 + tid;
    move_runs<SUB, false>(g, stage, const_cast<uint8_t *>(kin) + frame * g.out_stride, by, bx0,
                          nvalid);
    __syncthreads();
    if (tid >= nvalid) return;

    // The "memory" clobbers stop the LDS reads of later channels from being
    // hoisted above earlier channels' transforms (which spilled 128+ VGPRs).
    uint32_t Yv[32], Co[32], Cg[32];
    decode_channel<0, SUB, PERC>(stage, tid, Q, Yv);
    asm volatile("" ::: "memory");
    decode_channel<1, SUB, PERC>(stage, tid, Q, Co);
    asm volatile("" ::: "memory");
    decode_channel<2, SUB, PERC>(stage, tid, Q, Cg);
    asm volatile("" ::: "memory");

    uint8_t *dst = rgb + frame * g.in_stride;
#pragma unroll
    for (int y = 0; y < 8; ++y) {
        uint32_t px[24];
        to_rgb_row(Yv, Co, Cg, y, px);
        if (!PAD) {
            uint32_t w[6];
#pragma unroll
            for (int q = 0; q < 6; ++q)
                w[q] = px[4 * q] | (px[4 * q + 1] << 8) | (px[4 * q + 2] << 16) | (px[4 * q + 3] << 24);
            u32x2 *p = reinterpret_cast<u32x2 *>(dst + ((long long)(by * 8 + y) * g.W + bx * 8) * 3);
            __builtin_nontemporal_store(u32x2{w[0], w[1]}, p);
            __builtin_nontemporal_store(u32x2{w[2], w[3]}, p + 1);
            __builtin_nontemporal_store(u32x2{w[4], w[5]}, p + 2);
        } else {
            const int sy = by * 8 + y - g.top;
            if (sy < 0 || sy >= g.H) continue;
#pragma unroll
            for (int x = 0; x < 8; ++x) {
                const int sx = bx * 8 + x - g.left;
                if (sx < 0 || sx >= g.W) continue;
                uint8_t *p = dst + ((long long)sy * g.W + sx) * 3;
                p[0] = (uint8_t)px[3 * x];
                p[1] = (uint8_t)px[3 * x + 1];
                p[2] = (uint8_t)px[3 * x + 2];
            }
        }
        // one output row at a time (else all 192 samples are formed first and spill)
        __builtin_amdgcn_sched_barrier(0);
    }
}

int make_geom(int32_t H, int32_t W, Geom &g)
{
    g.H = H;
    g.W = W;
    g.Hp = (H + 7) / 8 * 8;
    g.Wp = (W + 7) / 8 * 8;
    g.top = (g.Hp - H) / 2;
    g.left = (g.Wp - W) / 2;
    g.nbx = g.Wp / 8;
    g.nby = g.Hp / 8;
    g.tiles_per_row = (g.nbx + kTile - 1) / kTile;
    g.in_stride = (long long)H * W * 3;
    g.out_stride = (long long)g.Hp * g.Wp * 3;
    // every subband run starts 16-B aligned and spans whole 16-B chunks iff
    // nbx % 16 == 0 (then Wp*3, nbx*3, 768 and the frame size are multiples of 16)
    g.vec = (g.nbx % 16 == 0) ? 1 : 0;
    return VCF_OK;
}

int check_args(const void *a, const void *b, int64_t n_frames, int32_t H, int32_t W,
               int32_t block_size, int32_t Q, uint32_t flags, bool decode)
{
    if (!a || !b) return set_error(VCF_ERR_INVALID, "null buffer");
    if (n_frames < 0) return set_error(VCF_ERR_INVALID, "n_frames < 0");
    if (H <= 0 || W <= 0)
        return set_error(VCF_ERR_INVALID, "Input image must be a 3D array (height, width, channels).");
    if (block_size != 8)
        return set_error(VCF_ERR_UNSUPPORTED, "block_size %d: only B=8 is implemented on the HIP path",
                         block_size);
    if (Q < 1 || (decode && Q > 32767))
        return set_error(VCF_ERR_INVALID, "quantization step %d out of range", Q);
    if (flags & ~(VCF_DCT_NO_SUBBANDS | VCF_DCT_PERCEPTUAL))
        return set_error(VCF_ERR_INVALID, "unknown flags 0x%x", flags);
    if ((long long)H * W > (1LL << 31) / 3)
        return set_error(VCF_ERR_INVALID, "frame too large");
    return VCF_OK;
}

}  // namespace
}  // namespace vcf

using namespace vcf;

#define VCF_ENC_CASE(P2, SB, PC, PD)                                                      \
    if (pow2 == P2 && sub == SB && perc == PC && pad == PD)                               \
        hipLaunchKernelGGL((dct_dz_encode_kernel<P2, SB, PC, PD>), grid, dim3(kTile), 0,  \
                           (hipStream_t)stream, rgb_dev + f0 * g.in_stride,               \
                           k_dev + f0 * g.out_stride, g, qd4);

#define VCF_DEC_CASE(SB, PC, PD)                                                          \
    if (sub == SB && perc == PC && pad == PD)                                             \
        hipLaunchKernelGGL((dct_dz_decode_kernel<SB, PC, PD>), grid, dim3(kTile), 0,      \
                           (hipStream_t)stream, k_dev + f0 * g.out_stride,                \
                           rgb_dev + f0 * g.in_stride, g, (int)Q);

extern "C" {

int vcf_dct_padded_shape(int32_t H, int32_t W, int32_t block_size, int32_t *Hp, int32_t *Wp)
{
    if (!Hp || !Wp) return set_error(VCF_ERR_INVALID, "null pointer");
    if (H <= 0 || W <= 0 || block_size <= 0)
        return set_error(VCF_ERR_INVALID, "bad shape %d x %d / block %d", H, W, block_size);
    *Hp = (H + block_size - 1) / block_size * block_size;
    *Wp = (W + block_size - 1) / block_size * block_size;
    return VCF_OK;
}

int vcf_dct_dz_encode(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W,
                      int32_t block_size, int32_t Q, uint32_t flags, uint8_t *k_dev, void *stream)
{
    int rc = check_args(rgb_dev, k_dev, n_frames, H, W, block_size, Q, flags, false);
    if (rc != VCF_OK) return rc;
    if (n_frames == 0) return VCF_OK;
    Geom g;
    make_geom(H, W, g);
    const bool pow2 = (Q & (Q - 1)) == 0;
    const bool sub = !(flags & VCF_DCT_NO_SUBBANDS);
    const bool perc = (flags & VCF_DCT_PERCEPTUAL) != 0;
    const bool pad = (g.Hp != H) || (g.Wp != W);
    // divisors Q*2^e (e = 3..6) or, for a power-of-two Q, their exact reciprocals
    float d[4];
    for (int e = 0; e < 4; ++e) {
        const double D = (double)Q * (double)(1 << (e + 3));
        d[e] = pow2 ? (float)(1.0 / D) : (float)D;
    }
    const float4 qd4 = make_float4(d[0], d[1], d[2], d[3]);
    for (int64_t f0 = 0; f0 < n_frames; f0 += 65535) {
        const dim3 grid(g.tiles_per_row * g.nby, (unsigned)std::min<int64_t>(65535, n_frames - f0));
        VCF_ENC_CASE(true, true, false, false) else VCF_ENC_CASE(true, true, false, true)
        else VCF_ENC_CASE(true, true, true, false) else VCF_ENC_CASE(true, true, true, true)
        else VCF_ENC_CASE(true, false, false, false) else VCF_ENC_CASE(true, false, false, true)
        else VCF_ENC_CASE(true, false, true, false) else VCF_ENC_CASE(true, false, true, true)
        else VCF_ENC_CASE(false, true, false, false) else VCF_ENC_CASE(false, true, false, true)
        else VCF_ENC_CASE(false, true, true, false) else VCF_ENC_CASE(false, true, true, true)
        else VCF_ENC_CASE(false, false, false, false) else VCF_ENC_CASE(false, false, false, true)
        else VCF_ENC_CASE(false, false, true, false) else VCF_ENC_CASE(false, false, true, true)
        rc = hip_check(hipGetLastError(), "dct_dz_encode_kernel launch");
        if (rc != VCF_OK) return rc;
    }
    return VCF_OK;
}

int vcf_dct_dz_decode(const uint8_t *k_dev, int64_t n_frames, int32_t H, int32_t W,
                      int32_t block_size, int32_t Q, uint32_t flags, uint8_t *rgb_dev, void *stream)
{
    int rc = check_args(k_dev, rgb_dev, n_frames, H, W, block_size, Q, flags, true);
    if (rc != VCF_OK) return rc;
    if (n_frames == 0) return VCF_OK;
    Geom g;
    make_geom(H, W, g);
    const bool sub = !(flags & VCF_DCT_NO_SUBBANDS);
    const bool perc = (flags & VCF_DCT_PERCEPTUAL) != 0;
    const bool pad = (g.Hp != H) || (g.Wp != W);
    for (int64_t f0 = 0; f0 < n_frames; f0 += 65535) {
        const dim3 grid(g.tiles_per_row * g.nby, (unsigned)std::min<int64_t>(65535, n_frames - f0));
        VCF_DEC_CASE(true, false, false) else VCF_DEC_CASE(true, false, true)
        else VCF_DEC_CASE(true, true, false) else VCF_DEC_CASE(true, true, true)
        else VCF_DEC_CASE(false, false, false) else VCF_DEC_CASE(false, false, true)
        else VCF_DEC_CASE(false, true, false) else VCF_DEC_CASE(false, true, true)
        rc = hip_check(hipGetLastError(), "dct_dz_decode_kernel launch");
        if (rc != VCF_OK) return rc;
    }
    return VCF_OK;
}

}  // extern "C"
