// vcf_dct_dz.hip -- fused DCT(B=8) + deadzone encode and decode kernels for
// gfx950, and the vcf_dct_dz_* entry points of the C ABI.
//
// What the kernels compute is src/2D-DCT.py encode_fn :276-361 and decode_fn
// :399-466 of the reference (see include/vcf_amd.h for the line map), with
// the upstream-package semantics A1-A5 of SURVEY.md Appendix A, bit-exact to
// oracle/vcf_oracle.c.  The per-block arithmetic lives in vcf_dct_block.h
// (host-testable); this file only moves memory around it.
//
// Layout and mapping:
//   * encode: a workgroup of 256 lanes owns 256 consecutive 8x8 blocks of a
//     frame (raster order); lane = block.  The 192 input bytes of a block sit
//     in 48 VGPRs; each YCoCg channel is built, transformed (column pass, then
//     row pass; packed fp32 for a power-of-two Q), quantized, and every index
//     byte is dropped from its register into an LDS image laid out exactly
//     like the output, which leaves with 16-byte coalesced stores (for a full
//     tile every (i, j) subband run is 768 contiguous bytes of the frame);
//   * decode: column-per-lane (8 lanes per block): coalesced 16-byte loads of
//     the runs into LDS, fp64 inverse transform per column then per row (LDS
//     transpose within the wave), packed int16 YCoCg->RGB, RGB rows written
//     straight from registers.
// The A/B variants measured against these live in the
// experimental library (csrc/ab/, libvcf_amd_ab.so), not here.
// The encode is VALU-issue bound (profiles/).  No MFMA: the
// transforms must follow pocketfft's rounding sequence exactly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "vcf_amd.h"
#include "vcf_dct8.h"
#include "vcf_dct_block.h"
#include "vcf_internal.h"

namespace vcf {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kTile = 256;                   // blocks (= lanes) per workgroup; a full tile's (i, j)
                                             // subband run is kTile * 3 bytes, its LDS image 48 KiB

struct Geom {
    int H, W, Hp, Wp, top, left, nbx, nby, tiles_per_row;
    int nblocks, tiles_per_frame;      // raster tiles: kTile consecutive blocks of a frame
    long long in_stride, out_stride;   // bytes per frame (RGB, coefficients)
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

// Raster tiles (encode variants 1/4, decode): a tile is kTile consecutive
// blocks of a frame in raster order and may wrap into the next block rows, so
// only a frame's last tile is partial.  Each lane publishes where its block's
// bytes start in the frame (`rowbase`: (by*Wp + bx)*3, or (by*8*Wp + bx*8)*3
// for -x); output run `seg` of the LDS image then maps to rowbase[block] +
// segment base.  With nbx % 16 == 0 block-row ends fall on 16-block
// boundaries of the tile, so a 16-byte chunk never straddles one.
__device__ __forceinline__ void tile_block(const Geom &g, int n, int &by, int &bx)
{
    by = n / g.nbx;
    bx = n - by * g.nbx;
}

template <bool SUB>
__device__ __forceinline__ uint32_t block_rowbase(const Geom &g, int by, int bx)
{
    return SUB ? ((uint32_t)by * (uint32_t)g.Wp + (uint32_t)bx) * 3u
               : ((uint32_t)by * 8u * (uint32_t)g.Wp + (uint32_t)bx * 8u) * 3u;
}

template <bool SUB>
__device__ __forceinline__ uint32_t seg_base(const Geom &g, int seg)
{
    if (!SUB) return (uint32_t)seg * (uint32_t)g.Wp * 3u;
    const uint32_t i = seg >> 3, j = seg & 7;
    return (i * (uint32_t)g.nby * (uint32_t)g.Wp + j * (uint32_t)g.nbx) * 3u;
}

template <bool SUB, bool TO_GLOBAL, int T = kTile>
__device__ __forceinline__ void move_runs_tab(const Geom &g, uint8_t *stage, const uint32_t *rowbase,
                                              uint8_t *frame, int nvalid)
{
    constexpr int nseg = SUB ? 64 : 8;
    constexpr int bpb = SUB ? 3 : 24;                  // bytes per block in a run
    constexpr int lds_stride = SUB ? T * 3 : T * 24;
    const int tid = threadIdx.x;
    if (g.vec) {
        const int cps = (nvalid * bpb) >> 4;           // nvalid is a multiple of 16
        // stage bytes are the low bytes of k: XOR 0x80 == +128 mod 256 (2D-DCT.py:348,361)
        const int total = nseg * cps;
#pragma clang loop unroll(disable) vectorize(disable) interleave(disable)
        for (int q = tid; q < total; q += T) {
            const int seg = q / cps;
            const int off = (q - seg * cps) << 4;
            const int blk = off / bpb;
            const uint32_t go = rowbase[blk] + seg_base<SUB>(g, seg) + (uint32_t)(off - blk * bpb);
            u32x4 *lp = reinterpret_cast<u32x4 *>(stage + seg * lds_stride + off);
            u32x4 *gp = reinterpret_cast<u32x4 *>(frame + go);
            if (TO_GLOBAL) __builtin_nontemporal_store(*lp ^ 0x80808080u, gp);   // k -> k + 128
            else *lp = __builtin_nontemporal_load(gp);
        }
    } else {
        const int seg_len = nvalid * bpb, total = nseg * seg_len;
#pragma clang loop unroll(disable) vectorize(disable) interleave(disable)
        for (int q = tid; q < total; q += T) {
            const int seg = q / seg_len;
            const int off = q - seg * seg_len;
            const int blk = off / bpb;
            const uint32_t go = rowbase[blk] + seg_base<SUB>(g, seg) + (uint32_t)(off - blk * bpb);
            if (TO_GLOBAL) frame[go] = stage[seg * lds_stride + off] ^ 0x80;
            else stage[seg * lds_stride + off] = frame[go];
        }
    }
}

// Copy-out of a full tile (nvalid == kTile, g.vec): compile-time chunk
// geometry (12 16-byte chunks per lane), every LDS read issued before the
// stores -- the generic loop above waits on each read in turn (4-5 % of the
// encode).  Plain stores, so the 128-byte lines a tile shares
// with its neighbours at run joins stay in the XCD's L2 until the neighbour's
// half arrives (the tile order keeps neighbours on one XCD, see
// dct_dz_encode_kernel); non-temporal stores wrote those lines twice, half at
// a time (2 % slower).  The chunk -> (run, offset, block) divisions are 24-bit
// multiply-shifts and the run bases come from two per-launch constants
// (full-rate v_mul_u32_u24 instead of quarter-rate 32-bit multiplies and
// 64-bit address arithmetic) whenever the frame's subband stride fits 24 bits.
// multiply-shift division q / cps for q < 64 cps (tiles of T = 256 blocks; 384- and
// 512-block tiles, m/s = 3641/18 and 2731/18, measured slower: DESIGN.md §6)
template <int T>
struct DivCps;
template <>
struct DivCps<256> { static constexpr uint32_t m = 2731, s = 17; };   // / 48

template <bool SUB, int T = kTile>
__device__ __forceinline__ void move_runs_full(const Geom &g, const uint8_t *stage, const uint32_t *rowbase,
                                               uint8_t *frame)
{
    constexpr int nseg = SUB ? 64 : 8;
    constexpr int bpb = SUB ? 3 : 24;
    constexpr int lds_stride = SUB ? T * 3 : T * 24;
    constexpr int cps = (T * bpb) >> 4;
    constexpr int per_lane = nseg * cps / T;
    static_assert(nseg * cps % T == 0, "whole stores per lane");
    const int tid = threadIdx.x;
    u32x4 v[per_lane];
    uint32_t go[per_lane];
    const uint32_t segA = (uint32_t)g.nby * (uint32_t)g.Wp * 3u, segB = (uint32_t)g.nbx * 3u;
    if (SUB && segA < (1u << 24)) {
        static_assert(!SUB || bpb == 3, "multiply-shift constants");
#pragma unroll
        for (int r = 0; r < per_lane; ++r) {
            const int q = tid + r * T;                                                  // < 64 cps
            const int seg = (int)(__umul24((uint32_t)q, DivCps<T>::m) >> DivCps<T>::s);   // q / cps
            const int off = (q - seg * cps) << 4;                                       // < 3 T
            const int blk = (int)(__umul24((uint32_t)off, 683u) >> 11);                 // off / 3
            go[r] = rowbase[blk] + __umul24((uint32_t)(seg >> 3), segA) + __umul24((uint32_t)(seg & 7), segB) +
                    (uint32_t)(off - blk * bpb);
            v[r] = *reinterpret_cast<const u32x4 *>(stage + seg * lds_stride + off);
        }
    } else {
#pragma unroll
        for (int r = 0; r < per_lane; ++r) {
            const int q = tid + r * T;
            const int seg = q / cps;
            const int off = (q - seg * cps) << 4;
            const int blk = off / bpb;
            go[r] = rowbase[blk] + seg_base<SUB>(g, seg) + (uint32_t)(off - blk * bpb);
            v[r] = *reinterpret_cast<const u32x4 *>(stage + seg * lds_stride + off);
        }
    }
#pragma unroll
    for (int r = 0; r < per_lane; ++r) *reinterpret_cast<u32x4 *>(frame + go[r]) = v[r] ^ 0x80808080u;   // k + 128
}

// Make raw[] look redefined *after* `dep` exists, so a channel's byte
// extractions can neither be CSE'd with the previous channel's nor hoisted
// above it (either keeps 2-3 channels' inputs live at once and spills).
__device__ __forceinline__ void opaque(uint32_t (&raw)[8][6], uint32_t dep)
{
#pragma unroll
    for (int y = 0; y < 8; ++y)
#pragma unroll
        for (int w = 0; w < 6; ++w) asm volatile("" : "+v"(raw[y][w]) : "v"(dep));
}

// The 192 bytes of block (by, bx), row y in raw[y][0..5] (little-endian);
// the padding (2D-DCT.py:187-229) reads as zero bytes like the reference's.
// Plain loads (non-temporal ones measured 2.7 % slower); the
// compiler merges each row's three 8-byte loads into one 16-byte and one
// 8-byte load.
template <bool PAD>
__device__ __forceinline__ void load_block(const Geom &g, const uint8_t *src, int by, int bx,
                                           uint32_t (&raw)[8][6])
{
    if (!PAD) {
        // one 64-bit block address, the rows at uniform (scalar) offsets y * 3W
        const uint8_t *blk = src + ((long long)by * 8 * g.W + bx * 8) * 3;
#pragma unroll
        for (int y = 0; y < 8; ++y) {
            const u32x2 *p = reinterpret_cast<const u32x2 *>(blk + (long long)y * (3LL * g.W));
            const u32x2 a = p[0], b = p[1], c = p[2];
            raw[y][0] = a.x; raw[y][1] = a.y; raw[y][2] = b.x;
            raw[y][3] = b.y; raw[y][4] = c.x; raw[y][5] = c.y;
        }
    } else {
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
}

template <bool POW2, bool SUB, bool PERC, bool PK, int T = kTile>
__device__ __forceinline__ void encode_block(uint32_t (&raw)[8][6], const EncConsts &K, const FinalK &rowk,
                                             uint8_t *stage, int tid)
{
    // each index byte goes from the low byte of its register straight into
    // the LDS image of the output (no conversion, no packing)
    auto s0 = [&](int i, int j, uint32_t w) {
        if (SUB) stage[(i * 8 + j) * (T * 3) + tid * 3 + 0] = (uint8_t)w;
        else stage[i * (T * 24) + tid * 24 + j * 3 + 0] = (uint8_t)w;
    };
    auto s1 = [&](int i, int j, uint32_t w) {
        if (SUB) stage[(i * 8 + j) * (T * 3) + tid * 3 + 1] = (uint8_t)w;
        else stage[i * (T * 24) + tid * 24 + j * 3 + 1] = (uint8_t)w;
    };
    auto s2 = [&](int i, int j, uint32_t w) {
        if (SUB) stage[(i * 8 + j) * (T * 3) + tid * 3 + 2] = (uint8_t)w;
        else stage[i * (T * 24) + tid * 24 + j * 3 + 2] = (uint8_t)w;
    };
    if constexpr (PK && POW2 && !PERC) {
        encode_block_channel_pk<0>(raw, rowk, K.qd[0], s0);
        opaque(raw, (uint32_t)tid);
        encode_block_channel_pk<1>(raw, rowk, K.qd[0], s1);
        opaque(raw, (uint32_t)tid);
        encode_block_channel_pk<2>(raw, rowk, K.qd[0], s2);
    } else {
        encode_block_channel_fold<0, POW2, PERC, true>(raw, rowk, K.qd, s0);
        opaque(raw, (uint32_t)tid);
        encode_block_channel_fold<1, POW2, PERC, true>(raw, rowk, K.qd, s1);
        opaque(raw, (uint32_t)tid);
        encode_block_channel_fold<2, POW2, PERC, true>(raw, rowk, K.qd, s2);
    }
}

// PK: packed-fp32 transforms (power-of-two Q, no -p).  Wave priority
// (s_setprio) 3 while the input loads issue and during the copy-out, 0 during
// the transforms: a workgroup entering or leaving its memory phase is not held
// behind the resident workgroups' VALU streams (1-2.5 % faster than none over
// three boxes, ABBA).
template <bool POW2, bool SUB, bool PERC, bool PAD, bool PK, int T = kTile>
__global__ __launch_bounds__(T) void dct_dz_encode_kernel(const uint8_t *__restrict__ rgb,
                                                          uint8_t *__restrict__ kout, Geom g,
                                                          EncConsts K, FinalK rowk)
{
    __shared__ __attribute__((aligned(16))) uint8_t stage[64 * T * 3];
    __shared__ uint32_t rowbase[T];
    const int tid = threadIdx.x;
    // each XCD takes a contiguous range of tiles (workgroups are dealt round
    // robin), so neighbouring tiles -- which share partial lines at run joins --
    // meet in one L2
    const unsigned n = gridDim.x * gridDim.y, gid = blockIdx.y * gridDim.x + blockIdx.x;
    const unsigned q = n >> 3, r = n & 7, xcd = gid & 7;
    const unsigned t = xcd * q + min(xcd, r) + (gid >> 3);
    const long long frame = t / gridDim.x;
    const int tile = (int)(t - (unsigned)frame * gridDim.x);
    const int n0 = tile * T;
    const int nvalid = min(T, g.nblocks - n0);
    if (tid < nvalid) {
        int by, bx;
        tile_block(g, n0 + tid, by, bx);
        rowbase[tid] = block_rowbase<SUB>(g, by, bx);
        uint32_t raw[8][6];
        __builtin_amdgcn_s_setprio(3);
        load_block<PAD>(g, rgb + frame * g.in_stride, by, bx, raw);
        __builtin_amdgcn_s_setprio(0);
        encode_block<POW2, SUB, PERC, PK, T>(raw, K, rowk, stage, tid);
    }
    __syncthreads();
    __builtin_amdgcn_s_setprio(3);
    if (nvalid == T && g.vec) move_runs_full<SUB, T>(g, stage, rowbase, kout + frame * g.out_stride);
    else move_runs_tab<SUB, true, T>(g, stage, rowbase, kout + frame * g.out_stride, nvalid);
}

// ---------------------------------------------------------------------------
// Column-per-lane decode.  A lane-per-block decode holds a block's 64 float64
// samples per lane (212+ VGPRs, 2 waves per SIMD), which leaves the float64
// pipe latency-bound.  Here 8 lanes share a block: a workgroup stages the
// index bytes of TB consecutive blocks of a block row in LDS with 16-byte
// loads; per channel, lane x dequantizes coefficient column x, runs its
// DCT-III (dct3_8r, pocketfft's float64 op sequence), the block's 8 lanes
// transpose through a per-block LDS tile (same wave: no workgroup barrier),
// lane x runs pixel row x and keeps its 8 truncated int16 samples; after the
// three channels each lane converts its row to RGB and stores its 24 bytes.
// ~60 VGPRs: 8 waves per SIMD.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wave_lds_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Offset of output run `seg` in the LDS image.  Lanes x = 0..7 of a block
// write runs 8 apart (SUB) or rows 1 apart (-x); runs of TB*3 = 384 bytes
// would put all eight in one bank, so every group of 8 runs (every row) is
// shifted by 32 bytes -- 8 banks -- keeping the 16-byte alignment.
template <int TB, bool SUB>
__device__ __forceinline__ int cols_stage_off(int seg)
{
    return SUB ? seg * (TB * 3) + (seg >> 3) * 32 : seg * (TB * 24) + seg * 32;
}

template <int TB>
struct DecColsSmem {
    double tr[TB][8][9];   // per-block transpose tile, pitch 9
    double lut[256];       // DQ 1: the dequantized int16 value of each index byte, / 16
    uint8_t stage[64 * TB * 3 + 8 * 32];
};

// Index bytes come in with plain loads (non-temporal ones measured 1.7 %
// slower), pixels leave with non-temporal stores, and the load phase runs at
// wave priority 3 (1 % faster than 0).  Dequantization (DQ 1):
// one LDS table of the 256 possible (int16)(Q*(k-128)) values, already divided
// by 16 -- a power of two commutes with every rounding of the transform (no
// value comes near the subnormal range), so the outputs are bit-identical and
// need no scaling; -p de-weights each value first (24-bit multiply).  The
// epilogue (EPI 1, aligned frames): to_RGB, += 128 and the clamp on pixel
// pairs in packed int16 arithmetic (v_pk_add/sub/max/min_i16 wrap exactly as
// numpy's int16), the 24 bytes formed with byte permutes; padded frames take
// one pixel at a time.
template <int TB, bool SUB, bool PERC, bool PAD>
__global__ __launch_bounds__(TB * 8) void dct_dz_decode_cols(const uint8_t *__restrict__ kin,
                                                              uint8_t *__restrict__ rgb, Geom g, int Q,
                                                              int tiles_per_row)
{
    constexpr bool NTL = false, NTS = true;
    constexpr int PRIO = 3, DQ = 1, EPI = 1;
    __shared__ __attribute__((aligned(16))) DecColsSmem<TB> sm;
    const int tid = threadIdx.x;
    const int lb = tid >> 3, x = tid & 7;
    const int by = blockIdx.x / tiles_per_row;
    const int bx0 = (blockIdx.x - by * tiles_per_row) * TB;
    const int nvalid = min(TB, g.nbx - bx0);
    const int bx = bx0 + lb;
    const uint8_t *src = kin + blockIdx.y * g.out_stride;
    uint8_t *dst = rgb + blockIdx.y * g.in_stride;

    // copy the tile's index bytes in: 64 runs of 3*nvalid bytes (or 8 rows of 24*nvalid)
    constexpr int nseg = SUB ? 64 : 8;
    auto seg_off = [&](int seg) -> uint32_t {
        return (uint32_t)(SUB ? seg_offset_sub(g, by, bx0, seg) : seg_offset_nosub(g, by, bx0, seg));
    };
    if (PRIO) __builtin_amdgcn_s_setprio(PRIO);
    // EPI 1 also takes the staging offsets in 24-bit arithmetic when the frame
    // allows it (wave-uniform): seg = q / cps by a multiply-shift, the run
    // offset from per-workgroup constants (no 32-bit multiplies per lane)
    const uint32_t runA = (uint32_t)g.nby * (uint32_t)g.Wp * 3u, runB = (uint32_t)g.nbx * 3u;
    const bool fast24 = EPI == 1 && SUB && runA < (1u << 24) && runB * 8u < (1u << 24);
    const uint32_t runBase = ((uint32_t)by * (uint32_t)g.Wp + (uint32_t)bx0) * 3u;
    if (g.vec && nvalid == TB && (TB * 3) % 16 == 0) {
        constexpr int cps = (SUB ? 3 * TB : 24 * TB) / 16, total = nseg * cps;
        constexpr uint32_t kDivM = ((1u << 18) + cps - 1) / cps;   // q / cps for q < total
        static_assert(total < 4096, "multiply-shift division range");
#pragma unroll
        for (int q0 = 0; q0 < total; q0 += TB * 8) {
            const int q = q0 + tid;
            if (total % (TB * 8) == 0 || q < total) {
                int seg, off;
                uint32_t so;
                if (fast24) {
                    seg = (int)(__umul24((uint32_t)q, kDivM) >> 18);
                    off = (q - seg * cps) << 4;
                    so = __umul24((uint32_t)(seg >> 3), runA) + __umul24((uint32_t)(seg & 7), runB) + runBase;
                } else {
                    seg = q / cps;
                    off = (q - seg * cps) << 4;
                    so = seg_off(seg);
                }
                const u32x4 *gp = reinterpret_cast<const u32x4 *>(src + so + off);
                *reinterpret_cast<u32x4 *>(sm.stage + cols_stage_off<TB, SUB>(seg) + off) =
                    NTL ? __builtin_nontemporal_load(gp) : *gp;
            }
        }
    } else {
        const int seg_len = SUB ? 3 * nvalid : 24 * nvalid, total = nseg * seg_len;
#pragma clang loop unroll(disable) vectorize(disable) interleave(disable)
        for (int q = tid; q < total; q += TB * 8) {
            const int seg = q / seg_len, off = q - seg * seg_len;
            sm.stage[cols_stage_off<TB, SUB>(seg) + off] = src[seg_off(seg) + off];
        }
    }
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    if constexpr (DQ == 1 && !PERC) {
        static_assert(TB * 8 >= 256, "one table entry per thread");
        if (tid < 256) sm.lut[tid] = (double)(int16_t)__mul24(Q, tid - 128) * 0.0625;
    }
    __syncthreads();
    if (lb >= nvalid) return;

    double (*tr)[9] = sm.tr[lb];
    int out[3][8];
#pragma unroll
    for (int C = 0; C < 3; ++C) {
        // :399-411 astype(int16) - 128, Q*k in int16 (A5); -p de-weighting (:421-435)
        double col[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int kb = SUB ? sm.stage[cols_stage_off<TB, SUB>(i * 8 + x) + lb * 3 + C]
                               : sm.stage[cols_stage_off<TB, SUB>(i) + lb * 24 + x * 3 + C];
            if constexpr (DQ == 1 && !PERC) {
                col[i] = sm.lut[kb];
                continue;
            }
            int16_t yv = (int16_t)(DQ ? __mul24(Q, kb - 128) : Q * (kb - 128));
            if (PERC) {
                const float f = (float)((double)(float)yv / pweight_rt(C, i * 8 + x));
                yv = (int16_t)(int)f;
            }
            col[i] = (double)yv;
        }
        // A wave whose 8 blocks are DC-only in this channel (quantized smooth
        // content: most blocks) decodes every pixel of a block to one value:
        // dct3_8r_k<1> per pass, the operations of dct3_8r whose results are
        // not known zeros (vcf_dct8.h; bit-identical int16 outputs).  The
        // branch is wave-uniform.  (64 x 4K S-smooth frames: 1.01 -> 0.756 ms;
        // uniform-random frames, no DC-only wave: 1.187 -> 1.262 ms, the AC
        // test; profiles/r03_dct_decode_dc_ab.log.)  The test: the OR of the
        // dequantized AC values' high words -- a double is +-0 iff its high
        // word is 0 or 0x80000000, and every nonzero input here is >= 1/16 in
        // magnitude, so a zero high word means a zero value; three v_or3 per
        // column instead of byte compares (round 4, decode A/B variant 10:
        // -1 % on both contents, profiles/r04_dct_decode_*_ab.log)
        uint32_t hw = x == 0 ? 0u : (uint32_t)__double2hiint(col[0]);
        hw = hw | (uint32_t)__double2hiint(col[1]) | (uint32_t)__double2hiint(col[2]);
        hw = hw | (uint32_t)__double2hiint(col[3]) | (uint32_t)__double2hiint(col[4]);
        hw = hw | (uint32_t)__double2hiint(col[5]) | (uint32_t)__double2hiint(col[6]);
        hw |= (uint32_t)__double2hiint(col[7]);
        if (__ballot((hw & 0x7FFFFFFFu) != 0u) == 0) {
            const int kb = sm.stage[cols_stage_off<TB, SUB>(0) + lb * (SUB ? 3 : 24) + C];
            double v;
            if constexpr (DQ == 1 && !PERC) {
                v = sm.lut[kb];
            } else {
                int16_t yv = (int16_t)__mul24(Q, kb - 128);
                if (PERC) yv = (int16_t)(int)(float)((double)(float)yv / pweight_rt(C, 0));
                v = (double)yv;
            }
            double r[8] = {v, 0, 0, 0, 0, 0, 0, 0};
            dct3_8r_k<1>(r);   // column pass: every output sqrt2 * v
            double q[8] = {r[0], 0, 0, 0, 0, 0, 0, 0};
            dct3_8r_k<1>(q);   // row pass: every output sqrt2 * (sqrt2 * v)
            const int o = (int16_t)(int)(DQ == 1 && !PERC ? q[0] : q[0] * 0.0625);
#pragma unroll
            for (int j = 0; j < 8; ++j) out[C][j] = o;
            continue;
        }
        // :440 synthesize_image (A2): axis 0 (this lane's column), then axis 1
        dct3_8r(col);
#pragma unroll
        for (int y = 0; y < 8; ++y) tr[y][x] = col[y];
        wave_lds_fence();
        double row[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) row[j] = tr[x][j];
        wave_lds_fence();   // the tile is rewritten by the next channel
        dct3_8r(row);
#pragma unroll
        for (int j = 0; j < 8; ++j)   // fct 1/4 per pass (already in the inputs for DQ 1); int16
            out[C][j] = (int16_t)(int)(DQ == 1 && !PERC ? row[j] : row[j] * 0.0625);
    }
    // :444 remove_padding, :449 to_RGB (int16), :454 += 128, :466 clip, uint8
    if constexpr (EPI == 1 && !PAD) {
        typedef short s2 __attribute__((ext_vector_type(2)));
        const s2 off = {128, 128}, zero = {0, 0}, top = {255, 255};
        uint32_t RG[4], Bq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const s2 Y = {(short)out[0][2 * q], (short)out[0][2 * q + 1]};
            const s2 Co = {(short)out[1][2 * q], (short)out[1][2 * q + 1]};
            const s2 Cg = {(short)out[2][2 * q], (short)out[2][2 * q + 1]};
            s2 R = Y + Co - Cg + off, G = Y + Cg + off, B = Y - Co - Cg + off;
            R = __builtin_elementwise_min(__builtin_elementwise_max(R, zero), top);
            G = __builtin_elementwise_min(__builtin_elementwise_max(G, zero), top);
            B = __builtin_elementwise_min(__builtin_elementwise_max(B, zero), top);
            // R(2q) G(2q) R(2q+1) G(2q+1); B(2q) and B(2q+1) sit in bytes 0 and 2 of Bq
            RG[q] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, G), __builtin_bit_cast(uint32_t, R),
                                          0x06020400u);
            Bq[q] = __builtin_bit_cast(uint32_t, B);
        }
        uint32_t w[6];
#pragma unroll
        for (int h = 0; h < 2; ++h) {   // pixels 4h .. 4h+3: 12 bytes
            const uint32_t a = RG[2 * h], b = Bq[2 * h], c = RG[2 * h + 1], d = Bq[2 * h + 1];
            w[3 * h + 0] = __builtin_amdgcn_perm(b, a, 0x02040100u);                 // R G B R
            const uint32_t t = __builtin_amdgcn_perm(b, a, 0x0c0c0603u);             // G B
            w[3 * h + 1] = __builtin_amdgcn_perm(c, t, 0x05040100u);                 // G B R G
            w[3 * h + 2] = __builtin_amdgcn_perm(d, c, 0x06030204u);                 // B R G B
        }
        u32x2 *p = reinterpret_cast<u32x2 *>(dst + ((uint32_t)(by * 8 + x) * (uint32_t)g.W + (uint32_t)bx * 8) * 3);
        if (NTS) {
            __builtin_nontemporal_store(u32x2{w[0], w[1]}, p);
            __builtin_nontemporal_store(u32x2{w[2], w[3]}, p + 1);
            __builtin_nontemporal_store(u32x2{w[4], w[5]}, p + 2);
        } else {
            p[0] = u32x2{w[0], w[1]};
            p[1] = u32x2{w[2], w[3]};
            p[2] = u32x2{w[4], w[5]};
        }
        return;
    }
    uint32_t px[24];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int yv = out[0][j], co = out[1][j], cg = out[2][j];
        px[3 * j + 0] = clip_u8((int16_t)(yv + co - cg));
        px[3 * j + 1] = clip_u8((int16_t)(yv + cg));
        px[3 * j + 2] = clip_u8((int16_t)(yv - co - cg));
    }
#pragma unroll
    for (int q = 0; q < 24; ++q) VCF_OPAQUE(px[q]);   // see to_rgb_row: avoids a gfx950 packing miscompile
    const int y = x;
    if (!PAD) {
        uint32_t w[6];
#pragma unroll
        for (int q = 0; q < 6; ++q)
            w[q] = px[4 * q] | (px[4 * q + 1] << 8) | (px[4 * q + 2] << 16) | (px[4 * q + 3] << 24);
        u32x2 *p = reinterpret_cast<u32x2 *>(dst + ((uint32_t)(by * 8 + y) * (uint32_t)g.W + (uint32_t)bx * 8) * 3);
        if (NTS) {
            __builtin_nontemporal_store(u32x2{w[0], w[1]}, p);
            __builtin_nontemporal_store(u32x2{w[2], w[3]}, p + 1);
            __builtin_nontemporal_store(u32x2{w[4], w[5]}, p + 2);
        } else {
            p[0] = u32x2{w[0], w[1]};
            p[1] = u32x2{w[2], w[3]};
            p[2] = u32x2{w[4], w[5]};
        }
    } else {
        const int sy = by * 8 + y - g.top;
        if (sy < 0 || sy >= g.H) return;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int sx = bx * 8 + j - g.left;
            if (sx < 0 || sx >= g.W) continue;
            uint8_t *p = dst + ((uint32_t)sy * (uint32_t)g.W + (uint32_t)sx) * 3;
            p[0] = (uint8_t)px[3 * j];
            p[1] = (uint8_t)px[3 * j + 1];
            p[2] = (uint8_t)px[3 * j + 2];
        }
    }
}

template <int TB>
int launch_decode_cols(const uint8_t *k_dev, int64_t n_frames, uint8_t *rgb_dev, const Geom &g, int Q, bool sub,
                       bool perc, bool pad, void *stream)
{
    const int tpr = (g.nbx + TB - 1) / TB;
    for (int64_t f0 = 0; f0 < n_frames; f0 += 65535) {
        const dim3 grid(tpr * g.nby, (unsigned)std::min<int64_t>(65535, n_frames - f0));
        const uint8_t *in = k_dev + f0 * g.out_stride;
        uint8_t *out = rgb_dev + f0 * g.in_stride;
#define VCF_DEC2(SB, PC, PD) \
        if (sub == SB && perc == PC && pad == PD) \
            hipLaunchKernelGGL((dct_dz_decode_cols<TB, SB, PC, PD>), grid, dim3(TB * 8), 0, (hipStream_t)stream, in, \
                               out, g, Q, tpr);
        VCF_DEC2(true, false, false) else VCF_DEC2(true, false, true)
        else VCF_DEC2(true, true, false) else VCF_DEC2(true, true, true)
        else VCF_DEC2(false, false, false) else VCF_DEC2(false, false, true)
        else VCF_DEC2(false, true, false) else VCF_DEC2(false, true, true)
#undef VCF_DEC2
        const int rc = hip_check(hipGetLastError(), "dct_dz_decode_cols launch");
        if (rc != VCF_OK) return rc;
    }
    return VCF_OK;
}

void make_geom(int32_t H, int32_t W, Geom &g)
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
    g.nblocks = g.nbx * g.nby;
    g.tiles_per_frame = (g.nblocks + kTile - 1) / kTile;
    g.in_stride = (long long)H * W * 3;
    g.out_stride = (long long)g.Hp * g.Wp * 3;
    // every subband run starts 16-B aligned and spans whole 16-B chunks iff
    // nbx % 16 == 0 (then Wp*3, nbx*3, 768 and the frame size are multiples of 16)
    g.vec = (g.nbx % 16 == 0) ? 1 : 0;
}

int check_args(const void *a, const void *b, int64_t n_frames, int32_t H, int32_t W,
               int32_t block_size, int32_t Q, uint32_t flags, bool decode)
{
    if (!a || !b) return set_error(VCF_ERR_INVALID, "null buffer");
    if (n_frames < 0) return set_error(VCF_ERR_INVALID, "n_frames < 0");
    if (H <= 0 || W <= 0)
        return set_error(VCF_ERR_INVALID, "Input image must be a 3D array (height, width, channels).");
    if (block_size != 8)
        return set_error(VCF_ERR_INVALID, "block_size %d: the 8x8 kernels need B=8", block_size);
    if (Q < 1 || (decode && Q > 32767))
        return set_error(VCF_ERR_INVALID, "quantization step %d out of range", Q);
    // the fp32 divisor Q*2^6 must be exact for a general (non power-of-two) Q
    if (!decode && (Q & (Q - 1)) != 0 && Q > (1 << 18))
        return set_error(VCF_ERR_UNSUPPORTED, "quantization step %d too large", Q);
    if (flags & ~(VCF_DCT_NO_SUBBANDS | VCF_DCT_PERCEPTUAL))
        return set_error(VCF_ERR_INVALID, "unknown flags 0x%x", flags);
    // the kernels address within a frame with 32-bit offsets
    if ((long long)((H + 7) & ~7) * ((W + 7) & ~7) * 3 >= (1LL << 31))
        return set_error(VCF_ERR_INVALID, "frame too large");
    return VCF_OK;
}

}  // namespace
}  // namespace vcf

using namespace vcf;

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
    if (block_size != 8)   // -B other than 8: vcf_dct_any.hip
        return dct_any_encode_u8(rgb_dev, n_frames, H, W, block_size, Q, flags, k_dev, stream);
    int rc = check_args(rgb_dev, k_dev, n_frames, H, W, block_size, Q, flags, false);
    if (rc != VCF_OK) return rc;
    if (n_frames == 0) return VCF_OK;
    Geom g;
    make_geom(H, W, g);
    const bool pow2 = (Q & (Q - 1)) == 0;
    const bool sub = !(flags & VCF_DCT_NO_SUBBANDS);
    const bool perc = (flags & VCF_DCT_PERCEPTUAL) != 0;
    const bool pad = (g.Hp != H) || (g.Wp != W);
    EncConsts K;
    make_enc_consts(K, Q);
    const FinalK rowk = pow2 ? row_final_k(Q) : final_k(1.0f, 1.0f);
    for (int64_t f0 = 0; f0 < n_frames; f0 += 65535) {
        const dim3 grid(g.tiles_per_frame, (unsigned)std::min<int64_t>(65535, n_frames - f0));
        const uint8_t *in = rgb_dev + f0 * g.in_stride;
        uint8_t *out = k_dev + f0 * g.out_stride;
        // packed-fp32 transforms for a power-of-two Q without -p, else the scalar ones
#define VCF_ENC(P2, SB, PC, PD, PK)                                                                          \
        if (pow2 == P2 && sub == SB && perc == PC && pad == PD)                                              \
            hipLaunchKernelGGL((dct_dz_encode_kernel<P2, SB, PC, PD, PK>), grid, dim3(kTile), 0,            \
                               (hipStream_t)stream, in, out, g, K, rowk);
        VCF_ENC(true, true, false, false, true) else VCF_ENC(true, true, false, true, true)
        else VCF_ENC(true, false, false, false, true) else VCF_ENC(true, false, false, true, true)
        else VCF_ENC(true, true, true, false, false) else VCF_ENC(true, true, true, true, false)
        else VCF_ENC(true, false, true, false, false) else VCF_ENC(true, false, true, true, false)
        else VCF_ENC(false, true, false, false, false) else VCF_ENC(false, true, false, true, false)
        else VCF_ENC(false, true, true, false, false) else VCF_ENC(false, true, true, true, false)
        else VCF_ENC(false, false, false, false, false) else VCF_ENC(false, false, false, true, false)
        else VCF_ENC(false, false, true, false, false) else VCF_ENC(false, false, true, true, false)
#undef VCF_ENC
        rc = hip_check(hipGetLastError(), "dct_dz_encode_kernel launch");
        if (rc != VCF_OK) return rc;
    }
    return VCF_OK;
}

int vcf_dct_dz_decode(const uint8_t *k_dev, int64_t n_frames, int32_t H, int32_t W,
                      int32_t block_size, int32_t Q, uint32_t flags, uint8_t *rgb_dev, void *stream)
{
    if (block_size != 8)   // -B other than 8: vcf_dct_any.hip
        return dct_any_decode_u8(k_dev, n_frames, H, W, block_size, Q, flags, rgb_dev, stream);
    int rc = check_args(k_dev, rgb_dev, n_frames, H, W, block_size, Q, flags, true);
    if (rc != VCF_OK) return rc;
    if (n_frames == 0) return VCF_OK;
    Geom g;
    make_geom(H, W, g);
    const bool sub = !(flags & VCF_DCT_NO_SUBBANDS);
    const bool perc = (flags & VCF_DCT_PERCEPTUAL) != 0;
    const bool pad = (g.Hp != H) || (g.Wp != W);
    return launch_decode_cols<32>(k_dev, n_frames, rgb_dev, g, (int)Q, sub, perc, pad, stream);
}

}  // extern "C"
