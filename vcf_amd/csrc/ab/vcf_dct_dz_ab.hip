// vcf_dct_dz_ab.hip -- A/B archive (libvcf_amd_ab.so; not the product library): the
// round-2/3 vcf_dct_dz.hip with every measured kernel variant, kept for the A/B
// scripts and cross-check tests.  Original header:
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
//   * encode variant 1 (default): a workgroup of 256 lanes owns one block row
//     (8 pixel rows) x 256 consecutive 8x8 blocks; lane = block.  The 192
//     input bytes of a block sit in 48 VGPRs; each YCoCg channel is built,
//     transformed (column pass, then row pass), quantized, and every index
//     byte is dropped from its register into an LDS image laid out exactly
//     like the output, which leaves with 16-byte coalesced stores (for a full
//     tile every (i, j) subband run is 768 contiguous bytes of the frame);
//   * encode variant 3: column-per-lane (8 lanes per block, LDS transpose
//     between the passes); cheaper arithmetic, weaker memory overlap;
//   * decode mirrors variant 1: coalesced 16-byte loads of the runs into LDS,
//     lane-per-block fp64 inverse transform, int16 YCoCg->RGB, RGB rows
//     written straight from registers.
// The encode is VALU-issue bound (profiles/).  No MFMA: the
// transforms must follow pocketfft's rounding sequence exactly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "vcf_amd.h"
#include "vcf_amd_ab.h"
#include "vcf_dct8.h"
#include "vcf_dct_block.h"
#include "vcf_internal.h"
#include "vcf_pipeline.h"

namespace vcf {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kTile = 256;                   // blocks (= lanes) per workgroup
constexpr int kSegBytes = kTile * 3;         // one (i, j) subband run of a full tile
constexpr int kStageBytes = 64 * kSegBytes;  // 48 KiB LDS image

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

template <bool SUB, bool TO_GLOBAL>
__device__ __forceinline__ void move_runs_tab(const Geom &g, uint8_t *stage, const uint32_t *rowbase,
                                              uint8_t *frame, int nvalid)
{
    constexpr int nseg = SUB ? 64 : 8;
    constexpr int bpb = SUB ? 3 : 24;                  // bytes per block in a run
    constexpr int lds_stride = SUB ? kSegBytes : kTile * 24;
    const int tid = threadIdx.x;
    if (g.vec) {
        const int cps = (nvalid * bpb) >> 4;           // nvalid is a multiple of 16
        // stage bytes are the low bytes of k: XOR 0x80 == +128 mod 256 (2D-DCT.py:348,361)
        const int total = nseg * cps;
#pragma clang loop unroll(disable) vectorize(disable) interleave(disable)
        for (int q = tid; q < total; q += kTile) {
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
        for (int q = tid; q < total; q += kTile) {
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
// encode).  Store policy (NT = 0, the default): plain stores,
// so the 128-byte lines a tile shares with its neighbours at run joins stay
// in the XCD's L2 until the neighbour's half arrives (the tile order keeps
// neighbours on one XCD, see dct_dz_encode_kernel); non-temporal stores
// wrote those lines twice, half at a time (2 % slower).
// FA: the chunk -> (run, offset, block) divisions as 24-bit multiply-shifts and
// the run bases from two per-launch constants (full-rate v_mul_u32_u24 instead
// of quarter-rate 32-bit multiplies and 64-bit address arithmetic) whenever the
// frame's subband stride fits 24 bits; FA = false is the earlier code (encode
// variant 17, A/B).
template <bool SUB, int NT = 1, bool FA = false>   // NT: 1 non-temporal stores, 0 plain, 2 plain within 128 B of a run's ends
__device__ __forceinline__ void move_runs_full(const Geom &g, const uint8_t *stage, const uint32_t *rowbase,
                                               uint8_t *frame)
{
    constexpr int nseg = SUB ? 64 : 8;
    constexpr int bpb = SUB ? 3 : 24;
    constexpr int lds_stride = SUB ? kSegBytes : kTile * 24;
    constexpr int cps = (kTile * bpb) >> 4;
    constexpr int per_lane = nseg * cps / kTile;
    static_assert(nseg * cps % kTile == 0, "whole stores per lane");
    const int tid = threadIdx.x;
    u32x4 v[per_lane];
    uint32_t go[per_lane];
    bool edge[per_lane];
    const uint32_t segA = (uint32_t)g.nby * (uint32_t)g.Wp * 3u, segB = (uint32_t)g.nbx * 3u;
    if (FA && SUB && segA < (1u << 24)) {
        static_assert(!SUB || (cps == 48 && bpb == 3), "multiply-shift constants");
#pragma unroll
        for (int r = 0; r < per_lane; ++r) {
            const int q = tid + r * kTile;                                   // < 3072
            const int seg = (int)(__umul24((uint32_t)q, 21846u) >> 20);      // q / 48
            const int off = (q - seg * cps) << 4;                            // < 768
            const int blk = (int)(__umul24((uint32_t)off, 43691u) >> 17);    // off / 3
            go[r] = rowbase[blk] + __umul24((uint32_t)(seg >> 3), segA) + __umul24((uint32_t)(seg & 7), segB) +
                    (uint32_t)(off - blk * bpb);
            v[r] = *reinterpret_cast<const u32x4 *>(stage + seg * lds_stride + off);
            edge[r] = off < 128 || off + 16 > cps * 16 - 128;
        }
    } else {
#pragma unroll
        for (int r = 0; r < per_lane; ++r) {
            const int q = tid + r * kTile;
            const int seg = q / cps;
            const int off = (q - seg * cps) << 4;
            const int blk = off / bpb;
            go[r] = rowbase[blk] + seg_base<SUB>(g, seg) + (uint32_t)(off - blk * bpb);
            v[r] = *reinterpret_cast<const u32x4 *>(stage + seg * lds_stride + off);
            edge[r] = off < 128 || off + 16 > cps * 16 - 128;
        }
    }
#pragma unroll
    for (int r = 0; r < per_lane; ++r) {
        if (NT == 1 || (NT == 2 && !edge[r]))
            __builtin_nontemporal_store(v[r] ^ 0x80808080u, reinterpret_cast<u32x4 *>(frame + go[r]));
        else
            *reinterpret_cast<u32x4 *>(frame + go[r]) = v[r] ^ 0x80808080u;
    }
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
// LD: 1 plain loads (default), 0 non-temporal loads (encode variant 11, an
// A/B record: 2.7 % slower).  The compiler merges each row's
// three 8-byte loads into one 16-byte and one 8-byte load either way.
template <bool PAD, int LD = 1, bool FA = false>
__device__ __forceinline__ void load_block(const Geom &g, const uint8_t *src, int by, int bx,
                                           uint32_t (&raw)[8][6])
{
    if (!PAD) {
        // FA: one 64-bit block address, the rows at uniform (scalar) offsets y * 3W
        const uint8_t *blk = src + ((long long)by * 8 * g.W + bx * 8) * 3;
#pragma unroll
        for (int y = 0; y < 8; ++y) {
            const u32x2 *p = reinterpret_cast<const u32x2 *>(
                FA ? blk + (long long)y * (3LL * g.W) : src + ((long long)(by * 8 + y) * g.W + bx * 8) * 3);
            const u32x2 a = LD == 0 ? __builtin_nontemporal_load(p) : p[0];
            const u32x2 b = LD == 0 ? __builtin_nontemporal_load(p + 1) : p[1];
            const u32x2 c = LD == 0 ? __builtin_nontemporal_load(p + 2) : p[2];
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

template <bool POW2, bool SUB, bool PERC, bool SDWA, bool PK = false, bool MEMONLY = false>
__device__ __forceinline__ void encode_block(uint32_t (&raw)[8][6], const EncConsts &K, const FinalK &rowk,
                                             uint8_t *stage, int tid)
{
    // each index byte goes from the low byte of its register straight into
    // the LDS image of the output (no conversion, no packing)
    auto s0 = [&](int i, int j, uint32_t w) {
        if (SUB) stage[(i * 8 + j) * kSegBytes + tid * 3 + 0] = (uint8_t)w;
        else stage[i * (kTile * 24) + tid * 24 + j * 3 + 0] = (uint8_t)w;
    };
    auto s1 = [&](int i, int j, uint32_t w) {
        if (SUB) stage[(i * 8 + j) * kSegBytes + tid * 3 + 1] = (uint8_t)w;
        else stage[i * (kTile * 24) + tid * 24 + j * 3 + 1] = (uint8_t)w;
    };
    auto s2 = [&](int i, int j, uint32_t w) {
        if (SUB) stage[(i * 8 + j) * kSegBytes + tid * 3 + 2] = (uint8_t)w;
        else stage[i * (kTile * 24) + tid * 24 + j * 3 + 2] = (uint8_t)w;
    };
    if constexpr (MEMONLY) {   // diagnostic: the same LDS and HBM traffic, no transform
#pragma unroll
        for (int n = 0; n < 64; ++n) {
            const uint32_t w = raw[n >> 3][(n * 3 / 4) % 6] >> (8 * (n & 3));
            s0(n >> 3, n & 7, w);
            s1(n >> 3, n & 7, w >> 1);
            s2(n >> 3, n & 7, w >> 2);
        }
    } else if constexpr (PK && POW2 && !PERC) {
        encode_block_channel_pk<0>(raw, rowk, K.qd[0], s0);
        opaque(raw, (uint32_t)tid);
        encode_block_channel_pk<1>(raw, rowk, K.qd[0], s1);
        opaque(raw, (uint32_t)tid);
        encode_block_channel_pk<2>(raw, rowk, K.qd[0], s2);
    } else {
        encode_block_channel_fold<0, POW2, PERC, SDWA>(raw, rowk, K.qd, s0);
        opaque(raw, (uint32_t)tid);
        encode_block_channel_fold<1, POW2, PERC, SDWA>(raw, rowk, K.qd, s1);
        opaque(raw, (uint32_t)tid);
        encode_block_channel_fold<2, POW2, PERC, SDWA>(raw, rowk, K.qd, s2);
    }
}

// PK: packed-fp32 transforms (power-of-two Q, no -p); MEMONLY: diagnostic
// with the same loads, LDS image and copy-out but no transforms.
// PRIO: wave priority (s_setprio) while the input loads issue (low 2 bits)
// and during the copy-out (bits 2-3), 0 during the transforms: a workgroup
// entering or leaving its memory phase is not held behind the resident
// workgroups' VALU streams (15, the default, measured 1-2.5 % faster than 0
// over three boxes, ABBA; variants 12-15 and 16 = PRIO 0 are the A/B records).
template <bool POW2, bool SUB, bool PERC, bool PAD, bool SDWA = true, bool PK = false, bool MEMONLY = false,
          int STREAMS = 0, int NT = 0, bool XCD = true, int LD = 1, int PRIO = 15, bool FA = true>
__global__ __launch_bounds__(kTile) void dct_dz_encode_kernel(const uint8_t *__restrict__ rgb,
                                                              uint8_t *__restrict__ kout, Geom g,
                                                              EncConsts K, FinalK rowk)
{
    __shared__ __attribute__((aligned(16))) uint8_t stage[kStageBytes];
    __shared__ uint32_t rowbase[kTile];
    const int tid = threadIdx.x;
    long long frame = blockIdx.y;
    int tile = blockIdx.x;
    if (XCD) {   // each XCD takes a contiguous range of tiles (workgroups are dealt round robin), so
                 // neighbouring tiles -- which share partial lines at run joins -- meet in one L2
        const unsigned n = gridDim.x * gridDim.y, gid = blockIdx.y * gridDim.x + blockIdx.x;
        const unsigned q = n >> 3, r = n & 7, x = gid & 7;
        const unsigned t = x * q + min(x, r) + (gid >> 3);
        frame = t / gridDim.x;
        tile = (int)(t - (unsigned)frame * gridDim.x);
    }
    const int n0 = tile * kTile;
    const int nvalid = min(kTile, g.nblocks - n0);
    if (tid < nvalid) {
        int by, bx;
        tile_block(g, n0 + tid, by, bx);
        rowbase[tid] = block_rowbase<SUB>(g, by, bx);
        uint32_t raw[8][6];
        if (PRIO & 3) __builtin_amdgcn_s_setprio(PRIO & 3);
        load_block<PAD, LD, FA>(g, rgb + frame * g.in_stride, by, bx, raw);
        if (PRIO & 3) __builtin_amdgcn_s_setprio(0);
        encode_block<POW2, SUB, PERC, SDWA, PK, MEMONLY>(raw, K, rowk, stage, tid);
    }
    __syncthreads();
    if (PRIO >> 2) __builtin_amdgcn_s_setprio(PRIO >> 2);
    if (STREAMS) {   // diagnostic: the image as 64 streams (run seg of tile t at seg*S + t*768 [+32]); wrong layout
        const long long S = (long long)g.out_stride * gridDim.y / 64 / 4096 * 4096;
        const long long t = (long long)blockIdx.y * gridDim.x + blockIdx.x;
        const int shift = STREAMS == 2 ? 32 : 0;
        if (nvalid == kTile)
#pragma unroll
            for (int r = 0; r < 12; ++r) {
                const int q = tid + r * kTile, seg = q / 48, off = (q - seg * 48) * 16;
                if (t * 768 + shift + off + 16 <= S)
                    __builtin_nontemporal_store(*reinterpret_cast<const u32x4 *>(stage + q * 16),
                                                reinterpret_cast<u32x4 *>(kout + seg * S + t * 768 + shift + off));
            }
        return;
    }
    if (nvalid == kTile && g.vec) move_runs_full<SUB, NT, FA>(g, stage, rowbase, kout + frame * g.out_stride);
    else move_runs_tab<SUB, true>(g, stage, rowbase, kout + frame * g.out_stride, nvalid);
}

// Diagnostic (encode variant 2): the same body with no memory traffic at all
// -- raw synthesised from the lane id, one word stored per lane -- to split
// kernel time into arithmetic and memory (scripts/bench_variants.py).
template <bool PK>
__global__ __launch_bounds__(kTile, 2) void dct_dz_encode_diag(uint8_t *__restrict__ kout, Geom g,
                                                               EncConsts K, FinalK rowk, long long nblocks)
{
    const long long gid = (long long)blockIdx.x * kTile + threadIdx.x;
    if (gid >= nblocks) return;
    uint32_t raw[8][6];
#pragma unroll
    for (int y = 0; y < 8; ++y)
#pragma unroll
        for (int w = 0; w < 6; ++w) raw[y][w] = (uint32_t)(gid * 2654435761u) ^ (y * 0x01010101u * (w + 1));
    uint32_t acc = 0;
    auto sink = [&](int i, int j, uint32_t w) { acc += w << ((i + j) & 7); };
    if constexpr (PK) {
        encode_block_channel_pk<0>(raw, rowk, K.qd[0], sink);
        opaque(raw, acc);
        encode_block_channel_pk<1>(raw, rowk, K.qd[0], sink);
        opaque(raw, acc);
        encode_block_channel_pk<2>(raw, rowk, K.qd[0], sink);
    } else {
        encode_block_channel_fold<0, true, false, true>(raw, rowk, K.qd, sink);
        opaque(raw, acc);
        encode_block_channel_fold<1, true, false, true>(raw, rowk, K.qd, sink);
        opaque(raw, acc);
        encode_block_channel_fold<2, true, false, true>(raw, rowk, K.qd, sink);
    }
    reinterpret_cast<uint32_t *>(kout)[gid] = acc;
}

// ---------------------------------------------------------------------------
// Column-per-lane encode (variant 3).  Lane-per-block needs ~120-165 VGPRs
// (48 for the block's bytes, 64 coefficients), i.e. 3 waves per SIMD, and a
// gfx950 SIMD needs >= 8 waves to issue a full-rate VALU op every ~2.3 cycles
// (one wave alone: every ~6.5; scripts/microbench).  Here 8 lanes share a
// block: lane x of a block loads pixel column x, runs that column's DCT-II,
// the 8 lanes transpose through LDS (same wave: no barrier), lane x then runs
// coefficient row x, quantizes it and drops its 8 index bytes into the
// workgroup's LDS image of the output, which leaves with coalesced stores.
// The column pass folds the factor 2 of outputs 0 and 4 into its last
// multiplications (2*hf, 2*tw3; exact), so every row is at the same scale and
// the quantizer divisor depends on (channel, j) only.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wave_lds_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

template <int TB>
struct ColsSmem {
    float tr[TB][8][9];       // per-block 8x8 transpose tile, pitch 9 (bank-conflict free)
    uint8_t stage[64 * TB * 3 + 8 * 32];
};

// Offset of output run `seg` in the LDS image.  Lanes x = 0..7 of a block
// write runs 8 apart (SUB) or rows 1 apart (-x); runs of TB*3 = 384 bytes
// would put all eight in one bank, so every group of 8 runs (every row) is
// shifted by 32 bytes -- 8 banks -- keeping the 16-byte alignment.
template <int TB, bool SUB>
__device__ __forceinline__ int cols_stage_off(int seg)
{
    return SUB ? seg * (TB * 3) + (seg >> 3) * 32 : seg * (TB * 24) + seg * 32;
}

template <int TB, bool POW2, bool SUB, bool PERC, bool PAD>
__global__ __launch_bounds__(TB * 8) void dct_dz_encode_cols(const uint8_t *__restrict__ rgb,
                                                              uint8_t *__restrict__ kout, Geom g,
                                                              EncConsts K, int tiles_per_row)
{
    __shared__ __attribute__((aligned(16))) ColsSmem<TB> sm;
    const int tid = threadIdx.x;
    const int lb = tid >> 3, x = tid & 7;
    const int by = blockIdx.x / tiles_per_row;
    const int bx0 = (blockIdx.x - by * tiles_per_row) * TB;
    const int nvalid = min(TB, g.nbx - bx0);
    const int bx = bx0 + lb;
    // frames are < 2 GiB (check_args): per-lane offsets stay 32-bit, the
    // frame bases are wave-uniform (SGPR) 64-bit pointers
    const uint8_t *src = rgb + blockIdx.y * g.in_stride;
    uint8_t *dst = kout + blockIdx.y * g.out_stride;
    if (lb < nvalid) {
        // the 3 bytes of pixel (y, x), as signed bytes R', G', B' in the low 24 bits
        uint32_t px[8];
        if (!PAD) {
            const int o = 3 * x;
            const uint32_t row_bytes = (uint32_t)g.W * 3;
            uint32_t off = (uint32_t)(by * 8) * row_bytes + (uint32_t)bx * 24 + (o & ~3);
            uint32_t lo[8], hi[8];
#pragma unroll
            for (int y = 0; y < 8; ++y, off += row_bytes) {
                const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(src + off));
                lo[y] = v.x;
                hi[y] = v.y;
            }
#pragma unroll
            for (int y = 0; y < 8; ++y)
                px[y] = __builtin_amdgcn_alignbyte(hi[y], lo[y], (uint32_t)(o & 3)) ^ 0x80808080u;
        } else {
            const int sx = bx * 8 + x - g.left;
#pragma unroll
            for (int y = 0; y < 8; ++y) {
                const int sy = by * 8 + y - g.top;
                uint32_t v = 0;
                if (sy >= 0 && sy < g.H && sx >= 0 && sx < g.W) {
                    const uint8_t *p = src + ((uint32_t)sy * (uint32_t)g.W + (uint32_t)sx) * 3;
                    v = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
                }
                px[y] = v ^ 0x80808080u;
            }
        }
        float (*tr)[9] = sm.tr[lb];
#pragma unroll
        for (int C = 0; C < 3; ++C) {
            float col[8];
#pragma unroll
            for (int y = 0; y < 8; ++y)
                col[y] = bits_as_float((uint32_t)sdot4(px[y], K.w[C][0], (int)K.cinit)) - K.csub[C];
            dct2_8k_colpass(col, K);
#pragma unroll
            for (int i = 0; i < 8; ++i) tr[i][x] = col[i];
            // the 8 lanes of a block are one wave, whose LDS operations
            // execute in order: only the compiler must not move the reads
            // above the other lanes' writes (nor the next channel's writes
            // above these reads)
            wave_lds_fence();
            float row[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) row[j] = tr[x][j];
            wave_lds_fence();
            dct2_8k(row, K);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float t = row[j];
                if (PERC) t = (float)((double)t * pweight_rt(C, x * 8 + j));
                // divisor Q * chs * 4 / s_j = Q * 2^e, e = log2(chs) + 2 + inv(j)
                const int e = (C == 1 ? 1 : 2) + 2 + dct2_inv_scale_log2(j);
                const float q = quant_div<POW2>(t, K.qd[e - 3]);
                const uint8_t b = (uint8_t)float_bits(trunc_f(q) + K.qmagic);
                if (SUB) sm.stage[cols_stage_off<TB, true>(x * 8 + j) + lb * 3 + C] = b;
                else sm.stage[cols_stage_off<TB, false>(x) + lb * 24 + j * 3 + C] = b;
            }
        }
    }
    __syncthreads();
    // copy the LDS image out: 64 runs of 3*nvalid bytes (or 8 rows of 24*nvalid)
    constexpr int nseg = SUB ? 64 : 8;
    auto seg_off = [&](int seg) -> uint32_t {
        return (uint32_t)(SUB ? seg_offset_sub(g, by, bx0, seg) : seg_offset_nosub(g, by, bx0, seg));
    };
    if (g.vec && nvalid == TB && (TB * 3) % 16 == 0) {
        // full tile: compile-time chunk geometry
        constexpr int cps = (SUB ? 3 * TB : 24 * TB) / 16, total = nseg * cps;
#pragma unroll
        for (int q0 = 0; q0 < total; q0 += TB * 8) {
            const int q = q0 + tid;
            if (total % (TB * 8) == 0 || q < total) {
                const int seg = q / cps, off = (q - seg * cps) << 4;
                __builtin_nontemporal_store(
                    *reinterpret_cast<const u32x4 *>(sm.stage + cols_stage_off<TB, SUB>(seg) + off),
                    reinterpret_cast<u32x4 *>(dst + seg_off(seg) + off));
            }
        }
    } else if (g.vec && (TB * 3) % 16 == 0) {
        const int cps = (SUB ? 3 * nvalid : 24 * nvalid) >> 4, total = nseg * cps;
#pragma clang loop unroll(disable) vectorize(disable) interleave(disable)
        for (int q = tid; q < total; q += TB * 8) {
            const int seg = q / cps, off = (q - seg * cps) << 4;
            __builtin_nontemporal_store(
                *reinterpret_cast<const u32x4 *>(sm.stage + cols_stage_off<TB, SUB>(seg) + off),
                reinterpret_cast<u32x4 *>(dst + seg_off(seg) + off));
        }
    } else {
        const int seg_len = SUB ? 3 * nvalid : 24 * nvalid, total = nseg * seg_len;
#pragma clang loop unroll(disable) vectorize(disable) interleave(disable)
        for (int q = tid; q < total; q += TB * 8) {
            const int seg = q / seg_len, off = q - seg * seg_len;
            dst[seg_off(seg) + off] = sm.stage[cols_stage_off<TB, SUB>(seg) + off];
        }
    }
}

// ---------------------------------------------------------------------------
// Column-per-lane decode (decode variant 2, the default).  The lane-per-block
// decode holds a block's 64 float64 samples per lane (212+ VGPRs, 2 waves per
// SIMD), which leaves the float64 pipe latency-bound.  Here 8 lanes share a
// block, as in encode variant 3: a workgroup stages the index bytes of TB
// consecutive blocks of a block row in LDS with 16-byte loads; per channel,
// lane x dequantizes coefficient column x, runs its DCT-III (dct3_8r, the same
// float64 op sequence), the block's 8 lanes transpose through a per-block LDS
// tile (same wave: no workgroup barrier), lane x runs pixel row x and keeps
// its 8 truncated int16 samples; after the three channels each lane converts
// its row to RGB and stores its 24 bytes.  ~60 VGPRs: 8 waves per SIMD.
// ---------------------------------------------------------------------------
template <int TB, bool TRH = false>
struct DecColsSmem {
    double tr[TB][TRH ? 4 : 8][9];   // per-block transpose tile, pitch 9 (TRH: half of it, used twice)
    double lut[256];                 // DQ 1: the dequantized int16 value of each index byte, / 16
    uint8_t stage[64 * TB * 3 + 8 * 32];
};

// NTL / NTS: non-temporal index loads / pixel stores.  Plain loads measured
// 1.7 % faster than non-temporal ones; the store hint does not matter
// (decode variants 3 and 4 are the A/B records).  PRIO: wave
// priority while the index loads issue (3: 1 % faster than 0, variant 5).
// DQ: how an index byte becomes the column pass's input.  0: (int16)(Q*(k-128))
// with a 32-bit multiply, converted, the transform's 1/16 applied to each
// output (ldexp); 2: the same with a 24-bit multiply (full rate); 1: one LDS
// table of the 256 possible values, already divided by 16 -- a power of two
// commutes with every rounding of the transform (no value comes near the
// subnormal range), so the outputs are bit-identical and need no scaling.
// 3: the 24-bit multiply with the 1/16 folded into the input (one multiply
// per input instead of per output; no table, no LDS reads).
// EPI 1 (aligned frames): to_RGB, += 128 and the clamp on pixel pairs in packed
// int16 arithmetic (v_pk_add/sub/max/min_i16 wrap exactly as numpy's int16),
// the 24 bytes formed with byte permutes; 0: one pixel at a time.
// ACT: the DC-only wave test (round 3).  0: none; 1: the product's (the OR and
// the AND of the AC index bytes); 2: the OR of the dequantized AC values' high
// words (a double is +-0 iff its high word is 0 or 0x80000000, and every
// nonzero input here is >= 1/16 in magnitude, so a zero high word means a zero
// value: three v_or3 per column, no byte compares).  TRH: the transpose tile
// halved (rows 0-3, then 4-7 through the same 4 rows): 9 KiB less LDS per
// workgroup, more workgroups per CU.
template <int TB, bool SUB, bool PERC, bool PAD, bool NTL = false, bool NTS = true, int PRIO = 3, int DQ = 0,
          int EPI = 0, int ACT = 0, bool TRH = false>
__global__ __launch_bounds__(TB * 8) void dct_dz_decode_cols(const uint8_t *__restrict__ kin,
                                                              uint8_t *__restrict__ rgb, Geom g, int Q,
                                                              int tiles_per_row)
{
    constexpr bool PREF = (DQ == 1 || DQ == 3) && !PERC;   // inputs already divided by 16
    __shared__ __attribute__((aligned(16))) DecColsSmem<TB, TRH> sm;
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
        uint32_t acor = 0, acand = 0xFFu;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int kb = SUB ? sm.stage[cols_stage_off<TB, SUB>(i * 8 + x) + lb * 3 + C]
                               : sm.stage[cols_stage_off<TB, SUB>(i) + lb * 24 + x * 3 + C];
            if constexpr (ACT == 1) {
                const uint32_t ac = (i == 0 && x == 0) ? 128u : (uint32_t)kb;
                acor |= ac;
                acand &= ac;
            }
            if constexpr (DQ == 1 && !PERC) {
                col[i] = sm.lut[kb];
                continue;
            }
            int16_t yv = (int16_t)(DQ ? __mul24(Q, kb - 128) : Q * (kb - 128));
            if (PERC) {
                const float f = (float)((double)(float)yv / pweight_rt(C, i * 8 + x));
                yv = (int16_t)(int)f;
            }
            col[i] = PREF ? (double)yv * 0.0625 : (double)yv;
        }
        bool dc_only = false;
        if constexpr (ACT == 1) dc_only = __ballot(acor != 128u || acand != 128u) == 0;
        if constexpr (ACT == 2) {
            uint32_t h = x == 0 ? 0u : (uint32_t)__double2hiint(col[0]);
            h = h | (uint32_t)__double2hiint(col[1]) | (uint32_t)__double2hiint(col[2]);
            h = h | (uint32_t)__double2hiint(col[3]) | (uint32_t)__double2hiint(col[4]);
            h = h | (uint32_t)__double2hiint(col[5]) | (uint32_t)__double2hiint(col[6]);
            h |= (uint32_t)__double2hiint(col[7]);
            dc_only = __ballot((h & 0x7FFFFFFFu) != 0u) == 0;
        }
        if (ACT && dc_only) {   // wave-uniform: every block of the wave DC-only in channel C
            double v = __shfl(col[0], __lane_id() & ~7);
            double r[8] = {v, 0, 0, 0, 0, 0, 0, 0};
            dct3_8r_k<1>(r);
            double q[8] = {r[0], 0, 0, 0, 0, 0, 0, 0};
            dct3_8r_k<1>(q);
            const int o = (int16_t)(int)(PREF ? q[0] : q[0] * 0.0625);
#pragma unroll
            for (int j = 0; j < 8; ++j) out[C][j] = o;
            continue;
        }
        // :440 synthesize_image (A2): axis 0 (this lane's column), then axis 1
        dct3_8r(col);
        double row[8];
        if constexpr (TRH) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
#pragma unroll
                for (int y = 0; y < 4; ++y) tr[y][x] = col[4 * h + y];
                wave_lds_fence();
                if ((x >> 2) == h) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) row[j] = tr[x & 3][j];
                }
                wave_lds_fence();
            }
        } else {
#pragma unroll
            for (int y = 0; y < 8; ++y) tr[y][x] = col[y];
            wave_lds_fence();
#pragma unroll
            for (int j = 0; j < 8; ++j) row[j] = tr[x][j];
            wave_lds_fence();   // the tile is rewritten by the next channel
        }
        dct3_8r(row);
#pragma unroll
        for (int j = 0; j < 8; ++j)   // fct 1/4 per pass (already in the inputs for DQ 1/3); int16
            out[C][j] = (int16_t)(int)(PREF ? row[j] : row[j] * 0.0625);
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

// dq: 1 (default) = the dequantization table with the packed int16 epilogue; 0 = the
// round-1 kernel (decode variant 2, A/B)
template <int TB>
int launch_decode_cols(const uint8_t *k_dev, int64_t n_frames, uint8_t *rgb_dev, const Geom &g, int Q, bool sub,
                       bool perc, bool pad, void *stream, int dq = 1)
{
    const int tpr = (g.nbx + TB - 1) / TB;
    for (int64_t f0 = 0; f0 < n_frames; f0 += 65535) {
        const dim3 grid(tpr * g.nby, (unsigned)std::min<int64_t>(65535, n_frames - f0));
        const uint8_t *in = k_dev + f0 * g.out_stride;
        uint8_t *out = rgb_dev + f0 * g.in_stride;
#define VCF_DEC2(SB, PC, PD) \
        if (sub == SB && perc == PC && pad == PD) { \
            if (dq == 1) \
                hipLaunchKernelGGL((dct_dz_decode_cols<TB, SB, PC, PD, false, true, 3, 1, 1>), grid, dim3(TB * 8), 0, \
                                   (hipStream_t)stream, in, out, g, Q, tpr); \
            else \
                hipLaunchKernelGGL((dct_dz_decode_cols<TB, SB, PC, PD>), grid, dim3(TB * 8), 0, \
                                   (hipStream_t)stream, in, out, g, Q, tpr); \
        }
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
    __shared__ uint32_t rowbase[kTile];
    const int tid = threadIdx.x;
    const long long frame = blockIdx.y;
    const int n0 = blockIdx.x * kTile;
    const int nvalid = min(kTile, g.nblocks - n0);
    int by = 0, bx = 0;
    if (tid < nvalid) {
        tile_block(g, n0 + tid, by, bx);
        rowbase[tid] = block_rowbase<SUB>(g, by, bx);
    }
    __syncthreads();
    move_runs_tab<SUB, false>(g, stage, rowbase, const_cast<uint8_t *>(kin) + frame * g.out_stride, nvalid);
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

template <int TB>
int launch_cols(const uint8_t *rgb_dev, int64_t n_frames, uint8_t *k_dev, const Geom &g,
                const EncConsts &K, bool pow2, bool sub, bool perc, bool pad, void *stream)
{
    const int tpr = (g.nbx + TB - 1) / TB;
    for (int64_t f0 = 0; f0 < n_frames; f0 += 65535) {
        const dim3 grid(tpr * g.nby, (unsigned)std::min<int64_t>(65535, n_frames - f0));
        const uint8_t *in = rgb_dev + f0 * g.in_stride;
        uint8_t *out = k_dev + f0 * g.out_stride;
#define VCF_ENC7(P2, SB, PC, PD) \
        if (pow2 == P2 && sub == SB && perc == PC && pad == PD) \
            hipLaunchKernelGGL((dct_dz_encode_cols<TB, P2, SB, PC, PD>), grid, dim3(TB * 8), 0, \
                               (hipStream_t)stream, in, out, g, K, tpr);
        VCF_ENC7(true, true, false, false) else VCF_ENC7(true, true, false, true)
        else VCF_ENC7(true, true, true, false) else VCF_ENC7(true, true, true, true)
        else VCF_ENC7(true, false, false, false) else VCF_ENC7(true, false, false, true)
        else VCF_ENC7(true, false, true, false) else VCF_ENC7(true, false, true, true)
        else VCF_ENC7(false, true, false, false) else VCF_ENC7(false, true, false, true)
        else VCF_ENC7(false, true, true, false) else VCF_ENC7(false, true, true, true)
        else VCF_ENC7(false, false, false, false) else VCF_ENC7(false, false, false, true)
        else VCF_ENC7(false, false, true, false) else VCF_ENC7(false, false, true, true)
#undef VCF_ENC7
        const int rc = hip_check(hipGetLastError(), "dct_dz_encode_cols launch");
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

#define VCF_ENC_CASE(P2, SB, PC, PD)                                                      \
    if (pow2 == P2 && sub == SB && perc == PC && pad == PD)                               \
        hipLaunchKernelGGL((dct_dz_encode_kernel<P2, SB, PC, PD>), grid, dim3(kTile), 0,  \
                           (hipStream_t)stream, rgb_dev + f0 * g.in_stride,               \
                           k_dev + f0 * g.out_stride, g, K, rowk);

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
    return vcf_dct_dz_encode_variant(0, rgb_dev, n_frames, H, W, block_size, Q, flags, k_dev, stream);
}

int vcf_dct_dz_encode_variant(int variant, const uint8_t *rgb_dev, int64_t n_frames, int32_t H,
                              int32_t W, int32_t block_size, int32_t Q, uint32_t flags,
                              uint8_t *k_dev, void *stream)
{
    if (block_size != 8 && variant == 0)   // -B other than 8: vcf_dct_any.hip
        return dct_any_encode_u8(rgb_dev, n_frames, H, W, block_size, Q, flags, k_dev, stream);
    int rc = check_args(rgb_dev, k_dev, n_frames, H, W, block_size, Q, flags, false);
    if (rc != VCF_OK) return rc;
    if (variant < 0 || variant > 19) return set_error(VCF_ERR_INVALID, "unknown encode variant %d", variant);
    if (n_frames == 0) return VCF_OK;
    Geom g;
    make_geom(H, W, g);
    if (variant == 18 || variant == 19) {   // A/B: variant 0 over two / four chunks of frames on two library streams
        const PipeShape ps{2, variant == 18 ? 2 : 4, false};
        return run_pipelined(n_frames, ps, (hipStream_t)stream,
                             [&](long long f0, long long n, hipStream_t cs, const PipeHook *) {
                                 return vcf_dct_dz_encode_variant(0, rgb_dev + f0 * g.in_stride, n, H, W, block_size,
                                                                  Q, flags, k_dev + f0 * g.out_stride, cs);
                             });
    }
    const bool pow2 = (Q & (Q - 1)) == 0;
    const bool sub = !(flags & VCF_DCT_NO_SUBBANDS);
    const bool perc = (flags & VCF_DCT_PERCEPTUAL) != 0;
    const bool pad = (g.Hp != H) || (g.Wp != W);
    EncConsts K;
    make_enc_consts(K, Q);
    const FinalK rowk = pow2 ? row_final_k(Q) : final_k(1.0f, 1.0f);
    if (variant == 2 || variant == 6) {   // 6: the diagnostic body with packed transforms
        if (!pow2) return set_error(VCF_ERR_INVALID, "diagnostic variant needs a power-of-two Q");
        const long long nblocks = (long long)n_frames * g.nbx * g.nby;
        if (variant == 6)
            hipLaunchKernelGGL(dct_dz_encode_diag<true>, dim3((unsigned)((nblocks + kTile - 1) / kTile)),
                               dim3(kTile), 0, (hipStream_t)stream, k_dev, g, K, rowk, nblocks);
        else
            hipLaunchKernelGGL(dct_dz_encode_diag<false>, dim3((unsigned)((nblocks + kTile - 1) / kTile)),
                               dim3(kTile), 0, (hipStream_t)stream, k_dev, g, K, rowk, nblocks);
        return hip_check(hipGetLastError(), "dct_dz_encode_diag launch");
    }
    if (variant == 4) {   // A/B reference: variant 1 with generic byte code for the colour conversion
        if (!(pow2 && sub && !perc && !pad)) return set_error(VCF_ERR_INVALID, "variant 4: pow2 Q, aligned, default flags");
        for (int64_t f0 = 0; f0 < n_frames; f0 += 65535) {
            const dim3 grid(g.tiles_per_frame, (unsigned)std::min<int64_t>(65535, n_frames - f0));
            hipLaunchKernelGGL((dct_dz_encode_kernel<true, true, false, false, false>), grid, dim3(kTile), 0,
                               (hipStream_t)stream, rgb_dev + f0 * g.in_stride, k_dev + f0 * g.out_stride, g, K, rowk);
        }
        return hip_check(hipGetLastError(), "variant 4 launch");
    }
    if (variant == 8 || variant == 9 || variant == 10) {   // diagnostics: memory traffic without the transforms
        if (!(sub && !pad)) return set_error(VCF_ERR_INVALID, "variant 8: aligned frames, subband layout");
        if (variant != 8 && n_frames > 65535) return set_error(VCF_ERR_INVALID, "variants 9/10: <= 65535 frames");
        for (int64_t f0 = 0; f0 < n_frames; f0 += 65535) {
            const dim3 grid(g.tiles_per_frame, (unsigned)std::min<int64_t>(65535, n_frames - f0));
            if (variant == 8)
                hipLaunchKernelGGL((dct_dz_encode_kernel<true, true, false, false, true, false, true>), grid,
                                   dim3(kTile), 0, (hipStream_t)stream, rgb_dev + f0 * g.in_stride,
                                   k_dev + f0 * g.out_stride, g, K, rowk);
            else if (variant == 9)   // 64 aligned streams continuing from tile to tile
                hipLaunchKernelGGL((dct_dz_encode_kernel<true, true, false, false, true, false, true, 1>), grid,
                                   dim3(kTile), 0, (hipStream_t)stream, rgb_dev, k_dev, g, K, rowk);
            else   // the same streams shifted by 32 bytes: partial lines at every tile join
                hipLaunchKernelGGL((dct_dz_encode_kernel<true, true, false, false, true, false, true, 2>), grid,
                                   dim3(kTile), 0, (hipStream_t)stream, rgb_dev, k_dev, g, K, rowk);
        }
        return hip_check(hipGetLastError(), "variant 8 launch");
    }
    if (variant >= 12 && variant <= 16) {   // A/B: wave priority for the load issue / copy-out (PRIO)
        if (!(pow2 && !perc && sub && !pad)) return set_error(VCF_ERR_INVALID, "variants 12-16: pow2 Q, aligned, default flags");
        if (n_frames > 65535) return set_error(VCF_ERR_INVALID, "variants 12-16: <= 65535 frames");
        const dim3 grid(g.tiles_per_frame, (unsigned)n_frames);
#define VCF_ENC_PRIO(V, P) \
        if (variant == V) \
            hipLaunchKernelGGL((dct_dz_encode_kernel<true, true, false, false, true, true, false, 0, 0, true, 1, P>), grid, \
                               dim3(kTile), 0, (hipStream_t)stream, rgb_dev, k_dev, g, K, rowk);
        VCF_ENC_PRIO(12, 15) VCF_ENC_PRIO(13, 5) VCF_ENC_PRIO(14, 12) VCF_ENC_PRIO(15, 3) VCF_ENC_PRIO(16, 0)
#undef VCF_ENC_PRIO
        return hip_check(hipGetLastError(), "variant 12-16 launch");
    }
    if (variant == 17) {   // A/B: the default with the earlier address arithmetic (FA = false)
        if (!(pow2 && !perc && sub && !pad)) return set_error(VCF_ERR_INVALID, "variant 17: pow2 Q, aligned, default flags");
        if (n_frames > 65535) return set_error(VCF_ERR_INVALID, "variant 17: <= 65535 frames");
        const dim3 grid(g.tiles_per_frame, (unsigned)n_frames);
        hipLaunchKernelGGL((dct_dz_encode_kernel<true, true, false, false, true, true, false, 0, 0, true, 1, 15, false>),
                           grid, dim3(kTile), 0, (hipStream_t)stream, rgb_dev, k_dev, g, K, rowk);
        return hip_check(hipGetLastError(), "variant 17 launch");
    }
    if (variant == 11) {   // A/B: variant 5 with the earlier non-temporal input loads
        if (!(pow2 && !perc && sub && !pad)) return set_error(VCF_ERR_INVALID, "variant 11: pow2 Q, aligned, default flags");
        if (n_frames > 65535) return set_error(VCF_ERR_INVALID, "variant 11: <= 65535 frames");
        const dim3 grid(g.tiles_per_frame, (unsigned)n_frames);
        hipLaunchKernelGGL((dct_dz_encode_kernel<true, true, false, false, true, true, false, 0, 0, true, 0>), grid,
                           dim3(kTile), 0, (hipStream_t)stream, rgb_dev, k_dev, g, K, rowk);
        return hip_check(hipGetLastError(), "variant 11 launch");
    }
    if (variant == 7 && pow2 && !perc && sub && !pad) {   // A/B: variant 5 with the earlier store policy
        if (n_frames > 65535) return set_error(VCF_ERR_INVALID, "variant 7: <= 65535 frames");
        const dim3 grid(g.tiles_per_frame, (unsigned)n_frames);
        hipLaunchKernelGGL((dct_dz_encode_kernel<true, true, false, false, true, true, false, 0, 1, false>), grid,
                           dim3(kTile), 0, (hipStream_t)stream, rgb_dev, k_dev, g, K, rowk);
        return hip_check(hipGetLastError(), "variant 7 launch");
    }
    if ((variant == 5 || (variant == 0 && pow2 && !perc)) && pow2 && !perc) {   // packed-fp32 transforms
        for (int64_t f0 = 0; f0 < n_frames; f0 += 65535) {
            const dim3 grid(g.tiles_per_frame, (unsigned)std::min<int64_t>(65535, n_frames - f0));
#define VCF_ENC_PK(SB, PD)                                                                                  \
    if (sub == SB && pad == PD)                                                                             \
        hipLaunchKernelGGL((dct_dz_encode_kernel<true, SB, false, PD, true, true>), grid, dim3(kTile), 0,   \
                           (hipStream_t)stream, rgb_dev + f0 * g.in_stride, k_dev + f0 * g.out_stride, g, K, rowk);
            VCF_ENC_PK(true, false) else VCF_ENC_PK(true, true) else VCF_ENC_PK(false, false) else VCF_ENC_PK(false, true)
#undef VCF_ENC_PK
            rc = hip_check(hipGetLastError(), "dct_dz_encode_kernel (packed) launch");
            if (rc != VCF_OK) return rc;
        }
        return VCF_OK;
    }
    if (variant == 3) return launch_cols<128>(rgb_dev, n_frames, k_dev, g, K, pow2, sub, perc, pad, stream);
    for (int64_t f0 = 0; f0 < n_frames; f0 += 65535) {
        const dim3 grid(g.tiles_per_frame, (unsigned)std::min<int64_t>(65535, n_frames - f0));
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
    return vcf_dct_dz_decode_variant(0, k_dev, n_frames, H, W, block_size, Q, flags, rgb_dev, stream);
}

int vcf_dct_dz_decode_variant(int variant, const uint8_t *k_dev, int64_t n_frames, int32_t H, int32_t W,
                              int32_t block_size, int32_t Q, uint32_t flags, uint8_t *rgb_dev, void *stream)
{
    if (block_size != 8 && variant == 0)   // -B other than 8: vcf_dct_any.hip
        return dct_any_decode_u8(k_dev, n_frames, H, W, block_size, Q, flags, rgb_dev, stream);
    int rc = check_args(k_dev, rgb_dev, n_frames, H, W, block_size, Q, flags, true);
    if (rc != VCF_OK) return rc;
    if (variant < 0 || variant > 13) return set_error(VCF_ERR_INVALID, "unknown decode variant %d", variant);
    if (n_frames == 0) return VCF_OK;
    Geom g;
    make_geom(H, W, g);
    const bool sub = !(flags & VCF_DCT_NO_SUBBANDS);
    const bool perc = (flags & VCF_DCT_PERCEPTUAL) != 0;
    const bool pad = (g.Hp != H) || (g.Wp != W);
    if (variant >= 3) {   // A/B: column-per-lane with other load/store hints (aligned, default flags)
        if (!(sub && !perc && !pad)) return set_error(VCF_ERR_INVALID, "decode variants 3/4: aligned, default flags");
        if (n_frames > 65535) return set_error(VCF_ERR_INVALID, "decode variants 3/4: <= 65535 frames");
        const int tpr = (g.nbx + 31) / 32;
        const dim3 grid(tpr * g.nby, (unsigned)n_frames);
        if (variant == 3)   // the earlier non-temporal index loads
            hipLaunchKernelGGL((dct_dz_decode_cols<32, true, false, false, true, true>), grid, dim3(256), 0,
                               (hipStream_t)stream, k_dev, rgb_dev, g, (int)Q, tpr);
        else if (variant == 4)   // plain pixel stores
            hipLaunchKernelGGL((dct_dz_decode_cols<32, true, false, false, false, false>), grid, dim3(256), 0,
                               (hipStream_t)stream, k_dev, rgb_dev, g, (int)Q, tpr);
        else if (variant == 5)   // no wave priority for the load phase
            hipLaunchKernelGGL((dct_dz_decode_cols<32, true, false, false, false, true, 0>), grid, dim3(256), 0,
                               (hipStream_t)stream, k_dev, rgb_dev, g, (int)Q, tpr);
        else if (variant == 6)   // dequantization table in LDS, 1/16 folded in
            hipLaunchKernelGGL((dct_dz_decode_cols<32, true, false, false, false, true, 3, 1>), grid, dim3(256), 0,
                               (hipStream_t)stream, k_dev, rgb_dev, g, (int)Q, tpr);
        else if (variant == 7)   // 24-bit multiply for the dequantization
            hipLaunchKernelGGL((dct_dz_decode_cols<32, true, false, false, false, true, 3, 2>), grid, dim3(256), 0,
                               (hipStream_t)stream, k_dev, rgb_dev, g, (int)Q, tpr);
        else if (variant == 8)   // the table and the packed int16 epilogue
            hipLaunchKernelGGL((dct_dz_decode_cols<32, true, false, false, false, true, 3, 1, 1>), grid, dim3(256),
                               0, (hipStream_t)stream, k_dev, rgb_dev, g, (int)Q, tpr);
        else if (variant == 9)   // 8 + the product's DC-only test
            hipLaunchKernelGGL((dct_dz_decode_cols<32, true, false, false, false, true, 3, 1, 1, 1>), grid,
                               dim3(256), 0, (hipStream_t)stream, k_dev, rgb_dev, g, (int)Q, tpr);
        else if (variant == 10)   // 8 + the high-word DC-only test
            hipLaunchKernelGGL((dct_dz_decode_cols<32, true, false, false, false, true, 3, 1, 1, 2>), grid,
                               dim3(256), 0, (hipStream_t)stream, k_dev, rgb_dev, g, (int)Q, tpr);
        else if (variant == 11)   // arithmetic dequantization (1/16 folded in) + the high-word test
            hipLaunchKernelGGL((dct_dz_decode_cols<32, true, false, false, false, true, 3, 3, 1, 2>), grid,
                               dim3(256), 0, (hipStream_t)stream, k_dev, rgb_dev, g, (int)Q, tpr);
        else if (variant == 12)   // 10 with the half transpose tile
            hipLaunchKernelGGL((dct_dz_decode_cols<32, true, false, false, false, true, 3, 1, 1, 2, true>), grid,
                               dim3(256), 0, (hipStream_t)stream, k_dev, rgb_dev, g, (int)Q, tpr);
        else   // 11 with the half transpose tile
            hipLaunchKernelGGL((dct_dz_decode_cols<32, true, false, false, false, true, 3, 3, 1, 2, true>), grid,
                               dim3(256), 0, (hipStream_t)stream, k_dev, rgb_dev, g, (int)Q, tpr);
        return hip_check(hipGetLastError(), "decode variant 3/4 launch");
    }
    if (variant != 1)
        return launch_decode_cols<32>(k_dev, n_frames, rgb_dev, g, (int)Q, sub, perc, pad, stream, variant == 2 ? 0 : 1);
    for (int64_t f0 = 0; f0 < n_frames; f0 += 65535) {
        const dim3 grid(g.tiles_per_frame, (unsigned)std::min<int64_t>(65535, n_frames - f0));
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
