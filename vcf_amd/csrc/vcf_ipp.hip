// vcf_ipp.hip -- the IPP temporal tools of src/IPP_DCT.py on gfx950:
// luma conversion, block matching (full search and --fast three-step search),
// motion compensation, residual and reconstruction; vcf_ipp_* of the C ABI.
//
// Bit-exact with the reference's own functions (tests/golden/make_golden_ipp.py
// runs them unmodified):
//   IPP.block_matching (:344-376): cv2 RGB2GRAY (assumption A10: OpenCV's
//     8-bit fixed point (4899 R + 9617 G + 1868 B + 8192) >> 14), then per
//     bs x bs block of the full-block area a motion vector (dx, dy);
//   _process_block_row full search (:207-246): dy outer, dx inner over
//     [-S, S], in-bounds candidates only, SAD in int16, the first strict
//     minimum wins -> argmin of (SAD, scan index);
//   _three_step_search (:159-204): serial, the centre moves inside the
//     8-neighbour loop; one wave per block evaluates the candidates in order;
//   IPP.motion_compensate (:378-395): block copy, out-of-bounds vectors fall
//     back to the co-located block, outside the full-block area zeros;
//   residual (:547-551): clip(cur - comp + 128, 0, 255) as uint8;
//   reconstruction (:559-561, :788-790): clip(comp + rec - 128, 0, 255).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "vcf_amd.h"
#include "vcf_internal.h"

namespace vcf {
namespace {

constexpr int kMaxBs = 64;
constexpr int kMaxSr = 32;

__device__ __forceinline__ uint32_t luma(const uint8_t *p)
{
    return (4899u * p[0] + 9617u * p[1] + 1868u * p[2] + 8192u) >> 14;
}

__global__ __launch_bounds__(256) void ipp_gray_kernel(const uint8_t *__restrict__ rgb, uint8_t *__restrict__ gray,
                                                       long long npx)
{
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < npx) gray[p] = (uint8_t)luma(rgb + 3 * p);
}

// Full search: one workgroup per block; the block and its search window in
// LDS (window rows/cols clipped to the frame; out-of-frame candidates are
// skipped exactly as the reference skips them).
__global__ __launch_bounds__(256) void ipp_full_search_kernel(const uint8_t *__restrict__ ref,
                                                              const uint8_t *__restrict__ cur, int H, int W,
                                                              int bs, int sr, float *__restrict__ mv)
{
    __shared__ uint8_t cb[kMaxBs * kMaxBs];
    __shared__ uint8_t win[(kMaxBs + 2 * kMaxSr) * (kMaxBs + 2 * kMaxSr)];
    __shared__ unsigned long long best[4];
    const int bx = blockIdx.x, by = blockIdx.y;
    const int i = by * bs, j = bx * bs;
    const int ws = bs + 2 * sr;
    for (int t = threadIdx.x; t < bs * bs; t += blockDim.x) cb[t] = cur[(long long)(i + t / bs) * W + j + t % bs];
    for (int t = threadIdx.x; t < ws * ws; t += blockDim.x) {
        const int y = i - sr + t / ws, x = j - sr + t % ws;
        win[t] = (y >= 0 && y < H && x >= 0 && x < W) ? ref[(long long)y * W + x] : 0;
    }
    __syncthreads();
    const int side = 2 * sr + 1, ncand = side * side;
    unsigned long long key = ~0ULL;
    for (int c = threadIdx.x; c < ncand; c += blockDim.x) {
        const int dy = c / side - sr, dx = c % side - sr;
        const int ry = i + dy, rx = j + dx;
        if (ry < 0 || ry + bs > H || rx < 0 || rx + bs > W) continue;
        uint32_t sad = 0;
        const uint8_t *w0 = win + (dy + sr) * ws + (dx + sr);
        for (int y = 0; y < bs; ++y) {
            const uint8_t *a = cb + y * bs, *b = w0 + y * ws;
            int x = 0;
            for (; x + 4 <= bs; x += 4) {
                const uint32_t av = a[x] | (a[x + 1] << 8) | (a[x + 2] << 16) | ((uint32_t)a[x + 3] << 24);
                const uint32_t bv = b[x] | (b[x + 1] << 8) | (b[x + 2] << 16) | ((uint32_t)b[x + 3] << 24);
                sad = __builtin_amdgcn_sad_u8(av, bv, sad);
            }
            for (; x < bs; ++x) sad += (uint32_t)abs((int)a[x] - (int)b[x]);
        }
        const unsigned long long k = ((unsigned long long)sad << 20) | (unsigned long long)c;
        key = k < key ? k : key;
    }
    // workgroup argmin of (SAD, scan index)
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(key, off, 64);
        key = o < key ? o : key;
    }
    if ((threadIdx.x & 63) == 0) best[threadIdx.x >> 6] = key;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long k = best[0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) k = best[w] < k ? best[w] : k;
        float dxv = 0.f, dyv = 0.f;   // no valid candidate cannot happen (0,0 is in bounds)
        if (k != ~0ULL) {
            const int c = (int)(k & 0xFFFFF);
            dyv = (float)(c / side - sr);
            dxv = (float)(c % side - sr);
        }
        float *m = mv + ((long long)by * gridDim.x + bx) * 2;
        m[0] = dxv;
        m[1] = dyv;
    }
}

// Full search on words (bs % 4 == 0, the default path): the block's rows and
// the search window sit in LDS as 32-bit words of 4 luma bytes; a thread owns
// one candidate (the workgroup has a lane per candidate, up to 1024) and
// forms each window word at its byte offset with one v_alignbyte, then
// v_sad_u8 adds 4 |differences| at a time -- 2 LDS reads, 1 align and 1 SAD
// per 4 pixels where the byte kernel above needs 8 byte reads and the
// packing.  The SAD is the same integer sum, the argmin the same (SAD, scan
// index) key, so the vectors are identical.
template <int WQ>   // words per block row (bs / 4); 0 = run-time
__global__ __launch_bounds__(1024) void ipp_full_search_words(const uint8_t *__restrict__ ref,
                                                              const uint8_t *__restrict__ cur, int H, int W,
                                                              int bs, int sr, float *__restrict__ mv)
{
    constexpr int kWinW = (kMaxBs + 2 * kMaxSr + 3) / 4 + 1;   // words per window row, max
    __shared__ uint32_t cbw[kMaxBs * kMaxBs / 4];
    __shared__ uint32_t winw[(kMaxBs + 2 * kMaxSr) * kWinW];
    __shared__ unsigned long long best[16];
    const int bx = blockIdx.x, by = blockIdx.y;
    const int i = by * bs, j = bx * bs;
    const int ws = bs + 2 * sr;
    const int wq = WQ ? WQ : bs >> 2;
    const int wp = (ws + 3) / 4 + 1;   // one spare word: a row's last aligned read
    const int tid = threadIdx.x, nthr = blockDim.x;
    for (int t = tid; t < bs * wq; t += nthr) {
        const int y = t / wq, q = t - y * wq;
        const uint8_t *p = cur + (long long)(i + y) * W + j + 4 * q;
        cbw[t] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
    }
    for (int t = tid; t < ws * wp; t += nthr) {
        const int r = t / wp, q = t - r * wp;
        const int y = i - sr + r;
        uint32_t v = 0;
        if (y >= 0 && y < H) {
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int x = j - sr + 4 * q + b;
                if (x >= 0 && x < W) v |= (uint32_t)ref[(long long)y * W + x] << (8 * b);
            }
        }
        winw[t] = v;
    }
    __syncthreads();
    const int side = 2 * sr + 1, ncand = side * side;
    unsigned long long key = ~0ULL;
    for (int c = tid; c < ncand; c += nthr) {
        const int dyi = c / side, dxi = c - dyi * side;   // window offsets dy + sr, dx + sr
        const int ry = i + dyi - sr, rx = j + dxi - sr;
        if (ry < 0 || ry + bs > H || rx < 0 || rx + bs > W) continue;
        const int w0 = dxi >> 2;
        const uint32_t sh = (uint32_t)(dxi & 3);
        uint32_t sad = 0;
        for (int y = 0; y < bs; ++y) {
            const uint32_t *a = cbw + y * wq;
            const uint32_t *b = winw + (dyi + y) * wp + w0;
            uint32_t lo = b[0];
            if (WQ) {
#pragma unroll
                for (int q = 0; q < WQ; ++q) {
                    const uint32_t hi = b[q + 1];
                    sad = __builtin_amdgcn_sad_u8(a[q], __builtin_amdgcn_alignbyte(hi, lo, sh), sad);
                    lo = hi;
                }
            } else {
                for (int q = 0; q < wq; ++q) {
                    const uint32_t hi = b[q + 1];
                    sad = __builtin_amdgcn_sad_u8(a[q], __builtin_amdgcn_alignbyte(hi, lo, sh), sad);
                    lo = hi;
                }
            }
        }
        const unsigned long long k = ((unsigned long long)sad << 20) | (unsigned long long)c;
        key = k < key ? k : key;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(key, off, 64);
        key = o < key ? o : key;
    }
    if ((tid & 63) == 0) best[tid >> 6] = key;
    __syncthreads();
    if (tid == 0) {
        unsigned long long k = best[0];
        for (int w = 1; w < (nthr >> 6); ++w) k = best[w] < k ? best[w] : k;
        float dxv = 0.f, dyv = 0.f;
        if (k != ~0ULL) {
            const int c = (int)(k & 0xFFFFF);
            dyv = (float)(c / side - sr);
            dxv = (float)(c % side - sr);
        }
        float *m = mv + ((long long)by * gridDim.x + bx) * 2;
        m[0] = dxv;
        m[1] = dyv;
    }
}

// SAD of the block at (i, j) against the reference at (ry, rx), one wave
__device__ uint32_t wave_sad(const uint8_t *cb, const uint8_t *ref, int W, int bs, int ry, int rx)
{
    uint32_t s = 0;
    for (int t = threadIdx.x; t < bs * bs; t += 64) {
        const int y = t / bs, x = t % bs;
        s += (uint32_t)abs((int)cb[t] - (int)ref[(long long)(ry + y) * W + rx + x]);
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    return s;
}

// Three-step search (--fast): one wave per block, the candidates in the
// reference's order because an improvement moves the centre immediately.
__global__ __launch_bounds__(64) void ipp_tss_kernel(const uint8_t *__restrict__ ref, const uint8_t *__restrict__ cur,
                                                     int H, int W, int bs, int sr, float *__restrict__ mv)
{
    __shared__ uint8_t cb[kMaxBs * kMaxBs];
    const int bx = blockIdx.x, by = blockIdx.y;
    const int i = by * bs, j = bx * bs;
    for (int t = threadIdx.x; t < bs * bs; t += 64) cb[t] = cur[(long long)(i + t / bs) * W + j + t % bs];
    __syncthreads();
    int step = sr / 2, cx = j, cy = i, bxv = 0, byv = 0;
    uint32_t best = wave_sad(cb, ref, W, bs, i, j);   // the block itself is always in bounds
    // a candidate may only improve on a finite minimum; the centre check ran, so min is finite
    while (step >= 1) {
        bool improved = false;
        for (int a = -1; a <= 1; ++a)
            for (int b = -1; b <= 1; ++b) {
                if (a == 0 && b == 0) continue;
                const int ry = cy + a * step, rx = cx + b * step;
                if (ry < 0 || ry + bs > H || rx < 0 || rx + bs > W) continue;
                const uint32_t s = wave_sad(cb, ref, W, bs, ry, rx);
                if (s < best) {
                    best = s;
                    bxv = rx - j;
                    byv = ry - i;
                    cx = rx;
                    cy = ry;
                    improved = true;
                }
            }
        step = improved ? (step / 2 > 1 ? step / 2 : 1) : step / 2;
    }
    if (threadIdx.x == 0) {
        float *m = mv + ((long long)by * gridDim.x + bx) * 2;
        m[0] = (float)bxv;
        m[1] = (float)byv;
    }
}

// Three-step search for bs = 16 (the default block size), same decisions as
// ipp_tss_kernel: the 8 neighbours of the current centre are evaluated in one
// parallel round (8 lanes per candidate, 2 block rows of 4 words per lane,
// v_alignbyte + v_sad_u8), then scanned in the reference's order; at the
// first improvement the centre moves and the candidates after it are
// evaluated again around the new centre, exactly as the serial loop would.
// Candidates read a (16 + 2R)^2 window of the reference staged in LDS as
// words; one outside it (a centre that wandered > R - step) takes the
// byte path from global memory.
constexpr int kTssR = 16;                          // window margin
constexpr int kTssWS = 16 + 2 * kTssR;             // window side (bytes)
constexpr int kTssWP = kTssWS / 4 + 1;             // words per window row (+1 spare)

__global__ __launch_bounds__(64) void ipp_tss16_kernel(const uint8_t *__restrict__ ref,
                                                       const uint8_t *__restrict__ cur, int H, int W, int sr,
                                                       float *__restrict__ mv)
{
    __shared__ uint32_t win[kTssWS * kTssWP];
    __shared__ uint32_t sads[9];
    const int bx = blockIdx.x, by = blockIdx.y, lane = threadIdx.x;
    const int i = by * 16, j = bx * 16;
    const int wy0 = i - kTssR, wx0 = j - kTssR;      // frame position of window (0, 0)
    // whole words straight from the frame when the window lies inside it and
    // rows are word aligned (W % 4 == 0; wx0 is a multiple of 16); else bytes
    const bool words = (W & 3) == 0 && wx0 >= 0 && wx0 + 4 * kTssWP <= W && wy0 >= 0 && wy0 + kTssWS <= H;
    for (int t = lane; t < kTssWS * kTssWP; t += 64) {
        const int r = t / kTssWP, q = t - r * kTssWP;
        const int y = wy0 + r;
        uint32_t v = 0;
        if (words) {
            v = *reinterpret_cast<const uint32_t *>(ref + (long long)y * W + wx0 + 4 * q);
        } else if (y >= 0 && y < H) {
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int x = wx0 + 4 * q + b;
                if (x >= 0 && x < W) v |= (uint32_t)ref[(long long)y * W + x] << (8 * b);
            }
        }
        win[t] = v;
    }
    // this lane's block words: rows 2g, 2g+1 (g = lane & 7), 4 words each
    const int g = lane & 7, cand = lane >> 3;
    uint32_t cw[8];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint8_t *p = cur + (long long)(i + 2 * g + r) * W + j + 4 * q;
            cw[r * 4 + q] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
        }
    __syncthreads();
    // SAD of this lane's 8 words against the reference block at frame (ry, rx)
    auto part_sad = [&](int ry, int rx) -> uint32_t {
        const int wy = ry - wy0, wx = rx - wx0;
        uint32_t s = 0;
        if (wy >= 0 && wy + 16 <= kTssWS && wx >= 0 && wx + 16 <= kTssWS) {
            const uint32_t sh = (uint32_t)(wx & 3);
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const uint32_t *b = win + (wy + 2 * g + r) * kTssWP + (wx >> 2);
                uint32_t lo = b[0];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t hi = b[q + 1];
                    s = __builtin_amdgcn_sad_u8(cw[r * 4 + q], __builtin_amdgcn_alignbyte(hi, lo, sh), s);
                    lo = hi;
                }
            }
        } else {   // outside the staged window (rare): bytes from global memory
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int x = 0; x < 16; ++x) {
                    const int a = (int)((cw[r * 4 + (x >> 2)] >> (8 * (x & 3))) & 0xFFu);
                    const int b = ref[(long long)(ry + 2 * g + r) * W + rx + x];
                    s += (uint32_t)abs(a - b);
                }
        }
        return s;
    };
    auto group_sum = [&](uint32_t s) -> uint32_t {   // sum over the 8 lanes of a candidate group
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        return s;
    };
    auto inb = [&](int ry, int rx) { return ry >= 0 && ry + 16 <= H && rx >= 0 && rx + 16 <= W; };
    // the centre's SAD (the block itself, always in bounds): every group computes it, group 0 publishes
    uint32_t best = group_sum(part_sad(i, j));
    int cy = i, cx = j, bxv = 0, byv = 0;
    int step = sr / 2;
    while (step >= 1) {
        bool improved = false;
        int k = 0;                   // next neighbour (scan order dy outer, dx inner, centre skipped)
        while (k < 8) {
            // neighbour m: (a, b) = offsets of the m-th of the 8 in scan order
            const int m = cand, mm = m + (m >= 4);   // skip the centre (index 4 of 3x3)
            const int ry = cy + (mm / 3 - 1) * step, rx = cx + (mm % 3 - 1) * step;
            uint32_t sv = 0xFFFFFFFFu;
            if (m >= k && inb(ry, rx)) sv = group_sum(part_sad(ry, rx));
            else group_sum(0u);      // keep the shuffles uniform
            if (g == 0) sads[m] = sv;
            __syncthreads();
            int moved = -1;
            for (int t = k; t < 8; ++t) {
                const uint32_t st = sads[t];
                if (st != 0xFFFFFFFFu && st < best) {
                    const int tt = t + (t >= 4);
                    best = st;
                    cy += (tt / 3 - 1) * step;
                    cx += (tt % 3 - 1) * step;
                    byv = cy - i;
                    bxv = cx - j;
                    improved = true;
                    moved = t;
                    break;
                }
            }
            __syncthreads();         // sads[] is rewritten by the next round
            if (moved < 0) break;
            k = moved + 1;
        }
        step = improved ? (step / 2 > 1 ? step / 2 : 1) : step / 2;
    }
    if (lane == 0) {
        float *o = mv + ((long long)by * gridDim.x + bx) * 2;
        o[0] = (float)bxv;
        o[1] = (float)byv;
    }
}

__global__ __launch_bounds__(256) void ipp_mc_kernel(const uint8_t *__restrict__ ref, const float *__restrict__ mv,
                                                     int H, int W, int bs, uint8_t *__restrict__ out)
{
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (long long)H * W) return;
    const int y = (int)(p / W), x = (int)(p % W);
    const int nbx = W / bs, nby = H / bs;
    const int by = y / bs, bx = x / bs;
    uint8_t *o = out + p * 3;
    if (by >= nby || bx >= nbx) {   // outside the full-block area: np.zeros_like
        o[0] = o[1] = o[2] = 0;
        return;
    }
    const float *m = mv + ((long long)by * nbx + bx) * 2;
    const int i = by * bs, j = bx * bs;
    int ry = (int)((float)i + m[1]), rx = (int)((float)j + m[0]);   // int(i + mv[1]) on float32
    if (!(ry >= 0 && ry + bs <= H && rx >= 0 && rx + bs <= W)) {
        ry = i;
        rx = j;
    }
    const uint8_t *s = ref + ((long long)(ry + (y - i)) * W + rx + (x - j)) * 3;
    o[0] = s[0];
    o[1] = s[1];
    o[2] = s[2];
}

__global__ __launch_bounds__(256) void ipp_residual_kernel(const uint8_t *__restrict__ cur,
                                                           const uint8_t *__restrict__ comp, long long n,
                                                           uint8_t *__restrict__ out)
{
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int v = (int)cur[p] - (int)comp[p] + 128;
    out[p] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

__global__ __launch_bounds__(256) void ipp_recon_kernel(const uint8_t *__restrict__ comp,
                                                        const uint8_t *__restrict__ rec, long long n,
                                                        uint8_t *__restrict__ out)
{
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int v = (int)comp[p] + (int)rec[p] - 128;
    out[p] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

unsigned blocks_for(long long n) { return (unsigned)((n + 255) / 256); }

int g_full_search_variant = 0;   // 0: word kernel when bs % 4 == 0; 1: byte kernel (A/B)
int ipp_full_search_variant() { return g_full_search_variant; }

}  // namespace
}  // namespace vcf

using namespace vcf;

extern "C" {

int vcf_ipp_block_match(const uint8_t *ref_rgb_dev, const uint8_t *cur_rgb_dev, int32_t H, int32_t W, int32_t bs,
                        int32_t sr, int32_t fast, float *mv_dev, uint8_t *gray_workspace_dev, void *stream)
{
    if (!ref_rgb_dev || !cur_rgb_dev || !mv_dev || !gray_workspace_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    if (H <= 0 || W <= 0) return set_error(VCF_ERR_INVALID, "bad frame shape");
    if (bs < 1 || bs > kMaxBs) return set_error(VCF_ERR_UNSUPPORTED, "block size %d (1..%d)", bs, kMaxBs);
    if (sr < 0 || sr > kMaxSr) return set_error(VCF_ERR_UNSUPPORTED, "search range %d (0..%d)", sr, kMaxSr);
    const int nbx = W / bs, nby = H / bs;
    if (nbx == 0 || nby == 0) return VCF_OK;
    hipStream_t s = (hipStream_t)stream;
    const long long npx = (long long)H * W;
    uint8_t *rg = gray_workspace_dev, *cg = gray_workspace_dev + npx;
    hipLaunchKernelGGL(ipp_gray_kernel, dim3(blocks_for(npx)), dim3(256), 0, s, ref_rgb_dev, rg, npx);
    hipLaunchKernelGGL(ipp_gray_kernel, dim3(blocks_for(npx)), dim3(256), 0, s, cur_rgb_dev, cg, npx);
    if (fast) {
        if (bs == 16 && ipp_full_search_variant() == 0)
            hipLaunchKernelGGL(ipp_tss16_kernel, dim3(nbx, nby), dim3(64), 0, s, rg, cg, H, W, sr, mv_dev);
        else
            hipLaunchKernelGGL(ipp_tss_kernel, dim3(nbx, nby), dim3(64), 0, s, rg, cg, H, W, bs, sr, mv_dev);
    } else if (bs % 4 != 0 || ipp_full_search_variant() == 1) {
        hipLaunchKernelGGL(ipp_full_search_kernel, dim3(nbx, nby), dim3(256), 0, s, rg, cg, H, W, bs, sr, mv_dev);
    } else {
        const int ncand = (2 * sr + 1) * (2 * sr + 1);
        const int nthr = std::min(1024, (ncand + 63) / 64 * 64);
        const dim3 grid(nbx, nby);
        switch (bs) {
        case 4: hipLaunchKernelGGL(ipp_full_search_words<1>, grid, dim3(nthr), 0, s, rg, cg, H, W, bs, sr, mv_dev); break;
        case 8: hipLaunchKernelGGL(ipp_full_search_words<2>, grid, dim3(nthr), 0, s, rg, cg, H, W, bs, sr, mv_dev); break;
        case 16: hipLaunchKernelGGL(ipp_full_search_words<4>, grid, dim3(nthr), 0, s, rg, cg, H, W, bs, sr, mv_dev); break;
        case 32: hipLaunchKernelGGL(ipp_full_search_words<8>, grid, dim3(nthr), 0, s, rg, cg, H, W, bs, sr, mv_dev); break;
        default: hipLaunchKernelGGL(ipp_full_search_words<0>, grid, dim3(nthr), 0, s, rg, cg, H, W, bs, sr, mv_dev); break;
        }
    }
    return hip_check(hipGetLastError(), "ipp block match launch");
}

int vcf_ipp_set_full_search_variant(int32_t variant)
{
    if (variant < 0 || variant > 1) return set_error(VCF_ERR_INVALID, "unknown full-search variant %d", variant);
    g_full_search_variant = variant;
    return VCF_OK;
}

int vcf_ipp_motion_compensate(const uint8_t *ref_rgb_dev, const float *mv_dev, int32_t H, int32_t W, int32_t bs,
                              uint8_t *out_rgb_dev, void *stream)
{
    if (!ref_rgb_dev || !mv_dev || !out_rgb_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    if (H <= 0 || W <= 0 || bs < 1) return set_error(VCF_ERR_INVALID, "bad arguments");
    const long long npx = (long long)H * W;
    hipLaunchKernelGGL(ipp_mc_kernel, dim3(blocks_for(npx)), dim3(256), 0, (hipStream_t)stream, ref_rgb_dev, mv_dev,
                       H, W, bs, out_rgb_dev);
    return hip_check(hipGetLastError(), "ipp mc launch");
}

int vcf_ipp_residual(const uint8_t *cur_dev, const uint8_t *comp_dev, int64_t n, uint8_t *out_dev, void *stream)
{
    if (n < 0 || (n > 0 && (!cur_dev || !comp_dev || !out_dev))) return set_error(VCF_ERR_INVALID, "bad arguments");
    if (n == 0) return VCF_OK;
    hipLaunchKernelGGL(ipp_residual_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, cur_dev, comp_dev,
                       (long long)n, out_dev);
    return hip_check(hipGetLastError(), "ipp residual launch");
}

int vcf_ipp_reconstruct(const uint8_t *comp_dev, const uint8_t *rec_dev, int64_t n, uint8_t *out_dev, void *stream)
{
    if (n < 0 || (n > 0 && (!comp_dev || !rec_dev || !out_dev))) return set_error(VCF_ERR_INVALID, "bad arguments");
    if (n == 0) return VCF_OK;
    hipLaunchKernelGGL(ipp_recon_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, comp_dev, rec_dev,
                       (long long)n, out_dev);
    return hip_check(hipGetLastError(), "ipp recon launch");
}

}  // extern "C"
