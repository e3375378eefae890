// vcf_cbaac_gpu.hip -- tiled CBAAC: the context-based adaptive arithmetic
// coder of src/CBAAC.py as a GPU-resident entropy stage (SURVEY.md §8(f)
// row 2).
//
// The reference codes the flattened frame as ONE stream (CBAAC.py:114-131):
// every interval depends on every earlier symbol, so that byte stream cannot
// be produced in parallel (vcf_cbaac.cpp keeps it, on the host).  The tiled
// variant splits the flattened symbols into consecutive segments of seg_len
// symbols and runs the reference's algorithm on each segment from scratch --
// a fresh ContextManager (:49-69, every model 256 frequencies of 1), history
// reset to `order` zeros (:119), the A8 coder from low = 0, high = 2^32 - 1,
// flushed at the segment's end (:130).  Each segment's bytes are therefore
// exactly what the serial coder (vcf_cbaac_encode) writes for that segment
// alone, and the container (vcf_amd/tcbaac.py) records each segment's size.
//
// Mapping: one wave per segment; the 64 lanes share one model.
//   - Order 0: the cumulative table C[0..256) of the model lives in VGPRs,
//     lane l holding C[4l .. 4l+3]; C[256] = total is wave-uniform.
//     get_range(s) (:40-41) is two v_readlane; update(s) (:32-36) adds 1 to
//     C[t] for t > s in every lane (4 compares, no cross-lane work); the
//     rescale (every ~16 k symbols: stale total >= 16384, f = (f >> 1) + 1)
//     rebuilds C with one wave prefix scan.  The decoder's
//     get_symbol_from_scaled_value (:43-47) becomes one ballot over the
//     lanes' interval ends (see the decode kernel).
//   - Order 1: the 256 context models (one per previous symbol) as 16-bit
//     cumulative tables in LDS (128 KiB + totals), the current context's row
//     read into the same four VGPRs per lane and written back after the
//     update.
//   - The coder state (low, high, pending bits, the bit writer) is
//     wave-uniform; floor(range * c / total) is a float64 multiply by an
//     estimated 1/total plus an exact correction (operands < 2^47).  Bits are packed MSB-first into
//     words that lane 0 stores (vector stores); symbols stream in 256 at a
//     time (one dword per lane, the next chunk prefetched).
// A second pass packs the segments back to back (a scan of their sizes and a
// copy), so only the compressed bytes need to leave HBM.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "vcf_amd.h"
#include "vcf_internal.h"

namespace vcf {
namespace {

constexpr uint32_t kMaxFreq = 16384;   // AdaptiveModel(max_freq=16384), CBAAC.py:18
constexpr uint32_t kQ1 = 0x40000000u;
constexpr int kChunk = 256;            // symbols (or bytes) per wave load: one dword per lane

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t lane)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

// ---- the model --------------------------------------------------------------------
// Lane l holds C[4l..4l+3] (C[s] = sum of freqs[0..s)) as packed u16 pairs:
// p0 = C[4l] | C[4l+1] << 16, p1 = C[4l+2] | C[4l+3] << 16 (every count
// <= 16385).  total = C[256] is wave-uniform.
struct Model {
    uint32_t p0, p1;
    uint32_t total;
};

__device__ __forceinline__ void model_reset(Model &m, uint32_t lane)
{
    m.p0 = (4 * lane) | ((4 * lane + 1) << 16);   // all frequencies 1
    m.p1 = (4 * lane + 2) | ((4 * lane + 3) << 16);
    m.total = 256;
}

// Prior-initialised models (orders 0 and 1, the `.tadpt_arith` version-2 container):
// every segment starts from the frame's prior frequencies f[s] = 1 +
// floor(hist[s] * kPriorScale / n) instead of 256 ones, then adapts by the
// reference's rules (CBAAC.py:32-36).  Short segments then stop paying the
// model's learning cost.
constexpr uint32_t kPriorScale = 8192;   // prior total <= 256 + 8192 < max_freq
constexpr int32_t kMaxClasses = 256;      // prior rows per frame (container version 3)

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t lane);

__device__ __forceinline__ void model_reset_prior(Model &m, const uint16_t *__restrict__ prior, uint32_t lane)
{
    const uint2 q = *reinterpret_cast<const uint2 *>(prior + 4 * lane);   // f[4l .. 4l+3]
    const uint32_t f0 = q.x & 0xFFFFu, f1 = q.x >> 16, f2 = q.y & 0xFFFFu, f3 = q.y >> 16;
    const uint32_t sum = f0 + f1 + f2 + f3;
    const uint32_t ex = wave_excl_scan(sum, lane);
    m.p0 = ex | ((ex + f0) << 16);
    m.p1 = (ex + f0 + f1) | ((ex + f0 + f1 + f2) << 16);
    m.total = rl(ex + sum, 63);
}

// C[4L..4L+4] of lane L as one 64-bit word + C[4L+4]
struct Quad {
    uint64_t w;
    uint32_t next;
};

__device__ __forceinline__ Quad model_quad(const Model &m, uint32_t L)
{
    Quad q;
    q.w = (uint64_t)rl(m.p0, L) | ((uint64_t)rl(m.p1, L) << 32);
    const uint32_t nx = rl(m.p0, (L + 1) & 63) & 0xFFFFu;
    q.next = L == 63 ? m.total : nx;
    return q;
}

// (cum[s], cum[s+1]) of get_range (CBAAC.py:40-41)
__device__ __forceinline__ void model_range(const Model &m, uint32_t s, uint32_t &lo, uint32_t &hi)
{
    const Quad q = model_quad(m, s >> 2);
    const uint32_t j = s & 3;
    lo = (uint32_t)(q.w >> (16 * j)) & 0xFFFFu;
    hi = j == 3 ? q.next : (uint32_t)(q.w >> (16 * j + 16)) & 0xFFFFu;
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t lane)
{
    uint32_t incl = v;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += o;
    }
    return incl - v;
}

// update(s) (CBAAC.py:32-36): freqs[s] += 1, i.e. C[t] += 1 for t > s; if the
// total *before* the increment is >= max_freq, every frequency becomes
// (f >> 1) + 1 and C is rebuilt.
__device__ __forceinline__ void model_update(Model &m, uint32_t s, uint32_t lane)
{
    const uint32_t L = s >> 2, j = s & 3;
    // increments of lane L's two words: entries 4L+j+1 .. 4L+3
    const uint32_t i0 = j == 0 ? 0x10000u : 0u;
    const uint32_t i1 = j <= 1 ? 0x10001u : (j == 2 ? 0x10000u : 0u);
    m.p0 += lane > L ? 0x10001u : (lane == L ? i0 : 0u);
    m.p1 += lane > L ? 0x10001u : (lane == L ? i1 : 0u);
    const uint32_t stale = m.total;
    m.total = stale + 1;
    if (stale >= kMaxFreq) {
        const uint32_t c0 = m.p0 & 0xFFFFu, c1 = m.p0 >> 16, c2 = m.p1 & 0xFFFFu, c3 = m.p1 >> 16;
        const uint32_t nxt0 = __shfl_down(c0, 1, 64);
        const uint32_t end = lane == 63 ? m.total : nxt0;
        const uint32_t f0 = ((c1 - c0) >> 1) + 1, f1 = ((c2 - c1) >> 1) + 1, f2 = ((c3 - c2) >> 1) + 1,
                       f3 = ((end - c3) >> 1) + 1;
        const uint32_t sum = f0 + f1 + f2 + f3;
        const uint32_t ex = wave_excl_scan(sum, lane);
        m.p0 = ex | ((ex + f0) << 16);
        m.p1 = (ex + f0 + f1) | ((ex + f0 + f1 + f2) << 16);
        m.total = rl(ex + sum, 63);
    }
}

// order-1 context tables: 256 models x 256 cumulative counts (u16) + totals, in LDS
struct Tables {
    uint2 c[256 * 64];     // row ctx: lane l's (p0, p1)
    uint32_t total[256];
};

// the order-1 kernels' LDS (a function-scope __shared__ variable is
// allocated in every kernel that calls get())
template <int ORDER>
struct Lds {
    __device__ static Tables *get() { return nullptr; }
};
template <>
struct Lds<1> {
    __device__ static Tables *get()
    {
        __shared__ Tables t;
        return &t;
    }
};

__device__ __forceinline__ void tables_reset(Tables &t, uint32_t lane)
{
    Model m;
    model_reset(m, lane);
    for (uint32_t r = 0; r < 256; ++r) t.c[r * 64 + lane] = make_uint2(m.p0, m.p1);
    for (uint32_t r = lane; r < 256; r += 64) t.total[r] = 256;
    __syncthreads();
}

// order 1 with a prior: every context's model starts from the frame's order-0 prior
__device__ __forceinline__ void tables_reset_prior(Tables &t, const uint16_t *__restrict__ prior, uint32_t lane)
{
    Model m;
    model_reset_prior(m, prior, lane);
    for (uint32_t r = 0; r < 256; ++r) t.c[r * 64 + lane] = make_uint2(m.p0, m.p1);
    for (uint32_t r = lane; r < 256; r += 64) t.total[r] = m.total;
    __syncthreads();
}

__device__ __forceinline__ void tables_read(const Tables &t, uint32_t ctx, uint32_t lane, Model &m)
{
    const uint2 v = t.c[ctx * 64 + lane];
    m.p0 = v.x;
    m.p1 = v.y;
    m.total = (uint32_t)__builtin_amdgcn_readfirstlane((int)t.total[ctx]);
}

__device__ __forceinline__ void tables_write(Tables &t, uint32_t ctx, uint32_t lane, const Model &m)
{
    t.c[ctx * 64 + lane] = make_uint2(m.p0, m.p1);
    if (lane == 0) t.total[ctx] = m.total;
}

// ---- the A8 coder's arithmetic ---------------------------------------------------------
// floor(a / t) for integers a < 2^47, 0 < t <= 2^19 held exactly in doubles,
// given inv ~= 1/t (relative error < 2^-50): q = trunc(a * inv) is within 1
// of the floor, r = a - q t is exact (an fma of integers < 2^47) and lies in
// (-t, 2t), and floor(r * inv + 2^-20) is the step (-1, 0 or +1) that fixes
// q: r / t = m + j/t with j in 0..t-1, and 2^-20 is below 1/t
// (t <= 2^19) and above the error of r * inv.
__device__ __forceinline__ double floordiv(double a, double t, double inv)
{
    const double q = __builtin_trunc(a * inv);
    const double r = __builtin_fma(-q, t, a);
    return q + __builtin_floor(__builtin_fma(r, inv, 0x1p-20));
}

// 1/t for 1 <= t < 2^33: the hardware estimate and two Newton steps
// (relative error far below the 2^-50 floordiv needs).
__device__ __forceinline__ double rcp_nr(double t)
{
    double x = __builtin_amdgcn_rcp(t);
    x = __builtin_fma(x, __builtin_fma(-t, x, 1.0), x);
    x = __builtin_fma(x, __builtin_fma(-t, x, 1.0), x);
    return x;
}

// MSB-first bit writer (bitarray endian='big'); lane 0 stores whole words.
// acc holds nb < 32 pending bits at its top.
struct BitWriter {
    uint32_t *out;
    uint64_t acc = 0;
    uint32_t nb = 0;
    uint64_t words = 0;

    // append the top k bits of v (1 <= k <= 32)
    __device__ __forceinline__ void bits(uint32_t v, uint32_t k, uint32_t lane)
    {
        if (k < 32) v &= ~(0xFFFFFFFFu >> k);
        acc |= (uint64_t)v << (32 - nb);
        nb += k;
        if (nb >= 32) {
            if (lane == 0) out[words] = __builtin_bswap32((uint32_t)(acc >> 32));
            ++words;
            acc <<= 32;
            nb -= 32;
        }
    }
    __device__ __forceinline__ void run(uint32_t bit, uint64_t count, uint32_t lane)
    {
        const uint32_t v = bit ? 0xFFFFFFFFu : 0u;
        for (; count >= 32; count -= 32) bits(v, 32, lane);
        if (count) bits(v, (uint32_t)count, lane);
    }
    __device__ __forceinline__ uint64_t finish(uint32_t lane)
    {
        if (nb && lane == 0) out[words] = __builtin_bswap32((uint32_t)(acc >> 32));
        return words * 32 + nb;
    }
};

// Encoder state: the interval and the pending (underflow) bits.
struct Encoder {
    uint32_t low = 0, high = 0xFFFFFFFFu;
    uint64_t pending = 0;

    // interval update + renormalisation of the A8 coder (vcf_cbaac.cpp's loop,
    // done in one step: the loop emits the common leading bits of low and
    // high, each followed by the pending bits after the first, then counts
    // the underflow steps while low = 01.. and high = 10..)
    __device__ __forceinline__ void code(uint32_t lo, uint32_t hi, double tot, double inv, BitWriter &w,
                                         uint32_t lane)
    {
        const double rng = (double)(high - low) + 1.0;
        const double qh = floordiv(rng * (double)hi, tot, inv);
        const double ql = floordiv(rng * (double)lo, tot, inv);
        high = low + (uint32_t)(qh - 1.0);
        low = low + (uint32_t)ql;
        const uint32_t d = __builtin_clz(low ^ high);   // high > low: d <= 31
        if (d) {
            const uint32_t b = low >> 31;
            w.bits(low, 1, lane);
            w.run(b ^ 1u, pending, lane);
            pending = 0;
            if (d > 1) w.bits(low << 1, d - 1, lane);
            low <<= d;
            high = (high << d) | ((1u << d) - 1u);
        }
        const uint32_t x = (low << 1) & ~(high << 1);
        const uint32_t p = __builtin_clz(~x);
        if (p) {
            pending += p;
            low = (low << p) & 0x7FFFFFFFu;
            high = (high << p) | ((1u << p) - 1u) | 0x80000000u;
        }
    }
    // flush (CBAAC.py:130 -> A8): one more pending bit and a disambiguating bit
    __device__ __forceinline__ void flush(BitWriter &w, uint32_t lane)
    {
        const uint32_t b = low < kQ1 ? 0u : 1u;
        w.bits(b << 31, 1, lane);
        w.run(b ^ 1u, pending + 1, lane);
    }
};

// Four symbols per lane.  Segment starts are multiples of 256 symbols from
// `sym`, so a dword load is aligned exactly when `sym` is (`aligned`,
// wave-uniform); a caller's pointer into the middle of a buffer (a frame of
// n % 4 != 0 symbols after the first) takes the byte loads.
__device__ __forceinline__ uint32_t load_sym4(const uint8_t *p, int64_t off, int64_t len, uint32_t lane, bool aligned)
{
    const int64_t i = off + 4 * (int64_t)lane;
    if (aligned && i + 3 < len) return *reinterpret_cast<const uint32_t *>(p + i);
    uint32_t v = 0;
    for (int j = 0; j < 4; ++j)
        if (i + j < len) v |= (uint32_t)p[i + j] << (8 * j);
    return v;
}

__device__ __forceinline__ double rcp_exact(uint32_t t) { return rcp_nr((double)t); }

// Frames of a batch (blockIdx.y = frame): frame f's symbols at sym + f *
// sym_stride, its prior at prior + f * prior_stride (0: one prior for all),
// its decoded symbols at out + f * out_stride, its packed segments at
// out + f * cap (encode)
struct Frames {
    int64_t sym_stride = 0, prior_stride = 0, out_stride = 0, cap = 0;
    int32_t nclass = 1;   // prior classes: segment s of nseg takes prior row s * nclass / nseg
};

// the prior row of segment `seg` of a frame's `nseg` (container version 3:
// nclass rows of 256, consecutive runs of segments share a row)
__device__ __forceinline__ const uint16_t *class_prior(const uint16_t *prior, int64_t seg, int64_t nseg, int32_t nclass)
{
    return prior + 256 * ((seg * nclass) / nseg);
}

template <int ORDER, bool TRACE>
__global__ __launch_bounds__(64) void cbaac_tiled_encode_kernel(const uint8_t *__restrict__ sym, int64_t n,
                                                                int64_t seg_len, uint32_t *__restrict__ slots,
                                                                int64_t slot_words, int64_t *__restrict__ seg_bits,
                                                                int32_t *__restrict__ trace,
                                                                const uint16_t *__restrict__ prior, Frames fr)
{
    Tables *tabs = Lds<ORDER>::get();
    {   // frame blockIdx.y of a batch
        const int64_t f = blockIdx.y, nsf = (n + seg_len - 1) / seg_len;
        sym += f * fr.sym_stride;
        slots += f * nsf * slot_words;
        seg_bits += f * nsf;
        if (prior) prior = class_prior(prior + f * fr.prior_stride, blockIdx.x, nsf, fr.nclass);
    }
    const int64_t seg = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    const int64_t start = seg * seg_len;
    const int64_t len = n - start < seg_len ? n - start : seg_len;
    const uint8_t *src = sym + start;

    Model m;
    if (prior) model_reset_prior(m, prior, lane);
    else model_reset(m, lane);
    if constexpr (ORDER == 1) {
        if (prior) tables_reset_prior(tabs[0], prior, lane);
        else tables_reset(tabs[0], lane);
    }
    uint32_t ctx = 0;

    BitWriter w;
    w.out = slots + seg * slot_words;
    Encoder e;

    const bool aligned = (reinterpret_cast<uintptr_t>(sym) & 3) == 0;
    uint32_t cur = load_sym4(src, 0, len, lane, aligned);
    for (int64_t off = 0; off < len; off += kChunk) {
        const uint32_t nxt = off + kChunk < len ? load_sym4(src, off + kChunk, len, lane, aligned) : 0u;
        const int cnt = len - off < kChunk ? (int)(len - off) : kChunk;
        for (int k = 0; k < cnt; ++k) {
            const uint32_t s = (rl(cur, k >> 2) >> (8 * (k & 3))) & 255u;
            if constexpr (ORDER == 1) tables_read(tabs[0], ctx, lane, m);
            const uint32_t tot = m.total;
            const double inv = rcp_exact(tot);
            uint32_t lo, hi;
            model_range(m, s, lo, hi);
            if constexpr (TRACE) {
                if (lane == 0) {
                    int32_t *t = trace + 3 * (start + off + k);
                    t[0] = (int32_t)lo;
                    t[1] = (int32_t)hi;
                    t[2] = (int32_t)tot;
                }
            }
            e.code(lo, hi, (double)tot, inv, w, lane);
            model_update(m, s, lane);
            if constexpr (ORDER == 1) {
                tables_write(tabs[0], ctx, lane, m);
                ctx = s;
            }
        }
        cur = nxt;
    }
    e.flush(w, lane);
    const uint64_t bits = w.finish(lane);
    if (lane == 0) seg_bits[seg] = (int64_t)bits;
}

// MSB-first bit reader over a segment's bytes, zeros past its end (A8).
// buf holds `avail` unread bits at its top; words come from 256-byte chunks
// held one big-endian dword per lane (the next chunk prefetched).
struct BitReader {
    const uint8_t *src;
    int64_t nbytes;
    int64_t chunk = 0;         // byte offset of `cur`
    uint32_t cur = 0, nxt = 0;
    uint32_t wi = 0;           // next word of `cur`
    uint64_t buf = 0;
    uint32_t avail = 0;

    __device__ __forceinline__ uint32_t load(int64_t off, uint32_t lane) const
    {
        uint32_t v = 0;
        for (int j = 0; j < 4; ++j) {
            const int64_t i = off + 4 * (int64_t)lane + j;
            v = (v << 8) | (i < nbytes ? (uint32_t)src[i] : 0u);
        }
        return v;
    }
    __device__ __forceinline__ void refill(uint32_t lane)
    {
        if (wi == 64) {
            wi = 0;
            chunk += kChunk;
            cur = nxt;
            nxt = load(chunk + kChunk, lane);
        }
        buf |= (uint64_t)rl(cur, wi++) << (32 - avail);
        avail += 32;
    }
    __device__ __forceinline__ void start(uint32_t lane)
    {
        cur = load(0, lane);
        nxt = load(kChunk, lane);
        refill(lane);
    }
    // the next k bits (1 <= k <= 32), right-aligned
    __device__ __forceinline__ uint32_t get(uint32_t k, uint32_t lane)
    {
        if (avail < k) refill(lane);
        const uint32_t v = (uint32_t)(buf >> (64 - k));
        buf <<= k;
        avail -= k;
        return v;
    }
};

template <int ORDER>
__global__ __launch_bounds__(64) void cbaac_tiled_decode_kernel(const uint8_t *__restrict__ in,
                                                                const int64_t *__restrict__ offs, int64_t n,
                                                                int64_t seg_len, uint8_t *__restrict__ out,
                                                                const uint16_t *__restrict__ prior, Frames fr)
{
    Tables *tabs = Lds<ORDER>::get();
    {
        const int64_t f = blockIdx.y, nsf = (n + seg_len - 1) / seg_len;
        offs += f * (nsf + 1);
        out += f * fr.out_stride;
        if (prior) prior = class_prior(prior + f * fr.prior_stride, blockIdx.x, nsf, fr.nclass);
    }
    const int64_t seg = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    const int64_t start = seg * seg_len;
    const int64_t len = n - start < seg_len ? n - start : seg_len;
    uint8_t *dst = out + start;
    const bool out_aligned = (reinterpret_cast<uintptr_t>(out) & 3) == 0;   // start is a multiple of 256

    Model m;
    if (prior) model_reset_prior(m, prior, lane);
    else model_reset(m, lane);
    if constexpr (ORDER == 1) {
        if (prior) tables_reset_prior(tabs[0], prior, lane);
        else tables_reset(tabs[0], lane);
    }
    uint32_t ctx = 0;

    BitReader br;
    br.src = in + offs[seg];
    br.nbytes = offs[seg + 1] - offs[seg];
    br.start(lane);
    uint32_t low = 0, high = 0xFFFFFFFFu, value = br.get(32, lane);

    uint32_t obuf = 0, acc = 0;
    for (int64_t i = 0; i < len; ++i) {
        if constexpr (ORDER == 1) tables_read(tabs[0], ctx, lane, m);
        const double tot = (double)m.total;
        const double inv = rcp_nr(tot);
        const uint32_t span = high - low;                 // range - 1
        const double rng = (double)span + 1.0;
        // The A8 decoder picks s with C[s] <= floor(((T + 1) total - 1) / range)
        // < C[s+1], T = value - low; for integers that is
        // floor(range C[s] / total) <= T < floor(range C[s+1] / total), and
        // those floors are the new interval's ends: every lane computes them
        // for its four counts, a ballot finds the lane, no division by range.
        const uint32_t T = value - low;
        const uint32_t f0 = (uint32_t)floordiv(rng * (double)(m.p0 & 0xFFFFu), tot, inv);
        const uint32_t f1 = (uint32_t)floordiv(rng * (double)(m.p0 >> 16), tot, inv);
        const uint32_t f2 = (uint32_t)floordiv(rng * (double)(m.p1 & 0xFFFFu), tot, inv);
        const uint32_t f3 = (uint32_t)floordiv(rng * (double)(m.p1 >> 16), tot, inv);
        const uint32_t L = (uint32_t)__popcll(__ballot(f0 <= T)) - 1;   // f0 increases with the lane
        const uint32_t g0 = rl(f0, L), g1 = rl(f1, L), g2 = rl(f2, L), g3 = rl(f3, L);
        const uint32_t g4m1 = L == 63 ? span : rl(f0, (L + 1) & 63) - 1;   // floor(range C[4L+4] / total) - 1
        const uint32_t j = (T >= g1 ? 1u : 0u) + (T >= g2 ? 1u : 0u) + (T >= g3 ? 1u : 0u);
        const uint32_t s = 4 * L + j;
        const uint32_t ql = j == 0 ? g0 : j == 1 ? g1 : j == 2 ? g2 : g3;
        const uint32_t qhm1 = j == 0 ? g1 - 1 : j == 1 ? g2 - 1 : j == 2 ? g3 - 1 : g4m1;
        high = low + qhm1;
        low = low + ql;
        const uint32_t d = __builtin_clz(low ^ high);
        if (d) {
            low <<= d;
            high = (high << d) | ((1u << d) - 1u);
            value = (value << d) | br.get(d, lane);
        }
        const uint32_t x = (low << 1) & ~(high << 1);
        const uint32_t p = __builtin_clz(~x);
        if (p) {
            low = (low << p) & 0x7FFFFFFFu;
            high = (high << p) | ((1u << p) - 1u) | 0x80000000u;
            value = ((value << p) ^ 0x80000000u) | br.get(p, lane);
        }
        model_update(m, s, lane);
        if constexpr (ORDER == 1) {
            tables_write(tabs[0], ctx, lane, m);
            ctx = s;
        }
        acc |= s << (8 * (i & 3));
        if ((i & 3) == 3) {
            obuf = lane == (uint32_t)((i >> 2) & 63) ? acc : obuf;
            acc = 0;
        }
        if ((i & (kChunk - 1)) == kChunk - 1) {   // a full chunk: one dword per lane
            uint8_t *q = dst + (i - (kChunk - 1)) + 4 * lane;
            if (out_aligned) {
                *reinterpret_cast<uint32_t *>(q) = obuf;
            } else {
                for (int j = 0; j < 4; ++j) q[j] = (uint8_t)(obuf >> (8 * j));
            }
        }
    }
    const int64_t done = len & ~(int64_t)(kChunk - 1);
    if (done < len) {   // the partial last chunk, byte by byte
        if (len & 3) obuf = lane == (uint32_t)(((len - 1) >> 2) & 63) ? acc : obuf;
        for (int j = 0; j < 4; ++j) {
            const int64_t i = done + 4 * (int64_t)lane + j;
            if (i < len) dst[i] = (uint8_t)(obuf >> (8 * j));
        }
    }
}

// segment sizes (bits) -> byte offsets (exclusive scan), sizes and the total
__global__ __launch_bounds__(1024) void cbaac_tiled_scan_kernel(const int64_t *__restrict__ seg_bits, int64_t nseg,
                                                                int64_t *__restrict__ offs,
                                                                int64_t *__restrict__ seg_bytes)
{
    seg_bits += (int64_t)blockIdx.x * nseg;   // frame blockIdx.x
    offs += (int64_t)blockIdx.x * (nseg + 1);
    seg_bytes += (int64_t)blockIdx.x * (nseg + 1);
    __shared__ int64_t part[1024];
    const int t = threadIdx.x;
    const int64_t per = (nseg + 1023) / 1024;
    const int64_t a = t * per, b = a + per < nseg ? a + per : nseg;
    int64_t sum = 0;
    for (int64_t i = a; i < b; ++i) sum += (seg_bits[i] + 7) >> 3;
    part[t] = sum;
    __syncthreads();
    if (t == 0) {
        int64_t run = 0;
        for (int i = 0; i < 1024; ++i) {
            const int64_t v = part[i];
            part[i] = run;
            run += v;
        }
        offs[nseg] = run;
        seg_bytes[nseg] = run;
    }
    __syncthreads();
    int64_t run = part[t];
    for (int64_t i = a; i < b; ++i) {
        const int64_t nb = (seg_bits[i] + 7) >> 3;
        offs[i] = run;
        seg_bytes[i] = nb;
        run += nb;
    }
}

__global__ __launch_bounds__(256) void cbaac_tiled_pack_kernel(const uint32_t *__restrict__ slots, int64_t slot_words,
                                                               const int64_t *__restrict__ offs, uint8_t *__restrict__ out,
                                                               int64_t capacity)
{
    const int64_t f = blockIdx.y;   // frame of a batch: gridDim.x segments each, out regions `capacity` apart
    slots += f * (int64_t)gridDim.x * slot_words;
    offs += f * ((int64_t)gridDim.x + 1);
    out += f * capacity;
    const int64_t seg = blockIdx.x;
    const uint8_t *src = reinterpret_cast<const uint8_t *>(slots + seg * slot_words);
    const int64_t o = offs[seg], nb = offs[seg + 1] - o;
    for (int64_t i = threadIdx.x; i < nb; i += 256)
        if (o + i < capacity) out[o + i] = src[i];
}

// order-0 histogram of the frame's symbols (LDS bins, one global atomic per bin and workgroup)
__global__ __launch_bounds__(256) void cbaac_hist_kernel(const uint8_t *__restrict__ sym, int64_t n,
                                                         uint32_t *__restrict__ hist, int64_t sym_stride)
{
    sym += (int64_t)blockIdx.y * sym_stride;   // frame blockIdx.y
    hist += 256 * blockIdx.y;
    __shared__ uint32_t bins[256];
    bins[threadIdx.x] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        atomicAdd(&bins[sym[i]], 1u);
    __syncthreads();
    if (bins[threadIdx.x]) atomicAdd(&hist[threadIdx.x], bins[threadIdx.x]);
}

__global__ __launch_bounds__(256) void cbaac_prior_kernel(const uint32_t *__restrict__ hist, int64_t n,
                                                          uint16_t *__restrict__ prior)
{
    hist += 256 * blockIdx.x;   // frame blockIdx.x
    prior += 256 * blockIdx.x;
    const uint32_t t = threadIdx.x;
    prior[t] = (uint16_t)(1u + (n > 0 ? (uint32_t)((uint64_t)hist[t] * kPriorScale / (uint64_t)n) : 0u));
}

// Version 3 (prior classes): per-class histograms, one workgroup per segment
// (its class is fixed), LDS bins, one global atomic per bin and segment
__global__ __launch_bounds__(256) void cbaac_hist_classes_kernel(const uint8_t *__restrict__ sym, int64_t n,
                                                                 int64_t seg_len, int32_t nclass,
                                                                 uint32_t *__restrict__ hist, int64_t sym_stride)
{
    const int64_t nseg = (n + seg_len - 1) / seg_len, seg = blockIdx.x;
    sym += (int64_t)blockIdx.y * sym_stride + seg * seg_len;   // frame blockIdx.y
    hist += 256 * ((int64_t)blockIdx.y * nclass + (seg * nclass) / nseg);
    const int64_t len = n - seg * seg_len < seg_len ? n - seg * seg_len : seg_len;
    __shared__ uint32_t bins[256];
    bins[threadIdx.x] = 0;
    __syncthreads();
    for (int64_t i = threadIdx.x; i < len; i += 256) atomicAdd(&bins[sym[i]], 1u);
    __syncthreads();
    if (bins[threadIdx.x]) atomicAdd(&hist[threadIdx.x], bins[threadIdx.x]);
}

// prior row of one (frame, class): f[s] = 1 + floor(hist[s] * 8192 / n_c), n_c
// the class's symbols (one class: the frame's n, version 2's formula)
__global__ __launch_bounds__(256) void cbaac_prior_classes_kernel(const uint32_t *__restrict__ hist,
                                                                  uint16_t *__restrict__ prior)
{
    hist += 256 * (int64_t)blockIdx.x;   // row (frame, class) blockIdx.x
    prior += 256 * (int64_t)blockIdx.x;
    __shared__ uint32_t part[4];
    const uint32_t t = threadIdx.x, h = hist[t];
    uint32_t v = h;
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if ((t & 63) == 0) part[t >> 6] = v;
    __syncthreads();
    const uint64_t nc = (uint64_t)part[0] + part[1] + part[2] + part[3];
    prior[t] = (uint16_t)(1u + (nc > 0 ? (uint32_t)((uint64_t)h * kPriorScale / nc) : 0u));
}

// ---- lane-per-segment coder (order 0) ----------------------------------------------
// One LANE per segment: a wave codes 64 segments at once, each with its own
// model and coder state, where the kernels above spend a whole wave on one
// segment's model.  Same algorithm, same bytes (the A8 coder and
// AdaptiveModel of CBAAC.py:17-47, 114-131 per segment).
// The model is two-level, u16 in LDS: C[b] (b = 0..15) = the frequencies of
// the symbols below 16 b summed (block starts), E[b][j] = those of 16 b ..
// 16 b + j - 1 (exclusive prefixes inside block b).  get_range(s) = (C[b] +
// E[b][j], C[b] + E[b][j + 1]) -- at j = 15 the upper end is C[b + 1], or the
// total at b = 15.  update(s) adds 1 to E[b][t > j] and to C[t > b]: an add
// of a mask to four 16-byte chunks (u16 entries never carry into the next:
// every count is below 2^15), and every frequency becomes (f >> 1) + 1 when
// the stale total reaches max_freq (CBAAC.py:32-36), rebuilt from the
// prefixes.  LDS units of 16 bytes are laid out [block][half][lane]: the b128
// accesses of a wave (one block and half per lane) are bank-conflict free.
constexpr int kLW = 64;   // segments (lanes) per workgroup

struct LaneLds {
    uint4 E[16][2][kLW];   // [block][half][lane]: entries 8 half .. 8 half + 7 of block `block`
    uint4 C[2][kLW];       // [half][lane]: block starts 8 half .. 8 half + 7
    uint4 M[16][2];        // M[i]: 1 in the u16 entries t > i
};

__device__ __forceinline__ uint4 add4(const uint4 &a, const uint4 &b)
{
    return make_uint4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// every lane's initial model (its segment's prior row, or 256 ones; lanes may
// sit in different prior classes) and the shared mask table
__device__ __forceinline__ void lane_model_init(LaneLds &L, const uint16_t *__restrict__ prior, uint32_t lane,
                                                uint32_t &total)
{
    if (lane >= 16 && lane < 48) {   // mask table
        const int i = (lane - 16) >> 1, h = (lane - 16) & 1;
        uint32_t d[4];
        for (int k = 0; k < 4; ++k) {
            const int t = 8 * h + 2 * k;
            d[k] = (t > i ? 1u : 0u) | (t + 1 > i ? 0x10000u : 0u);
        }
        L.M[i][h] = make_uint4(d[0], d[1], d[2], d[3]);
    }
    uint32_t run = 0, c[16];
    for (int b = 0; b < 16; ++b) {
        uint32_t acc = 0, e[16];
        if (prior) {
            const uint2 *q = reinterpret_cast<const uint2 *>(prior + 16 * b);   // f[16b .. 16b+15], 8-B aligned
            const uint2 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
            const uint32_t w[8] = {q0.x, q0.y, q1.x, q1.y, q2.x, q2.y, q3.x, q3.y};
            for (int k = 0; k < 16; ++k) {
                e[k] = acc;
                acc += (k & 1) ? w[k >> 1] >> 16 : w[k >> 1] & 0xFFFFu;
            }
        } else {
            for (int k = 0; k < 16; ++k) e[k] = k;
            acc = 16;
        }
        L.E[b][0][lane] = make_uint4(e[0] | e[1] << 16, e[2] | e[3] << 16, e[4] | e[5] << 16, e[6] | e[7] << 16);
        L.E[b][1][lane] = make_uint4(e[8] | e[9] << 16, e[10] | e[11] << 16, e[12] | e[13] << 16, e[14] | e[15] << 16);
        c[b] = run;
        run += acc;
    }
    L.C[0][lane] = make_uint4(c[0] | c[1] << 16, c[2] | c[3] << 16, c[4] | c[5] << 16, c[6] | c[7] << 16);
    L.C[1][lane] = make_uint4(c[8] | c[9] << 16, c[10] | c[11] << 16, c[12] | c[13] << 16, c[14] | c[15] << 16);
    total = run;
    __syncthreads();
}

// every frequency -> (f >> 1) + 1 (CBAAC.py:34-36), from the prefixes; returns the new total
__device__ __attribute__((noinline)) uint32_t lane_model_rescale(LaneLds &L, uint32_t lane, uint32_t total)
{
    uint32_t cs[17];
    {
        const uint4 c0 = L.C[0][lane], c1 = L.C[1][lane];
        const uint32_t w[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        for (int k = 0; k < 8; ++k) {
            cs[2 * k] = w[k] & 0xFFFFu;
            cs[2 * k + 1] = w[k] >> 16;
        }
        cs[16] = total;
    }
    uint32_t run = 0, cn[16];
    for (int b = 0; b < 16; ++b) {
        const uint4 e0 = L.E[b][0][lane], e1 = L.E[b][1][lane];
        const uint32_t w[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
        uint32_t e[17];
        for (int k = 0; k < 8; ++k) {
            e[2 * k] = w[k] & 0xFFFFu;
            e[2 * k + 1] = w[k] >> 16;
        }
        e[16] = cs[b + 1] - cs[b];
        cn[b] = run;
        uint32_t acc = 0, ne[16];
        for (int t = 0; t < 16; ++t) {
            ne[t] = acc;
            acc += ((e[t + 1] - e[t]) >> 1) + 1;
        }
        run += acc;
        L.E[b][0][lane] = make_uint4(ne[0] | ne[1] << 16, ne[2] | ne[3] << 16, ne[4] | ne[5] << 16, ne[6] | ne[7] << 16);
        L.E[b][1][lane] =
            make_uint4(ne[8] | ne[9] << 16, ne[10] | ne[11] << 16, ne[12] | ne[13] << 16, ne[14] | ne[15] << 16);
    }
    L.C[0][lane] = make_uint4(cn[0] | cn[1] << 16, cn[2] | cn[3] << 16, cn[4] | cn[5] << 16, cn[6] | cn[7] << 16);
    L.C[1][lane] =
        make_uint4(cn[8] | cn[9] << 16, cn[10] | cn[11] << 16, cn[12] | cn[13] << 16, cn[14] | cn[15] << 16);
    return run;
}

// per-lane MSB-first bit writer: acc holds nb < 32 pending bits at its top, whole
// words go to the lane's own slot (bitarray endian='big')
struct LaneBits {
    uint32_t *out;
    uint64_t acc = 0;
    uint32_t nb = 0, words = 0;
    __device__ __forceinline__ void bits(uint32_t v, uint32_t k)   // the top k bits of v, 1 <= k <= 32
    {
        if (k < 32) v &= ~(0xFFFFFFFFu >> k);
        acc |= (uint64_t)v << (32 - nb);
        nb += k;
        if (nb >= 32) {
            out[words++] = __builtin_bswap32((uint32_t)(acc >> 32));
            acc <<= 32;
            nb -= 32;
        }
    }
    __device__ __forceinline__ void run(uint32_t bit, uint32_t count)
    {
        const uint32_t v = bit ? 0xFFFFFFFFu : 0u;
        for (; count >= 32; count -= 32) bits(v, 32);
        if (count) bits(v, count);
    }
};

template <bool PRIOR>
__global__ __launch_bounds__(kLW) void cbaac_lane_encode_kernel(const uint8_t *__restrict__ sym, int64_t n,
                                                                int64_t seg_len, int64_t nseg,
                                                                uint32_t *__restrict__ slots, int64_t slot_words,
                                                                int64_t *__restrict__ seg_bits,
                                                                const uint16_t *__restrict__ prior, Frames fr)
{
    __shared__ LaneLds L;
    {   // frame blockIdx.y of a batch (nseg segments each)
        const int64_t f = blockIdx.y;
        sym += f * fr.sym_stride;
        slots += f * nseg * slot_words;
        seg_bits += f * nseg;
        if (prior) prior += f * fr.prior_stride;
    }
    const uint32_t lane = threadIdx.x;
    const int64_t seg = (int64_t)blockIdx.x * kLW + lane;
    const bool act = seg < nseg;
    const int64_t start = act ? seg * seg_len : 0;
    const int64_t len = act ? (n - start < seg_len ? n - start : seg_len) : 0;
    uint32_t total;
    lane_model_init(L, PRIOR ? class_prior(prior, act ? seg : 0, nseg, fr.nclass) : nullptr, lane, total);
    double inv = rcp_nr((double)total);
    LaneBits w;
    w.out = slots + (act ? seg : 0) * slot_words;
    uint32_t low = 0, high = 0xFFFFFFFFu, pending = 0;
    const uint8_t *src = sym + start;
    const bool aligned = (reinterpret_cast<uintptr_t>(src) & 15) == 0;
    auto load16 = [&](int64_t off) -> uint4 {   // symbols off .. off + 15 (zeros past the segment)
        if (aligned && off + 16 <= len) return *reinterpret_cast<const uint4 *>(src + off);
        uint32_t d[4] = {0, 0, 0, 0};
        for (int k = 0; k < 16; ++k)
            if (off + k < len) d[k >> 2] |= (uint32_t)src[off + k] << (8 * (k & 3));
        return make_uint4(d[0], d[1], d[2], d[3]);
    };
    const int64_t seg0 = (int64_t)blockIdx.x * kLW;
    const int64_t wave_len = n - seg0 * seg_len < seg_len ? n - seg0 * seg_len : seg_len;   // the longest lane's
    uint4 cur = load16(0);
    char *const Eb = reinterpret_cast<char *>(&L.E[0][0][lane]);
    char *const Cb = reinterpret_cast<char *>(&L.C[0][lane]);
    constexpr uint32_t kHalfStride = kLW * 16;   // bytes from (b, half) to (b, half + 1) of a lane
    // get_range(s) of the model as it stands (u16 reads of the lane's tables)
    auto query = [&](uint32_t s, uint32_t tot, uint32_t &lo, uint32_t &hi) {
        const uint32_t b = s >> 4, j = s & 15u, j1 = j < 15 ? j + 1 : 15, b1 = b < 15 ? b + 1 : 15;
        const uint32_t eb = b * (2 * kHalfStride);
        const uint32_t e_lo = *reinterpret_cast<const uint16_t *>(Eb + eb + (j >> 3) * kHalfStride + (j & 7) * 2);
        const uint32_t e_hi = *reinterpret_cast<const uint16_t *>(Eb + eb + (j1 >> 3) * kHalfStride + (j1 & 7) * 2);
        const uint32_t c_lo = *reinterpret_cast<const uint16_t *>(Cb + (b >> 3) * kHalfStride + (b & 7) * 2);
        const uint32_t c_hi = *reinterpret_cast<const uint16_t *>(Cb + (b1 >> 3) * kHalfStride + (b1 & 7) * 2);
        lo = c_lo + e_lo;
        hi = j < 15 ? c_lo + e_hi : (b < 15 ? c_hi : tot);
    };
    // Software pipeline: symbol i+1's range is read from the model BEFORE
    // symbol i's update and corrected afterwards (the update adds one to every
    // cumulative count above s_i and to the total): get_range(s') after
    // update(s) = (cum[s'] + [s' > s], cum[s' + 1] + [s' >= s]), total + 1.
    // So the model's LDS round trips run beside the coder's arithmetic chain,
    // not in front of it.  A rescale (the stale total at max_freq) reads again.
    uint32_t s_cur = cur.x & 0xFFu, lo_cur = 0, hi_cur = 0;
    if (len > 0) query(s_cur, total, lo_cur, hi_cur);
    for (int64_t off = 0; off < wave_len; off += 16) {
        const uint4 nxt = off + 16 < wave_len ? load16(off + 16) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (off + k < len) {
                const uint32_t s = s_cur;
                const uint32_t s_n = k < 15 ? ((k + 1 < 4 ? cur.x : k + 1 < 8 ? cur.y : k + 1 < 12 ? cur.z : cur.w) >>
                                               (8 * ((k + 1) & 3))) & 0xFFu
                                            : nxt.x & 0xFFu;
                const bool more = off + k + 1 < len;
                const uint32_t b = s >> 4, j = s & 15u;
                const uint32_t tot_i = total;
                const bool resc = tot_i >= kMaxFreq;            // the stale total (CBAAC.py:34)
                const double inv_n = rcp_nr((double)(tot_i + 1));   // the next symbol's, off the chain
                uint32_t lo_n = 0, hi_n = 0;
                if (more) query(s_n, tot_i, lo_n, hi_n);         // before this symbol's update
                // update(s): the four chunks plus the mask rows
                const uint4 e0 = L.E[b][0][lane], e1 = L.E[b][1][lane];
                const uint4 c0 = L.C[0][lane], c1 = L.C[1][lane];
                const uint4 mj0 = L.M[j][0], mj1 = L.M[j][1], mb0 = L.M[b][0], mb1 = L.M[b][1];
                L.E[b][0][lane] = add4(e0, mj0);
                L.E[b][1][lane] = add4(e1, mj1);
                L.C[0][lane] = add4(c0, mb0);
                L.C[1][lane] = add4(c1, mb1);
                // the A8 interval update (the wave kernel's Encoder::code, per lane)
                const double rng = (double)(high - low) + 1.0, tot = (double)tot_i;
                const double qh = floordiv(rng * (double)hi_cur, tot, inv);
                const double ql = floordiv(rng * (double)lo_cur, tot, inv);
                high = low + (uint32_t)(qh - 1.0);
                low = low + (uint32_t)ql;
                const uint32_t d = __builtin_clz(low ^ high);
                if (d) {
                    const uint32_t bit = low >> 31;
                    w.bits(low, 1);
                    w.run(bit ^ 1u, pending);
                    pending = 0;
                    if (d > 1) w.bits(low << 1, d - 1);
                    low <<= d;
                    high = (high << d) | ((1u << d) - 1u);
                }
                const uint32_t x = (low << 1) & ~(high << 1);
                const uint32_t p = __builtin_clz(~x);
                if (p) {
                    pending += p;
                    low = (low << p) & 0x7FFFFFFFu;
                    high = (high << p) | ((1u << p) - 1u) | 0x80000000u;
                }
                total = tot_i + 1;
                lo_n += s_n > s ? 1u : 0u;
                hi_n += s_n >= s ? 1u : 0u;
                inv = inv_n;
                if (resc) {   // rare: every frequency halved, read the next range again
                    total = lane_model_rescale(L, lane, total);
                    inv = rcp_nr((double)total);
                    if (more) query(s_n, total, lo_n, hi_n);
                }
                s_cur = s_n;
                lo_cur = lo_n;
                hi_cur = hi_n;
            }
        }
        cur = nxt;
    }
    if (act) {
        const uint32_t bit = low < kQ1 ? 0u : 1u;   // flush (CBAAC.py:130 -> A8)
        w.bits(bit << 31, 1);
        w.run(bit ^ 1u, pending + 1);
        if (w.nb) w.out[w.words] = __builtin_bswap32((uint32_t)(w.acc >> 32));
        seg_bits[seg] = (int64_t)w.words * 32 + w.nb;
    }
}

// floor(a / t) for integers a < 2^47, 1 <= t <= 2^32 held exactly in doubles,
// inv ~= 1/t: the quotient estimate is within one of the floor, the remainder
// (an exact fma) says which way
__device__ __forceinline__ double floordiv_big(double a, double t, double inv)
{
    double q = __builtin_trunc(a * inv);
    const double r = __builtin_fma(-q, t, a);
    q = r < 0.0 ? q - 1.0 : (r >= t ? q + 1.0 : q);
    return q;
}

// the 16 u16 entries of (a, b): how many are <= v (entries start at 0 and
// increase strictly), the last of those and the first above v (`none` if none)
__device__ __forceinline__ void scan16(const uint4 &a, const uint4 &b, uint32_t v, uint32_t none, uint32_t &cnt,
                                       uint32_t &le, uint32_t &gt)
{
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    cnt = 0;
    le = 0;
    gt = none;
#pragma unroll
    for (int t = 15; t >= 0; --t) {
        const uint32_t x = (t & 1) ? w[t >> 1] >> 16 : w[t >> 1] & 0xFFFFu;
        const bool in = x <= v;
        cnt += in ? 1u : 0u;
        gt = in ? gt : x;
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const uint32_t x = (t & 1) ? w[t >> 1] >> 16 : w[t >> 1] & 0xFFFFu;
        le = x <= v ? x : le;
    }
}

// per-lane MSB-first bit reader over a segment's bytes, zeros past its end (A8)
struct LaneReader {
    const uint8_t *p;
    int64_t nbytes, pos = 0;
    uint64_t buf = 0;
    uint32_t avail = 0;
    __device__ __forceinline__ void refill()
    {
        while (avail <= 56) {
            const uint32_t byte = pos < nbytes ? p[pos] : 0u;
            buf |= (uint64_t)byte << (56 - avail);
            ++pos;
            avail += 8;
        }
    }
    __device__ __forceinline__ uint32_t get(uint32_t k)   // 1 <= k <= 32, right-aligned
    {
        if (avail < k) refill();
        const uint32_t v = (uint32_t)(buf >> (64 - k));
        buf <<= k;
        avail -= k;
        return v;
    }
};

template <bool PRIOR>
__global__ __launch_bounds__(kLW) void cbaac_lane_decode_kernel(const uint8_t *__restrict__ in,
                                                                const int64_t *__restrict__ offs, int64_t n,
                                                                int64_t seg_len, int64_t nseg,
                                                                uint8_t *__restrict__ out,
                                                                const uint16_t *__restrict__ prior, Frames fr)
{
    __shared__ LaneLds L;
    {
        const int64_t f = blockIdx.y;
        offs += f * (nseg + 1);
        out += f * fr.out_stride;
        if (prior) prior += f * fr.prior_stride;
    }
    const uint32_t lane = threadIdx.x;
    const int64_t seg = (int64_t)blockIdx.x * kLW + lane;
    const bool act = seg < nseg;
    const int64_t start = act ? seg * seg_len : 0;
    const int64_t len = act ? (n - start < seg_len ? n - start : seg_len) : 0;
    uint32_t total;
    lane_model_init(L, PRIOR ? class_prior(prior, act ? seg : 0, nseg, fr.nclass) : nullptr, lane, total);
    double tinv = 1.0 / (double)total;   // (unused until the first symbol; recomputed per symbol)
    (void)tinv;
    LaneReader br;
    br.p = in + (act ? offs[seg] : 0);
    br.nbytes = act ? offs[seg + 1] - offs[seg] : 0;
    uint32_t low = 0, high = 0xFFFFFFFFu, value = br.get(32);
    uint8_t *dst = out + start;
    const bool aligned = (reinterpret_cast<uintptr_t>(dst) & 15) == 0;
    uint4 c0 = L.C[0][lane], c1 = L.C[1][lane];
    const int64_t seg0 = (int64_t)blockIdx.x * kLW;
    const int64_t wave_len = n - seg0 * seg_len < seg_len ? n - seg0 * seg_len : seg_len;
    for (int64_t off = 0; off < wave_len; off += 16) {
        uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (off + k < len) {
                const double rng = (double)(high - low) + 1.0, tot = (double)total;
                const uint32_t T = value - low;
                const double scaled = floordiv_big(((double)T + 1.0) * tot - 1.0, rng, rcp_nr(rng));
                const uint32_t sv = (uint32_t)scaled;
                uint32_t nb, cb, cb1;
                scan16(c0, c1, sv, total, nb, cb, cb1);   // C lives in registers: no LDS round trip
                const uint32_t b = nb - 1;
                const uint4 e0 = L.E[b][0][lane], e1 = L.E[b][1][lane];
                const uint4 mb0 = L.M[b][0], mb1 = L.M[b][1];
                uint32_t nj, elo, ehi;
                scan16(e0, e1, sv - cb, cb1 - cb, nj, elo, ehi);
                const uint32_t j = nj - 1;
                const uint32_t lo = cb + elo, hi = cb + ehi;
                const uint4 mj0 = L.M[j][0], mj1 = L.M[j][1];
                const double inv = rcp_nr(tot);
                const double qh = floordiv(rng * (double)hi, tot, inv);
                const double ql = floordiv(rng * (double)lo, tot, inv);
                high = low + (uint32_t)(qh - 1.0);
                low = low + (uint32_t)ql;
                const uint32_t d = __builtin_clz(low ^ high);
                if (d) {
                    low <<= d;
                    high = (high << d) | ((1u << d) - 1u);
                    value = (value << d) | br.get(d);
                }
                const uint32_t x = (low << 1) & ~(high << 1);
                const uint32_t p = __builtin_clz(~x);
                if (p) {
                    low = (low << p) & 0x7FFFFFFFu;
                    high = (high << p) | ((1u << p) - 1u) | 0x80000000u;
                    value = ((value << p) ^ 0x80000000u) | br.get(p);
                }
                L.E[b][0][lane] = add4(e0, mj0);
                L.E[b][1][lane] = add4(e1, mj1);
                c0 = add4(c0, mb0);
                c1 = add4(c1, mb1);
                const uint32_t stale = total++;
                if (stale >= kMaxFreq) {   // rare: the rebuild reads and writes C through LDS
                    L.C[0][lane] = c0;
                    L.C[1][lane] = c1;
                    total = lane_model_rescale(L, lane, total);
                    c0 = L.C[0][lane];
                    c1 = L.C[1][lane];
                }
                o[k >> 2] |= (16 * b + j) << (8 * (k & 3));
            }
        }
        if (off < len) {
            if (aligned && off + 16 <= len) {
                *reinterpret_cast<uint4 *>(dst + off) = make_uint4(o[0], o[1], o[2], o[3]);
            } else {
                for (int k = 0; k < 16; ++k)
                    if (off + k < len) dst[off + k] = (uint8_t)(o[k >> 2] >> (8 * (k & 3)));
            }
        }
    }
}

int64_t slot_words_for(int64_t seg_len) { return (vcf_cbaac_bound(seg_len) + 3) / 4; }

// 0 = automatic (order 0: one lane per segment from kLaneMinEncode /
// kLaneMinDecode segments on), 1 = one wave per segment, 2 = one lane per
// segment (order 0; A/B)
int g_tiled_variant = 0;
// Crossovers measured on MI355X at 32768-symbol segments (scripts/
// bench_tcbaac_lane.py, profiles/r03_tcbaac_lane.jsonl): a wave per segment
// fills the 1024 SIMDs from ~1000 segments on and then grows linearly (encode
// 16.3 ms at 3038 segments, 39.0 at 12150; decode 21.9 / 63.0), a lane per
// segment stays at one segment's latency until 64k segments (encode ~20 ms,
// decode ~35 ms)
constexpr int64_t kLaneMinEncode = 4608, kLaneMinDecode = 6144;

int check_args(int64_t n, int32_t order, int64_t seg_len)
{
    if (n < 0) return set_error(VCF_ERR_INVALID, "negative symbol count");
    if (seg_len <= 0 || seg_len % kChunk) return set_error(VCF_ERR_INVALID, "seg_len must be a positive multiple of %d", kChunk);
    if (order < 0) return set_error(VCF_ERR_INVALID, "negative order");
    if (order > 1) return set_error(VCF_ERR_UNSUPPORTED, "tiled CBAAC on the GPU: orders 0 and 1 (got %d)", order);
    return VCF_OK;
}

}  // namespace
}  // namespace vcf

using namespace vcf;

extern "C" {

int vcf_cbaac_tiled_set_variant(int32_t variant)
{
    if (variant < 0 || variant > 2) return set_error(VCF_ERR_INVALID, "tiled CBAAC variant %d (0, 1, 2)", variant);
    g_tiled_variant = variant;
    return VCF_OK;
}

int64_t vcf_cbaac_tiled_segments(int64_t n, int64_t seg_len)
{
    if (n <= 0 || seg_len <= 0) return 0;
    return (n + seg_len - 1) / seg_len;
}

int64_t vcf_cbaac_tiled_workspace(int64_t n, int64_t seg_len)
{
    const int64_t ns = vcf_cbaac_tiled_segments(n, seg_len);
    if (ns == 0) return 0;
    // slots, per-segment bit counts, byte offsets (ns + 1)
    return ns * slot_words_for(seg_len) * 4 + ns * 8 + (ns + 1) * 8;
}

int64_t vcf_cbaac_tiled_bound(int64_t n, int64_t seg_len)
{
    return vcf_cbaac_tiled_segments(n, seg_len) * slot_words_for(seg_len > 0 ? seg_len : 1) * 4;
}

int64_t vcf_cbaac_tiled_frames_workspace(int64_t n_frames, int64_t frame_symbols, int64_t seg_len)
{
    return n_frames <= 0 ? 0 : n_frames * vcf_cbaac_tiled_workspace(frame_symbols, seg_len);
}

// one lane per segment when there are enough segments to fill waves with them
// (a lane codes a symbol in about twice a wave's time, but 64 segments at once)
static bool use_lanes(int32_t order, int64_t total_segments, bool decode)
{
    if (order != 0 || g_tiled_variant == 1) return false;
    return g_tiled_variant == 2 || total_segments >= (decode ? kLaneMinDecode : kLaneMinEncode);
}

static int tiled_encode(const uint8_t *sym_dev, int64_t n_frames, int64_t n, int64_t sym_stride, int32_t order,
                        int64_t seg_len, uint8_t *out_dev, int64_t out_capacity, int64_t *seg_bytes_dev,
                        int32_t *trace_dev, void *ws_dev, void *stream, const uint16_t *prior_dev = nullptr,
                        int64_t prior_stride = 0, int32_t nclass = 1)
{
    if (int s = check_args(n, order, seg_len)) return s;
    if (n_frames < 1 || n_frames > 65535) return set_error(VCF_ERR_INVALID, "n_frames %lld (1 .. 65535)", (long long)n_frames);
    const int64_t ns = vcf_cbaac_tiled_segments(n, seg_len);
    if (!seg_bytes_dev) return set_error(VCF_ERR_INVALID, "null seg_bytes");
    hipStream_t st = (hipStream_t)stream;
    if (ns == 0) return hip_check(hipMemsetAsync(seg_bytes_dev, 0, 8 * n_frames, st), "hipMemsetAsync");
    if (!sym_dev || !ws_dev || (!trace_dev && !out_dev)) return set_error(VCF_ERR_INVALID, "null buffer");
    if (ns > 0x7FFFFFFF) return set_error(VCF_ERR_INVALID, "too many segments");
    const int64_t sw = slot_words_for(seg_len);
    uint32_t *slots = (uint32_t *)ws_dev;
    int64_t *bits = (int64_t *)(slots + n_frames * ns * sw);
    int64_t *offs = bits + n_frames * ns;
    Frames fr;
    fr.sym_stride = sym_stride;
    fr.prior_stride = prior_stride;
    fr.nclass = nclass;
    const dim3 grid((unsigned)ns, (unsigned)n_frames);
    if (!trace_dev && use_lanes(order, ns * n_frames, false)) {   // one lane per segment
        const dim3 lg((unsigned)((ns + kLW - 1) / kLW), (unsigned)n_frames);
        if (prior_dev) cbaac_lane_encode_kernel<true><<<lg, kLW, 0, st>>>(sym_dev, n, seg_len, ns, slots, sw, bits, prior_dev, fr);
        else cbaac_lane_encode_kernel<false><<<lg, kLW, 0, st>>>(sym_dev, n, seg_len, ns, slots, sw, bits, nullptr, fr);
    } else if (trace_dev) {
        if (n_frames != 1) return set_error(VCF_ERR_INVALID, "traces take one frame");
        if (order == 0) cbaac_tiled_encode_kernel<0, true><<<grid, 64, 0, st>>>(sym_dev, n, seg_len, slots, sw, bits, trace_dev, prior_dev, fr);
        else cbaac_tiled_encode_kernel<1, true><<<grid, 64, 0, st>>>(sym_dev, n, seg_len, slots, sw, bits, trace_dev, prior_dev, fr);
    } else {
        if (order == 0) cbaac_tiled_encode_kernel<0, false><<<grid, 64, 0, st>>>(sym_dev, n, seg_len, slots, sw, bits, nullptr, prior_dev, fr);
        else cbaac_tiled_encode_kernel<1, false><<<grid, 64, 0, st>>>(sym_dev, n, seg_len, slots, sw, bits, nullptr, prior_dev, fr);
    }
    if (int s = hip_check(hipGetLastError(), "cbaac_tiled_encode_kernel")) return s;
    cbaac_tiled_scan_kernel<<<(unsigned)n_frames, 1024, 0, st>>>(bits, ns, offs, seg_bytes_dev);
    if (int s = hip_check(hipGetLastError(), "cbaac_tiled_scan_kernel")) return s;
    if (out_dev) {
        cbaac_tiled_pack_kernel<<<grid, 256, 0, st>>>(slots, sw, offs, out_dev, out_capacity);
        if (int s = hip_check(hipGetLastError(), "cbaac_tiled_pack_kernel")) return s;
    }
    return VCF_OK;
}

int vcf_cbaac_tiled_encode(const uint8_t *sym_dev, int64_t n, int32_t order, int64_t seg_len, uint8_t *out_dev,
                           int64_t out_capacity, int64_t *seg_bytes_dev, void *ws_dev, void *stream)
{
    if (out_capacity < 0) return set_error(VCF_ERR_INVALID, "negative capacity");
    if (n > 0 && !out_dev) return set_error(VCF_ERR_INVALID, "null output buffer");
    return tiled_encode(sym_dev, 1, n, 0, order, seg_len, out_dev, out_capacity, seg_bytes_dev, nullptr, ws_dev,
                        stream);
}

int vcf_cbaac_tiled_trace(const uint8_t *sym_dev, int64_t n, int32_t order, int64_t seg_len, int32_t *triples_dev,
                          int64_t *seg_bytes_dev, void *ws_dev, void *stream)
{
    if (n > 0 && !triples_dev) return set_error(VCF_ERR_INVALID, "null trace buffer");
    return tiled_encode(sym_dev, 1, n, 0, order, seg_len, nullptr, 0, seg_bytes_dev, triples_dev, ws_dev, stream);
}

static int tiled_decode(const uint8_t *in_dev, const int64_t *seg_offsets_dev, int64_t n_frames, int64_t n,
                        int32_t order, int64_t seg_len, uint8_t *sym_dev, int64_t out_stride, void *stream,
                        const uint16_t *prior_dev, int64_t prior_stride, int32_t nclass = 1)
{
    if (int s = check_args(n, order, seg_len)) return s;
    if (n_frames < 1 || n_frames > 65535) return set_error(VCF_ERR_INVALID, "n_frames %lld (1 .. 65535)", (long long)n_frames);
    const int64_t ns = vcf_cbaac_tiled_segments(n, seg_len);
    if (ns == 0) return VCF_OK;
    if (!in_dev || !seg_offsets_dev || !sym_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    if (ns > 0x7FFFFFFF) return set_error(VCF_ERR_INVALID, "too many segments");
    hipStream_t st = (hipStream_t)stream;
    Frames fr;
    fr.out_stride = out_stride;
    fr.prior_stride = prior_stride;
    fr.nclass = nclass;
    const dim3 grid((unsigned)ns, (unsigned)n_frames);
    if (use_lanes(order, ns * n_frames, true)) {   // one lane per segment
        const dim3 lg((unsigned)((ns + kLW - 1) / kLW), (unsigned)n_frames);
        if (prior_dev)
            cbaac_lane_decode_kernel<true><<<lg, kLW, 0, st>>>(in_dev, seg_offsets_dev, n, seg_len, ns, sym_dev, prior_dev, fr);
        else
            cbaac_lane_decode_kernel<false><<<lg, kLW, 0, st>>>(in_dev, seg_offsets_dev, n, seg_len, ns, sym_dev, nullptr, fr);
        return hip_check(hipGetLastError(), "cbaac_lane_decode_kernel");
    }
    if (order == 0) cbaac_tiled_decode_kernel<0><<<grid, 64, 0, st>>>(in_dev, seg_offsets_dev, n, seg_len, sym_dev, prior_dev, fr);
    else cbaac_tiled_decode_kernel<1><<<grid, 64, 0, st>>>(in_dev, seg_offsets_dev, n, seg_len, sym_dev, prior_dev, fr);
    return hip_check(hipGetLastError(), "cbaac_tiled_decode_kernel");
}

int vcf_cbaac_tiled_decode(const uint8_t *in_dev, const int64_t *seg_offsets_dev, int64_t n, int32_t order,
                           int64_t seg_len, uint8_t *sym_dev, void *stream)
{
    return tiled_decode(in_dev, seg_offsets_dev, 1, n, order, seg_len, sym_dev, 0, stream, nullptr, 0);
}

static int tiled_prior(const uint8_t *sym_dev, int64_t n_frames, int64_t n, int64_t sym_stride, uint16_t *prior_dev,
                       uint32_t *hist_dev, void *stream)
{
    if (n < 0) return set_error(VCF_ERR_INVALID, "negative symbol count");
    if (n_frames < 1 || n_frames > 65535) return set_error(VCF_ERR_INVALID, "n_frames %lld (1 .. 65535)", (long long)n_frames);
    if (!prior_dev || !hist_dev || (n > 0 && !sym_dev)) return set_error(VCF_ERR_INVALID, "null buffer");
    if (reinterpret_cast<uintptr_t>(prior_dev) & 7) return set_error(VCF_ERR_INVALID, "prior_dev not 8-byte aligned");
    hipStream_t st = (hipStream_t)stream;
    if (int s = hip_check(hipMemsetAsync(hist_dev, 0, 256 * sizeof(uint32_t) * n_frames, st), "hipMemsetAsync"))
        return s;
    if (n > 0) {
        const int64_t blocks = std::min<int64_t>((n + 4095) / 4096, 2048);
        cbaac_hist_kernel<<<dim3((unsigned)blocks, (unsigned)n_frames), 256, 0, st>>>(sym_dev, n, hist_dev, sym_stride);
        if (int s = hip_check(hipGetLastError(), "cbaac_hist_kernel")) return s;
    }
    cbaac_prior_kernel<<<(unsigned)n_frames, 256, 0, st>>>(hist_dev, n, prior_dev);
    return hip_check(hipGetLastError(), "cbaac_prior_kernel");
}

int vcf_cbaac_tiled_prior(const uint8_t *sym_dev, int64_t n, uint16_t *prior_dev, uint32_t *hist_dev, void *stream)
{
    return tiled_prior(sym_dev, 1, n, 0, prior_dev, hist_dev, stream);
}

int vcf_cbaac_tiled_encode_prior(const uint8_t *sym_dev, int64_t n, int32_t order, const uint16_t *prior_dev,
                                 int64_t seg_len, uint8_t *out_dev, int64_t out_capacity, int64_t *seg_bytes_dev,
                                 void *ws_dev, void *stream)
{
    if (out_capacity < 0) return set_error(VCF_ERR_INVALID, "negative capacity");
    if (n > 0 && (!out_dev || !prior_dev)) return set_error(VCF_ERR_INVALID, "null buffer");
    if (reinterpret_cast<uintptr_t>(prior_dev) & 7) return set_error(VCF_ERR_INVALID, "prior_dev not 8-byte aligned");
    return tiled_encode(sym_dev, 1, n, 0, order, seg_len, out_dev, out_capacity, seg_bytes_dev, nullptr, ws_dev, stream,
                        prior_dev);
}

int vcf_cbaac_tiled_decode_prior(const uint8_t *in_dev, const int64_t *seg_offsets_dev, int64_t n, int32_t order,
                                 const uint16_t *prior_dev, int64_t seg_len, uint8_t *sym_dev, void *stream)
{
    if (n > 0 && !prior_dev) return set_error(VCF_ERR_INVALID, "null prior");
    if (reinterpret_cast<uintptr_t>(prior_dev) & 7) return set_error(VCF_ERR_INVALID, "prior_dev not 8-byte aligned");
    return tiled_decode(in_dev, seg_offsets_dev, 1, n, order, seg_len, sym_dev, 0, stream, prior_dev, 0);
}

// ---- batches of frames: one launch per stage for all of them -------------------------
int vcf_cbaac_tiled_prior_frames(const uint8_t *sym_dev, int64_t n_frames, int64_t frame_symbols,
                                 int64_t frame_stride, uint16_t *priors_dev, uint32_t *hist_dev, void *stream)
{
    return tiled_prior(sym_dev, n_frames, frame_symbols, frame_stride, priors_dev, hist_dev, stream);
}

int vcf_cbaac_tiled_encode_frames(const uint8_t *sym_dev, int64_t n_frames, int64_t frame_symbols,
                                  int64_t frame_stride, int32_t order, const uint16_t *priors_dev, int64_t seg_len,
                                  uint8_t *out_dev, int64_t out_frame_capacity, int64_t *seg_bytes_dev, void *ws_dev,
                                  void *stream)
{
    if (out_frame_capacity < 0) return set_error(VCF_ERR_INVALID, "negative capacity");
    if (frame_symbols > 0 && !out_dev) return set_error(VCF_ERR_INVALID, "null output buffer");
    if (priors_dev && (reinterpret_cast<uintptr_t>(priors_dev) & 7))
        return set_error(VCF_ERR_INVALID, "priors_dev not 8-byte aligned");
    return tiled_encode(sym_dev, n_frames, frame_symbols, frame_stride, order, seg_len, out_dev, out_frame_capacity,
                        seg_bytes_dev, nullptr, ws_dev, stream, priors_dev, priors_dev ? 256 : 0);
}

int vcf_cbaac_tiled_decode_frames(const uint8_t *in_dev, const int64_t *seg_offsets_dev, int64_t n_frames,
                                  int64_t frame_symbols, int32_t order, const uint16_t *priors_dev, int64_t seg_len,
                                  uint8_t *sym_dev, int64_t out_frame_stride, void *stream)
{
    if (priors_dev && (reinterpret_cast<uintptr_t>(priors_dev) & 7))
        return set_error(VCF_ERR_INVALID, "priors_dev not 8-byte aligned");
    return tiled_decode(in_dev, seg_offsets_dev, n_frames, frame_symbols, order, seg_len, sym_dev, out_frame_stride,
                        stream, priors_dev, priors_dev ? 256 : 0);
}

// ---- version 3: prior classes (consecutive runs of segments share a prior row) ----
static int check_classes(int32_t nclass, const void *priors_dev)
{
    if (nclass < 1 || nclass > kMaxClasses) return set_error(VCF_ERR_INVALID, "nclass %d (1 .. %d)", nclass, kMaxClasses);
    if (priors_dev && (reinterpret_cast<uintptr_t>(priors_dev) & 7))
        return set_error(VCF_ERR_INVALID, "priors_dev not 8-byte aligned");
    return VCF_OK;
}

int vcf_cbaac_tiled_prior_classes(const uint8_t *sym_dev, int64_t n_frames, int64_t frame_symbols,
                                  int64_t frame_stride, int64_t seg_len, int32_t nclass, uint16_t *priors_dev,
                                  uint32_t *hist_dev, void *stream)
{
    if (int s = check_args(frame_symbols, 0, seg_len)) return s;
    if (int s = check_classes(nclass, priors_dev)) return s;
    if (n_frames < 1 || n_frames > 65535) return set_error(VCF_ERR_INVALID, "n_frames %lld (1 .. 65535)", (long long)n_frames);
    if (!priors_dev || !hist_dev || (frame_symbols > 0 && !sym_dev)) return set_error(VCF_ERR_INVALID, "null buffer");
    hipStream_t st = (hipStream_t)stream;
    const int64_t rows = n_frames * nclass;
    if (int s = hip_check(hipMemsetAsync(hist_dev, 0, 256 * sizeof(uint32_t) * rows, st), "hipMemsetAsync")) return s;
    const int64_t ns = vcf_cbaac_tiled_segments(frame_symbols, seg_len);
    if (ns > 0x7FFFFFFF) return set_error(VCF_ERR_INVALID, "too many segments");
    if (ns > 0) {
        cbaac_hist_classes_kernel<<<dim3((unsigned)ns, (unsigned)n_frames), 256, 0, st>>>(sym_dev, frame_symbols, seg_len,
                                                                                          nclass, hist_dev, frame_stride);
        if (int s = hip_check(hipGetLastError(), "cbaac_hist_classes_kernel")) return s;
    }
    cbaac_prior_classes_kernel<<<(unsigned)rows, 256, 0, st>>>(hist_dev, priors_dev);
    return hip_check(hipGetLastError(), "cbaac_prior_classes_kernel");
}

int vcf_cbaac_tiled_encode_classes(const uint8_t *sym_dev, int64_t n_frames, int64_t frame_symbols,
                                   int64_t frame_stride, int32_t order, const uint16_t *priors_dev, int32_t nclass,
                                   int64_t seg_len, uint8_t *out_dev, int64_t out_frame_capacity,
                                   int64_t *seg_bytes_dev, void *ws_dev, void *stream)
{
    if (int s = check_classes(nclass, priors_dev)) return s;
    if (out_frame_capacity < 0) return set_error(VCF_ERR_INVALID, "negative capacity");
    if (frame_symbols > 0 && (!out_dev || !priors_dev)) return set_error(VCF_ERR_INVALID, "null buffer");
    return tiled_encode(sym_dev, n_frames, frame_symbols, frame_stride, order, seg_len, out_dev, out_frame_capacity,
                        seg_bytes_dev, nullptr, ws_dev, stream, priors_dev, 256LL * nclass, nclass);
}

int vcf_cbaac_tiled_decode_classes(const uint8_t *in_dev, const int64_t *seg_offsets_dev, int64_t n_frames,
                                   int64_t frame_symbols, int32_t order, const uint16_t *priors_dev, int32_t nclass,
                                   int64_t seg_len, uint8_t *sym_dev, int64_t out_frame_stride, void *stream)
{
    if (int s = check_classes(nclass, priors_dev)) return s;
    if (frame_symbols > 0 && !priors_dev) return set_error(VCF_ERR_INVALID, "null prior");
    return tiled_decode(in_dev, seg_offsets_dev, n_frames, frame_symbols, order, seg_len, sym_dev, out_frame_stride,
                        stream, priors_dev, 256LL * nclass, nclass);
}

}  // extern "C"
