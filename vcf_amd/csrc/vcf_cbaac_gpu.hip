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
//     get_symbol_from_scaled_value (:43-47) is one ballot of C[4l] <= v plus
//     four readlanes.
//   - Order 1: the 256 context models (one per previous symbol) as 16-bit
//     cumulative tables in LDS (128 KiB + totals), the current context's row
//     read into the same four VGPRs per lane and written back after the
//     update.
//   - The coder state (low, high, pending bits, the bit writer) is
//     wave-uniform; floor(range * c / total) is one float64 division plus an
//     exact correction (operands < 2^47).  Bits are packed MSB-first into
//     words that lane 0 stores (vector stores); symbols stream in 256 at a
//     time (one dword per lane, the next chunk prefetched).
// A second pass packs the segments back to back (a scan of their sizes and a
// copy), so only the compressed bytes need to leave HBM.
#include <hip/hip_runtime.h>

#include "vcf_amd.h"
#include "vcf_internal.h"

namespace vcf {
namespace {

constexpr uint32_t kMaxFreq = 16384;   // AdaptiveModel(max_freq=16384), CBAAC.py:18
constexpr uint32_t kHalf = 0x80000000u, kQ1 = 0x40000000u, kQ3 = 0xC0000000u;
constexpr int kChunk = 256;            // symbols (or bytes) per wave load: one dword per lane

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t lane)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

// floor(a / b) for a < 2^53, 0 < b < 2^33: the correctly rounded float64
// quotient is floor(a/b) or floor(a/b) + 1 (a and b are exact doubles and
// RN is monotonic), one multiply-compare picks the right one.
__device__ __forceinline__ uint64_t udiv(uint64_t a, uint64_t b)
{
    uint64_t q = (uint64_t)((double)a / (double)b);
    if (q * b > a) --q;
    return q;
}

// lane l holds C[4l + j], j = 0..3; total = C[256] (uniform)
struct Model {
    uint32_t c[4];
    uint32_t total;
};

__device__ __forceinline__ uint32_t pick(const Model &m, uint32_t j)
{
    return j == 0 ? m.c[0] : j == 1 ? m.c[1] : j == 2 ? m.c[2] : m.c[3];
}

__device__ __forceinline__ void model_reset(Model &m, uint32_t lane)
{
    for (int j = 0; j < 4; ++j) m.c[j] = 4 * lane + j;   // all frequencies 1
    m.total = 256;
}

// (cum[s], cum[s+1]) of get_range (CBAAC.py:40-41)
__device__ __forceinline__ void model_range(const Model &m, uint32_t s, uint32_t &lo, uint32_t &hi)
{
    lo = rl(pick(m, s & 3), s >> 2);
    hi = s == 255 ? m.total : rl(pick(m, (s + 1) & 3), (s + 1) >> 2);
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

// update(s) (CBAAC.py:32-36): freqs[s] += 1; if the total *before* the
// increment is >= max_freq, every frequency becomes (f >> 1) + 1.
__device__ __forceinline__ void model_update(Model &m, uint32_t s, uint32_t lane)
{
    const uint32_t stale = m.total;
    for (int j = 0; j < 4; ++j) m.c[j] += (4 * lane + j > s) ? 1u : 0u;
    m.total = stale + 1;
    if (stale >= kMaxFreq) {
        const uint32_t nxt0 = __shfl_down(m.c[0], 1, 64);
        const uint32_t end = lane == 63 ? m.total : nxt0;
        uint32_t f[4] = {m.c[1] - m.c[0], m.c[2] - m.c[1], m.c[3] - m.c[2], end - m.c[3]};
        uint32_t sum = 0;
        for (int j = 0; j < 4; ++j) {
            f[j] = (f[j] >> 1) + 1;
            sum += f[j];
        }
        const uint32_t ex = wave_excl_scan(sum, lane);
        m.c[0] = ex;
        m.c[1] = ex + f[0];
        m.c[2] = m.c[1] + f[1];
        m.c[3] = m.c[2] + f[2];
        m.total = rl(ex + sum, 63);
    }
}

// get_symbol_from_scaled_value (CBAAC.py:43-47): the s with C[s] <= v < C[s+1]
__device__ __forceinline__ uint32_t model_find(const Model &m, uint32_t v, uint32_t &lo, uint32_t &hi)
{
    const uint64_t mask = __ballot(m.c[0] <= v);   // a prefix of the lanes (C is increasing)
    const uint32_t L = (uint32_t)__popcll(mask) - 1;
    const uint32_t a0 = rl(m.c[0], L), a1 = rl(m.c[1], L), a2 = rl(m.c[2], L), a3 = rl(m.c[3], L);
    const uint32_t a4 = L == 63 ? m.total : rl(m.c[0], L + 1);
    if (v < a1) { lo = a0; hi = a1; return 4 * L; }
    if (v < a2) { lo = a1; hi = a2; return 4 * L + 1; }
    if (v < a3) { lo = a2; hi = a3; return 4 * L + 2; }
    lo = a3;
    hi = a4;
    return 4 * L + 3;
}

// order-1 context tables: 256 models x 256 cumulative counts (u16: every
// count <= 16385) + 256 totals, in LDS
struct Tables {
    uint16_t c[256 * 256];
    uint16_t total[256];
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
    for (uint32_t r = 0; r < 256; ++r) {
        uint2 v;
        v.x = (4 * lane) | ((4 * lane + 1) << 16);
        v.y = (4 * lane + 2) | ((4 * lane + 3) << 16);
        *reinterpret_cast<uint2 *>(&t.c[r * 256 + 4 * lane]) = v;
    }
    for (uint32_t r = lane; r < 256; r += 64) t.total[r] = 256;
    __syncthreads();
}

__device__ __forceinline__ void tables_read(const Tables &t, uint32_t ctx, uint32_t lane, Model &m)
{
    const uint2 v = *reinterpret_cast<const uint2 *>(&t.c[ctx * 256 + 4 * lane]);
    m.c[0] = v.x & 0xFFFFu;
    m.c[1] = v.x >> 16;
    m.c[2] = v.y & 0xFFFFu;
    m.c[3] = v.y >> 16;
    m.total = (uint32_t)__builtin_amdgcn_readfirstlane((int)t.total[ctx]);
}

__device__ __forceinline__ void tables_write(Tables &t, uint32_t ctx, uint32_t lane, const Model &m)
{
    uint2 v;
    v.x = m.c[0] | (m.c[1] << 16);
    v.y = m.c[2] | (m.c[3] << 16);
    *reinterpret_cast<uint2 *>(&t.c[ctx * 256 + 4 * lane]) = v;
    if (lane == 0) t.total[ctx] = (uint16_t)m.total;
}

// MSB-first bit writer (bitarray endian='big'); lane 0 stores whole words
struct BitWriter {
    uint32_t *out;
    uint32_t acc = 0, nb = 0;
    uint64_t words = 0;

    __device__ __forceinline__ void flush_word(uint32_t lane)
    {
        if (lane == 0) out[words] = __builtin_bswap32(acc);
        ++words;
        acc = 0;
        nb = 0;
    }
    __device__ __forceinline__ void put(uint32_t bit, uint32_t lane)
    {
        acc |= bit << (31 - nb);
        if (++nb == 32) flush_word(lane);
    }
    __device__ __forceinline__ void run(uint32_t bit, uint64_t count, uint32_t lane)
    {
        while (count) {
            const uint32_t room = 32 - nb;
            const uint32_t take = count < room ? (uint32_t)count : room;
            if (bit) acc |= (take == 32 ? 0xFFFFFFFFu : ((1u << take) - 1u)) << (room - take);
            nb += take;
            count -= take;
            if (nb == 32) flush_word(lane);
        }
    }
    __device__ __forceinline__ uint64_t finish(uint32_t lane)
    {
        const uint64_t bits = words * 32 + nb;
        if (nb && lane == 0) out[words] = __builtin_bswap32(acc);
        return bits;
    }
};

__device__ __forceinline__ uint32_t load_sym4(const uint8_t *p, int64_t off, int64_t len, uint32_t lane)
{
    const int64_t i = off + 4 * (int64_t)lane;
    if (i + 3 < len) return *reinterpret_cast<const uint32_t *>(p + i);   // segment starts are 256-aligned
    uint32_t v = 0;
    for (int j = 0; j < 4; ++j)
        if (i + j < len) v |= (uint32_t)p[i + j] << (8 * j);
    return v;
}

template <int ORDER, bool TRACE>
__global__ __launch_bounds__(64) void cbaac_tiled_encode_kernel(const uint8_t *__restrict__ sym, int64_t n,
                                                                int64_t seg_len, uint32_t *__restrict__ slots,
                                                                int64_t slot_words, int64_t *__restrict__ seg_bits,
                                                                int32_t *__restrict__ trace)
{
    Tables *tabs = Lds<ORDER>::get();
    const int64_t seg = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    const int64_t start = seg * seg_len;
    const int64_t len = n - start < seg_len ? n - start : seg_len;
    const uint8_t *src = sym + start;

    Model m;
    model_reset(m, lane);
    if constexpr (ORDER == 1) tables_reset(tabs[0], lane);
    uint32_t ctx = 0;

    BitWriter w;
    w.out = slots + seg * slot_words;
    uint32_t low = 0, high = 0xFFFFFFFFu;
    uint64_t pending = 0;

    uint32_t cur = load_sym4(src, 0, len, lane);
    for (int64_t off = 0; off < len; off += kChunk) {
        const uint32_t nxt = off + kChunk < len ? load_sym4(src, off + kChunk, len, lane) : 0u;
        const int cnt = len - off < kChunk ? (int)(len - off) : kChunk;
        for (int k = 0; k < cnt; ++k) {
            const uint32_t s = (rl(cur, k >> 2) >> (8 * (k & 3))) & 255u;
            if constexpr (ORDER == 1) tables_read(tabs[0], ctx, lane, m);
            uint32_t lo, hi;
            model_range(m, s, lo, hi);
            const uint32_t tot = m.total;
            if constexpr (TRACE) {
                if (lane == 0) {
                    int32_t *t = trace + 3 * (start + off + k);
                    t[0] = (int32_t)lo;
                    t[1] = (int32_t)hi;
                    t[2] = (int32_t)tot;
                }
            }
            // A8 interval update (vcf_cbaac.cpp, encode)
            const uint64_t range = (uint64_t)(high - low) + 1;
            high = low + (uint32_t)(udiv(range * hi, tot) - 1);
            low = low + (uint32_t)udiv(range * lo, tot);
            for (;;) {
                if (high < kHalf) {
                    w.put(0, lane);
                    w.run(1, pending, lane);
                    pending = 0;
                } else if (low >= kHalf) {
                    w.put(1, lane);
                    w.run(0, pending, lane);
                    pending = 0;
                    low -= kHalf;
                    high -= kHalf;
                } else if (low >= kQ1 && high < kQ3) {
                    ++pending;
                    low -= kQ1;
                    high -= kQ1;
                } else {
                    break;
                }
                low <<= 1;
                high = (high << 1) | 1u;
            }
            model_update(m, s, lane);
            if constexpr (ORDER == 1) {
                tables_write(tabs[0], ctx, lane, m);
                ctx = s;
            }
        }
        cur = nxt;
    }
    // flush (CBAAC.py:130 -> A8): one more pending bit and a disambiguating bit
    ++pending;
    const uint32_t b = low < kQ1 ? 0u : 1u;
    w.put(b, lane);
    w.run(b ^ 1u, pending, lane);
    const uint64_t bits = w.finish(lane);
    if (lane == 0) seg_bits[seg] = (int64_t)bits;
}

// MSB-first bit reader over a segment's bytes, zeros past its end (A8)
struct BitReader {
    const uint8_t *src;
    int64_t nbytes;
    int64_t chunk = 0;         // byte offset of `cur`
    uint32_t cur = 0, nxt = 0; // 256 bytes each, one big-endian dword per lane
    uint32_t wi = 0, word = 0, used = 0;

    __device__ __forceinline__ uint32_t load(int64_t off, uint32_t lane) const
    {
        uint32_t v = 0;
        for (int j = 0; j < 4; ++j) {
            const int64_t i = off + 4 * (int64_t)lane + j;
            v = (v << 8) | (i < nbytes ? (uint32_t)src[i] : 0u);
        }
        return v;
    }
    __device__ __forceinline__ void start(uint32_t lane)
    {
        cur = load(0, lane);
        nxt = load(kChunk, lane);
        wi = 0;
        word = rl(cur, 0);
        used = 32;   // the first 32 bits go straight into `value`
    }
    __device__ __forceinline__ uint32_t get(uint32_t lane)
    {
        if (used == 32) {
            if (++wi == 64) {
                wi = 0;
                chunk += kChunk;
                cur = nxt;
                nxt = load(chunk + kChunk, lane);
            }
            word = rl(cur, wi);
            used = 0;
        }
        return (word >> (31 - used++)) & 1u;
    }
};

template <int ORDER>
__global__ __launch_bounds__(64) void cbaac_tiled_decode_kernel(const uint8_t *__restrict__ in,
                                                                const int64_t *__restrict__ offs, int64_t n,
                                                                int64_t seg_len, uint8_t *__restrict__ out)
{
    Tables *tabs = Lds<ORDER>::get();
    const int64_t seg = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    const int64_t start = seg * seg_len;
    const int64_t len = n - start < seg_len ? n - start : seg_len;
    uint8_t *dst = out + start;

    Model m;
    model_reset(m, lane);
    if constexpr (ORDER == 1) tables_reset(tabs[0], lane);
    uint32_t ctx = 0;

    BitReader br;
    br.src = in + offs[seg];
    br.nbytes = offs[seg + 1] - offs[seg];
    br.start(lane);
    uint32_t low = 0, high = 0xFFFFFFFFu, value = br.word;

    uint32_t obuf = 0, acc = 0;
    for (int64_t i = 0; i < len; ++i) {
        if constexpr (ORDER == 1) tables_read(tabs[0], ctx, lane, m);
        const uint64_t range = (uint64_t)(high - low) + 1;
        const uint32_t tot = m.total;
        const uint32_t v = (uint32_t)udiv(((uint64_t)(value - low) + 1) * tot - 1, range);
        uint32_t lo, hi;
        const uint32_t s = model_find(m, v, lo, hi);
        high = low + (uint32_t)(udiv(range * hi, tot) - 1);
        low = low + (uint32_t)udiv(range * lo, tot);
        for (;;) {
            if (high < kHalf) {
            } else if (low >= kHalf) {
                low -= kHalf;
                high -= kHalf;
                value -= kHalf;
            } else if (low >= kQ1 && high < kQ3) {
                low -= kQ1;
                high -= kQ1;
                value -= kQ1;
            } else {
                break;
            }
            low <<= 1;
            high = (high << 1) | 1u;
            value = (value << 1) | br.get(lane);
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
        if ((i & (kChunk - 1)) == kChunk - 1)   // a full chunk: one dword per lane
            *reinterpret_cast<uint32_t *>(dst + (i - (kChunk - 1)) + 4 * lane) = obuf;
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
    const int64_t seg = blockIdx.x;
    const uint8_t *src = reinterpret_cast<const uint8_t *>(slots + seg * slot_words);
    const int64_t o = offs[seg], nb = offs[seg + 1] - o;
    for (int64_t i = threadIdx.x; i < nb; i += 256)
        if (o + i < capacity) out[o + i] = src[i];
}

int64_t slot_words_for(int64_t seg_len) { return (vcf_cbaac_bound(seg_len) + 3) / 4; }

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

static int tiled_encode(const uint8_t *sym_dev, int64_t n, int32_t order, int64_t seg_len, uint8_t *out_dev,
                        int64_t out_capacity, int64_t *seg_bytes_dev, int32_t *trace_dev, void *ws_dev,
                        void *stream)
{
    if (int s = check_args(n, order, seg_len)) return s;
    const int64_t ns = vcf_cbaac_tiled_segments(n, seg_len);
    if (!seg_bytes_dev) return set_error(VCF_ERR_INVALID, "null seg_bytes");
    hipStream_t st = (hipStream_t)stream;
    if (ns == 0) return hip_check(hipMemsetAsync(seg_bytes_dev, 0, 8, st), "hipMemsetAsync");
    if (!sym_dev || !ws_dev || (!trace_dev && !out_dev)) return set_error(VCF_ERR_INVALID, "null buffer");
    if (ns > 0x7FFFFFFF) return set_error(VCF_ERR_INVALID, "too many segments");
    const int64_t sw = slot_words_for(seg_len);
    uint32_t *slots = (uint32_t *)ws_dev;
    int64_t *bits = (int64_t *)(slots + ns * sw);
    int64_t *offs = bits + ns;
    const dim3 grid((unsigned)ns);
    if (trace_dev) {
        if (order == 0) cbaac_tiled_encode_kernel<0, true><<<grid, 64, 0, st>>>(sym_dev, n, seg_len, slots, sw, bits, trace_dev);
        else cbaac_tiled_encode_kernel<1, true><<<grid, 64, 0, st>>>(sym_dev, n, seg_len, slots, sw, bits, trace_dev);
    } else {
        if (order == 0) cbaac_tiled_encode_kernel<0, false><<<grid, 64, 0, st>>>(sym_dev, n, seg_len, slots, sw, bits, nullptr);
        else cbaac_tiled_encode_kernel<1, false><<<grid, 64, 0, st>>>(sym_dev, n, seg_len, slots, sw, bits, nullptr);
    }
    if (int s = hip_check(hipGetLastError(), "cbaac_tiled_encode_kernel")) return s;
    cbaac_tiled_scan_kernel<<<1, 1024, 0, st>>>(bits, ns, offs, seg_bytes_dev);
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
    return tiled_encode(sym_dev, n, order, seg_len, out_dev, out_capacity, seg_bytes_dev, nullptr, ws_dev, stream);
}

int vcf_cbaac_tiled_trace(const uint8_t *sym_dev, int64_t n, int32_t order, int64_t seg_len, int32_t *triples_dev,
                          int64_t *seg_bytes_dev, void *ws_dev, void *stream)
{
    if (n > 0 && !triples_dev) return set_error(VCF_ERR_INVALID, "null trace buffer");
    return tiled_encode(sym_dev, n, order, seg_len, nullptr, 0, seg_bytes_dev, triples_dev, ws_dev, stream);
}

int vcf_cbaac_tiled_decode(const uint8_t *in_dev, const int64_t *seg_offsets_dev, int64_t n, int32_t order,
                           int64_t seg_len, uint8_t *sym_dev, void *stream)
{
    if (int s = check_args(n, order, seg_len)) return s;
    const int64_t ns = vcf_cbaac_tiled_segments(n, seg_len);
    if (ns == 0) return VCF_OK;
    if (!in_dev || !seg_offsets_dev || !sym_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    if (ns > 0x7FFFFFFF) return set_error(VCF_ERR_INVALID, "too many segments");
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)ns);
    if (order == 0) cbaac_tiled_decode_kernel<0><<<grid, 64, 0, st>>>(in_dev, seg_offsets_dev, n, seg_len, sym_dev);
    else cbaac_tiled_decode_kernel<1><<<grid, 64, 0, st>>>(in_dev, seg_offsets_dev, n, seg_len, sym_dev);
    return hip_check(hipGetLastError(), "cbaac_tiled_decode_kernel");
}

}  // extern "C"
