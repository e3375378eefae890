// vcf_cbaac.cpp -- context-based adaptive arithmetic coding (src/CBAAC.py),
// native host code, and the vcf_cbaac_* entry points of the C ABI.
//
// The model is the reference's, exactly (pinned against traces of its own
// classes, tests/golden/make_golden_cbaac.py):
//   AdaptiveModel (CBAAC.py:17-47): 256 frequencies initialised to 1;
//     update(s): freqs[s] += 1, and if the total *before* that increment is
//     >= 16384, every frequency becomes (f >> 1) + 1; get_range(s) =
//     (cum[s], cum[s+1], total).
//   ContextManager (:49-69): one model per distinct tuple of the previous
//     `order` symbols (history starts as `order` zeros), created on first use.
// The arithmetic coder (package arithmetic_coding, not vendored) is
// assumption A8 of SURVEY.md: a 32-bit Witten-Neal-Cleary integer coder
// with pending (underflow) bits, bits emitted MSB-first into bytes
// (bitarray endian='big', zero padded), flush = one more pending bit and a
// disambiguating bit.  The decoder reads zeros past the end.
//
// The coder is inherently serial (every symbol's interval depends on all
// previous ones), so this is host code; prefix sums are a Fenwick tree
// (log2 256 = 8 steps per symbol instead of the reference's 256-entry
// cumulative rebuild), rebuilt only when the model rescales.
//
// Per-symbol costs (round 6; the bytes are unchanged, pinned by
// tests/test_cbaac.py against the A8 stand-in coder and the fixtures):
//   * the interval's two divisions by the model total become a multiply by
//     an exact reciprocal (Divider, below: totals <= 16384 by the halving rule);
//   * renormalisation is done in bulk: the common leading bits of low and
//     high (the E1/E2 steps) by one count-leading-zeros, then the underflow
//     (E3) steps by another, instead of one loop trip per bit;
//   * bits go through a 64-bit accumulator, 32 at a time;
//   * the decoder first tests the model's most probable symbol with two
//     multiplications (lo * range <= num < hi * range is exactly
//     lo <= floor(num / range) < hi), and only otherwise divides by the
//     range and walks the Fenwick tree.
#include <cstdint>
#include <cstring>
#include <memory>
#include <new>
#include <unordered_map>
#include <vector>

#include "vcf_amd.h"
#include "vcf_internal.h"

namespace vcf {
namespace {

constexpr int kSymbols = 256;
constexpr uint32_t kMaxFreq = 16384;   // AdaptiveModel(max_freq=16384)

// The reference's AdaptiveModel with its cumulative counts in a Fenwick tree.
// DCT index streams are dominated by one symbol (98.6 % of a 1080p frame's), so
// the model keeps a most probable symbol `mps` aside: its cumulative count
// lo_mps is maintained directly, and its increments are held back (`pend`)
// instead of walking the tree, which then lacks them until they are needed --
// for another symbol's count above mps (added), the tree descent of find(), a
// change of mps or a rescale (flushed).  freq[] and total are always exact.
struct Model {
    uint32_t freq[kSymbols];
    uint32_t tree[kSymbols + 1];   // Fenwick tree over freq (1-based), less `pend` at mps
    uint32_t total;
    int mps = 0;                   // a most probable symbol (the decoder's first guess)
    uint32_t lo_mps = 0;           // cum(mps), exact
    uint32_t pend = 0;             // increments of mps not yet in the tree

    Model() { reset(); }
    void reset()
    {
        for (int i = 0; i < kSymbols; ++i) freq[i] = 1;
        rebuild();
    }
    void rebuild()
    {
        total = 0;
        mps = 0;
        pend = 0;
        for (int i = 1; i <= kSymbols; ++i) tree[i] = 0;
        for (int i = 0; i < kSymbols; ++i) {
            total += freq[i];
            if (freq[i] > freq[mps]) mps = i;
            for (int k = i + 1; k <= kSymbols; k += k & -k) tree[k] += freq[i];
        }
        lo_mps = tree_cum(mps);
    }
    void init(const uint16_t *prior)   // the tiled container's prior-initialised model (order 0)
    {
        for (int i = 0; i < kSymbols; ++i) freq[i] = prior[i];
        rebuild();
    }
    uint32_t tree_cum(int s) const
    {
        uint32_t r = 0;
        for (int k = s; k > 0; k -= k & -k) r += tree[k];
        return r;
    }
    void flush()   // the held-back increments of mps into the tree
    {
        if (!pend) return;
        for (int k = mps + 1; k <= kSymbols; k += k & -k) tree[k] += pend;
        pend = 0;
    }
    uint32_t cum(int s) const   // sum of freq[0..s)
    {
        if (s == mps) return lo_mps;
        return tree_cum(s) + (s > mps ? pend : 0u);
    }
    void update(int s)
    {
        const uint32_t stale = total;   // CBAAC.py:34: tests self.total before recomputing
        ++freq[s];
        if (stale >= kMaxFreq) {
            for (int i = 0; i < kSymbols; ++i) freq[i] = (freq[i] >> 1) + 1;
            rebuild();
            return;
        }
        ++total;
        if (s == mps) {
            ++pend;
            return;
        }
        for (int k = s + 1; k <= kSymbols; k += k & -k) ++tree[k];
        if (s < mps) ++lo_mps;
        if (freq[s] > freq[mps]) {
            flush();
            mps = s;
            lo_mps = tree_cum(s);
        }
    }
    // largest s with cum(s) <= v (v < total): CBAAC.py get_symbol_from_scaled_value
    int find(uint32_t v, uint32_t &lo)
    {
        flush();
        int pos = 0;
        uint32_t acc = 0;
        for (int step = kSymbols; step > 0; step >>= 1) {
            const int nxt = pos + step;
            if (nxt <= kSymbols && acc + tree[nxt] <= v) {
                pos = nxt;
                acc += tree[nxt];
            }
        }
        lo = acc;
        return pos;   // symbol index (0-based) whose range contains v
    }
};

class Contexts {
  public:
    explicit Contexts(int order) : order_(order)
    {
        if (order_ <= 1) flat_.resize(order_ == 0 ? 1 : kSymbols);
    }
    Model &get(uint64_t key)
    {
        if (order_ <= 1) return flat_[key];
        auto it = map_.find(key);
        if (it == map_.end()) it = map_.emplace(key, std::unique_ptr<Model>(new Model())).first;
        return *it->second;
    }
    uint64_t push(uint64_t key, int s) const
    {
        if (order_ == 0) return 0;
        const uint64_t mask = order_ >= 8 ? ~0ULL : ((1ULL << (8 * order_)) - 1);
        return ((key << 8) | (uint64_t)s) & mask;
    }

  private:
    int order_;
    std::vector<Model> flat_;
    std::unordered_map<uint64_t, std::unique_ptr<Model>> map_;
};

constexpr uint32_t kHalf = 0x80000000u, kQ1 = 0x40000000u, kQ3 = 0xC0000000u;

// x / d for the coder's numerators x = range * cum < 2^32 * d and d = the model
// total: with m = floor(2^64 / d) + 1 and e = m d - 2^64 (0 < e <= d),
// floor(x m / 2^64) = floor(x / d + x e / (d 2^64)), and x e < 2^64 keeps the
// added term below 1/d, too small to cross the next multiple of 1/d: exact
// whenever x d < 2^64, i.e. for every total below 2^16.  The halving rule keeps
// totals <= 16384; a larger prior-seeded total (only before its first update)
// divides.
constexpr uint32_t kRecipMax = 1u << 16;
struct Divider {
    uint64_t m[kRecipMax];
    Divider()
    {
        m[0] = m[1] = 0;
        for (uint32_t d = 2; d < kRecipMax; ++d) m[d] = ~0ULL / d + ((~0ULL % d) + 1 == d ? 2 : 1);
    }
    static const Divider &get()
    {
        static const Divider *t = new Divider();   // thread-safe, once per process
        return *t;
    }
    uint32_t div(uint64_t x, uint32_t d) const
    {
        if (d < kRecipMax && d > 1) return (uint32_t)(((unsigned __int128)x * m[d]) >> 64);
        return (uint32_t)(x / d);
    }
};

// MSB-first bits into bytes (bitarray endian='big'), 32 at a time
struct BitWriter {
    uint8_t *buf;
    int64_t cap;
    int64_t nbits = 0;          // bits written in all
    uint64_t acc = 0;           // the last (nbits & 31) bits, in its low bits
    bool overflow = false;
    void put(uint32_t v, int n)   // v's low n bits, 0 <= n <= 32
    {
        if (n == 0) return;
        const int have = (int)(nbits & 31);
        acc = (acc << n) | (n == 32 ? (uint64_t)v : ((uint64_t)v & ((1ULL << n) - 1)));
        nbits += n;
        if (have + n >= 32) {   // a whole word: the 32 bits above the (have + n - 32) newest
            const uint32_t w = (uint32_t)(acc >> (have + n - 32));
            const int64_t at = (nbits >> 5 << 2) - 4;
            if (at + 4 <= cap) {
                buf[at] = (uint8_t)(w >> 24);
                buf[at + 1] = (uint8_t)(w >> 16);
                buf[at + 2] = (uint8_t)(w >> 8);
                buf[at + 3] = (uint8_t)w;
            } else {
                for (int i = 0; i < 4; ++i)
                    if (at + i < cap) buf[at + i] = (uint8_t)(w >> (24 - 8 * i));
                    else overflow = true;
            }
        }
    }
    void repeat(int b, uint64_t count)   // count copies of bit b
    {
        const uint32_t word = b ? 0xFFFFFFFFu : 0u;
        for (; count >= 32; count -= 32) put(word, 32);
        put(word, (int)count);
    }
    void finish()   // the partial last word, zero padded to whole bytes
    {
        const int have = (int)(nbits & 31);
        if (!have) return;
        const uint32_t w = (uint32_t)(acc << (32 - have));
        const int64_t at = nbits >> 5 << 2;
        for (int i = 0; i < (have + 7) / 8; ++i) {
            if (at + i < cap) buf[at + i] = (uint8_t)(w >> (24 - 8 * i));
            else overflow = true;
        }
    }
};

// MSB-first bits, zeros past the end
struct BitReader {
    const uint8_t *buf;
    int64_t nbytes, pos = 0;    // next byte to load
    uint64_t bits = 0;          // left-aligned
    int n = 0;                  // valid bits in `bits`
    void refill()
    {
        while (n <= 56) {
            const uint64_t b = pos < nbytes ? buf[pos] : 0u;
            ++pos;
            bits |= b << (56 - n);
            n += 8;
        }
    }
    uint32_t get(int k)   // 0 <= k <= 32
    {
        if (k == 0) return 0;
        if (n < k) refill();
        const uint32_t v = (uint32_t)(bits >> (64 - k));
        bits <<= k;
        n -= k;
        return v;
    }
};

// the coder's renormalisation, in bulk: E1/E2 (low and high share their top bit)
// for all the leading bits they share, then E3 (low = 01.., high = 10..) for all
// the underflow steps that follow; returns the number of bits shifted in (the
// decoder reads that many), with the shared prefix in *prefix (its top bit
// first) and the E3 count in *e3
inline int renorm(uint32_t &low, uint32_t &high, uint32_t &prefix, int &n_prefix, int &e3)
{
    n_prefix = __builtin_clz(low ^ high);   // low < high, so low ^ high != 0
    prefix = n_prefix ? low >> (32 - n_prefix) : 0u;
    if (n_prefix) {
        low <<= n_prefix;
        high = (high << n_prefix) | ((1u << n_prefix) - 1u);
    }
    e3 = 0;
    if (low >= kQ1 && high < kQ3) {   // low = 01^k.., high = 10^k..
        const int ones = __builtin_clz(~(low << 1)), zeros = __builtin_clz((high << 1) | 1u);
        e3 = ones < zeros ? ones : zeros;
        low = (low << e3) & 0x7FFFFFFFu;
        high = (high << e3) | kHalf | ((1u << e3) - 1u);
    }
    return n_prefix + e3;
}

}  // namespace
}  // namespace vcf

using namespace vcf;

extern "C" {

int64_t vcf_cbaac_bound(int64_t n_symbols)
{
    // each symbol narrows the interval by at most total/1 <= 2^15 -> <= 17 bits incl. carry-over
    return n_symbols < 0 ? 0 : (n_symbols * 17 + 7) / 8 + 16;
}

static int cbaac_encode(const uint8_t *symbols, int64_t n, int32_t order, uint8_t *out, int64_t out_capacity,
                        int64_t *out_bytes, int64_t *out_bits, const uint16_t *prior)
{
    if (n < 0 || order < 0 || order > 8) return set_error(VCF_ERR_INVALID, "bad n or order (0..8)");
    if ((n > 0 && !symbols) || !out || !out_bytes) return set_error(VCF_ERR_INVALID, "null buffer");
    try {
        Contexts ctx(order);
        if (prior)   // orders 0 / 1: every context's model (1 or 256, all created up front) from the prior
            for (uint64_t c = 0; c < (order == 0 ? 1u : 256u); ++c) ctx.get(c).init(prior);
        BitWriter bw{out, out_capacity};
        const Divider &dv = Divider::get();
        uint32_t low = 0, high = 0xFFFFFFFFu;
        uint64_t pending = 0, key = 0;
        for (int64_t i = 0; i < n; ++i) {
            const int s = symbols[i];
            Model &m = ctx.get(key);
            const uint32_t lo = m.cum(s), hi = lo + m.freq[s], tot = m.total;
            const uint64_t range = (uint64_t)(high - low) + 1;
            high = low + dv.div(range * hi, tot) - 1;
            low = low + dv.div(range * lo, tot);
            uint32_t prefix;
            int np, e3;
            renorm(low, high, prefix, np, e3);
            if (np) {   // the first shared bit, the pending bits (its complement), the rest
                const uint32_t b = prefix >> (np - 1);
                bw.put(b, 1);
                if (pending) {
                    bw.repeat(!b, pending);
                    pending = 0;
                }
                bw.put(prefix, np - 1);
            }
            pending += (uint64_t)e3;
            m.update(s);
            key = ctx.push(key, s);
            if (bw.overflow) return set_error(VCF_ERR_INVALID, "output buffer too small");
        }
        {   // flush: one more pending bit and the disambiguating bit
            const uint32_t b = low < kQ1 ? 0u : 1u;
            bw.put(b, 1);
            bw.repeat(!b, pending + 1);
        }
        bw.finish();
        if (bw.overflow) return set_error(VCF_ERR_INVALID, "output buffer too small");
        *out_bytes = (bw.nbits + 7) >> 3;
        if (out_bits) *out_bits = bw.nbits;
    } catch (const std::bad_alloc &) {
        return set_error(VCF_ERR_INVALID, "out of host memory (context order %d)", order);
    }
    return VCF_OK;
}

int vcf_cbaac_encode(const uint8_t *symbols, int64_t n, int32_t order, uint8_t *out, int64_t out_capacity,
                     int64_t *out_bytes, int64_t *out_bits)
{
    return cbaac_encode(symbols, n, order, out, out_capacity, out_bytes, out_bits, nullptr);
}

// orders 0 / 1 from the tiled container's prior frequencies (vcf_cbaac_gpu.hip)
int vcf_cbaac_encode_prior(const uint8_t *symbols, int64_t n, int32_t order, const uint16_t *prior, uint8_t *out,
                           int64_t out_capacity, int64_t *out_bytes, int64_t *out_bits)
{
    if (!prior) return set_error(VCF_ERR_INVALID, "null prior");
    if (order < 0 || order > 1) return set_error(VCF_ERR_UNSUPPORTED, "prior-seeded models: orders 0 and 1");
    for (int i = 0; i < kSymbols; ++i)
        if (prior[i] == 0) return set_error(VCF_ERR_INVALID, "prior frequency 0 (symbol %d)", i);
    return cbaac_encode(symbols, n, order, out, out_capacity, out_bytes, out_bits, prior);
}

static int cbaac_decode(const uint8_t *bytes, int64_t nbytes, int64_t n, int32_t order, uint8_t *symbols_out,
                        const uint16_t *prior)
{
    if (n < 0 || nbytes < 0 || order < 0 || order > 8) return set_error(VCF_ERR_INVALID, "bad arguments");
    if ((n > 0 && !symbols_out) || (nbytes > 0 && !bytes)) return set_error(VCF_ERR_INVALID, "null buffer");
    try {
        Contexts ctx(order);
        if (prior)   // orders 0 / 1: every context's model (1 or 256, all created up front) from the prior
            for (uint64_t c = 0; c < (order == 0 ? 1u : 256u); ++c) ctx.get(c).init(prior);
        BitReader br{bytes, nbytes};
        const Divider &dv = Divider::get();
        uint32_t low = 0, high = 0xFFFFFFFFu, value = br.get(32);
        uint64_t key = 0;
        for (int64_t i = 0; i < n; ++i) {
            Model &m = ctx.get(key);
            const uint64_t range = (uint64_t)(high - low) + 1;
            const uint32_t tot = m.total;
            // the reference's scaled value is floor(num / range); its symbol s has
            // cum(s) <= scaled < cum(s) + freq(s), i.e. cum(s) range <= num < (cum(s) + freq(s)) range
            const uint64_t num = ((uint64_t)(value - low) + 1) * tot - 1;
            int s = m.mps;
            uint32_t lo = m.cum(s);
            if (!((uint64_t)lo * range <= num && num < (uint64_t)(lo + m.freq[s]) * range))
                s = m.find((uint32_t)(num / range), lo);
            const uint32_t hi = lo + m.freq[s];
            high = low + dv.div(range * hi, tot) - 1;
            low = low + dv.div(range * lo, tot);
            uint32_t prefix;
            int np, e3;
            renorm(low, high, prefix, np, e3);
            if (np) value = (np == 32 ? 0u : value << np) | br.get(np);
            if (e3) value = (value & kHalf) | ((value << e3) & 0x7FFFFFFFu) | br.get(e3);
            symbols_out[i] = (uint8_t)s;
            m.update(s);
            key = ctx.push(key, s);
        }
    } catch (const std::bad_alloc &) {
        return set_error(VCF_ERR_INVALID, "out of host memory (context order %d)", order);
    }
    return VCF_OK;
}

int vcf_cbaac_decode(const uint8_t *bytes, int64_t nbytes, int64_t n, int32_t order, uint8_t *symbols_out)
{
    return cbaac_decode(bytes, nbytes, n, order, symbols_out, nullptr);
}

int vcf_cbaac_decode_prior(const uint8_t *bytes, int64_t nbytes, int64_t n, int32_t order, const uint16_t *prior,
                           uint8_t *symbols_out)
{
    if (!prior) return set_error(VCF_ERR_INVALID, "null prior");
    if (order < 0 || order > 1) return set_error(VCF_ERR_UNSUPPORTED, "prior-seeded models: orders 0 and 1");
    for (int i = 0; i < kSymbols; ++i)
        if (prior[i] == 0) return set_error(VCF_ERR_INVALID, "prior frequency 0 (symbol %d)", i);
    return cbaac_decode(bytes, nbytes, n, order, symbols_out, prior);
}

// The model alone, for parity tests: (low, high, total) handed to the coder
// for every symbol (what CBAAC.py's _encode passes to encode_symbol).
int vcf_cbaac_model_trace(const uint8_t *symbols, int64_t n, int32_t order, int32_t *triples)
{
    if (n < 0 || order < 0 || order > 8) return set_error(VCF_ERR_INVALID, "bad n or order");
    if (n > 0 && (!symbols || !triples)) return set_error(VCF_ERR_INVALID, "null buffer");
    Contexts ctx(order);
    uint64_t key = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int s = symbols[i];
        Model &m = ctx.get(key);
        const uint32_t lo = m.cum(s);
        triples[3 * i] = (int32_t)lo;
        triples[3 * i + 1] = (int32_t)(lo + m.freq[s]);
        triples[3 * i + 2] = (int32_t)m.total;
        m.update(s);
        key = ctx.push(key, s);
    }
    return VCF_OK;
}

/* Container version 3 index pieces (vcf_amd/tcbaac.py), per row of values:
 * the segment sizes as unsigned LEB128 varints, row r's bytes ending at
 * out[row_end[r]]. */
int vcf_leb128_encode_rows(const int64_t *v, int64_t rows, int64_t cols, uint8_t *out, int64_t capacity,
                           int64_t *row_end)
{
    if (rows < 0 || cols < 0 || capacity < 0) return set_error(VCF_ERR_INVALID, "negative size");
    if ((rows * cols > 0 && (!v || !out)) || (rows > 0 && !row_end)) return set_error(VCF_ERR_INVALID, "null buffer");
    int64_t o = 0;
    for (int64_t r = 0; r < rows; ++r) {
        for (int64_t c = 0; c < cols; ++c) {
            uint64_t x = (uint64_t)v[r * cols + c];
            if (v[r * cols + c] < 0) return set_error(VCF_ERR_INVALID, "negative value");
            do {
                if (o >= capacity) return set_error(VCF_ERR_INVALID, "output buffer too small");
                const uint8_t b = (uint8_t)(x & 0x7F);
                x >>= 7;
                out[o++] = x ? (uint8_t)(b | 0x80) : b;
            } while (x);
        }
        row_end[r] = o;
    }
    return VCF_OK;
}

/* Version 3's prior rows of `frames` frames (nclass x 256 uint16 each): per
 * frame uint32 nclass, then per row uint16 m and the m symbols whose
 * frequency is not 1 (uint8, ascending) and their m frequencies (uint16);
 * frame f's bytes end at out[frame_end[f]]. */
int vcf_prior_rows_sparse(const uint16_t *priors, int64_t frames, int32_t nclass, uint8_t *out, int64_t capacity,
                          int64_t *frame_end)
{
    if (frames < 0 || nclass < 1 || capacity < 0) return set_error(VCF_ERR_INVALID, "bad size");
    if (frames > 0 && (!priors || !out || !frame_end)) return set_error(VCF_ERR_INVALID, "null buffer");
    int64_t o = 0;
    auto put = [&](uint32_t v, int nb) -> bool {
        if (o + nb > capacity) return false;
        for (int i = 0; i < nb; ++i) out[o++] = (uint8_t)(v >> (8 * i));
        return true;
    };
    for (int64_t f = 0; f < frames; ++f) {
        if (!put((uint32_t)nclass, 4)) return set_error(VCF_ERR_INVALID, "output buffer too small");
        for (int32_t c = 0; c < nclass; ++c) {
            const uint16_t *row = priors + (f * nclass + c) * 256;
            uint32_t m = 0;
            for (int s = 0; s < 256; ++s) m += row[s] != 1;
            if (!put(m, 2)) return set_error(VCF_ERR_INVALID, "output buffer too small");
            for (int s = 0; s < 256; ++s)
                if (row[s] != 1 && !put((uint32_t)s, 1)) return set_error(VCF_ERR_INVALID, "output buffer too small");
            for (int s = 0; s < 256; ++s)
                if (row[s] != 1 && !put(row[s], 2)) return set_error(VCF_ERR_INVALID, "output buffer too small");
        }
        frame_end[f] = o;
    }
    return VCF_OK;
}

}  // extern "C"
