// vcf_cbahc.cpp -- context-based adaptive Huffman coding (src/CBAHC.py),
// native host code, and the vcf_cbahc_* entry points of the C ABI.
//
// Bit-exact with the reference (tests/golden/make_golden_cbahc.py runs its
// unmodified CoDec): for every symbol, a Huffman tree is built from the
// current counts of its context (_ContextModel, CBAHC.py:123-155: 256 counts
// starting at 1, one model per tuple of the previous `order` symbols padded
// with 256), the symbol's code is appended (left = 0, right = 1, root first,
// _build_codebook :81-106), then its count is incremented.
//
// _build_huffman_tree_from_freq (:38-78) pops the two smallest (freq, uid)
// pairs of a heap (leaf uid = symbol, the dict's insertion order; internal
// uid = 256, 257, ... in creation order) and makes them left / right of a new
// node.  (freq, uid) pairs are unique, so the tree does not depend on the
// heap; the linear two-queue construction yields the same pops: leaves kept
// sorted by (freq, symbol), internal nodes in a FIFO (their (freq, uid) are
// created in increasing order), a leaf winning a frequency tie because its
// uid is below 256.  O(256) per symbol instead of the reference's heap and
// dictionary walk.
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

constexpr int kSym = 256;
constexpr int kPad = 256;   // _ContextModel.PAD

struct HufModel {
    uint32_t freq[kSym];
    uint16_t sorted[kSym];   // symbols by (freq, symbol) ascending
    uint16_t pos[kSym];      // position of each symbol in `sorted`

    HufModel()
    {
        for (int s = 0; s < kSym; ++s) {
            freq[s] = 1;
            sorted[s] = (uint16_t)s;
            pos[s] = (uint16_t)s;
        }
    }
    bool less(int a, int b) const { return freq[a] < freq[b] || (freq[a] == freq[b] && a < b); }
    void update(int s)
    {
        ++freq[s];
        int p = pos[s];
        while (p + 1 < kSym && less(sorted[p + 1], s)) {
            sorted[p] = sorted[p + 1];
            pos[sorted[p]] = (uint16_t)p;
            ++p;
        }
        sorted[p] = (uint16_t)s;
        pos[s] = (uint16_t)p;
    }
};

// The tree of one model: nodes 0..255 are leaves (symbols), 256..510 internal.
struct Tree {
    int16_t left[2 * kSym], right[2 * kSym], parent[2 * kSym];
    int root;

    void build(const HufModel &m)
    {
        uint64_t f[2 * kSym];
        for (int s = 0; s < kSym; ++s) f[s] = m.freq[s];
        int li = 0;              // next leaf in m.sorted
        int qh = kSym, qt = kSym;   // internal FIFO [qh, qt)
        auto pick = [&]() -> int {
            // leaf vs internal front: smaller (freq, uid); leaf uid < internal uid
            if (li < kSym && (qh == qt || f[m.sorted[li]] <= f[qh])) return m.sorted[li++];
            return qh++;
        };
        for (int k = 0; k < kSym - 1; ++k) {
            const int a = pick();
            const int b = pick();
            const int n = qt++;
            f[n] = f[a] + f[b];
            left[n] = (int16_t)a;
            right[n] = (int16_t)b;
            parent[a] = (int16_t)n;
            parent[b] = (int16_t)n;
        }
        root = qt - 1;
        parent[root] = -1;
    }
    // code of symbol s, root first: bits[0..len)
    int code(int s, uint8_t *bits) const
    {
        int len = 0;
        for (int n = s; n != root; n = parent[n]) bits[len++] = (right[parent[n]] == n) ? 1 : 0;
        for (int i = 0; i < len / 2; ++i) {
            const uint8_t t = bits[i];
            bits[i] = bits[len - 1 - i];
            bits[len - 1 - i] = t;
        }
        return len;
    }
};

class HufContexts {
  public:
    explicit HufContexts(int order) : order_(order)
    {
        key_ = 0;
        for (int i = 0; i < order_; ++i) key_ = (key_ << 9) | kPad;
    }
    HufModel &get()
    {
        auto it = map_.find(key_);
        if (it == map_.end()) it = map_.emplace(key_, std::unique_ptr<HufModel>(new HufModel())).first;
        return *it->second;
    }
    void push(int s)
    {
        if (order_ == 0) return;
        const uint64_t mask = (order_ >= 7) ? ~0ULL : ((1ULL << (9 * order_)) - 1);
        key_ = ((key_ << 9) | (uint64_t)s) & mask;
    }

  private:
    int order_;
    uint64_t key_;
    std::unordered_map<uint64_t, std::unique_ptr<HufModel>> map_;
};

}  // namespace
}  // namespace vcf

using namespace vcf;

extern "C" {

int64_t vcf_cbahc_bound(int64_t n_symbols)
{
    return n_symbols < 0 ? 0 : n_symbols * 32 + 16;   // a code is at most 255 bits
}

int vcf_cbahc_encode(const uint8_t *symbols, int64_t n, int32_t order, uint8_t *out, int64_t out_capacity,
                     int64_t *out_bytes, int64_t *out_bits)
{
    if (n < 0 || order < 0 || order > 7) return set_error(VCF_ERR_INVALID, "bad n or order (0..7)");
    if ((n > 0 && !symbols) || !out || !out_bytes) return set_error(VCF_ERR_INVALID, "null buffer");
    try {
        HufContexts ctx(order);
        std::unique_ptr<Tree> tree(new Tree());
        uint8_t bits[kSym];
        int64_t nb = 0;
        for (int64_t i = 0; i < n; ++i) {
            HufModel &m = ctx.get();
            tree->build(m);
            const int s = symbols[i];
            const int len = tree->code(s, bits);
            if (((nb + len + 7) >> 3) > out_capacity) return set_error(VCF_ERR_INVALID, "output buffer too small");
            for (int k = 0; k < len; ++k, ++nb) {
                if ((nb & 7) == 0) out[nb >> 3] = 0;
                if (bits[k]) out[nb >> 3] |= (uint8_t)(0x80u >> (nb & 7));
            }
            m.update(s);
            ctx.push(s);
        }
        *out_bytes = (nb + 7) >> 3;
        if (out_bits) *out_bits = nb;
    } catch (const std::bad_alloc &) {
        return set_error(VCF_ERR_INVALID, "out of host memory (context order %d)", order);
    }
    return VCF_OK;
}

int vcf_cbahc_decode(const uint8_t *bytes, int64_t nbits, int64_t n, int32_t order, uint8_t *symbols_out)
{
    if (n < 0 || nbits < 0 || order < 0 || order > 7) return set_error(VCF_ERR_INVALID, "bad arguments");
    if ((n > 0 && !symbols_out) || (nbits > 0 && !bytes)) return set_error(VCF_ERR_INVALID, "null buffer");
    try {
        HufContexts ctx(order);
        std::unique_ptr<Tree> tree(new Tree());
        int64_t p = 0;
        for (int64_t i = 0; i < n; ++i) {
            HufModel &m = ctx.get();
            tree->build(m);
            int node = tree->root;
            while (node >= kSym) {
                if (p >= nbits) return set_error(VCF_ERR_INVALID, "Truncated bitstream while decoding");
                const int b = (bytes[p >> 3] >> (7 - (p & 7))) & 1;
                ++p;
                node = b ? tree->right[node] : tree->left[node];
            }
            symbols_out[i] = (uint8_t)node;
            m.update(node);
            ctx.push(node);
        }
    } catch (const std::bad_alloc &) {
        return set_error(VCF_ERR_INVALID, "out of host memory (context order %d)", order);
    }
    return VCF_OK;
}

}  // extern "C"
