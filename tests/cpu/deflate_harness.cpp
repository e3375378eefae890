// Host build of vcf_amd/csrc/vcf_deflate.h (the GPU deflate's parse, trees and
// bit layout) with a sequential hash-chain matcher, so that the restatement can
// be checked against zlib.compress(data, level) itself on the CPU
// (tests/test_deflate.py).  Test infrastructure only.
#include <string.h>

#include <vector>

#include "vcf_deflate.h"

using namespace vcf::dfl;

#ifdef DH_STATS
#include <algorithm>
// diagnostic build only: [0] longest_match calls, [1] candidates visited, [2..5] calls whose
// farthest candidate is beyond 8 / 12 / 16 / 24 KiB, [8..23] candidates by distance (2 KiB bins)
extern "C" {
unsigned long long dh_stats[32];
}
#endif

namespace {

struct BitOut {
    std::vector<uint8_t> bytes;
    uint64_t buf = 0;
    int nbits = 0;
    void operator()(uint32_t v, int n) { put64(v, n); }
    void put64(uint64_t v, int n)
    {
        if (n == 0) return;
        buf |= (v & ((n == 64) ? ~0ull : ((1ull << n) - 1))) << nbits;
        nbits += n;
        while (nbits >= 8) {
            bytes.push_back((uint8_t)buf);
            buf >>= 8;
            nbits -= 8;
        }
    }
    void windup()
    {
        if (nbits > 0) bytes.push_back((uint8_t)buf);
        buf = 0;
        nbits = 0;
    }
};

struct HostOps {
    const uint8_t *in;
    uint32_t n;
    std::vector<uint8_t> win;      // the window as longest_match reads it (view past the end)
    std::vector<uint32_t> prevpos;
    std::vector<uint32_t> syms;
    BlockTrees T;
    std::vector<uint16_t> store;
    std::vector<int16_t> heap;
    std::vector<uint8_t> depth;
    BitOut out;

    HostOps(const uint8_t *src, uint32_t len) : in(src), n(len)
    {
        win.assign((size_t)n + MAX_MATCH + 8, 0);   // fill_window's high_water zeroing past the end
        memcpy(win.data(), in, n);
        prevpos.assign(n + 1, 0);
        std::vector<uint32_t> head(1 << 15, 0);
        for (uint32_t p = 0; p + 2 < n; ++p) {       // INSERT_STRING for every position 0..n-3
            const uint32_t h = (((uint32_t)in[p] << 10) ^ ((uint32_t)in[p + 1] << 5) ^ in[p + 2]) & 0x7fff;
            prevpos[p] = head[h];
            head[h] = p;
        }
        const int nl = HEAP_SIZE, nd = 2 * D_CODES + 1, nb = 2 * BL_CODES + 1;
        store.assign(4 * (nl + nd + nb) + 16 + 3 * 8, 0);
        uint16_t *s = store.data();
        auto take = [&](int k) { uint16_t *r = s; s += k; return r; };
        T.l = {take(nl), take(nl), take(nl), take(nl), L_CODES, MAX_BITS, 0, 0};
        T.d = {take(nd), take(nd), take(nd), take(nd), D_CODES, MAX_BITS, 1, 0};
        T.bl = {take(nb), take(nb), take(nb), take(nb), BL_CODES, MAX_BL_BITS, 2, 0};
        T.w.bl_count = take(MAX_BITS + 1);
        heap.assign(HEAP_SIZE, 0);
        depth.assign(HEAP_SIZE, 0);
        T.w.heap = heap.data();
        T.w.depth = depth.data();
        init_block(T);
    }
    uint8_t byte(uint32_t p) const { return win[p]; }
    uint32_t head(uint32_t p) const { return prevpos[p]; }
    void slide()
    {
        // after zlib's slide the bytes past the end are the stale copy wsize back
        for (uint32_t P = n; P < n + MAX_MATCH; ++P) win[P] = win[P - WSIZE];
    }
    uint32_t lcp(uint32_t a, uint32_t b) const
    {
        uint32_t l = 0;
        while (l < (uint32_t)MAX_MATCH && win[a + l] == win[b + l]) ++l;
        return l;
    }
    bool longest(uint32_t p, uint32_t cur, uint32_t best, uint32_t chain, uint32_t nice, uint32_t limit,
                 uint32_t &len, uint32_t &pos)
    {
        bool found = false;
#ifdef DH_STATS
        uint32_t far = 0;
        ++dh_stats[0];
#endif
        do {
#ifdef DH_STATS
            far = p - cur > far ? p - cur : far;
            ++dh_stats[1];
            ++dh_stats[8 + std::min<uint32_t>((p - cur) >> 11, 15)];
#endif
            const uint32_t l = lcp(cur, p);
            if (l > best) {
                pos = cur;
                best = l;
                found = true;
                if (l >= nice) break;
            }
        } while ((cur = prevpos[cur]) > limit && --chain != 0);
#ifdef DH_STATS
        dh_stats[2] += far > 8192;
        dh_stats[3] += far > 12288;
        dh_stats[4] += far > 16384;
        dh_stats[5] += far > 24576;
#endif
        len = best;
        return found;
    }
    bool tally(uint32_t dist, uint32_t lc)
    {
        syms.push_back(dist << 8 | lc);
        vcf::dfl::tally(T, dist, lc);
        return syms.size() == (size_t)LIT_BUFSIZE - 1;
    }
    void flush(uint32_t stored_len, bool buf_ok, uint32_t block_start, bool last)
    {
        int max_blindex = 0;
        const int kind = plan_block(T, stored_len, buf_ok, max_blindex);
        if (kind == 0) {
            out(last ? 1 : 0, 3);
            out.windup();
            out(stored_len & 0xffff, 16);
            out(~stored_len & 0xffff, 16);
            for (uint32_t i = 0; i < stored_len; ++i) out(in[block_start + i], 8);
        } else {
            std::vector<uint16_t> lc(L_CODES + 2), ll(L_CODES + 2), dc(D_CODES), dl(D_CODES);
            if (kind == 1) {
                out(2 + (last ? 1 : 0), 3);
                for (int i = 0; i < L_CODES + 2; ++i) lc[i] = (uint16_t)static_lcode(i), ll[i] = (uint16_t)static_llen(i);
                for (int i = 0; i < D_CODES; ++i) dc[i] = (uint16_t)static_dcode(i), dl[i] = 5;
            } else {
                out(4 + (last ? 1 : 0), 3);
                send_all_trees(T, max_blindex, out);
                for (int i = 0; i <= T.l.max_code; ++i) lc[i] = T.l.code[i], ll[i] = T.l.len[i];
                for (int i = 0; i <= T.d.max_code; ++i) dc[i] = T.d.code[i], dl[i] = T.d.len[i];
            }
            for (uint32_t s : syms) {
                uint64_t v;
                int nb;
                symbol_bits(s, lc.data(), ll.data(), dc.data(), dl.data(), v, nb);
                out.put64(v, nb);
            }
            out.put64(lc[END_BLOCK], ll[END_BLOCK]);
        }
        syms.clear();
        init_block(T);
        if (last) out.windup();
    }
};

}  // namespace

extern "C" long long dh_compress(const uint8_t *in, long long n, int level, uint8_t *out, long long cap)
{
    Config cfg;
    if (!level_config(level, cfg) || n < 0 || n > MAX_STRIP) return -1;
    HostOps ops(in, (uint32_t)n);
    const uint32_t hdr = zlib_header(level);
    ops.out(hdr >> 8, 8);
    ops.out(hdr & 0xff, 8);
    deflate_slow(ops, (uint32_t)n, cfg);
    uint64_t sb = 0, swb = 0;
    for (long long i = 0; i < n; ++i) sb += in[i], swb += (uint64_t)(n - i) * in[i];
    const uint32_t ad = adler32_from_sums(sb, swb, (uint64_t)n);
    for (int k = 3; k >= 0; --k) ops.out((ad >> (8 * k)) & 0xff, 8);
    const std::vector<uint8_t> &b = ops.out.bytes;
    if ((long long)b.size() > cap) return -2;
    memcpy(out, b.data(), b.size());
    return (long long)b.size();
}
