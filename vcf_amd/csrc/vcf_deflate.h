// vcf_deflate.h -- zlib's deflate (levels 4-9: deflate_slow) restated so that
// a GPU wave can produce, for one TIFF strip, exactly the bytes of
// zlib.compress(strip, level) (zlib 1.2.11, windowBits 15, memLevel 8,
// Z_DEFAULT_STRATEGY).  The reference's default entropy codec is TIFF.py:29
// (tifffile.imwrite(..., compression='zlib') -> one zlib stream per ~64 KB
// strip at level 6); the host path (vcf_amd/codec/tiff.py) calls system zlib.
//
// What is restated, and from where (zlib 1.2.11, Jean-loup Gailly and Mark
// Adler, zlib licence -- see THIRD_PARTY_NOTICES.md).  The trees.c part is a
// close transliteration of zlib's own functions (same control flow and
// variable roles, so that every tie and overflow resolves as zlib's does):
//   * deflate.c deflate_slow: lazy evaluation, the TOO_FAR rule, the hash
//     insertion of every position, FLUSH_BLOCK after lit_bufsize-1 symbols;
//     fill_window's one slide for strips longer than wsize+MAX_DIST (the
//     window's stale bytes past the end, read by the matcher, are reproduced);
//   * deflate.c longest_match: the chain walk in hash-chain order with
//     max_chain (>> 2 once prev_length >= good_match), nice_match (clamped to
//     the lookahead), the limit MAX_DIST back, "first candidate longer than
//     the best so far";
//   * trees.c: build_tree (heap with the (freq, depth) tie rule), gen_bitlen
//     (with the overflow fix-up), gen_codes, scan_tree / send_tree /
//     build_bl_tree / send_all_trees, _tr_flush_block's stored / static /
//     dynamic choice, _tr_stored_block, compress_block, bi_windup;
//   * deflate.c deflate(): the 2-byte zlib header and the adler32 trailer.
//
// The one structural change: zlib's hash chains do not
// depend on the parse -- every position 0..n-3 is inserted, in order, and a
// position's hash is a function of its 3 bytes (hash_shift 5, hash_bits 15)
// -- so the chain of position p is "the earlier positions with p's hash,
// newest first".  The GPU builds those lists for all positions at once
// (positions bucketed by hash, stable) and evaluates up to 64 chain
// candidates per step in parallel; this header holds everything else, shared
// by the kernel (vcf_deflate.hip) and the host harness that checks it against
// zlib itself (tests/cpu/deflate_harness.cpp, tests/test_deflate.py).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define VD_HD __host__ __device__
#else
#define VD_HD
#endif

namespace vcf {
namespace dfl {

constexpr int MIN_MATCH = 3, MAX_MATCH = 258;
constexpr int WSIZE = 32768;                                  // windowBits 15
constexpr int MIN_LOOKAHEAD = MAX_MATCH + MIN_MATCH + 1;      // 262
constexpr int MAX_DIST = WSIZE - MIN_LOOKAHEAD;               // 32506
constexpr int TOO_FAR = 4096;
constexpr int LIT_BUFSIZE = 1 << (8 + 6);                     // memLevel 8
constexpr int MAX_STRIP = 2 * WSIZE;                          // whole strip read by the first fill_window
constexpr int L_CODES = 286, D_CODES = 30, BL_CODES = 19;
constexpr int HEAP_SIZE = 2 * L_CODES + 1;
constexpr int END_BLOCK = 256, REP_3_6 = 16, REPZ_3_10 = 17, REPZ_11_138 = 18;
constexpr int MAX_BITS = 15, MAX_BL_BITS = 7;

struct Config {
    int good, lazy, nice, chain;
};

// deflate.c configuration_table for the deflate_slow levels
VD_HD inline bool level_config(int level, Config &c)
{
    switch (level) {
    case 4: c = {4, 4, 16, 16}; return true;
    case 5: c = {8, 16, 32, 32}; return true;
    case 6: c = {8, 16, 128, 128}; return true;
    case 7: c = {8, 32, 128, 256}; return true;
    case 8: c = {32, 128, 258, 1024}; return true;
    case 9: c = {32, 258, 258, 4096}; return true;
    default: return false;
    }
}

// zlib header (deflate.c deflate(), no dictionary): CMF 0x78, level flags
VD_HD inline uint32_t zlib_header(int level)
{
    const uint32_t lf = level < 6 ? 1 : level == 6 ? 2 : 3;
    uint32_t h = (0x78u << 8) | (lf << 6);
    h += 31 - (h % 31);
    return h;
}

// ---- RFC 1951 code tables, computed (trees.c tr_static_init builds the same) ----
VD_HD inline int ilog2(uint32_t v) { return 31 - __builtin_clz(v); }
// length code 0..28 of lc = length - 3 (_length_code; 258 uses code 285)
VD_HD inline int length_code(int lc)
{
    if (lc < 8) return lc;
    if (lc == 255) return 28;
    const int b = ilog2((uint32_t)lc);
    return 4 * (b - 1) + ((lc >> (b - 2)) & 3);
}
VD_HD inline int extra_lbits(int c) { return (c < 8 || c == 28) ? 0 : (c - 4) >> 2; }
VD_HD inline int base_length(int c) { return c < 8 ? c : c == 28 ? 0 : (4 + (c & 3)) << ((c - 4) >> 2); }
// distance code of d = distance - 1 (d_code)
VD_HD inline int dist_code(int d)
{
    if (d < 4) return d;
    const int b = ilog2((uint32_t)d);
    return 2 * b + ((d >> (b - 1)) & 1);
}
VD_HD inline int extra_dbits(int c) { return c < 4 ? 0 : (c - 2) >> 1; }
VD_HD inline int base_dist(int c) { return c < 4 ? c : (2 + (c & 1)) << ((c - 2) >> 1); }
VD_HD inline int extra_blbits(int c) { return c == 16 ? 2 : c == 17 ? 3 : c == 18 ? 7 : 0; }
VD_HD inline int bl_order(int r)
{
    if (r < 3) return 16 + r;
    if (r == 3) return 0;
    return (r & 1) ? 7 - ((r - 5) >> 1) : 8 + ((r - 4) >> 1);
}
VD_HD inline uint32_t bi_reverse(uint32_t code, int len)
{
    uint32_t res = 0;
    do {
        res |= code & 1;
        code >>= 1;
        res <<= 1;
    } while (--len > 0);
    return res >> 1;
}
VD_HD inline int static_llen(int n) { return n < 144 ? 8 : n < 256 ? 9 : n < 280 ? 7 : 8; }
VD_HD inline uint32_t static_lcode(int n)
{
    const uint32_t canon = n < 144 ? 0x30u + n : n < 256 ? 0x190u + (n - 144) : n < 280 ? (uint32_t)(n - 256)
                                                                                         : 0xc0u + (n - 280);
    return bi_reverse(canon, static_llen(n));
}
VD_HD inline uint32_t static_dcode(int n) { return bi_reverse((uint32_t)n, 5); }

// ---- trees.c --------------------------------------------------------------
// One tree's arrays (zlib's ct_data unions split into separate arrays: Freq /
// Code and Dad / Len are never live at the same time, see build_tree).
struct Tree {
    uint16_t *freq;    // [2*elems+1] node frequencies
    uint16_t *dad;     // [2*elems+1]
    uint16_t *len;     // [2*elems+1] (index max_code+1 holds scan_tree's guard)
    uint16_t *code;    // [elems]
    int elems, max_length, kind;   // kind 0 literal/length, 1 distance, 2 bit lengths
    int max_code;
};

struct TreeWork {
    int16_t *heap;      // [HEAP_SIZE]
    uint8_t *depth;     // [HEAP_SIZE]
    uint16_t *bl_count; // [MAX_BITS+1]
    int heap_len, heap_max;
    uint64_t opt_len, static_len;   // ulg in zlib; the forced-node decrements wrap and come back
};

VD_HD inline int xbits_of(int kind, int n)
{
    if (kind == 0) return n >= 257 ? extra_lbits(n - 257) : 0;
    if (kind == 1) return extra_dbits(n);
    return extra_blbits(n);
}
VD_HD inline int stree_len(int kind, int n) { return kind == 0 ? static_llen(n) : 5; }

VD_HD inline bool smaller(const Tree &t, const TreeWork &w, int n, int m)
{
    return t.freq[n] < t.freq[m] || (t.freq[n] == t.freq[m] && w.depth[n] <= w.depth[m]);
}

VD_HD inline void pqdownheap(const Tree &t, TreeWork &w, int k)
{
    const int v = w.heap[k];
    int j = k << 1;
    while (j <= w.heap_len) {
        if (j < w.heap_len && smaller(t, w, w.heap[j + 1], w.heap[j])) j++;
        if (smaller(t, w, v, w.heap[j])) break;
        w.heap[k] = w.heap[j];
        k = j;
        j <<= 1;
    }
    w.heap[k] = (int16_t)v;
}

VD_HD inline void gen_bitlen(Tree &t, TreeWork &w)
{
    const int max_code = t.max_code, max_length = t.max_length;
    int overflow = 0;
    for (int bits = 0; bits <= MAX_BITS; bits++) w.bl_count[bits] = 0;
    t.len[w.heap[w.heap_max]] = 0;   // root
    int h;
    for (h = w.heap_max + 1; h < HEAP_SIZE; h++) {
        const int n = w.heap[h];
        int bits = t.len[t.dad[n]] + 1;
        if (bits > max_length) bits = max_length, overflow++;
        t.len[n] = (uint16_t)bits;
        if (n > max_code) continue;   // not a leaf
        w.bl_count[bits]++;
        const int xb = xbits_of(t.kind, n);
        const uint64_t f = t.freq[n];
        w.opt_len += f * (uint64_t)(bits + xb);
        if (t.kind != 2) w.static_len += f * (uint64_t)(stree_len(t.kind, n) + xb);
    }
    if (overflow == 0) return;
    do {
        int bits = max_length - 1;
        while (w.bl_count[bits] == 0) bits--;
        w.bl_count[bits]--;
        w.bl_count[bits + 1] += 2;
        w.bl_count[max_length]--;
        overflow -= 2;
    } while (overflow > 0);
    h = HEAP_SIZE;
    for (int bits = max_length; bits != 0; bits--) {
        int n = w.bl_count[bits];
        while (n != 0) {
            const int m = w.heap[--h];
            if (m > max_code) continue;
            if (t.len[m] != (uint16_t)bits) {
                w.opt_len += ((uint64_t)bits - t.len[m]) * (uint64_t)t.freq[m];
                t.len[m] = (uint16_t)bits;
            }
            n--;
        }
    }
}

VD_HD inline void gen_codes(Tree &t, const uint16_t *bl_count)
{
    uint16_t next_code[MAX_BITS + 1];
    uint32_t code = 0;
    for (int bits = 1; bits <= MAX_BITS; bits++) {
        code = (code + bl_count[bits - 1]) << 1;
        next_code[bits] = (uint16_t)code;
    }
    for (int n = 0; n <= t.max_code; n++) {
        const int len = t.len[n];
        if (len == 0) continue;
        t.code[n] = (uint16_t)bi_reverse(next_code[len]++, len);
    }
}

VD_HD inline void build_tree(Tree &t, TreeWork &w)
{
    const int elems = t.elems;
    int max_code = -1;
    w.heap_len = 0;
    w.heap_max = HEAP_SIZE;
    for (int n = 0; n < elems; n++) {
        if (t.freq[n] != 0) {
            w.heap[++(w.heap_len)] = (int16_t)(max_code = n);
            w.depth[n] = 0;
        } else {
            t.len[n] = 0;
        }
    }
    // the pkzip format needs at least one distance code; at least two codes of any kind
    while (w.heap_len < 2) {
        const int node = w.heap[++(w.heap_len)] = (int16_t)(max_code < 2 ? ++max_code : 0);
        t.freq[node] = 1;
        w.depth[node] = 0;
        w.opt_len--;
        if (t.kind != 2) w.static_len -= (uint64_t)stree_len(t.kind, node);
    }
    t.max_code = max_code;
    for (int n = w.heap_len / 2; n >= 1; n--) pqdownheap(t, w, n);
    int node = elems;
    do {
        // pqremove
        const int n = w.heap[1];
        w.heap[1] = w.heap[w.heap_len--];
        pqdownheap(t, w, 1);
        const int m = w.heap[1];
        w.heap[--(w.heap_max)] = (int16_t)n;
        w.heap[--(w.heap_max)] = (int16_t)m;
        t.freq[node] = (uint16_t)(t.freq[n] + t.freq[m]);
        w.depth[node] = (uint8_t)((w.depth[n] >= w.depth[m] ? w.depth[n] : w.depth[m]) + 1);
        t.dad[n] = t.dad[m] = (uint16_t)node;
        w.heap[1] = (int16_t)node++;
        pqdownheap(t, w, 1);
    } while (w.heap_len >= 2);
    w.heap[--(w.heap_max)] = w.heap[1];
    gen_bitlen(t, w);
    gen_codes(t, w.bl_count);
}

VD_HD inline void scan_tree(Tree &t, int max_code, Tree &bl)
{
    int prevlen = -1, nextlen = t.len[0], count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    t.len[max_code + 1] = 0xffff;   // guard
    for (int n = 0; n <= max_code; n++) {
        const int curlen = nextlen;
        nextlen = t.len[n + 1];
        if (++count < max_count && curlen == nextlen) {
            continue;
        } else if (count < min_count) {
            bl.freq[curlen] += count;
        } else if (curlen != 0) {
            if (curlen != prevlen) bl.freq[curlen]++;
            bl.freq[REP_3_6]++;
        } else if (count <= 10) {
            bl.freq[REPZ_3_10]++;
        } else {
            bl.freq[REPZ_11_138]++;
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

// send_tree with a bit sink: put(value, nbits)
template <class Put>
VD_HD inline void send_tree(const Tree &t, int max_code, const Tree &bl, Put &put)
{
    int prevlen = -1, nextlen = t.len[0], count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    for (int n = 0; n <= max_code; n++) {
        const int curlen = nextlen;
        nextlen = t.len[n + 1];
        if (++count < max_count && curlen == nextlen) {
            continue;
        } else if (count < min_count) {
            do { put(bl.code[curlen], bl.len[curlen]); } while (--count != 0);
        } else if (curlen != 0) {
            if (curlen != prevlen) {
                put(bl.code[curlen], bl.len[curlen]);
                count--;
            }
            put(bl.code[REP_3_6], bl.len[REP_3_6]);
            put((uint32_t)(count - 3), 2);
        } else if (count <= 10) {
            put(bl.code[REPZ_3_10], bl.len[REPZ_3_10]);
            put((uint32_t)(count - 3), 3);
        } else {
            put(bl.code[REPZ_11_138], bl.len[REPZ_11_138]);
            put((uint32_t)(count - 11), 7);
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

// The three trees of a block and their work arrays (caller-owned storage:
// LDS on the GPU).
struct BlockTrees {
    Tree l, d, bl;
    TreeWork w;
};

// init_block: zero the frequencies, END_BLOCK counts once
VD_HD inline void init_block(BlockTrees &T)
{
    for (int n = 0; n < L_CODES; n++) T.l.freq[n] = 0;
    for (int n = 0; n < D_CODES; n++) T.d.freq[n] = 0;
    for (int n = 0; n < BL_CODES; n++) T.bl.freq[n] = 0;
    T.l.freq[END_BLOCK] = 1;
}

// _tr_flush_block's tree half: builds the trees and decides the block type.
// Returns 0 = stored, 1 = static, 2 = dynamic; max_blindex for send_all_trees.
VD_HD inline int plan_block(BlockTrees &T, uint32_t stored_len, bool buf_ok, int &max_blindex)
{
    T.w.opt_len = 0;
    T.w.static_len = 0;
    build_tree(T.l, T.w);
    build_tree(T.d, T.w);
    // build_bl_tree
    scan_tree(T.l, T.l.max_code, T.bl);
    scan_tree(T.d, T.d.max_code, T.bl);
    build_tree(T.bl, T.w);
    for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
        if (T.bl.len[bl_order(max_blindex)] != 0) break;
    T.w.opt_len += 3 * ((uint64_t)max_blindex + 1) + 5 + 5 + 4;
    uint64_t opt_lenb = (T.w.opt_len + 3 + 7) >> 3;
    const uint64_t static_lenb = (T.w.static_len + 3 + 7) >> 3;
    if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
    if ((uint64_t)stored_len + 4 <= opt_lenb && buf_ok) return 0;
    if (static_lenb == opt_lenb) return 1;
    return 2;
}

// send_all_trees after the 3-bit block header of a dynamic block
template <class Put>
VD_HD inline void send_all_trees(const BlockTrees &T, int max_blindex, Put &put)
{
    const int lcodes = T.l.max_code + 1, dcodes = T.d.max_code + 1, blcodes = max_blindex + 1;
    put((uint32_t)(lcodes - 257), 5);
    put((uint32_t)(dcodes - 1), 5);
    put((uint32_t)(blcodes - 4), 4);
    for (int rank = 0; rank < blcodes; rank++) put(T.bl.len[bl_order(rank)], 3);
    send_tree(T.l, lcodes - 1, T.bl, put);
    send_tree(T.d, dcodes - 1, T.bl, put);
}

// Bits of one tallied symbol (compress_block): value LSB-first and its
// length (at most 15+5+15+13 = 48).  sym = dist << 8 | lc (dist 0 = literal lc).
VD_HD inline void symbol_bits(uint32_t sym, const uint16_t *lcode, const uint16_t *llen, const uint16_t *dcode,
                              const uint16_t *dlen, uint64_t &val, int &nbits)
{
    const uint32_t dist = sym >> 8, lc = sym & 0xff;
    if (dist == 0) {
        val = lcode[lc];
        nbits = llen[lc];
        return;
    }
    const int code = length_code((int)lc);
    uint64_t v = lcode[code + 257];
    int n = llen[code + 257];
    const int el = extra_lbits(code);
    if (el) {
        v |= (uint64_t)(lc - (uint32_t)base_length(code)) << n;
        n += el;
    }
    const uint32_t d = dist - 1;
    const int dc = dist_code((int)d);
    v |= (uint64_t)dcode[dc] << n;
    n += dlen[dc];
    const int ed = extra_dbits(dc);
    if (ed) {
        v |= (uint64_t)(d - (uint32_t)base_dist(dc)) << n;
        n += ed;
    }
    val = v;
    nbits = n;
}

// _tr_tally's frequency update (the symbol itself is stored by the caller)
VD_HD inline void tally(BlockTrees &T, uint32_t dist, uint32_t lc)
{
    if (dist == 0) {
        T.l.freq[lc]++;
    } else {
        T.l.freq[length_code((int)lc) + 257]++;
        T.d.freq[dist_code((int)(dist - 1))]++;
    }
}

// adler32 of n bytes from partial sums: s1 = 1 + sum b_i, s2 = n + sum (n-i) b_i
VD_HD inline uint32_t adler32_from_sums(uint64_t sum_b, uint64_t sum_wb, uint64_t n)
{
    const uint32_t s1 = (uint32_t)((1 + sum_b) % 65521u);
    const uint32_t s2 = (uint32_t)((n + sum_wb) % 65521u);
    return (s2 << 16) | s1;
}

// ---- deflate_slow ----------------------------------------------------------
// The parse, with the input wholly in the window (strips <= MAX_STRIP bytes:
// fill_window's first call reads all of it).  Ops supplies:
//   uint32_t head(p)                     most recent earlier position with p's hash (0 = NIL)
//   bool longest(p, head, prev_len, chain, nice, limit, &len, &pos)
//                                        longest_match's scan: true when a candidate longer
//                                        than prev_len was found (len = its length before
//                                        the lookahead clamp, pos = its position)
//   uint8_t byte(p)
//   void slide()                         fill_window's slide (window bytes past the end change)
//   bool tally(dist, lc)                 _tr_tally; true when lit_bufsize-1 symbols are buffered
//   void flush(stored_len, buf_ok, block_start, last)   _tr_flush_block
// Positions are input offsets throughout; zlib's window offsets differ from
// them by the slide, which every distance, TOO_FAR and limit test is invariant
// to -- except the NIL mapping of the head entry at input WSIZE, handled below.
template <class Ops>
VD_HD inline void deflate_slow(Ops &ops, uint32_t n, const Config &cfg)
{
    uint32_t strstart = 0, lookahead = n;
    uint32_t block_start = 0;
    uint32_t match_length = MIN_MATCH - 1, prev_length = MIN_MATCH - 1, match_start = 0, prev_match = 0;
    bool match_available = false, slid = false;
    auto flush_block = [&](bool last) {
        // block_start >= 0 in zlib's window offsets, i.e. not before the slid-out half
        const bool buf_ok = !slid || block_start >= (uint32_t)WSIZE;
        ops.flush(strstart - block_start, buf_ok, block_start, last);
        block_start = strstart;
    };
    for (;;) {
        if (lookahead < (uint32_t)MIN_LOOKAHEAD) {
            // fill_window: the input is all in; it only slides, once, at strstart >= wsize + MAX_DIST
            if (!slid && strstart >= (uint32_t)(WSIZE + MAX_DIST)) {
                slid = true;
                ops.slide();
            }
            if (lookahead == 0) break;
        }
        uint32_t hash_head = 0;
        if (lookahead >= (uint32_t)MIN_MATCH) hash_head = ops.head(strstart);
        // slide_hash maps every head entry m <= wsize (window offsets) to NIL:
        // input position WSIZE is window offset 0 after the slide, and is not
        // searched even though its distance from strstart = wsize + MAX_DIST
        // is exactly MAX_DIST (earlier entries are farther than MAX_DIST anyway)
        if (slid && hash_head <= (uint32_t)WSIZE) hash_head = 0;
        prev_length = match_length;
        prev_match = match_start;
        match_length = MIN_MATCH - 1;
        if (hash_head != 0 && prev_length < (uint32_t)cfg.lazy && strstart - hash_head <= (uint32_t)MAX_DIST) {
            uint32_t chain = (uint32_t)cfg.chain;
            if (prev_length >= (uint32_t)cfg.good) chain >>= 2;
            uint32_t nice = (uint32_t)cfg.nice;
            if (nice > lookahead) nice = lookahead;
            const uint32_t limit = strstart > (uint32_t)MAX_DIST ? strstart - MAX_DIST : 0;
            uint32_t best_len = prev_length, pos = 0;
            if (ops.longest(strstart, hash_head, prev_length, chain, nice, limit, best_len, pos)) match_start = pos;
            else best_len = prev_length;
            match_length = best_len <= lookahead ? best_len : lookahead;
            if (match_length <= 5 && match_length == (uint32_t)MIN_MATCH && strstart - match_start > (uint32_t)TOO_FAR)
                match_length = MIN_MATCH - 1;
        }
        if (prev_length >= (uint32_t)MIN_MATCH && match_length <= prev_length) {
            const bool bflush = ops.tally(strstart - 1 - prev_match, prev_length - MIN_MATCH);
            lookahead -= prev_length - 1;
            strstart += prev_length - 1;
            match_available = false;
            match_length = MIN_MATCH - 1;
            if (bflush) flush_block(false);
        } else if (match_available) {
            const bool bflush = ops.tally(0, ops.byte(strstart - 1));
            if (bflush) flush_block(false);
            strstart++;
            lookahead--;
        } else {
            match_available = true;
            strstart++;
            lookahead--;
        }
    }
    if (match_available) (void)ops.tally(0, ops.byte(strstart - 1));
    flush_block(true);
}

}  // namespace dfl
}  // namespace vcf
