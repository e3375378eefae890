// vcf_deflate.hip -- the reference's default entropy stage on the GPU: every
// TIFF strip deflated exactly as zlib.compress(strip, level) would
// (TIFF.py:29 -> tifffile.imwrite(..., compression='zlib') -> zlib level 6,
// one stream per RowsPerStrip strip; the host path is vcf_amd/codec/tiff.py).
//
// One wave (64 lanes, one workgroup) per strip; two strips per CU (76 KB LDS
// each).  Three phases per strip:
//   A  hash-chain order for all positions at once: every position 0..n-3 is
//      bucketed by its zlib hash, stably (histogram, scan, ordered scatter in
//      groups of 64 with an exact same-hash lane mask).  sorted[] lists the
//      positions bucket by bucket in increasing order, idx[p] is p's slot,
//      so zlib's chain of p -- earlier positions with p's hash, newest first --
//      is sorted[idx[p]-1], sorted[idx[p]-2], ... while the hash stays p's.
//   B  the strip is copied into LDS (the bytes past its end as zlib's window
//      holds them) and the wave runs deflate_slow (vcf_deflate.h) with
//      uniform state; longest_match evaluates the chain head with one
//      wave-wide 256-byte compare and, when that is not already a nice match,
//      up to 64 candidates at a time, one per lane.
//   C  per block: trees built by lane 0 (trees.c restated), the block and
//      tree headers written serially, the symbols packed in parallel (64 per
//      step: per-lane code bits, prefix sum of their lengths, LDS OR into
//      staging words, whole words stored).
// The wave ends with the adler32 trailer; sizes_dev[s] = the stream's length.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "vcf_amd.h"
#include "vcf_deflate.h"
#include "vcf_internal.h"

namespace vcf {
namespace {

using namespace dfl;

constexpr int kWinBytes = MAX_STRIP + 320;      // strip + the window bytes past its end
constexpr int kStgWords = 128;                  // staging for one 64-symbol step (<= 3072 + 31 bits)
constexpr int64_t kWsPerStrip = (int64_t)MAX_STRIP * 2 * 2 + (int64_t)LIT_BUFSIZE * 4;   // idx, sorted, symbols

struct DflSmem {
    union {
        uint32_t cnt[1 << 14];                  // phase A: 32768 u16 counters, packed in pairs
        uint32_t win32[kWinBytes / 4];          // phase B/C: the window
    } u;
    uint16_t lfreq[HEAP_SIZE], ldad[HEAP_SIZE], llen[HEAP_SIZE], lcode[L_CODES + 2];
    uint16_t dfreq[2 * D_CODES + 1], ddad[2 * D_CODES + 1], dlen[2 * D_CODES + 1], dcode[D_CODES + 2];
    uint16_t bfreq[2 * BL_CODES + 1], bdad[2 * BL_CODES + 1], blen[2 * BL_CODES + 1], bcode[BL_CODES + 2];
    int16_t heap[HEAP_SIZE];
    uint8_t depth[HEAP_SIZE];
    uint16_t bl_count[MAX_BITS + 1];
    uint32_t stg[kStgWords];
    uint32_t bcast[4];
};

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint32_t lane_val(uint32_t v, uint32_t l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)uni(l));
}
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_s_barrier();
}
__device__ __forceinline__ uint32_t excl_scan(uint32_t v, uint32_t &total)
{
    uint32_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, 64);
        if ((int)lane_id() >= d) incl += o;
    }
    total = (uint32_t)__shfl(incl, 63, 64);
    return incl - v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d, 64));
    return v;
}
template <class T>
__device__ __forceinline__ T ld_l2(const T *p)   // coherent with the other lanes' earlier stores (not via L1)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct Wave {
    DflSmem &sm;
    const uint8_t *src;
    uint32_t n;
    uint16_t *idx, *sorted;
    uint32_t *syms;
    uint32_t *out32;
    uint32_t out_words;           // slot capacity in words
    uint32_t bitpos = 0;          // bits written so far (uniform)
    uint32_t nsym = 0;            // symbols of the current block (uniform)
    uint32_t wbase = 0xffffffffu, idxw = 0;   // idx[wbase + lane]
    uint32_t last_ip = 0;
    bool overflow = false;
    BlockTrees T;

    __device__ Wave(DflSmem &s, const uint8_t *in, uint32_t len, uint16_t *ix, uint16_t *so, uint32_t *sy,
                    uint32_t *o, uint32_t ow)
        : sm(s), src(in), n(len), idx(ix), sorted(so), syms(sy), out32(o), out_words(ow)
    {
        T.l = {sm.lfreq, sm.ldad, sm.llen, sm.lcode, L_CODES, MAX_BITS, 0, 0};
        T.d = {sm.dfreq, sm.ddad, sm.dlen, sm.dcode, D_CODES, MAX_BITS, 1, 0};
        T.bl = {sm.bfreq, sm.bdad, sm.blen, sm.bcode, BL_CODES, MAX_BL_BITS, 2, 0};
        T.w.heap = sm.heap;
        T.w.depth = sm.depth;
        T.w.bl_count = sm.bl_count;
    }

    __device__ uint8_t *win() { return reinterpret_cast<uint8_t *>(sm.u.win32); }
    __device__ uint32_t wbyte(uint32_t p) { return win()[p]; }
    __device__ uint32_t hash_at(uint32_t p) { return ((wbyte(p) << 10) ^ (wbyte(p + 1) << 5) ^ wbyte(p + 2)) & 0x7fffu; }
    // 4 window bytes from any byte offset: two aligned LDS words and a funnel shift
    __device__ uint32_t ld4(uint32_t a)
    {
        const uint32_t w0 = sm.u.win32[a >> 2], w1 = sm.u.win32[(a >> 2) + 1];
        return __builtin_amdgcn_alignbyte(w1, w0, a & 3);
    }

    // ---- bit output ----------------------------------------------------
    __device__ void store_words(uint32_t first, uint32_t count)   // stg[0..count) -> out32[first..)
    {
        for (uint32_t i = lane_id(); i < count; i += 64) {
            if (first + i < out_words) out32[first + i] = sm.stg[i];
            else overflow = true;
        }
    }
    // every lane contributes nbits (<= 57) bits of val; lanes in order
    __device__ void emit_par(uint64_t val, uint32_t nbits)
    {
        uint32_t tot;
        const uint32_t off = excl_scan(nbits, tot);
        const uint32_t base_w = bitpos >> 5, pos = bitpos + off;
        const uint32_t li = (pos >> 5) - base_w, sh = pos & 31;
        if (nbits) {
            atomicOr(&sm.stg[li], (uint32_t)(val << sh));
            if (sh + nbits > 32) atomicOr(&sm.stg[li + 1], (uint32_t)(val >> (32 - sh)));
            if (sh + nbits > 64) atomicOr(&sm.stg[li + 2], (uint32_t)(val >> (64 - sh)));
        }
        wave_sync();
        const uint32_t end = bitpos + tot, nfull = (end >> 5) - base_w;
        if (nfull) {
            store_words(base_w, nfull);
            const uint32_t carry = sm.stg[nfull];
            wave_sync();
            for (uint32_t i = lane_id(); i <= nfull + 2 && i < (uint32_t)kStgWords; i += 64) sm.stg[i] = 0;
            wave_sync();
            if (lane_id() == 0) sm.stg[0] = carry;
            wave_sync();
        }
        bitpos = end;
    }
    // lane-0 serial writer over the same state (block and tree headers)
    struct Serial {
        Wave &w;
        uint64_t acc;
        uint32_t accbits, word;
        __device__ void operator()(uint32_t v, int nb)
        {
            acc |= (uint64_t)(v & ((1u << nb) - 1u)) << accbits;
            accbits += nb;
            if (accbits >= 32) {
                if (word < w.out_words) w.out32[word] = (uint32_t)acc;
                else w.overflow = true;
                ++word;
                acc >>= 32;
                accbits -= 32;
            }
        }
    };
    __device__ Serial serial_begin() { return Serial{*this, sm.stg[0], bitpos & 31, bitpos >> 5}; }
    __device__ void serial_end(const Serial &s)   // lane 0 publishes; all lanes pick up bitpos
    {
        sm.stg[0] = (uint32_t)s.acc;
        sm.bcast[0] = s.word * 32 + s.accbits;
    }
    __device__ void windup()   // bi_windup: to a byte boundary (the bits above are zero)
    {
        const uint32_t nb = (bitpos + 7) & ~7u;
        if ((nb >> 5) != (bitpos >> 5)) {   // the partial word became whole: store it, start a new one
            store_words(bitpos >> 5, 1);
            wave_sync();
            if (lane_id() == 0) sm.stg[0] = 0;
            wave_sync();
        }
        bitpos = nb;
    }

    // ---- deflate_slow's Ops ----------------------------------------------
    __device__ uint32_t byte(uint32_t p) { return wbyte(p); }
    __device__ uint32_t idx_at(uint32_t p)
    {
        const uint32_t b = p & ~63u;
        if (b != wbase) {
            wbase = b;
            const uint32_t q = b + lane_id();
            idxw = q < n ? ld_l2(idx + q) : 0u;
        }
        return lane_val(idxw, p - b);
    }
    __device__ uint32_t head(uint32_t p)
    {
        const uint32_t ip = idx_at(p);
        last_ip = ip;
        if (ip == 0) return 0;
        const uint32_t c = uni(ld_l2(sorted + (ip - 1)));
        return hash_at(c) == hash_at(p) ? c : 0u;
    }
    __device__ void slide()
    {
        for (uint32_t P = n + lane_id(); P < n + MAX_MATCH; P += 64) win()[P] = win()[P - WSIZE];
        wave_sync();
    }
    // common prefix of the strings at a and b, up to MAX_MATCH: one wave-wide compare
    __device__ uint32_t wave_lcp(uint32_t a, uint32_t b)
    {
        const uint32_t x = ld4(a + 4 * lane_id()) ^ ld4(b + 4 * lane_id());
        const uint64_t m = __ballot(x != 0);
        if (m) {
            const uint32_t f = (uint32_t)__ffsll((unsigned long long)m) - 1;
            return 4 * f + ((uint32_t)__builtin_ctz(lane_val(x, f)) >> 3);
        }
        uint32_t l = 256;
        if (wbyte(a + 256) == wbyte(b + 256)) l = wbyte(a + 257) == wbyte(b + 257) ? 258 : 257;
        return l;
    }
    __device__ uint32_t lane_lcp(uint32_t a, uint32_t b)
    {
        uint32_t l = 0;
        while (l < (uint32_t)MAX_MATCH) {
            const uint32_t x = ld4(a + l) ^ ld4(b + l);
            if (x) {
                l += (uint32_t)__builtin_ctz(x) >> 3;
                break;
            }
            l += 4;
        }
        return min(l, (uint32_t)MAX_MATCH);
    }
    // longest_match: the first candidate (chain order) reaching max(nice, prev_len+1),
    // else the first reaching the longest length found, if longer than prev_len
    __device__ bool longest(uint32_t p, uint32_t hd, uint32_t prev_len, uint32_t chain, uint32_t nice,
                            uint32_t limit, uint32_t &len, uint32_t &pos)
    {
        const uint32_t T = max(nice, prev_len + 1);
        const uint32_t l1 = wave_lcp(hd, p);
        if (l1 >= T) {
            len = l1;
            pos = hd;
            return true;
        }
        const uint32_t hp = hash_at(p), ip = last_ip;
        uint32_t best = prev_len, bpos = 0;
        bool found = false;
        for (uint32_t b = 0; b < chain; b += 64) {
            const uint32_t gk = b + lane_id();
            bool v = gk < chain && gk < ip;
            uint32_t c = v ? (uint32_t)ld_l2(sorted + (ip - 1 - gk)) : 0u;
            v = v && (gk == 0 || c > limit) && hash_at(c) == hp;
            const uint64_t stop = __ballot(!v);
            const uint32_t nv = stop ? (uint32_t)__ffsll((unsigned long long)stop) - 1 : 64u;
            v = lane_id() < nv;
            const uint32_t l = v ? (gk == 0 ? l1 : lane_lcp(c, p)) : 0u;
            const uint64_t hit = __ballot(v && l >= T);
            if (hit) {
                const uint32_t k = (uint32_t)__ffsll((unsigned long long)hit) - 1;
                len = lane_val(l, k);
                pos = lane_val(c, k);
                return true;
            }
            const uint32_t m = uni(wave_max(l));
            if (m > best) {
                const uint32_t k = (uint32_t)__ffsll((unsigned long long)__ballot(v && l == m)) - 1;
                best = m;
                bpos = lane_val(c, k);
                found = true;
            }
            if (nv < 64) break;
        }
        len = best;
        pos = bpos;
        return found;
    }
    __device__ bool tally(uint32_t dist, uint32_t lc)
    {
        if (lane_id() == 0) {
            syms[nsym] = dist << 8 | lc;
            dfl::tally(T, dist, lc);
        }
        ++nsym;
        return nsym == (uint32_t)LIT_BUFSIZE - 1;
    }
    __device__ void init_freqs()
    {
        for (uint32_t i = lane_id(); i < (uint32_t)L_CODES; i += 64) sm.lfreq[i] = i == END_BLOCK ? 1 : 0;
        if (lane_id() < (uint32_t)D_CODES) sm.dfreq[lane_id()] = 0;
        if (lane_id() < (uint32_t)BL_CODES) sm.bfreq[lane_id()] = 0;
        wave_sync();
    }
    __device__ void flush(uint32_t stored_len, bool buf_ok, uint32_t block_start, bool last)
    {
        __threadfence();   // the block's symbols (lane 0's stores) before the other lanes read them
        wave_sync();
        if (lane_id() == 0) {
            int max_blindex = 0;
            const int kind = plan_block(T, stored_len, buf_ok, max_blindex);
            Serial s = serial_begin();
            if (kind == 0) {
                s((last ? 1u : 0u), 3);
                if (s.accbits & 7) s(0, 8 - (s.accbits & 7));   // bi_windup
                s(stored_len & 0xffff, 16);
                s(~stored_len & 0xffff, 16);
            } else if (kind == 1) {
                s(2u + (last ? 1u : 0u), 3);
            } else {
                s(4u + (last ? 1u : 0u), 3);
                send_all_trees(T, max_blindex, s);
            }
            serial_end(s);
            sm.bcast[1] = (uint32_t)kind;
        }
        wave_sync();
        bitpos = uni(sm.bcast[0]);
        const uint32_t kind = uni(sm.bcast[1]);
        if (kind == 0) {
            for (uint32_t i = 0; i < stored_len; i += 64) {
                const uint32_t q = i + lane_id();
                emit_par(q < stored_len ? wbyte(block_start + q) : 0u, q < stored_len ? 8u : 0u);
            }
        } else {
            if (kind == 1) {
                for (uint32_t i = lane_id(); i < (uint32_t)L_CODES; i += 64) {
                    sm.lcode[i] = (uint16_t)static_lcode((int)i);
                    sm.llen[i] = (uint16_t)static_llen((int)i);
                }
                if (lane_id() < (uint32_t)D_CODES) {
                    sm.dcode[lane_id()] = (uint16_t)static_dcode((int)lane_id());
                    sm.dlen[lane_id()] = 5;
                }
                wave_sync();
            }
            for (uint32_t i = 0; i < nsym; i += 64) {
                const uint32_t q = i + lane_id();
                uint64_t v = 0;
                int nb = 0;
                if (q < nsym) symbol_bits(ld_l2(syms + q), sm.lcode, sm.llen, sm.dcode, sm.dlen, v, nb);
                emit_par(v, (uint32_t)nb);
            }
            emit_par(lane_id() == 0 ? sm.lcode[END_BLOCK] : 0u, lane_id() == 0 ? sm.llen[END_BLOCK] : 0u);
        }
        nsym = 0;
        init_freqs();
        if (last) windup();
    }
};

// Phase A: sorted[] / idx[] (the chains of every position) and the adler32 sums
__device__ void hash_order(DflSmem &sm, const uint8_t *src, uint32_t n, uint16_t *idx, uint16_t *sorted)
{
    const uint32_t lane = lane_id();
    for (uint32_t i = lane; i < (1u << 14); i += 64) sm.u.cnt[i] = 0;
    wave_sync();
    const uint32_t np = n >= 3 ? n - 2 : 0;   // positions 0..n-3 are inserted
    auto hash_g = [&](uint32_t p) {
        return (((uint32_t)src[p] << 10) ^ ((uint32_t)src[p + 1] << 5) ^ (uint32_t)src[p + 2]) & 0x7fffu;
    };
    for (uint32_t p = lane; p < np; p += 64) {
        const uint32_t h = hash_g(p);
        atomicAdd(&sm.u.cnt[h >> 1], 1u << ((h & 1) * 16));
    }
    wave_sync();
    // exclusive scan of the 32768 counters (each < 65536 in total: u16 starts)
    uint32_t s = 0;
    for (uint32_t i = 0; i < 256; ++i) {
        const uint32_t w = sm.u.cnt[lane * 256 + i];
        s += (w & 0xffffu) + (w >> 16);
    }
    uint32_t tot;
    uint32_t run = excl_scan(s, tot);
    for (uint32_t i = 0; i < 256; ++i) {
        const uint32_t w = sm.u.cnt[lane * 256 + i];
        const uint32_t c0 = w & 0xffffu, c1 = w >> 16;
        sm.u.cnt[lane * 256 + i] = run | ((run + c0) << 16);
        run += c0 + c1;
    }
    wave_sync();
    // ordered scatter, 64 positions at a time
    for (uint32_t p0 = 0; p0 < np; p0 += 64) {
        const uint32_t p = p0 + lane;
        const bool v = p < np;
        const uint32_t h = v ? hash_g(p) : 0u;
        uint64_t rem = __ballot(v), mine = 0;
        while (rem) {
            const uint32_t l = (uint32_t)__ffsll((unsigned long long)rem) - 1;
            const uint32_t hl = lane_val(h, l);
            const uint64_t m = __ballot(v && h == hl);
            if (v && h == hl) mine = m;
            rem &= ~m;
        }
        if (v) {
            const uint32_t rank = (uint32_t)__popcll(mine & ((1ull << lane) - 1));
            const uint32_t sh = (h & 1) * 16;
            const uint32_t slot = ((sm.u.cnt[h >> 1] >> sh) & 0xffffu) + rank;
            idx[p] = (uint16_t)slot;
            sorted[slot] = (uint16_t)p;
            if (rank == 0) atomicAdd(&sm.u.cnt[h >> 1], (uint32_t)__popcll(mine) << sh);
        }
        wave_sync();
    }
    __threadfence();
    wave_sync();
}

__global__ __launch_bounds__(64) void zlib_strips_kernel(const uint8_t *__restrict__ in, int64_t frame_bytes,
                                                        int32_t strip_bytes, int32_t spf, int32_t level,
                                                        uint8_t *__restrict__ out, int64_t slot_bytes,
                                                        int32_t *__restrict__ sizes, uint8_t *__restrict__ ws)
{
    __shared__ __attribute__((aligned(16))) DflSmem sm;
    const int64_t s = blockIdx.x;
    const int64_t f = s / spf, k = s - f * spf;
    const int64_t off = k * (int64_t)strip_bytes;
    const uint32_t n = (uint32_t)min((int64_t)strip_bytes, frame_bytes - off);
    const uint8_t *src = in + f * frame_bytes + off;
    uint8_t *w = ws + s * kWsPerStrip;
    uint16_t *idx = reinterpret_cast<uint16_t *>(w);
    uint16_t *sorted = idx + MAX_STRIP;
    uint32_t *syms = reinterpret_cast<uint32_t *>(sorted + MAX_STRIP);
    Config cfg;
    level_config(level, cfg);

    hash_order(sm, src, n, idx, sorted);

    // adler32 sums; the window: the strip, then zeros (fill_window's high_water zeroing)
    const uint32_t lane = lane_id();
    uint64_t sb = 0, swb = 0;
    uint8_t *win = reinterpret_cast<uint8_t *>(sm.u.win32);
    for (uint32_t p = lane; p < (uint32_t)kWinBytes; p += 64) {
        const uint32_t b = p < n ? src[p] : 0u;
        win[p] = (uint8_t)b;
        sb += b;
        swb += (uint64_t)(n - min(p, n)) * b;
    }
    for (int d = 32; d >= 1; d >>= 1) {
        sb += __shfl_xor(sb, d, 64);
        swb += __shfl_xor(swb, d, 64);
    }
    for (uint32_t i = lane; i < (uint32_t)kStgWords; i += 64) sm.stg[i] = 0;
    Wave wv(sm, src, n, idx, sorted, syms, reinterpret_cast<uint32_t *>(out + s * slot_bytes),
            (uint32_t)(slot_bytes >> 2));
    wv.init_freqs();   // includes the barrier for the window and the staging words

    const uint32_t hdr = zlib_header(level);
    wv.emit_par(lane == 0 ? ((hdr >> 8) | ((hdr & 0xffu) << 8)) : 0u, lane == 0 ? 16u : 0u);
    deflate_slow(wv, n, cfg);
    const uint32_t ad = adler32_from_sums(sb, swb, n);
    const uint32_t be = (ad >> 24) | ((ad >> 8) & 0xff00u) | ((ad << 8) & 0xff0000u) | (ad << 24);
    wv.emit_par(lane == 0 ? be : 0u, lane == 0 ? 32u : 0u);
    if (wv.bitpos & 31) wv.store_words(wv.bitpos >> 5, 1);
    const bool ovf = __ballot(wv.overflow) != 0;
    if (lane == 0) sizes[s] = ovf ? -1 : (int32_t)(wv.bitpos >> 3);
}

}  // namespace
}  // namespace vcf

using namespace vcf;

extern "C" {

int64_t vcf_zlib_bound(int64_t strip_bytes)
{
    if (strip_bytes < 0) return -1;
    // deflateBound's general formula (stored blocks worst case) + the zlib wrapper, in whole 16-B units
    const int64_t b = strip_bytes + ((strip_bytes + 7) >> 3) + ((strip_bytes + 63) >> 6) + 5 + 6;
    return (b + 15) / 16 * 16 + 16;
}

int64_t vcf_zlib_workspace(int64_t n_strips) { return n_strips < 0 ? -1 : n_strips * kWsPerStrip; }

int64_t vcf_zlib_strip_count(int64_t frame_bytes, int32_t strip_bytes)
{
    if (frame_bytes < 0 || strip_bytes <= 0) return -1;
    return frame_bytes == 0 ? 0 : (frame_bytes + strip_bytes - 1) / strip_bytes;
}

int vcf_zlib_strips(const uint8_t *in_dev, int64_t n_frames, int64_t frame_bytes, int32_t strip_bytes, int32_t level,
                    uint8_t *out_dev, int64_t slot_bytes, int32_t *sizes_dev, void *ws_dev, void *stream)
{
    if (!in_dev || !out_dev || !sizes_dev || !ws_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    if (n_frames < 0 || frame_bytes < 0) return set_error(VCF_ERR_INVALID, "negative count");
    if (strip_bytes <= 0 || strip_bytes > dfl::MAX_STRIP)
        return set_error(VCF_ERR_UNSUPPORTED, "strip of %d bytes: the GPU deflate takes strips of 1..%d bytes",
                         strip_bytes, dfl::MAX_STRIP);
    dfl::Config cfg;
    if (!dfl::level_config(level, cfg))
        return set_error(VCF_ERR_UNSUPPORTED, "zlib level %d: the GPU deflate implements levels 4-9 (deflate_slow)",
                         level);
    if (slot_bytes < vcf_zlib_bound(strip_bytes) || (slot_bytes & 3))
        return set_error(VCF_ERR_INVALID, "slot_bytes %lld: need a multiple of 4 >= vcf_zlib_bound(%d) = %lld",
                         (long long)slot_bytes, strip_bytes, (long long)vcf_zlib_bound(strip_bytes));
    if (((uintptr_t)out_dev & 3) || ((uintptr_t)ws_dev & 3) || ((uintptr_t)sizes_dev & 3))
        return set_error(VCF_ERR_INVALID, "out_dev, sizes_dev and ws_dev must be 4-byte aligned");
    if (n_frames == 0 || frame_bytes == 0) return VCF_OK;
    const int64_t spf = vcf_zlib_strip_count(frame_bytes, strip_bytes);
    const int64_t total = spf * n_frames;
    if (total > (int64_t)INT32_MAX) return set_error(VCF_ERR_INVALID, "too many strips");
    hipLaunchKernelGGL(zlib_strips_kernel, dim3((unsigned)total), dim3(64), 0, (hipStream_t)stream, in_dev,
                       frame_bytes, strip_bytes, (int32_t)spf, level, out_dev, slot_bytes, sizes_dev,
                       (uint8_t *)ws_dev);
    return hip_check(hipGetLastError(), "zlib_strips_kernel launch");
}

}  // extern "C"
