// vcf_inflate.hip -- the decode side of the reference's default entropy stage
// on the GPU: every TIFF strip inflated (TIFF.py:33-39 -> tifffile.imread ->
// zlib.decompress per strip), one wave per strip, straight into the index
// frames in HBM that the DCT decode reads.
//
// What is decoded is RFC 1950/1951 (zlib wrapper, stored / fixed / dynamic
// Huffman blocks), written from the format specification:
//   * the compressed strip is staged in a 4 KiB LDS ring (1 KiB chunks, loaded
//     coalesced ahead of the bit reader); the bit buffer is wave-uniform;
//   * a Huffman symbol is decoded without tables: canonical codes of length L
//     are the integers first[L] .. first[L] + count[L] - 1 (MSB-first), so lane
//     L (1..15) tests the next L bits (bit-reversed from the LSB-first stream)
//     against its own length's range, and the lowest lane that matches gives the
//     code length; the symbol is sorted[offs[L] + code - first[L]] (one LDS
//     read), symbols sorted by (length, value) when the tree is built;
//   * the output's last 32 KiB live in an LDS ring, so a match copy reads its
//     source there: lane i of a 64-byte round takes byte p - dist + (i mod dist)
//     (never the match's own output, so a round has no internal dependence);
//     completed 1 KiB chunks go to HBM with 16-byte stores;
//   * the adler32 trailer is checked (sums over the flushed bytes, reduced at
//     the end), and the output length against the strip's expected length.
// status[s] = 0, or a negative code for a stream that is not what zlib would
// accept (corrupt data, wrong length, adler mismatch, an over-subscribed or
// incomplete code-length set as inflate_table rejects it, a dynamic block
// without an end-of-block code, a negative strip length).
//
// Window-check diagnostic (VCF_INFLATE_WINCHECK_BUILD, compiled into the A/B
// library as vcf_inflate_strips_wincheck): every back-reference read and
// every flush read of the 32 KiB output ring is checked against the ring's
// valid span -- the byte was written (q < p + i) and not yet overwritten
// (p + i - q <= 32 KiB) -- and the violations are counted per strip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "vcf_amd.h"
#include "vcf_internal.h"

namespace vcf {
namespace {

constexpr uint32_t kOutRing = 32768, kOutMask = kOutRing - 1;
constexpr uint32_t kInRing = 4096, kInMask = kInRing - 1, kInChunk = 1024;

// RFC 1951 3.2.5: length codes 257..285 and distance codes 0..29
__constant__ uint16_t c_len_base[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                        31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_len_extra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dist_base[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                         193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dist_extra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
// order of the code length code lengths (3.2.7)
__constant__ uint8_t c_clen_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

enum : int32_t {
    kOk = 0,
    kErrHeader = -1,
    kErrBlock = -2,
    kErrCode = -3,
    kErrDistance = -4,
    kErrLength = -5,
    kErrAdler = -6,
    kErrInput = -7,
    kErrTree = -8,   // over-subscribed / incomplete code lengths (zlib: "invalid code lengths set" etc.)
    kErrEob = -9,    // dynamic block without a code for symbol 256 ("invalid code -- missing end-of-block")
    kErrArgs = -10,  // negative compressed or output length
};

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_s_barrier();
}

struct InflateSmem {
    uint8_t out[kOutRing];      // the last 32 KiB of output
    uint8_t in[kInRing];        // compressed bytes, a ring of 1 KiB chunks
    uint16_t sorted_ll[288];    // symbols by (code length, value): literal/length tree
    uint16_t sorted_d[32];      // distance tree
    uint16_t sorted_cl[19];     // code-length tree
    uint8_t lens[336];          // the code-length code's 19 lengths, then the 286 + 30 literal/length + distance lengths
    uint32_t cursor[16];        // per-length placement cursors of the tree build
};

// One canonical Huffman tree as the lanes hold it: lane L (1..15) keeps
// first[L], count[L] and offs[L]; the symbols in (length, value) order in LDS.
struct Tree {
    uint32_t first, count, offs;   // this lane's length
    uint16_t *sorted;
    bool ok;                       // inflate_table would accept the lengths
};

// inflate_table's checks (zlib inftrees.c): left = 1; left = 2 left - count[L]
// for L = 1..15, over-subscribed if it ever goes negative; an incomplete set
// (left > 0 at the end) is accepted only for the literal/length and distance
// trees with a single code of length 1 (max == 1), never for the code-length
// tree.  No code at all (max == 0) is accepted: decoding then fails on use.
enum TreeKind { kCodes, kLensOrDists };

struct Inflater {
    InflateSmem &sm;
    const uint8_t *src;
    uint32_t src_len;
    uint32_t staged = 0;       // bytes of src loaded into the ring
    uint32_t rpos = 0;         // next byte of src the bit buffer takes
    uint64_t bb = 0;           // bit buffer (LSB first), uniform
    uint32_t nb = 0;           // bits in it
    bool bad_input = false;

    __device__ Inflater(InflateSmem &s, const uint8_t *in, uint32_t n) : sm(s), src(in), src_len(n) {}

    // load source chunk [staged, staged + kInChunk) into the ring (16 B per lane)
    __device__ __forceinline__ void stage_chunk()
    {
        const uint32_t base = staged, o = 16 * lane_id();
        uint8_t b[16];
        if (base + o + 16 <= src_len && (((uintptr_t)(src + base + o)) & 3) == 0) {
            const uint4 v = *reinterpret_cast<const uint4 *>(src + base + o);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int i = 0; i < 16; ++i) b[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) b[i] = base + o + i < src_len ? src[base + o + i] : 0u;
        }
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = b[4 * i] | b[4 * i + 1] << 8 | b[4 * i + 2] << 16 | (uint32_t)b[4 * i + 3] << 24;
        *reinterpret_cast<uint4 *>(sm.in + ((base + o) & kInMask)) = make_uint4(w[0], w[1], w[2], w[3]);
        staged = base + kInChunk;
    }
    __device__ __forceinline__ void refill()   // at least 32 bits in the buffer
    {
        if (nb >= 32) return;
        // keep two chunks staged ahead of the reader (the ring holds four)
        while (staged < rpos + 2 * kInChunk && staged < src_len + kInChunk) {
            stage_chunk();
            wave_sync();
        }
        const uint32_t *w32 = reinterpret_cast<const uint32_t *>(sm.in);
        const uint32_t a = rpos & kInMask;
        const uint32_t lo = w32[a >> 2], hi = w32[((a >> 2) + 1) & (kInMask >> 2)];
        const uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, a & 3);
        bb |= (uint64_t)v << nb;
        nb += 32;
        rpos += 4;
        if (rpos > src_len + 8) bad_input = true;   // ran past the stream (corrupt data)
    }
    __device__ __forceinline__ uint32_t bits(uint32_t n)   // n <= 32
    {
        refill();
        const uint32_t v = (uint32_t)bb & (n == 32 ? 0xffffffffu : ((1u << n) - 1u));
        bb >>= n;
        nb -= n;
        return v;
    }
    __device__ __forceinline__ void align_byte()
    {
        const uint32_t k = nb & 7;
        bb >>= k;
        nb -= k;
    }
    // bytes of src consumed so far (the bit buffer holds whole bytes after align_byte)
    __device__ __forceinline__ uint32_t byte_pos() const { return rpos - nb / 8; }

    // build a tree from code lengths lens[0..n) (LDS, uniform n <= 288)
    __device__ __forceinline__ Tree build(const uint8_t *lens, uint32_t n, uint16_t *sorted, TreeKind kind)
    {
        const uint32_t lane = lane_id();
        if (lane < 16) sm.cursor[lane] = 0;
        wave_sync();
        for (uint32_t s = lane; s < n; s += 64)
            if (lens[s]) atomicAdd(&sm.cursor[lens[s]], 1u);
        wave_sync();
        // lane L: count[L]; canonical first code and symbol offset by a scan over lengths
        const uint32_t cnt = lane >= 1 && lane <= 15 ? sm.cursor[lane] : 0u;
        uint32_t off = cnt;
        // exclusive prefix sum of the counts (offsets), and the canonical first codes
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const uint32_t o = __shfl_up(off, d, 64);
            if ((int)lane >= d) off += o;
        }
        off -= cnt;
        // first[L] = (first[L-1] + count[L-1]) << 1, first[1] = 0: serial over 15 lengths
        uint32_t fl = 0, f = 0, c_prev = 0, maxlen = 0;
        int32_t left = 1;
        bool over = false;
        for (uint32_t L = 1; L <= 15; ++L) {
            const uint32_t cL = (uint32_t)__shfl((int)cnt, (int)L, 64);
            f = (f + c_prev) << 1;
            if (lane == L) fl = f;
            c_prev = cL;
            left = 2 * left - (int32_t)cL;
            over = over || left < 0;
            if (cL) maxlen = L;
        }
        const bool incomplete = maxlen != 0 && left > 0 && (kind == kCodes || maxlen != 1);
        Tree t{fl, cnt, off, sorted, !over && !incomplete};
        wave_sync();
        if (lane >= 1 && lane <= 15) sm.cursor[lane] = off;
        wave_sync();
        // symbols in value order within a length: 64 at a time, rank among the group's lanes of the same length
        for (uint32_t s0 = 0; s0 < n; s0 += 64) {
            const uint32_t s = s0 + lane;
            const uint32_t L = s < n ? lens[s] : 0u;
            uint64_t same = __ballot(s < n);
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint64_t m = __ballot(s < n && ((L >> b) & 1));
                same &= ((L >> b) & 1) ? m : ~m;
            }
            const uint32_t rank = (uint32_t)__popcll(same & ((1ull << lane) - 1));
            const uint32_t base = L ? sm.cursor[L] : 0u;
            wave_sync();
            if (s < n && L) {
                sorted[base + rank] = (uint16_t)s;
                if (((same >> lane) >> 1) == 0) sm.cursor[L] = base + rank + 1;   // the group's last of length L
            }
            wave_sync();
        }
        return t;
    }
    // decode one symbol (uniform); returns 0xffff on an invalid code
    __device__ __forceinline__ uint32_t decode(const Tree &t)
    {
        refill();
        const uint32_t lane = lane_id();
        const uint32_t rev = __builtin_bitreverse32((uint32_t)bb) >> 17;   // the next 15 stream bits, MSB first
        const uint32_t c = rev >> (15 - (lane & 15));
        const bool ok = lane >= 1 && lane <= 15 && c - t.first < t.count;
        const uint64_t m = __ballot(ok);
        if (!m) return 0xffffu;
        const uint32_t L = (uint32_t)__ffsll((unsigned long long)m) - 1;
        const uint32_t idx = uni(__shfl((int)(t.offs + c - t.first), (int)L, 64));
        bb >>= L;
        nb -= L;
        return t.sorted[idx];
    }
};

template <bool WC>
__global__ __launch_bounds__(64) void inflate_kernel(const uint8_t *__restrict__ comp, const int64_t *__restrict__ comp_off,
                                                    const int32_t *__restrict__ comp_len, uint8_t *__restrict__ out,
                                                    const int64_t *__restrict__ out_off,
                                                    const int32_t *__restrict__ out_len, int32_t *__restrict__ status,
                                                    uint32_t *__restrict__ viol)
{
    __shared__ __attribute__((aligned(16))) InflateSmem sm;
    const uint32_t s = blockIdx.x, lane = lane_id();
    if (comp_len[s] < 0 || out_len[s] < 0) {   // nothing is read or written for such a strip
        if (lane == 0) status[s] = kErrArgs;
        if (WC && lane == 0) viol[s] = 0;
        return;
    }
    const uint32_t n_in = (uint32_t)comp_len[s], n_out = (uint32_t)out_len[s];
    uint8_t *dst = out + out_off[s];
    Inflater in(sm, comp + comp_off[s], n_in);
    int32_t err = kOk;
    uint32_t p = 0, flushed = 0;
    uint32_t nviol = 0;        // WC: ring reads outside the valid span (this lane's count)
    uint64_t s1 = 0, s2 = 0;   // this lane's adler terms: sum b, sum i*b over flushed bytes
    auto flush = [&](uint32_t upto) {   // output [flushed, upto) from the ring to HBM (upto - flushed <= 32 KiB)
        upto = min(upto, n_out);
        // WC: every byte still to flush must be in the ring (written, not overwritten)
        if (WC && (upto > p || p - flushed > kOutRing)) ++nviol;
        while (flushed < upto) {
            const uint32_t end = min(upto, (flushed & ~(kInChunk - 1)) + kInChunk);
            const uint32_t o = flushed + 16 * lane;
            if (o < end) {
                uint8_t b[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) b[i] = sm.out[(o + i) & kOutMask];
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (o + i < end) {
                        s1 += b[i];
                        s2 += (uint64_t)(o + i) * b[i];
                    }
                if (o + 16 <= end && (((uintptr_t)(dst + o)) & 15) == 0) {
                    uint32_t w[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        w[i] = b[4 * i] | b[4 * i + 1] << 8 | b[4 * i + 2] << 16 | (uint32_t)b[4 * i + 3] << 24;
                    *reinterpret_cast<uint4 *>(dst + o) = make_uint4(w[0], w[1], w[2], w[3]);
                } else {
                    for (int i = 0; i < 16; ++i)
                        if (o + i < end) dst[o + i] = b[i];
                }
            }
            flushed = end;
        }
    };
    // zlib header (RFC 1950): CM 8, CINFO <= 7, no preset dictionary, FCHECK
    {
        const uint32_t cmf = in.bits(8), flg = in.bits(8);
        if ((cmf & 15) != 8 || (cmf >> 4) > 7 || (flg & 0x20) || ((cmf << 8) | flg) % 31 != 0) err = kErrHeader;
    }
    bool last = false;
    while (err == kOk && !last) {
        last = in.bits(1) != 0;
        const uint32_t type = in.bits(2);
        if (type == 0) {   // stored
            in.align_byte();
            const uint32_t len = in.bits(16), nlen = in.bits(16);
            if ((len ^ 0xffffu) != nlen) {
                err = kErrBlock;
                break;
            }
            for (uint32_t i = 0; i < len; ++i) {   // byte at a time through the bit buffer (stored blocks are rare here)
                const uint32_t v = in.bits(8);
                if (lane == 0) sm.out[p & kOutMask] = (uint8_t)v;
                ++p;
                if (p - flushed >= kInChunk) {
                    wave_sync();
                    flush(p & ~(kInChunk - 1));
                }
            }
        } else if (type == 1 || type == 2) {
            Tree tl, td;
            if (type == 1) {   // fixed trees (3.2.6)
                for (uint32_t i = lane; i < 318; i += 64)
                    sm.lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : i < 288 ? 8 : 5;
                wave_sync();
                tl = in.build(sm.lens, 288, sm.sorted_ll, kLensOrDists);
                td = in.build(sm.lens + 288, 30, sm.sorted_d, kLensOrDists);
            } else {   // dynamic trees (3.2.7)
                const uint32_t hlit = in.bits(5) + 257, hdist = in.bits(5) + 1, hclen = in.bits(4) + 4;
                if (hlit > 286 || hdist > 30) {
                    err = kErrBlock;
                    break;
                }
                if (lane < 19) sm.lens[lane] = 0;
                wave_sync();
                for (uint32_t i = 0; i < hclen; ++i) {
                    const uint32_t v = in.bits(3);
                    if (lane == 0) sm.lens[c_clen_order[i]] = (uint8_t)v;
                }
                wave_sync();
                const Tree tc = in.build(sm.lens, 19, sm.sorted_cl, kCodes);
                if (!tc.ok) {
                    err = kErrTree;
                    break;
                }
                uint32_t k = 0, prev = 0;
                uint8_t *ln = sm.lens + 19;   // the decoded lengths land after the 19 code-length lengths
                while (k < hlit + hdist) {
                    const uint32_t sym = in.decode(tc);
                    uint32_t rep = 1, val = 0;
                    if (sym < 16) {
                        val = prev = sym;
                    } else if (sym == 16) {
                        if (k == 0) {
                            err = kErrBlock;
                            break;
                        }
                        rep = 3 + in.bits(2);
                        val = prev;
                    } else if (sym == 17) {
                        rep = 3 + in.bits(3);
                        prev = 0;
                    } else if (sym == 18) {
                        rep = 11 + in.bits(7);
                        prev = 0;
                    } else {
                        err = kErrCode;
                        break;
                    }
                    if (k + rep > hlit + hdist) {
                        err = kErrBlock;
                        break;
                    }
                    for (uint32_t i = lane; i < rep; i += 64) ln[k + i] = (uint8_t)val;
                    k += rep;
                    wave_sync();
                }
                if (err != kOk) break;
                if (ln[256] == 0) {
                    err = kErrEob;
                    break;
                }
                tl = in.build(ln, hlit, sm.sorted_ll, kLensOrDists);
                td = in.build(ln + hlit, hdist, sm.sorted_d, kLensOrDists);
                if (!tl.ok || !td.ok) {
                    err = kErrTree;
                    break;
                }
            }
            // the block's symbols
            for (;;) {
                const uint32_t sym = in.decode(tl);
                if (sym < 256) {
                    if (lane == 0) sm.out[p & kOutMask] = (uint8_t)sym;
                    ++p;
                } else if (sym == 256) {
                    break;
                } else if (sym <= 285) {
                    const uint32_t li = sym - 257;
                    const uint32_t len = c_len_base[li] + in.bits(c_len_extra[li]);
                    const uint32_t ds = in.decode(td);
                    if (ds >= 30) {
                        err = kErrCode;
                        break;
                    }
                    const uint32_t dist = c_dist_base[ds] + in.bits(c_dist_extra[ds]);
                    if (dist > p) {
                        err = kErrDistance;
                        break;
                    }
                    wave_sync();   // the literals before the match are in the ring
                    for (uint32_t r = 0; r < len; r += 64) {
                        const uint32_t i = r + lane;
                        uint8_t v = 0;
                        if (i < len) {
                            const uint32_t q = p - dist + (i % dist);
                            // WC: q was written (q < p + i) and its slot not yet reused (p + i - q <= 32 KiB)
                            if (WC && (q >= p + i || p + i - q > kOutRing)) ++nviol;
                            v = sm.out[q & kOutMask];
                        }
                        if (i < len) sm.out[(p + i) & kOutMask] = v;
                    }
                    p += len;
                    wave_sync();
                } else {
                    err = kErrCode;
                    break;
                }
                if (p > n_out) {
                    err = kErrLength;
                    break;
                }
                if (in.bad_input) {
                    err = kErrInput;
                    break;
                }
                if (p - flushed >= 2 * kInChunk) {
                    wave_sync();
                    flush(p & ~(kInChunk - 1));
                }
            }
        } else {
            err = kErrBlock;
        }
        if (in.bad_input && err == kOk) err = kErrInput;
    }
    if (err == kOk && p != n_out) err = kErrLength;
    wave_sync();
    flush(p);
    if (err == kOk) {   // adler32 trailer, big-endian, after the byte-aligned end of the deflate data
        in.align_byte();
        const uint32_t t = in.bits(8) << 24 | in.bits(8) << 16 | in.bits(8) << 8 | in.bits(8);
        for (int d = 32; d >= 1; d >>= 1) {
            s1 += __shfl_xor(s1, d, 64);
            s2 += __shfl_xor(s2, d, 64);
        }
        // s1 = 1 + sum b, s2 = n + sum (n - i) b_i  (mod 65521)
        const uint64_t sb = s1, sib = s2, nn = n_out;
        const uint32_t a1 = (uint32_t)((1 + sb) % 65521u);
        const uint32_t a2 = (uint32_t)((nn % 65521u + (nn % 65521u) * (sb % 65521u) % 65521u + 65521u -
                                        sib % 65521u) % 65521u);
        if (((a2 << 16) | a1) != t) err = kErrAdler;
        if (in.byte_pos() > n_in) err = kErrInput;
    }
    if (lane == 0) status[s] = err;
    if (WC) {
        for (int d = 32; d >= 1; d >>= 1) nviol += __shfl_xor(nviol, d, 64);
        if (lane == 0) viol[s] = nviol;
    }
}

template <bool WC>
int launch_inflate(const uint8_t *comp_dev, const int64_t *comp_off_dev, const int32_t *comp_len_dev, int64_t n_strips,
                   uint8_t *out_dev, const int64_t *out_off_dev, const int32_t *out_len_dev, int32_t *status_dev,
                   uint32_t *viol_dev, void *stream)
{
    if (n_strips < 0) return set_error(VCF_ERR_INVALID, "n_strips < 0");
    if (n_strips == 0) return VCF_OK;
    if (!comp_dev || !comp_off_dev || !comp_len_dev || !out_dev || !out_off_dev || !out_len_dev || !status_dev)
        return set_error(VCF_ERR_INVALID, "null buffer");
    for (int64_t s0 = 0; s0 < n_strips; s0 += 65535) {
        const unsigned cnt = (unsigned)std::min<int64_t>(65535, n_strips - s0);
        hipLaunchKernelGGL(inflate_kernel<WC>, dim3(cnt), dim3(64), 0, (hipStream_t)stream, comp_dev,
                           comp_off_dev + s0, comp_len_dev + s0, out_dev, out_off_dev + s0, out_len_dev + s0,
                           status_dev + s0, WC ? viol_dev + s0 : nullptr);
        const int rc = hip_check(hipGetLastError(), "inflate_kernel launch");
        if (rc != VCF_OK) return rc;
    }
    return VCF_OK;
}

}  // namespace
}  // namespace vcf

using namespace vcf;

extern "C" {

#ifndef VCF_INFLATE_WINCHECK_BUILD
int vcf_inflate_strips(const uint8_t *comp_dev, const int64_t *comp_off_dev, const int32_t *comp_len_dev,
                       int64_t n_strips, uint8_t *out_dev, const int64_t *out_off_dev, const int32_t *out_len_dev,
                       int32_t *status_dev, void *stream)
{
    return launch_inflate<false>(comp_dev, comp_off_dev, comp_len_dev, n_strips, out_dev, out_off_dev, out_len_dev,
                                 status_dev, nullptr, stream);
}
#else
// the diagnostic build (csrc/ab/vcf_inflate_wincheck.hip, include/vcf_amd_ab.h)
int vcf_inflate_strips_wincheck(const uint8_t *comp_dev, const int64_t *comp_off_dev, const int32_t *comp_len_dev,
                                int64_t n_strips, uint8_t *out_dev, const int64_t *out_off_dev,
                                const int32_t *out_len_dev, int32_t *status_dev, uint32_t *viol_dev, void *stream)
{
    if (!viol_dev) return set_error(VCF_ERR_INVALID, "null violation counter buffer");
    return launch_inflate<true>(comp_dev, comp_off_dev, comp_len_dev, n_strips, out_dev, out_off_dev, out_len_dev,
                                status_dev, viol_dev, stream);
}
#endif

}  // extern "C"
