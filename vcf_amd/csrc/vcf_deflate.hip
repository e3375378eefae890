// vcf_deflate.hip -- the reference's default entropy stage on the GPU: every
// TIFF strip deflated exactly as zlib.compress(strip, level) would
// (TIFF.py:29 -> tifffile.imwrite(..., compression='zlib') -> zlib level 6,
// one stream per RowsPerStrip strip; the host path is vcf_amd/codec/tiff.py).
//
// zlib's serial loop is split where its data dependences allow (DESIGN.md
// §4.9; the restatement and its proofs of equivalence are vcf_deflate.h):
//   K1 zlib_sort_kernel, eight waves per strip: the positions 0..n-3 sorted
//      by zlib's hash, stably (two counting passes over 8 + 7 hash bits, the
//      strip's tiles split between the waves).  zlib inserts every position,
//      in order, and a position's hash depends on its 3 bytes only, so the
//      hash chains do not depend on the parse: the chain of p is the earlier
//      positions of p's bucket, newest first -- contiguous in sorted[].  Also
//      hd[p], the chain's head (zlib's head[] as p is inserted), and the
//      adler32 sums.
//   K2 zlib_match_kernel, 16 consecutive positions per thread, 4096 per
//      workgroup: longest_match at p for both chain limits deflate_slow can
//      use (max_chain, and max_chain >> 2 once prev_length >= good_match).
//      Every call whose result can matter has the early-exit threshold
//      min(nice, lookahead), independent of prev_length (vcf_deflate.h), so
//      two (length, distance) pairs per position carry all of it; "found" is
//      length > prev_length, decided in K3.  K2a resolves a position from
//      its chain head alone when that is exact (a nice match, or inside a
//      run of one byte value reaching max_chain back) and lists the others;
//      K2b walks the listed chains, one position per wave, 64 candidates
//      from sorted[] per step, zlib's scan_end test before a full compare.
//      The window (32 KB back + the span, K2b the whole strip) in LDS, the
//      bytes past the strip's end as zlib's window holds them (zeros, or
//      after its one slide the stale copy 32 KB back).
//   K3 zlib_parse_kernel, one wave per strip: deflate_slow with uniform state
//      over 512-position register windows of hd[], the K2 results and the
//      bytes; per block the trees built by lane 0 (trees.c restated), the
//      block and tree headers written serially, the symbols packed 64 at a
//      time (per-lane code bits, prefix sum of their lengths, LDS OR into
//      staging words, whole words stored); the adler32 trailer.
// sizes_dev[s] = the stream's length.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <type_traits>

#include "vcf_amd.h"
#include "vcf_deflate.h"
#include "vcf_internal.h"
#include "vcf_pipeline.h"

namespace vcf {
namespace {

using namespace dfl;

constexpr int kStgWords = 128;       // bit staging for one 64-symbol step (<= 3072 + 31 bits)
constexpr int kK2Threads = 256;
constexpr int kPer = 16;             // K2: consecutive positions per thread
constexpr int kChunk = kK2Threads * kPer;                 // K2: positions per workgroup
constexpr int kK2Win = WSIZE + kChunk + MAX_MATCH + 64;   // K2's LDS window
// workspace per strip: idx (u16; K2 turns it into hd, zlib's head[] per position),
// sorted (u16), hd (u16), K2's worklist (u16), full- and reduced-chain results (u32),
// symbols (u32), adler sums
constexpr int64_t kIdxOff = 0;
constexpr int64_t kSortOff = kIdxOff + (int64_t)MAX_STRIP * 2;
constexpr int64_t kHdOff = kSortOff + (int64_t)MAX_STRIP * 2;
constexpr int64_t kListOff = kHdOff + (int64_t)MAX_STRIP * 2;
constexpr int64_t kRfOff = kListOff + (int64_t)MAX_STRIP * 2;
constexpr int64_t kRrOff = kRfOff + (int64_t)MAX_STRIP * 4;
constexpr int64_t kSymOff = kRrOff + (int64_t)MAX_STRIP * 4;
// adler sums (2 x u64), K2's worklist length, the parse order (lazy or not), K1's distinct-hash
// count, the lazy parse's dispatch order, the round's list of non-lazy strips (entry i in slot
// i), their count (slot 0) (u32 each)
constexpr int64_t kSumOff = kSymOff + (int64_t)LIT_BUFSIZE * 4;
constexpr int64_t kWsPerStrip = kSumOff + 48;
// Rounds: the strips of a call are processed in rounds whose workspace stays
// under the budget, one round after the other on the caller's stream.  Every
// round ends in a tail (the last strips' serial parses on a draining GPU), so
// fewer, larger rounds are faster: the budget is a quarter of the device memory
// that is free when the library first sizes it (MI355X with the bench's buffers
// resident: 40 GB, C4's 25 344 strips in one round, 317 -> 245 ms against round
// 4's fixed 3.9 GB), at least 3.9 GB and at most 40 GB.  It is fixed per device
// on first use, so vcf_zlib_workspace and vcf_zlib_strips agree; a caller that
// cannot hold it sets a smaller one with vcf_zlib_set_workspace_budget (the
// strips then run in more rounds) and asks vcf_zlib_workspace again.  (Rounds
// in flight on library streams, each with its own workspace slot, measured
// slower -- 517 vs 453 ms for C4 -- and produced a wrong strip now and then on
// MI355X)
constexpr int64_t kWsBudget = 3900000000LL, kWsBudgetMax = 40000000000LL;
constexpr int kMaxDevices = 64;
std::atomic<int64_t> g_ws_override[kMaxDevices];   // > 0: the caller's budget (vcf_zlib_set_workspace_budget)
inline int current_device()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) dev = 0;
    return dev;
}
// the budget in effect on the current device (VCF_ZX_BUDGET bytes overrides the
// default: A/B of the round size); thread-safe, computed once per device
inline int64_t ws_budget()
{
    const int dev = current_device();
    const int64_t o = g_ws_override[dev].load(std::memory_order_relaxed);
    if (o > 0) return o;
    static std::once_flag once[kMaxDevices];
    static int64_t dflt[kMaxDevices];
    std::call_once(once[dev], [dev] {
        int64_t v = kWsBudget;
        size_t free_b = 0, total = 0;
        if (hipMemGetInfo(&free_b, &total) == hipSuccess)
            v = std::min(kWsBudgetMax, std::max(kWsBudget, (int64_t)(free_b / 4)));
        const char *e = getenv("VCF_ZX_BUDGET");
        dflt[dev] = e && atoll(e) > 0 ? atoll(e) : v;
    });
    return dflt[dev];
}
// A call's strips in rounds of `per` strips (at most 65535: the y grid dimension of
// the K2a launch), the workspace of one round within the budget.
struct ZRounds {
    int64_t rounds, per;
    explicit ZRounds(int64_t total)
    {
        const int64_t round_max = std::min<int64_t>(65535, std::max<int64_t>(1, ws_budget() / kWsPerStrip));
        rounds = std::max<int64_t>(1, (total + round_max - 1) / round_max);
        per = std::max<int64_t>(1, (total + rounds - 1) / rounds);
    }
};
constexpr int kK2bThreads = 1024;    // K2b: 16 waves per strip, one listed position per wave at a time
#ifndef VCF_ZX_K2BSPLIT   // A/B (diagnostic builds): K2b workgroups per strip
#define VCF_ZX_K2BSPLIT 4
#endif
constexpr int kK2bSplit = VCF_ZX_K2BSPLIT;   // K2b: workgroups per strip, the listed positions split between them
// A strip is parsed LAZY (on demand, zlib's order of work) when K1 finds fewer than
// one distinct hash per kLazyDiv positions among its 64-position groups: such
// repetitive content leaves most positions inside long matches, which zlib -- and
// the lazy parse -- never search, while K2 would search them all.  Both orders
// produce the same bytes; only the time differs.  kLazyDiv 2
// (round 4: 4) sends C4's borderline strips -- 3 % of them -- to the lazy parse
// too: its side stream of K2a/K2b/K3 no longer competes with the lazy parse for
// the CUs (C4 deflate 160 -> 107 ms), and raw RGB strips still take K2 (561 ms
// either way; every strip lazy: 864 ms).
#ifndef VCF_ZX_LAZYDIV   // A/B (diagnostic builds)
#define VCF_ZX_LAZYDIV 2
#endif
constexpr uint32_t kLazyDiv = VCF_ZX_LAZYDIV;

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

#ifndef VCF_ZLIB_PROF
#define VCF_ZLIB_PROF 0
#endif
#ifndef VCF_ZX_NOCAP   // A/B (diagnostic builds): lane compares run on to MAX_MATCH
#define VCF_ZX_NOCAP 0
#endif
#ifndef VCF_ZX_NOPRIO   // A/B (diagnostic builds): the side stream at normal priority
#define VCF_ZX_NOPRIO 0
#endif
#ifndef VCF_ZX_COHERENT   // A/B (diagnostic builds): agent-scope loads of the K1 / head tables in the lazy parse
#define VCF_ZX_COHERENT 0
#endif
#ifndef VCF_ZX_WINCHECK   // (diagnostic) the lazy window checked against the strip at every call
#define VCF_ZX_WINCHECK 0
#endif
#if VCF_ZX_WINCHECK
// first failure: [0] 1 + kind (1: window at p, 2: window at a candidate), [1] strip, [2] p,
// [3] position, [4] window byte, [5] strip byte, [6] wbase, [7] count of failures
__device__ unsigned int g_zdbg[8];
#endif
#ifndef VCF_ZX_LDSZERO
#define VCF_ZX_LDSZERO 0
#endif
#ifndef VCF_ZX_EARLY0   // A/B (diagnostic builds): round 0's candidate reads before the head compare
// (round 6: 0 -- the head compare no longer waits for the candidate list and the far
// candidates' bytes, and round 0's far reads share one round trip with its scan_end
// bytes: C4 deflate 102.3 -> 97.2 ms, ABBA, profiles/r06_zab_v2.json)
#define VCF_ZX_EARLY0 0
#endif
#ifndef VCF_ZX_PREDICT   // A/B (diagnostic builds): prefetch the exactly predicted next call position
// (round 6: 1 -- 70 % -> 93 % of the calls find their candidates prefetched; C4 deflate
// 101.3 -> 95.3 ms, ABBA, profiles/r06_zab_v3.json; 2: also p + 1, 98.4 ms)
#define VCF_ZX_PREDICT 1
#endif
#ifndef VCF_ZX_SERIAL   // A/B (diagnostic builds): every kernel of a round on the caller's stream
#define VCF_ZX_SERIAL 0
#endif
#if VCF_ZLIB_PROF
// diagnostic build only (scripts/zprof_build.sh): per-phase clock totals of the parse kernels
// [0] lazy total, [1] lazy longest, [2] lazy flush, [3] longest calls, [4] chain rounds,
// [5] window shifts, [6] lazy strips, [7] K3 (non-lazy) total, [8] lazy longest up to the end
// of the head compare, [9] lane compare steps (the wave's maximum per round), [10] candidates
// passing the scan_end test, [11] calls served by the prefetch, [12] cycles then waiting for
// the first two rounds' candidates, [13..15] chain-round cycles: to the chain ballot, to the
// lengths, the rest (rounds that end the call with a hit excluded from [15])
// [16] calls ending at the head compare, [17] chain rounds holding a far lane, [18] lanes entering
// far_lcp, [19] far wave_lcp_at calls, [20] calls whose chain head is far, [21] calls finding nothing
// [40..45] K1's phases (thread 0's clock at the barriers): pass-1 counts, scan, pass-1
// placement, scan, pass-2 placement, the tiles' first elements; [47] K1 workgroups
__device__ unsigned long long g_zprof[48];
#define VCF_ZPROF_COUNT(x) (++(x))
#else
#define VCF_ZPROF_COUNT(x) ((void)0)
#endif
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint32_t lane_val(uint32_t v, uint32_t l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)uni(l));
}
// The parse kernels' workgroups hold VCF_ZX_WG waves, one strip each, every wave with
// its own LDS section and no data shared between them: a wave's LDS writes and reads
// need only the ordering of its own instructions (the LDS serves one wave's DS
// instructions in order) and the fence's wait counts -- no workgroup barrier, which
// would tie the waves' independent control flows together.
#ifndef VCF_ZX_WG   // A/B (diagnostic builds): strips (waves) per parse workgroup
#define VCF_ZX_WG 1
#endif
constexpr int kParseWG = VCF_ZX_WG;
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    if (kParseWG == 1) __builtin_amdgcn_s_barrier();
    else __builtin_amdgcn_wave_barrier();
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
// Data a wave stores and later reads back in the same kernel (the parse's symbol
// buffer) goes through agent-scope accesses on both sides.  An agent-scope load
// must see other XCDs' writes, so on gfx950 it does not take this XCD's L2 copy,
// and a plain store stays in that (write-back) L2: a plain store followed by an
// agent-scope load can read what the address held before the store -- here, the
// previous round's strip in the same workspace slot (seen as rare, run-dependent
// wrong strips).  Both accesses at agent scope meet at the coherent level.
template <class T>
__device__ __forceinline__ T ld_l2(const T *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void st_l2(T *p, T v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct Strip {
    const uint8_t *src;
    uint32_t n;
    uint8_t *ws;
};
__device__ __forceinline__ bool strip_lazy(const Strip &S)
{
    return *reinterpret_cast<const uint32_t *>(S.ws + kSumOff + 20) != 0;
}
// strip s of the batch; its workspace is slot s - s0 of the round's workspace
// (rounds of at most kRound strips reuse one workspace)
__device__ __forceinline__ Strip strip_of(const uint8_t *in, int64_t frame_bytes, int32_t strip_bytes, int32_t spf,
                                          uint8_t *ws, int64_t s0, int64_t s)
{
    const int64_t f = s / spf, k = s - f * spf;
    const int64_t off = k * (int64_t)strip_bytes;
    return {in + f * frame_bytes + off, (uint32_t)min((int64_t)strip_bytes, frame_bytes - off),
            ws + (s - s0) * kWsPerStrip};
}

// The round's non-lazy strips, listed by K1: the side kernels (K2a, K2b, K3) loop over
// this list on small grids instead of launching a workgroup per strip of the round that
// returns at once for a lazy strip -- half a million such workgroups per C4 call
// (K2a's with 36 KB of LDS, K2b's with 64 KB) competed with the lazy parse for
// dispatch and CUs: 2-5 ms of a 65 ms call, different from one library load to the next.
__device__ __forceinline__ uint32_t side_count(const uint8_t *ws)
{
    return *reinterpret_cast<const uint32_t *>(ws + kSumOff + 40);
}
__device__ __forceinline__ uint32_t side_strip(const uint8_t *ws, uint32_t i)
{
    return *reinterpret_cast<const uint32_t *>(ws + (int64_t)i * kWsPerStrip + kSumOff + 32);
}

// ---- K1: hash-bucket order of the positions, and the adler32 sums ----------
// sorted[] lists the positions 0..n-3 bucket by bucket (buckets in hash order,
// positions increasing inside a bucket) and idx[p] is p's slot, so zlib's chain
// of p -- the earlier positions with p's hash, newest first -- is
// sorted[idx[p]-1], sorted[idx[p]-2], ... while the hash stays p's; hd[p] is
// its first element (zlib's head[] as p is inserted, 0 = NIL).
__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c)   // zlib UPDATE_HASH x3
{
    return (a << 10 ^ b << 5 ^ c) & 0x7fffu;
}

// Round 6 form: the hash order by a two-pass LSD radix sort.  Round 5's K1 built
// the order with 32768 bucket counters in LDS and an ordered scatter in which each
// wave owned an eighth of the hash space -- and repetitive content puts most
// positions' hashes in one wave's part: that wave acted on ~250 of the strip's 256
// groups while the others waited at each chunk's barrier (K1 27 ms of a C4 call, 80 %
// of it in the scatter; a separate pass then wrote hd[]).  Sorting the positions by hash with two
// stable counting passes over 8 + 7 hash bits instead splits the work by position:
// the strip's tiles of 2048 positions go to the eight waves in turn, a tile's digit
// counts are known before it is placed, the per-(tile, digit) cursors come from one
// column scan, and each wave then places its tiles' positions with no exchange
// between waves.  Inside a tile a group of 64 positions takes its ranks from
// same-digit lane masks built from one ballot per digit bit (bits equal on every
// lane skipped) and the tile's cursors in LDS, read by every lane and advanced by
// each digit's first lane -- the LDS serves one wave's instructions in order.
//   pass 1 (low 8 bits): the tile's bytes staged in LDS (all its loads in flight);
//     the digit counts, then hash << 16 | position to the K2 result area rf[] (K2
//     writes it only after this kernel) in digit order -- and each position's
//     pass-2 (tile, digit) counted at its new slot, so pass 2 needs no count pass;
//   pass 2 (high 7 bits) reads rf[] in that order, which keeps equal hashes in
//     position order, and writes sorted[] and idx[].  The element before a
//     position in the final order -- its bucket predecessor when the hashes match:
//     zlib's head[] as p is inserted, hd[p] -- is the lane below it with the same
//     digit, or for a digit's first lane the digit's last element of the tile's
//     earlier groups (a per-wave LDS row); a digit's first element in a tile is
//     completed after the pass from sorted[] and the strip bytes.
// hd[] also gives each 64-position group's distinct hashes (the lazy-parse test): a
// position is its hash's first in the group unless its bucket predecessor lies in it.
constexpr int kSortWaves = 8;
constexpr uint32_t kSortT = 2048;                  // positions per tile (both passes)
constexpr uint32_t kSortTiles = MAX_STRIP / kSortT;
constexpr uint32_t kSortH = 1024;                  // pass 1 stages a tile in halves
constexpr uint32_t kSortStg = kSortH / 4 + 4;      // a wave's staged half tile, dwords (+ the 2 bytes after it)
struct SortSmem {
    uint32_t tab1[kSortTiles * 256 / 2];   // pass 1: u16 [t * 256 + d], digit d's count, then cursor, in tile t
    uint32_t tab2[kSortTiles * 128 / 2];   // pass 2: u16 [t * 128 + d]
    uint32_t stg[kSortWaves][kSortStg];    // pass 1: the wave's half tile of strip bytes; pass 2: its last key per digit
    uint32_t dsum[kSortWaves];
    uint64_t sums[kSortWaves][2];
    uint32_t distinct[kSortWaves];
};
// the valid lanes whose digit equals this lane's: one ballot per digit bit, the bits
// equal on every valid lane skipped (a scalar branch)
template <int BITS>
__device__ __forceinline__ uint64_t digit_mask(uint32_t d, bool valid)
{
    const uint64_t vm = __ballot(valid);
    uint64_t m = vm;
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
        const uint32_t bit = (d >> b) & 1u;
        const uint64_t B = __ballot(valid && bit);
        if (B == 0 || B == vm) continue;
        m &= ~(B ^ (bit ? ~0ull : 0ull));
    }
    return valid ? m : 0ull;
}
// the same mask from one round per distinct digit (a lane's digit compared with a
// leader's by readlane + ballot): fewer instructions when a group holds few digits, as
// repetitive content does; past kDigitRounds rounds the bit-sliced form finishes
#ifndef VCF_ZX_DIGITLOOP   // A/B (diagnostic builds)
#define VCF_ZX_DIGITLOOP 1
#endif
constexpr int kDigitRounds = 6;
template <int BITS>
__device__ __forceinline__ uint64_t digit_mask_r(uint32_t d, bool valid)
{
    if (!VCF_ZX_DIGITLOOP) return digit_mask<BITS>(d, valid);
    uint64_t rem = __ballot(valid), m0 = 0;
    for (int r = 0; r < kDigitRounds && rem; ++r) {
        const uint32_t hl = lane_val(d, (uint32_t)__ffsll((unsigned long long)rem) - 1);
        const bool eq = valid && d == hl;
        const uint64_t m = __ballot(eq);
        if (eq) m0 = m;
        rem &= ~m;
    }
    if (rem) {   // many digits (e.g. raw RGB): the rest bit-sliced
        const uint64_t mb = digit_mask<BITS>(d, valid);
        if ((rem >> lane_id()) & 1) m0 = mb;
    }
    return m0;
}
// a group's counts into the u16 table entries a: a run of one entry over consecutive
// lanes (runs of one byte value) adds its length with one atomic from its first lane;
// the valid lanes are a prefix
__device__ __forceinline__ void tile_count(uint32_t *tab, uint32_t a, bool valid, uint32_t lane)
{
    const uint32_t aprev = (uint32_t)__shfl_up((int)a, 1, 64);
    const bool head = valid && (lane == 0 || aprev != a);
    const uint64_t heads = __ballot(head), vmask = __ballot(valid);
    if (head) {
        const uint64_t above = heads & ~((2ull << lane) - 1);
        const uint32_t end = above ? (uint32_t)__ffsll((unsigned long long)above) - 1 : (uint32_t)__popcll(vmask);
        atomicAdd(&tab[a >> 1], (end - lane) << ((a & 1) * 16));
    }
}
// counts -> cursors: per digit (one thread each) the exclusive prefix over the tiles,
// plus the digit's start (the exclusive prefix of the digit totals)
template <uint32_t D>
__device__ __forceinline__ void tile_scan(SortSmem &sm, uint16_t *tab16, uint32_t ntiles, uint32_t tid, uint32_t w,
                                          uint32_t lane)
{
    uint32_t tot = 0;
    if (tid < D)
        for (uint32_t t = 0; t < ntiles; ++t) {
            const uint32_t x = tab16[t * D + tid];
            tab16[t * D + tid] = (uint16_t)tot;
            tot += x;
        }
    uint32_t wsum;
    uint32_t ex = excl_scan(tot, wsum);
    if (lane == 0) sm.dsum[w] = wsum;
    __syncthreads();
    if (tid < D) {
        for (uint32_t v = 0; v < w; ++v) ex += sm.dsum[v];
        for (uint32_t t = 0; t < ntiles; ++t) tab16[t * D + tid] = (uint16_t)(tab16[t * D + tid] + ex);
    }
    __syncthreads();
}

__global__ __launch_bounds__(64 * kSortWaves) void zlib_sort_kernel(const uint8_t *__restrict__ in, int64_t frame_bytes,
                                                                   int32_t strip_bytes, int32_t spf,
                                                                   uint8_t *__restrict__ ws, int64_t s0)
{
    __shared__ __attribute__((aligned(16))) SortSmem sm;
    const Strip S = strip_of(in, frame_bytes, strip_bytes, spf, ws, s0, s0 + blockIdx.x);
    uint16_t *idx = reinterpret_cast<uint16_t *>(S.ws + kIdxOff);
    uint16_t *sorted = reinterpret_cast<uint16_t *>(S.ws + kSortOff);
    uint16_t *hd = reinterpret_cast<uint16_t *>(S.ws + kHdOff);
    uint32_t *tmp = reinterpret_cast<uint32_t *>(S.ws + kRfOff);
    uint16_t *tab1 = reinterpret_cast<uint16_t *>(sm.tab1), *tab2 = reinterpret_cast<uint16_t *>(sm.tab2);
    constexpr uint32_t NT = 64 * kSortWaves;
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6, n = S.n;
    const uint32_t np = n >= 3 ? n - 2 : 0;   // positions 0..n-3 are inserted
    const uint64_t lt = (1ull << lane) - 1;
    const uint32_t nt1 = (n + kSortT - 1) / kSortT, nt2 = (np + kSortT - 1) / kSortT;
    const uint8_t *src = S.src;
    const bool al4 = (((uintptr_t)src) & 3) == 0;
    const uint8_t *stg = reinterpret_cast<const uint8_t *>(sm.stg[w]);
    uint32_t *lastk = sm.stg[w];
#if VCF_ZLIB_PROF
    unsigned long long ck[8];
    int nck = 0;
#define VCF_SORT_CLK() (ck[nck++] = clock64())
#else
#define VCF_SORT_CLK() ((void)0)
#endif
    // bytes [b0, b0 + H + 4) of the strip (zeros past n) into registers, every dword load in
    // flight at once; then into the wave's staging area.  A wave's half tiles in order are
    // k = 0, 1, ...: tile w + 8 (k / 2), half k % 2; the next one is fetched while the
    // current one is processed.
    constexpr uint32_t kSV = (kSortStg + 63) / 64;
    auto fetch = [&](uint32_t b0, uint32_t (&v)[kSV]) {
#pragma unroll
        for (uint32_t k = 0; k < kSV; ++k) {
            const uint32_t q = b0 + 4 * (lane + 64 * k);
            if (al4 && q + 4 <= n) {
                v[k] = *reinterpret_cast<const uint32_t *>(src + q);
            } else {
                v[k] = 0;
                for (uint32_t i = 0; i < 4; ++i) v[k] |= (q + i < n ? (uint32_t)src[q + i] : 0u) << (8 * i);
            }
        }
    };
    auto commit = [&](const uint32_t (&v)[kSV]) {
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (uint32_t k = 0; k < kSV; ++k)
            if (lane + 64 * k < kSortStg) sm.stg[w][lane + 64 * k] = v[k];
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    };
    auto half_base = [&](uint32_t k) { return (w + kSortWaves * (k >> 1)) * kSortT + (k & 1) * kSortH; };
    for (uint32_t i = tid; i < (uint32_t)(sizeof(sm.tab1) / 4); i += NT) sm.tab1[i] = 0;
    for (uint32_t i = tid; i < (uint32_t)(sizeof(sm.tab2) / 4); i += NT) sm.tab2[i] = 0;
    __syncthreads();
    VCF_SORT_CLK();
    // pass 1 counts (low 8 hash bits) and the adler32 sums over every byte
    uint64_t sb = 0, swb = 0;
    uint32_t sv[kSV];
    if (half_base(0) < n) fetch(half_base(0), sv);
    for (uint32_t k = 0, hb = half_base(0); hb < n; hb = half_base(++k)) {
        const uint32_t t = hb / kSortT;
        commit(sv);
        if (half_base(k + 1) < n) fetch(half_base(k + 1), sv);
        // four consecutive positions per lane (a quad of 256 positions per step): a run of
        // one digit adds its length with one atomic from its first position, the run's end
        // being the next run's first position -- in this lane, else the next lane holding
        // one (its first), else the quad's valid end
        uint32_t qsb = 0, qswb = 0;   // this half tile's adler32 terms (< 2^32 over 1024 bytes)
        for (uint32_t Q = 0; Q < kSortH / 256 && hb + Q * 256 < n; ++Q) {
            const uint32_t j0 = Q * 256 + 4 * lane;
            const uint64_t bb = (uint64_t)sm.stg[w][Q * 64 + lane + 1] << 32 | sm.stg[w][Q * 64 + lane];
            const uint32_t V = np > hb + Q * 256 ? min(256u, np - (hb + Q * 256)) : 0u;   // valid positions
            uint32_t d[4], hm = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t b = (uint32_t)(bb >> (8 * k)) & 0xffu, p = hb + j0 + k;
                if (p < n) {
                    qsb += b;
                    qswb += (n - p) * b;
                }
                d[k] = hash3(b, (uint32_t)(bb >> (8 * k + 8)) & 0xffu, (uint32_t)(bb >> (8 * k + 16)) & 0xffu) & 255u;
            }
            const uint32_t dl = (uint32_t)__shfl_up((int)d[3], 1, 64);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool head = 4 * lane + k < V && (k ? d[k - 1] != d[k] : (lane == 0 || dl != d[0]));
                hm |= (head ? 1u : 0u) << k;
            }
            const uint64_t above = __ballot(hm != 0) & ~((2ull << lane) - 1);
            const int l2 = above ? __ffsll((unsigned long long)above) - 1 : (int)lane;
            const uint32_t fh2 = (uint32_t)__shfl((int)(hm ? __builtin_ctz(hm) : 0u), l2, 64);
            const uint32_t nxt = above ? 4u * (uint32_t)l2 + fh2 : V;   // the next lane's first run
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if ((hm >> k) & 1u) {
                    const uint32_t rest = hm >> (k + 1);
                    const uint32_t end = rest ? 4 * lane + k + 1 + __builtin_ctz(rest) : nxt;
                    const uint32_t a = t * 256 + d[k];
                    atomicAdd(&sm.tab1[a >> 1], (end - 4 * lane - k) << ((a & 1) * 16));
                }
        }
        sb += qsb;
        swb += qswb;
        __builtin_amdgcn_wave_barrier();   // the staging area is rewritten next
    }
    __syncthreads();
    VCF_SORT_CLK();
    tile_scan<256>(sm, tab1, nt1, tid, w, lane);
    VCF_SORT_CLK();
    // pass 1 placement: hash << 16 | position to tmp[] in low-digit order; pass 2's counts
    if (half_base(0) < np) fetch(half_base(0), sv);
    for (uint32_t k = 0, hb = half_base(0); hb < np; hb = half_base(++k)) {
        const uint32_t t = hb / kSortT;
        commit(sv);
        if (half_base(k + 1) < np) fetch(half_base(k + 1), sv);
        for (uint32_t g = 0; g < kSortH && hb + g < np; g += 64) {
            const uint32_t j = g + lane, p = hb + j;
            const bool valid = p < np;
            const uint32_t h = hash3(stg[j], stg[j + 1], stg[j + 2]), d = h & 255u;
            const uint64_t m = digit_mask_r<8>(d, valid);
            const uint32_t a = t * 256 + d;
            const uint32_t cur = valid ? (uint32_t)tab1[a] : 0u;
            if (valid && (m & lt) == 0) tab1[a] = (uint16_t)(cur + (uint32_t)__popcll(m));
            const uint32_t slot = cur + (uint32_t)__popcll(m & lt);
            if (valid) tmp[slot] = h << 16 | p;
            // pass 2's count at the new slot (equal hashes over consecutive lanes have
            // consecutive slots: a run in one tile adds with one atomic)
            tile_count(sm.tab2, (slot / kSortT) * 128 + (h >> 8), valid, lane);
        }
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    VCF_SORT_CLK();
    tile_scan<128>(sm, tab2, nt2, tid, w, lane);
    VCF_SORT_CLK();
    // pass 2 placement (high 7 bits): sorted[], idx[], hd[] but for each digit's first element of a tile
    uint32_t distinct = 0;
    for (uint32_t t = w; t < nt2; t += kSortWaves) {
        lastk[lane] = 0xffffffffu;   // no element of any digit yet in this tile
        lastk[lane + 64] = 0xffffffffu;
        for (uint32_t half = 0; half < kSortT / 1024 && t * kSortT + half * 1024 < np; ++half) {
            uint32_t e[16];   // the half tile's 16 groups, all loads in flight at once
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) {
                const uint32_t i = t * kSortT + half * 1024 + 64 * k + lane;
                e[k] = i < np ? tmp[i] : 0u;
            }
            for (uint32_t k = 0; k < 16 && t * kSortT + half * 1024 + 64 * k < np; ++k) {
                const uint32_t i = t * kSortT + half * 1024 + 64 * k + lane;
                const bool valid = i < np;
                const uint32_t ek = e[k], d = ek >> 24;
                const uint64_t m = digit_mask_r<7>(d, valid);
                const uint32_t a = t * 128 + d;
                const uint64_t below = m & lt;
                const bool lead = valid && below == 0;
                const uint32_t cur = valid ? (uint32_t)tab2[a] : 0u;
                const uint32_t lk = lead ? lastk[d] : 0u;   // read before this group's update below
                if (lead) tab2[a] = (uint16_t)(cur + (uint32_t)__popcll(m));
                if (valid && (m >> lane) == 1) lastk[d] = ek;   // the digit's last lane in the group
                const int pl = below ? 63 - __clzll((long long)below) : (int)lane;
                const uint32_t ebelow = (uint32_t)__shfl((int)ek, pl, 64);
                if (valid) {
                    const uint32_t slot = cur + (uint32_t)__popcll(below), p = ek & 0xffffu;
                    sorted[slot] = (uint16_t)p;
                    idx[p] = (uint16_t)slot;
                    const uint32_t prev = lead ? lk : ebelow;
                    if (prev != 0xffffffffu) {
                        const bool same = (prev >> 16) == (ek >> 16);
                        hd[p] = same ? (uint16_t)(prev & 0xffffu) : (uint16_t)0;
                        distinct += same && (prev & 0xffffu) >= (p & ~63u) ? 0u : 1u;
                    }
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    VCF_SORT_CLK();
    // each digit's first element of a tile: its predecessor is the slot before it (another
    // tile's, or another digit's: then the hashes differ), the hashes from the strip bytes
    for (uint32_t pr = tid; pr < nt2 * 128; pr += NT) {
        const uint32_t t = pr >> 7, d = pr & 127u;
        const uint32_t end = tab2[pr];
        const uint32_t start = t ? (uint32_t)tab2[pr - 128] : d ? (uint32_t)tab2[(nt2 - 1) * 128 + d - 1] : 0u;
        if (end > start) {
            const uint32_t p = sorted[start];
            const uint32_t q = start ? (uint32_t)sorted[start - 1] : 0u;
            const bool same = start && hash3(src[p], src[p + 1], src[p + 2]) == hash3(src[q], src[q + 1], src[q + 2]);
            hd[p] = same ? (uint16_t)q : (uint16_t)0;
            distinct += same && q >= (p & ~63u) ? 0u : 1u;
        }
    }
    for (int dd = 32; dd >= 1; dd >>= 1) {
        sb += __shfl_xor(sb, dd, 64);
        swb += __shfl_xor(swb, dd, 64);
        distinct += (uint32_t)__shfl_xor((int)distinct, dd, 64);
    }
    if (lane == 0) {
        sm.sums[w][0] = sb;
        sm.sums[w][1] = swb;
        sm.distinct[w] = distinct;
    }
    __syncthreads();
    VCF_SORT_CLK();
#if VCF_ZLIB_PROF
    if (tid == 0) {
        for (int i = 0; i + 1 < nck && i < 7; ++i) atomicAdd(&g_zprof[40 + i], ck[i + 1] - ck[i]);
        atomicAdd(&g_zprof[47], 1ull);
    }
#endif
#undef VCF_SORT_CLK
    if (tid == 0) {
        uint64_t a = 0, b = 0;
        uint32_t dsum = 0;
        for (int v = 0; v < kSortWaves; ++v) {
            a += sm.sums[v][0];
            b += sm.sums[v][1];
            dsum += sm.distinct[v];
        }
        uint64_t *sums = reinterpret_cast<uint64_t *>(S.ws + kSumOff);
        sums[0] = a;
        sums[1] = b;
        *reinterpret_cast<uint32_t *>(S.ws + kSumOff + 16) = 0;   // K2's worklist length
        *reinterpret_cast<uint32_t *>(S.ws + kSumOff + 24) = dsum;   // the lazy parse's dispatch order key
#ifdef VCF_ZX_LAZYALL   // A/B (diagnostic builds): every strip through the lazy parse
        const bool lazy = true;
#else
        const bool lazy = dsum * kLazyDiv < np;
#endif
        *reinterpret_cast<uint32_t *>(S.ws + kSumOff + 20) = lazy ? 1u : 0u;   // parse order
        if (!lazy) {   // onto the side kernels' list
            const uint32_t i = atomicAdd(reinterpret_cast<uint32_t *>(ws + kSumOff + 40), 1u);
            *reinterpret_cast<uint32_t *>(ws + (int64_t)i * kWsPerStrip + kSumOff + 32) = blockIdx.x;
        }
    }
}

// ---- K2: longest_match at every position, both chain limits ----------------
// A thread takes kPer consecutive positions.  zlib's own shortcuts, exact:
// a candidate can only beat the best length L so far if it matches at bytes
// L-1 and L (longest_match's scan_end test), and when the first candidate of
// p+1 is the first candidate of p plus one, its common prefix is p's minus
// one (one byte is checked when p's reached the MAX_MATCH cap).
__device__ __forceinline__ void k2a_strip(const uint8_t *__restrict__ in, int64_t frame_bytes, int32_t strip_bytes,
                                          int32_t spf, int32_t level, uint8_t *__restrict__ ws, int64_t s0, int64_t s,
                                          uint32_t *win32)
{
    uint8_t *win = reinterpret_cast<uint8_t *>(win32);
    const Strip S = strip_of(in, frame_bytes, strip_bytes, spf, ws, s0, s);
    const uint32_t n = S.n, p0 = blockIdx.x * kChunk;
    const uint32_t np = n >= 3 ? n - 2 : 0;
    if (p0 >= np) return;
    Config cfg;
    level_config(level, cfg);
    const uint16_t *hd = reinterpret_cast<const uint16_t *>(S.ws + kHdOff);
    uint16_t *list = reinterpret_cast<uint16_t *>(S.ws + kListOff);
    uint32_t *nlist = reinterpret_cast<uint32_t *>(S.ws + kSumOff + 16);
    uint32_t *rf = reinterpret_cast<uint32_t *>(S.ws + kRfOff);
    uint32_t *rr = reinterpret_cast<uint32_t *>(S.ws + kRrOff);
    // window [w0, wend): 32 KB back (every candidate is > p - MAX_DIST) and the
    // chunk's strings; past n the bytes zlib's window holds there: zeros before its
    // slide, after it (at strstart >= slide_at) the stale copy WSIZE back
    const uint32_t w0 = p0 > (uint32_t)WSIZE ? p0 - WSIZE : 0u;
    const uint32_t wend = min(np, p0 + kChunk) + MAX_MATCH + 16;
    const uint32_t slide_at = n == (uint32_t)MAX_STRIP ? WSIZE + MAX_DIST + 1 : WSIZE + MAX_DIST;
    if ((((uintptr_t)(S.src + w0)) & 3) == 0 && wend <= n) {
        const uint32_t *s32 = reinterpret_cast<const uint32_t *>(S.src + w0);
        for (uint32_t q = threadIdx.x; q < (wend - w0 + 3) / 4; q += kK2Threads)
            win32[q] = w0 + 4 * q + 4 <= n ? s32[q] : 0u;
        for (uint32_t q = threadIdx.x; q < 4; q += kK2Threads) win32[(wend - w0 + 3) / 4 + q] = 0;
    } else {
        for (uint32_t p = w0 + threadIdx.x; p < wend + 16; p += kK2Threads) win[p - w0] = p < n ? S.src[p] : 0u;
    }
    __syncthreads();
    const uint32_t cfull = (uint32_t)cfg.chain;
    auto ld4 = [&](uint32_t a) {
        return __builtin_amdgcn_alignbyte(win32[(a >> 2) + 1], win32[a >> 2], a & 3);
    };
    auto lcp_fast = [&](uint32_t a, uint32_t b, uint32_t from) -> uint32_t {   // window offsets; from: bytes known equal
        uint32_t len = from;
        while (len < (uint32_t)MAX_MATCH) {
            uint32_t x = 0, q = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t xu = ld4(a + len + 4 * u) ^ ld4(b + len + 4 * u);
                if (x == 0) {
                    x = xu;
                    q = 4 * u;
                }
            }
            if (x) {
                len += q + ((uint32_t)__builtin_ctz(x) >> 3);
                break;
            }
            len += 16;
        }
        return min(len, (uint32_t)MAX_MATCH);
    };
    // the thread's positions' chain heads (zlib's head[] as each is inserted), one round of loads
    const uint32_t pbeg = p0 + threadIdx.x * kPer;
    const uint32_t pn = pbeg < np ? min((uint32_t)kPer, np - pbeg) : 0u;
    uint32_t c1v[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) c1v[u] = (uint32_t)u < pn ? (uint32_t)hd[pbeg + u] : 0u;
    uint32_t prev_c = 0, prev_l = 0;   // the previous position's first candidate and its common prefix
    // run: how many bytes before p equal p's (counted up to cfull)
    uint32_t run = 0;
    if (pn) {
        const uint32_t b = win[pbeg - w0];
        while (run < cfull && pbeg - run > w0 && win[pbeg - run - 1 - w0] == b) ++run;
    }
#pragma unroll 1
    for (uint32_t u = 0; u < pn; ++u) {
        const uint32_t p = pbeg + u;
        if (u) run = win[p - w0] == win[p - 1 - w0] ? min(run + 1, cfull) : 0u;
        // (register arrays indexed by a loop variable: select through a switch-free scan)
        uint32_t cur = 0;
#pragma unroll
        for (int t = 0; t < kPer; ++t)
            if ((uint32_t)t == u) cur = c1v[t];
        uint32_t rfull = 0, rred = 0;
        if (cur != 0 && p - cur <= (uint32_t)MAX_DIST) {
            const uint32_t nice = min((uint32_t)cfg.nice, n - p);
            const bool tail = p + MAX_MATCH + 16 > n;     // compares may read past the end
            const bool post = p >= slide_at;              // ... as zlib's window holds it after the slide
            auto vb = [&](uint32_t P) -> uint32_t {
                if (P < n) return win[P - w0];
                return post ? (uint32_t)win[P - WSIZE - w0] : 0u;
            };
            auto lcp = [&](uint32_t c, uint32_t from) -> uint32_t {
                if (!tail) return lcp_fast(c - w0, p - w0, from);
                uint32_t len = from;
                while (len < (uint32_t)MAX_MATCH && vb(c + len) == vb(p + len)) ++len;
                return len;
            };
            uint32_t len;
            if (!tail && cur == prev_c + 1 && prev_l > 0) {
                len = prev_l < (uint32_t)MAX_MATCH ? prev_l - 1 : lcp(cur, MAX_MATCH - 1);
            } else {
                len = lcp(cur, 0);
            }
            prev_c = cur;
            prev_l = len;
            uint32_t bf = len, bfp = cur, br = len, brp = cur;
            // Inside a run of one byte value b reaching cfull positions back with
            // len >= 3 (p's bytes are b b b), the chain's first cfull candidates are
            // p-1, ..., p-cfull (the only positions there, all b b b: p's hash) and
            // each matches exactly up to the run's end, as the first does: no walk.
            const bool in_run = cur == p - 1 && run >= cfull && len >= 3;
            if (len < nice && !in_run && hd[cur] > (p > (uint32_t)MAX_DIST ? p - MAX_DIST : 0u)) {
                // the rest of the chain may hold a longer match: K2b walks it (rf/rr keep
                // the first candidate meanwhile)
                list[atomicAdd(nlist, 1u)] = (uint16_t)p;
            }
            if (bf) rfull = bf << 16 | (p - bfp);
            if (br) rred = br << 16 | (p - brp);
        } else {
            prev_c = 0;
            prev_l = 0;
        }
        rf[p] = rfull;
        rr[p] = rred;
    }
}

constexpr unsigned kSideK2a = 256, kSideK2b = 128, kSideK3 = 4096;   // side kernels' strips in flight
__global__ __launch_bounds__(kK2Threads) void zlib_match_kernel(const uint8_t *__restrict__ in, int64_t frame_bytes,
                                                               int32_t strip_bytes, int32_t spf, int32_t level,
                                                               uint8_t *__restrict__ ws, int64_t s0)
{
    __shared__ __attribute__((aligned(16))) uint32_t win32[kK2Win / 4 + 4];
    const uint32_t cnt = side_count(ws);
    for (uint32_t i = blockIdx.y; i < cnt; i += gridDim.y) {
        k2a_strip(in, frame_bytes, strip_bytes, spf, level, ws, s0, s0 + side_strip(ws, i), win32);
        __syncthreads();   // the window is refilled for the next strip
    }
}

// ---- K2b: the listed positions' chains, 64 candidates per wave step ----------
// One workgroup of 16 waves per strip, the whole strip in LDS; a wave takes one
// listed position at a time.  Lane t evaluates candidate k = 1 + t (+64 per
// round) of the chain; only a candidate matching p at bytes len1-1 and len1 can
// beat the first candidate's length len1 (longest_match's scan_end test), so
// only those do the full compare.  The reductions keep zlib's order: the first
// candidate reaching nice, else the first reaching the longest length.
__device__ __forceinline__ void k2b_strip(const uint8_t *__restrict__ in, int64_t frame_bytes, int32_t strip_bytes,
                                          int32_t spf, int32_t level, uint8_t *__restrict__ ws, int64_t s0, int64_t s,
                                          uint32_t *win32)
{
    uint8_t *win = reinterpret_cast<uint8_t *>(win32);
    const Strip S = strip_of(in, frame_bytes, strip_bytes, spf, ws, s0, s);
    const uint32_t n = S.n;
    const uint32_t cnt = *reinterpret_cast<const uint32_t *>(S.ws + kSumOff + 16);
    if (cnt == 0) return;
    Config cfg;
    level_config(level, cfg);
    const uint16_t *idx = reinterpret_cast<const uint16_t *>(S.ws + kIdxOff);
    const uint16_t *sorted = reinterpret_cast<const uint16_t *>(S.ws + kSortOff);
    const uint16_t *list = reinterpret_cast<const uint16_t *>(S.ws + kListOff);
    uint32_t *rf = reinterpret_cast<uint32_t *>(S.ws + kRfOff);
    uint32_t *rr = reinterpret_cast<uint32_t *>(S.ws + kRrOff);
    const uint32_t wend = min(n + MAX_MATCH + 32, (uint32_t)(MAX_STRIP + MAX_MATCH + 60));
    if (((uintptr_t)S.src & 3) == 0) {
        const uint32_t *s32 = reinterpret_cast<const uint32_t *>(S.src);
        for (uint32_t q = threadIdx.x; q < wend / 4; q += kK2bThreads) win32[q] = 4 * q + 4 <= n ? s32[q] : 0u;
        __syncthreads();
        for (uint32_t p = (n & ~3u) + threadIdx.x; p < min(n, (n & ~3u) + 4); p += kK2bThreads) win[p] = S.src[p];
    } else {
        for (uint32_t p = threadIdx.x; p < wend; p += kK2bThreads) win[p] = p < n ? S.src[p] : 0u;
    }
    __syncthreads();
    const uint32_t slide_at = n == (uint32_t)MAX_STRIP ? WSIZE + MAX_DIST + 1 : WSIZE + MAX_DIST;
    const uint32_t cfull = (uint32_t)cfg.chain, cred = (uint32_t)cfg.chain >> 2;
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
    // the strip's list is split over gridDim.y workgroups (each with its own copy of
    // the strip in LDS): a round has few such strips, one workgroup each left most CUs idle
    constexpr uint32_t kWaves = kK2bThreads / 64;
    for (uint32_t i = blockIdx.y * kWaves + wave; i < cnt; i += kWaves * gridDim.y) {
        const uint32_t p = list[i];
        const uint32_t ip = idx[p];
        const uint32_t hp = ((uint32_t)win[p] << 10 ^ (uint32_t)win[p + 1] << 5 ^ win[p + 2]) & 0x7fffu;
        const uint32_t r1 = rf[p], len1 = r1 >> 16, c1 = p - (r1 & 0xffffu);
        const uint32_t nice = min((uint32_t)cfg.nice, n - p);
        const uint32_t limit = p > (uint32_t)MAX_DIST ? p - MAX_DIST : 0u;
        const bool post = p >= slide_at;
        auto vb = [&](uint32_t P) -> uint32_t {   // the window as zlib's longest_match reads it
            if (P < n) return win[P];
            return post ? (uint32_t)win[P - WSIZE] : 0u;
        };
        const bool tail = p + MAX_MATCH + 16 > n;
        auto lcp = [&](uint32_t c) -> uint32_t {
            uint32_t len = 0;
            if (!tail) {
                while (len < (uint32_t)MAX_MATCH) {
                    uint32_t x = 0, q = 0;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const uint32_t a = c + len + 4 * u, b = p + len + 4 * u;
                        const uint32_t xu = __builtin_amdgcn_alignbyte(win32[(a >> 2) + 1], win32[a >> 2], a & 3) ^
                                            __builtin_amdgcn_alignbyte(win32[(b >> 2) + 1], win32[b >> 2], b & 3);
                        if (x == 0) {
                            x = xu;
                            q = 4 * u;
                        }
                    }
                    if (x) {
                        len += q + ((uint32_t)__builtin_ctz(x) >> 3);
                        break;
                    }
                    len += 16;
                }
                return min(len, (uint32_t)MAX_MATCH);
            }
            while (len < (uint32_t)MAX_MATCH && vb(c + len) == vb(p + len)) ++len;
            return len;
        };
        uint32_t bf = len1, bfp = c1, br = len1, brp = c1;
        bool done_f = false, done_r = false;   // a nice match found (the scans stop there)
        for (uint32_t k0 = 1; k0 < cfull && !done_f; k0 += 64) {
            const uint32_t k = k0 + lane;
            const bool in_arr = k < cfull && k + 1 <= ip;   // slot ip-1-k >= 0
            const uint32_t c = in_arr ? (uint32_t)sorted[ip - 1 - k] : 0u;
            // still p's bucket (its hash) and newer than the limit
            const bool in_chain = in_arr && c > limit &&
                                  (((uint32_t)win[c] << 10 ^ (uint32_t)win[c + 1] << 5 ^ win[c + 2]) & 0x7fffu) == hp;
            const uint64_t stop = __ballot(!in_chain);
            const uint32_t nv = stop ? (uint32_t)__ffsll((unsigned long long)stop) - 1 : 64u;
            const bool v = lane < nv;
            // scan_end against the first candidate: only then can the match be longer than len1
            const bool cand = v && (len1 == 0 || (vb(c + len1) == vb(p + len1) && vb(c + len1 - 1) == vb(p + len1 - 1)));
            const uint32_t l = cand ? lcp(c) : 0u;
            // full chain: the first reaching nice, else the first reaching the longest length
            const uint64_t hit = __ballot(cand && l > bf && l >= nice);
            uint32_t m = l;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor(m, d, 64));
            const uint32_t hk = hit ? (uint32_t)__ffsll((unsigned long long)hit) - 1 : 64u;
            // the reduced chain (k < cred), evaluated before the full one moves on
            if (!done_r && k0 < cred) {
                const bool inr = cand && k < cred;
                const uint64_t hr = __ballot(inr && l > br && l >= nice);
                if (hr) {
                    const uint32_t t = (uint32_t)__ffsll((unsigned long long)hr) - 1;
                    br = lane_val(l, t);
                    brp = lane_val(c, t);
                    done_r = true;
                } else {
                    uint32_t mr = inr ? l : 0u;
#pragma unroll
                    for (int d = 32; d >= 1; d >>= 1) mr = max(mr, (uint32_t)__shfl_xor(mr, d, 64));
                    mr = uni(mr);
                    if (mr > br) {
                        const uint32_t t = (uint32_t)__ffsll((unsigned long long)__ballot(inr && l == mr)) - 1;
                        br = mr;
                        brp = lane_val(c, t);
                    }
                }
            }
            if (hk < 64) {
                bf = lane_val(l, hk);
                bfp = lane_val(c, hk);
                done_f = true;
            } else {
                m = uni(m);
                if (m > bf) {
                    const uint32_t t = (uint32_t)__ffsll((unsigned long long)__ballot(cand && l == m)) - 1;
                    bf = m;
                    bfp = lane_val(c, t);
                }
            }
            if (nv < 64) break;
        }
        if (lane == 0) {
            rf[p] = bf << 16 | (p - bfp);
            rr[p] = br << 16 | (p - brp);
        }
    }
}
__global__ __launch_bounds__(kK2bThreads) void zlib_chain_kernel(const uint8_t *__restrict__ in, int64_t frame_bytes,
                                                                int32_t strip_bytes, int32_t spf, int32_t level,
                                                                uint8_t *__restrict__ ws, int64_t s0)
{
    __shared__ __attribute__((aligned(16))) uint32_t win32[(MAX_STRIP + MAX_MATCH + 64) / 4];
    const uint32_t cnt = side_count(ws);
    for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
        k2b_strip(in, frame_bytes, strip_bytes, spf, level, ws, s0, s0 + side_strip(ws, i), win32);
        __syncthreads();   // the strip copy is refilled for the next strip
    }
}

// ---- K3: the parse, the trees, the bits ------------------------------------
// The trees' Freq and Code share storage, as in zlib's ct_data union: a tree's
// codes are written by gen_codes after its last frequency read, and the next
// block's counts start from zero after its last code read.  The block's symbol
// counts go straight into the frequency arrays (packed 16-bit LDS adds).
// stg[0] carries the output's partial word from one block to the next; everything from
// lfreq on is used only while a block is flushed (the frequencies are counted from the
// block's symbols at its flush), so the lazy parse lays its window over that part
// (ParseShared<true>) and reloads the window after each flush
struct ParseSmem {
    uint32_t stg[kStgWords];
    uint32_t bcast[4];
    uint16_t lfreq[HEAP_SIZE + 1], ldad[HEAP_SIZE], llen[HEAP_SIZE];
    uint16_t dfreq[2 * D_CODES + 1 + 1], ddad[2 * D_CODES + 1], dlen[2 * D_CODES + 1];
    uint16_t bfreq[2 * BL_CODES + 1 + 1], bdad[2 * BL_CODES + 1], blen[2 * BL_CODES + 1];
    int16_t heap[HEAP_SIZE];
    uint8_t depth[HEAP_SIZE];
    uint16_t bl_count[MAX_BITS + 1];
};
static_assert(offsetof(ParseSmem, lfreq) % 16 == 0, "packed adds into lfreq; the lazy window over it");
// the lazy parse's sliding window of the strip: [wbase, wbase + kLazyWin) holds
// the bytes longest_match reads near the current position (back to p -
// kNearDist, ahead to p + MAX_MATCH + 62); the parse shifts it forward in
// 256-byte steps.  Candidates farther back (zlib's chains reach p - MAX_DIST)
// read the strip in HBM.  Round 4 held all of [p - MAX_DIST, p + 320) (34.5 KB,
// four strips per CU); the lazy parse is a per-wave dependency chain whose
// throughput follows the strips a CU holds, so smaller windows buy more than
// their far reads cost, down to the 3 840-byte window that makes 16 strips per
// CU (C4 deflate, ms: 34 560 B 245, 18 432 B 212, 14 080 B 189, 9 984 B 182,
// 8 448 B 176, 7 168 B 172, 5 120 B 165, 3 840 B 161; 3 072 / 2 304 B 161 / 159:
// no more than 16 workgroups reside on a CU).  Round 6 lays the window over the
// flush-only part of ParseSmem (VCF_ZX_ALIAS): 9 216 bytes at the same 16 strips per CU.
#ifndef VCF_ZX_ALIAS   // A/B (diagnostic builds): the lazy window laid over the flush-only LDS
// (round 6: 1 -- the window grows from 3 840 to 9 216 bytes at the same 16 strips per CU,
// so chain candidates up to 7 872 bytes back read LDS instead of HBM)
#define VCF_ZX_ALIAS 1
#endif
#ifndef VCF_ZX_LAZYWIN   // A/B (diagnostic builds): the window's bytes (a multiple of 256)
#define VCF_ZX_LAZYWIN (VCF_ZX_ALIAS ? 9216 : 3840)
#endif
constexpr uint32_t kLazyWin = VCF_ZX_LAZYWIN;
#ifndef VCF_ZX_LWIN   // A/B (diagnostic builds): positions per lazy hd[] / idx[] register window (512 or 256)
// (round 6: 256 -- uint2 windows, two readlanes per lookup instead of four, 8 fewer VGPRs:
// C4 deflate 95.5 -> 89.5 ms, ABBA, profiles/r06_zab_v5.json)
#define VCF_ZX_LWIN 256
#endif
constexpr uint32_t kLWin = VCF_ZX_LWIN;
static_assert(kLWin == 512 || kLWin == 256, "lazy windows of 512 or 256 positions");
using LVec = std::conditional_t<kLWin == 512, uint4, uint2>;
constexpr uint32_t kLazyAhead = 320;
// the near distance the window keeps behind p after a shift: candidates at most
// this far back read the window, farther ones (zlib reaches MAX_DIST back) read
// the strip in HBM (Wave::far_*); shifts come every ~1 KB
#ifndef VCF_ZX_SLACK   // A/B (diagnostic builds): bytes a window shift leaves ahead
#define VCF_ZX_SLACK (kLazyWin >= 8192 ? 1024 : 512)
#endif
constexpr uint32_t kShiftSlack = VCF_ZX_SLACK;   // bytes a shift leaves ahead
constexpr uint32_t kNearDist = kLazyWin >= MAX_DIST + kLazyAhead + kShiftSlack ? (uint32_t)MAX_DIST
                                                                               : kLazyWin - kLazyAhead - kShiftSlack;
static_assert(kLazyWin % 256 == 0 && kNearDist >= 512, "window too short");

// LAZY (strips K1 found repetitive, kLazyDiv below): zlib's own order of work --
// the strip in LDS and longest_match evaluated only where deflate_slow calls it
// (the chain head with one wave-wide compare, then 64 candidates of sorted[] per
// step, one per lane), so positions inside long matches cost nothing.  Otherwise
// the K2 results are read from register windows.  Same bytes either way.
template <bool LAZY>
struct Wave {
    ParseSmem &sm;
    const uint8_t *src;
    uint32_t n;
    const uint16_t *hd;
    const uint32_t *rf, *rr;
    uint32_t *syms;
    uint32_t *out32;
    uint32_t out_words;           // slot capacity in words
    uint32_t good;                // cfg.good: the reduced-chain results from prev_length >= good
    uint32_t lazy = 0;            // cfg.lazy (VCF_ZX_PREDICT)
    uint32_t bitpos = 0;          // bits written so far (uniform)
    uint32_t nsym = 0;            // symbols of the current block (uniform)
    // 512-position windows: lane l holds positions base + 8l .. base + 8l + 7
    uint32_t base = 0x80000000u;  // p - base >= 512: not loaded
    uint4 hv, fv0, fv1, rv0, rv1;
    uint32_t bv0, bv1;
    bool overflow = false;
    BlockTrees T;
    // LAZY: the sliding window in LDS, the bucket order, and a 512-position window of idx[]
    uint8_t *lwin = nullptr;      // window byte i is input position wbase + i
    uint32_t wbase = 0;
    bool wslid = false;           // zlib's window has slid: the bytes past n are the stale copy WSIZE back
    const uint16_t *idx = nullptr, *sorted = nullptr;
    uint32_t ibase = 0x80000000u;
    uint4 iv;
    // the chain candidates of the positions the next call will most likely be at (p + 1,
    // and p + the match length), requested at the end of a call: their global latency
    // overlaps the parse step in between (~70 % of the calls are at one of the two)
    uint32_t pfa_p = 0xffffffffu, pfa0 = 0, pfa1 = 0, pfb_p = 0xffffffffu, pfb0 = 0, pfb1 = 0;
#if VCF_ZX_WINCHECK
    uint32_t dbg_strip = 0;
    __device__ __forceinline__ void wincheck(uint32_t kind, uint32_t P, bool bad, uint32_t got, uint32_t want)
    {
        const uint64_t m = __ballot(bad);
        if (!m) return;
        const uint32_t k = (uint32_t)__ffsll((unsigned long long)m) - 1;
        if (lane_id() == k) {
            atomicAdd(&g_zdbg[7], 1u);
            if (atomicCAS(&g_zdbg[0], 0u, kind) == 0u) {
                g_zdbg[1] = dbg_strip; g_zdbg[2] = cur_p; g_zdbg[3] = P; g_zdbg[4] = got; g_zdbg[5] = want;
                g_zdbg[6] = wbase;
            }
        }
    }
    uint32_t cur_p = 0;
#endif

    __device__ __forceinline__ Wave(ParseSmem &s, const uint8_t *in, uint32_t len, const uint8_t *w, uint32_t g, uint32_t *o,
                    uint32_t ow)
        : sm(s), src(in), n(len), hd(reinterpret_cast<const uint16_t *>(w + kHdOff)),
          rf(reinterpret_cast<const uint32_t *>(w + kRfOff)), rr(reinterpret_cast<const uint32_t *>(w + kRrOff)),
          syms(reinterpret_cast<uint32_t *>(const_cast<uint8_t *>(w) + kSymOff)), out32(o), out_words(ow), good(g)
    {
        T.l = {sm.lfreq, sm.ldad, sm.llen, sm.lfreq, L_CODES, MAX_BITS, 0, 0};
        T.d = {sm.dfreq, sm.ddad, sm.dlen, sm.dfreq, D_CODES, MAX_BITS, 1, 0};
        T.bl = {sm.bfreq, sm.bdad, sm.blen, sm.bfreq, BL_CODES, MAX_BL_BITS, 2, 0};
        T.w.heap = sm.heap;
        T.w.depth = sm.depth;
        T.w.bl_count = sm.bl_count;
    }

    // ---- the windows ---------------------------------------------------
    // LAZY: 512-aligned windows of hd[] and idx[], each with the next window requested
    // as soon as the current one is in use (the parse only moves forward, at most
    // MAX_MATCH positions at a time, so it always enters the next window)
    uint4 hv_n, iv_n;
    // VCF_ZX_COHERENT (A/B): the workspace tables K1 wrote, read at agent scope
    __device__ __forceinline__ static uint4 wload4(const uint16_t *a)
    {
#if VCF_ZX_COHERENT
        const uint32_t *v = reinterpret_cast<const uint32_t *>(a);
        return make_uint4(ld_l2(v), ld_l2(v + 1), ld_l2(v + 2), ld_l2(v + 3));
#else
        return *reinterpret_cast<const uint4 *>(a);
#endif
    }
    __device__ __forceinline__ static uint32_t wload16(const uint16_t *a)
    {
#if VCF_ZX_COHERENT
        return ld_l2(a);
#else
        return *a;
#endif
    }
    // VCF_ZX_LWIN = 256 (A/B): the lazy windows of hd[] / idx[] as 256 positions, 4 per lane in
    // a uint2 (8 fewer VGPRs than 512 in uint4s: room for more waves per SIMD)
    LVec lhv, liv, lhv_n, liv_n;
    __device__ __forceinline__ static LVec wloadL(const uint16_t *a)
    {
#if VCF_ZX_LWIN == 512
        return wload4(a);
#else
        return *reinterpret_cast<const uint2 *>(a);
#endif
    }
    __device__ __forceinline__ static uint32_t pickL(const LVec &v, uint32_t l, uint32_t d)   // dword d of lane l
    {
#if VCF_ZX_LWIN == 512
        return pick4(v, l, d);
#else
        const uint32_t a = lane_val(v.x, l), b = lane_val(v.y, l);
        return d == 0 ? a : b;
#endif
    }
    __device__ __forceinline__ void lazy_windows(uint32_t p)
    {
        constexpr uint32_t per = kLWin / 64;   // positions per lane
        if (p - base < kLWin) return;
        const uint32_t nb = p & ~(kLWin - 1);
        if (nb == base + kLWin) {
            lhv = lhv_n;
            liv = liv_n;
        } else {
            lhv = wloadL(hd + nb + per * lane_id());
            liv = wloadL(idx + nb + per * lane_id());
        }
        base = ibase = nb;
        lhv_n = wloadL(hd + nb + kLWin + per * lane_id());
        liv_n = wloadL(idx + nb + kLWin + per * lane_id());
    }
    __device__ __forceinline__ void window(uint32_t p)
    {
        if constexpr (LAZY) {
            lazy_windows(p);
            return;
        }
        if (p - base < 512u) return;
        base = p & ~7u;
        const uint32_t q = base + 8 * lane_id();
        hv = *reinterpret_cast<const uint4 *>(hd + q);
        fv0 = *reinterpret_cast<const uint4 *>(rf + q);
        fv1 = *reinterpret_cast<const uint4 *>(rf + q + 4);
        rv0 = *reinterpret_cast<const uint4 *>(rr + q);
        rv1 = *reinterpret_cast<const uint4 *>(rr + q + 4);
        uint32_t b[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = q + j < n ? src[q + j] : 0u;
        bv0 = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24;
        bv1 = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
    }
    __device__ __forceinline__ static uint32_t pick4(const uint4 &v, uint32_t l, uint32_t e)   // dword e (0..3) of lane l
    {
        const uint32_t a = lane_val(v.x, l), b = lane_val(v.y, l), c = lane_val(v.z, l), d = lane_val(v.w, l);
        return e == 0 ? a : e == 1 ? b : e == 2 ? c : d;
    }
    __device__ __forceinline__ uint32_t u32_at(const uint4 &v0, const uint4 &v1, uint32_t p)
    {
        const uint32_t off = p - base, l = off >> 3, e = off & 7;
        return e < 4 ? pick4(v0, l, e) : pick4(v1, l, e - 4);
    }

    // ---- bit output ----------------------------------------------------
    __device__ __forceinline__ void store_words(uint32_t first, uint32_t count)   // stg[0..count) -> out32[first..)
    {
        for (uint32_t i = lane_id(); i < count; i += 64) {
            if (first + i < out_words) out32[first + i] = sm.stg[i];
            else overflow = true;
        }
    }
    // every lane contributes nbits (<= 57) bits of val; lanes in order
    __device__ __forceinline__ void emit_par(uint64_t val, uint32_t nbits)
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
        __device__ __forceinline__ void operator()(uint32_t v, int nb)
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
    __device__ __forceinline__ Serial serial_begin() { return Serial{*this, sm.stg[0], bitpos & 31, bitpos >> 5}; }
    __device__ __forceinline__ void serial_end(const Serial &s)   // lane 0 publishes; all lanes pick up bitpos
    {
        sm.stg[0] = (uint32_t)s.acc;
        sm.bcast[0] = s.word * 32 + s.accbits;
    }
    __device__ __forceinline__ void windup()   // bi_windup: to a byte boundary (the bits above are zero)
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
    __device__ __forceinline__ uint32_t byte(uint32_t p)
    {
        if constexpr (LAZY) {
            ensure(p);
            return lwin[p - wbase];
        }
        window(p);
        const uint32_t off = p - base, l = off >> 3, e = off & 7;
        const uint32_t w = e < 4 ? lane_val(bv0, l) : lane_val(bv1, l);
        return (w >> ((e & 3) * 8)) & 0xffu;
    }
    // zlib's head[] as p is inserted (0 = NIL)
    __device__ __forceinline__ uint32_t head(uint32_t p)
    {
        window(p);
        if constexpr (LAZY) {
            constexpr uint32_t per = kLWin / 64;
            const uint32_t off = p - base, l = off / per, e = off % per;
            return (pickL(lhv, l, e >> 1) >> ((e & 1) * 16)) & 0xffffu;
        }
        const uint32_t off = p - base, l = off >> 3, e = off & 7;
        const uint32_t w = pick4(hv, l, e >> 1);
        return (w >> ((e & 1) * 16)) & 0xffffu;
    }
    __device__ __forceinline__ void slide()   // fill_window's slide: past the end, the stale copy WSIZE back
    {
        if constexpr (LAZY) {
            wslid = true;
            for (uint32_t P = max(n, wbase) + lane_id(); P < min(n + MAX_MATCH, wbase + kLazyWin); P += 64)
                lwin[P - wbase] = src[P - WSIZE];
            wave_sync();
        }   // (K2 compared against the slid window already)
    }
    // the byte zlib's window holds at input position P (P < wbase + kLazyWin):
    // the strip, then zeros (fill_window's high_water zeroing) or, once slid, the stale copy
    __device__ __forceinline__ uint32_t win_src(uint32_t P) const
    {
        return P < n ? (uint32_t)src[P] : (wslid && P - WSIZE < n ? (uint32_t)src[P - WSIZE] : 0u);
    }
    __device__ __forceinline__ void fill(uint32_t from, uint32_t to)   // window bytes of input positions [from, to)
    {
        for (uint32_t P = from + lane_id(); P < to; P += 64) lwin[P - wbase] = (uint8_t)win_src(P);
    }
    // the whole window [wbase, wbase + kLazyWin) again (after a flush, whose tree arrays share
    // its LDS): 16 bytes per lane from the strip where they lie inside it, the rest one at a time
    __device__ __forceinline__ void reload()
    {
        wave_sync();
        uint4 *w = reinterpret_cast<uint4 *>(lwin);
        uint32_t from = wbase;
        const uint32_t to = wbase + kLazyWin;
        if ((((uintptr_t)(src + from)) & 15) == 0) {
            const uint32_t vend = min(to, n & ~15u);
            for (uint32_t P = from + 16 * lane_id(); P < vend; P += 1024)
                w[(P - wbase) >> 4] = *reinterpret_cast<const uint4 *>(src + P);
            from = max(from, vend);
        }
        fill(from, to);
        wave_sync();
    }
    // keep [p - kNearDist, p + kLazyAhead) in the window: shift it forward when p runs
    // ahead (chain candidates farther back than the window read the strip in HBM:
    // Wave::g4 / far_lcp / wave_lcp_at)
    __device__ __forceinline__ void ensure(uint32_t p)
    {
        if (p + kLazyAhead <= wbase + kLazyWin) return;
        const uint32_t nb = (p > kNearDist ? p - kNearDist : 0u) & ~255u;
        const uint32_t d = nb - wbase;   // > 0, a multiple of 256
        VCF_ZPROF_COUNT(n_shift);
        uint4 *w = reinterpret_cast<uint4 *>(lwin);
        // forward copy in increasing order: chunk k reads at >= d + 1024 k, writes below d + 1024 k
        for (uint32_t o = 16 * lane_id(); o < kLazyWin - d; o += 1024) w[o >> 4] = w[(o + d) >> 4];
        wave_sync();
        const uint32_t old_end = wbase + kLazyWin;
        wbase = nb;
        // the new bytes: 16 per lane from the strip where they lie inside it (the range is
        // 256-aligned), the rest (past the end: zeros or the slid copy) one at a time
        uint32_t from = old_end;
        const uint32_t to = nb + kLazyWin;
        if ((((uintptr_t)(src + from)) & 15) == 0) {
            const uint32_t vend = min(to, n & ~15u);
            for (uint32_t P = from + 16 * lane_id(); P < vend; P += 1024)
                w[(P - wbase) >> 4] = *reinterpret_cast<const uint4 *>(src + P);
            from = max(from, vend);
        }
        fill(from, to);
        wave_sync();
    }
    // ---- candidates farther back than the window: the strip's bytes in HBM
    // (c + 274 < p <= n for every such read: real strip bytes, never the
    // zeros or the slid copy past the end)
    __device__ __forceinline__ uint32_t g4(uint32_t P) const   // 4 bytes at input position P (unaligned)
    {
        uint32_t d;
        __builtin_memcpy(&d, src + P, 4);
        return d;
    }
    // far_lcp: lane_lcp with the first string at input position c in HBM
    __device__ __forceinline__ uint32_t far_lcp(uint32_t c, uint32_t b, uint32_t cap, uint32_t from)
    {
        uint32_t l = from;
        while (l < cap) {
            const uint32_t x0 = g4(c + l) ^ ld4(b + l), x1 = g4(c + l + 4) ^ ld4(b + l + 4);
            const uint32_t x2 = g4(c + l + 8) ^ ld4(b + l + 8), x3 = g4(c + l + 12) ^ ld4(b + l + 12);
            if (x0 | x1 | x2 | x3) {
                l += x0 ? 0 : x1 ? 4 : x2 ? 8 : 12;
                l += (uint32_t)__builtin_ctz(x0 ? x0 : x1 ? x1 : x2 ? x2 : x3) >> 3;
                break;
            }
            l += 16;
        }
        return min(l, (uint32_t)MAX_MATCH);
    }
    // wave_lcp with the first string at input position c: from the window when it is there
    __device__ __forceinline__ uint32_t wave_lcp_at(uint32_t c, uint32_t b)
    {
        if (c >= wbase) return wave_lcp(c - wbase, b);
        const uint32_t x = g4(c + 4 * lane_id()) ^ ld4(b + 4 * lane_id());
        const uint64_t m = __ballot(x != 0);
        if (m) {
            const uint32_t f = (uint32_t)__ffsll((unsigned long long)m) - 1;
            return 4 * f + ((uint32_t)__builtin_ctz(lane_val(x, f)) >> 3);
        }
        uint32_t l = 256;
        if (src[c + 256] == lwin[b + 256]) l = src[c + 257] == lwin[b + 257] ? 258 : 257;
        return l;
    }
    __device__ __forceinline__ uint32_t ld4(uint32_t a)   // window offsets
    {
        const uint32_t *w32 = reinterpret_cast<const uint32_t *>(lwin);
        return __builtin_amdgcn_alignbyte(w32[(a >> 2) + 1], w32[a >> 2], a & 3);
    }
    __device__ __forceinline__ uint32_t hash_at(uint32_t q) { return hash3(lwin[q], lwin[q + 1], lwin[q + 2]); }   // window offset
    // common prefix of the strings at a and b, up to MAX_MATCH: one wave-wide compare
    __device__ __forceinline__ uint32_t wave_lcp(uint32_t a, uint32_t b)
    {
        const uint32_t x = ld4(a + 4 * lane_id()) ^ ld4(b + 4 * lane_id());
        const uint64_t m = __ballot(x != 0);
        if (m) {
            const uint32_t f = (uint32_t)__ffsll((unsigned long long)m) - 1;
            return 4 * f + ((uint32_t)__builtin_ctz(lane_val(x, f)) >> 3);
        }
        uint32_t l = 256;
        if (lwin[a + 256] == lwin[b + 256]) l = lwin[a + 257] == lwin[b + 257] ? 258 : 257;
        return l;
    }
    // one lane, 16 bytes per step, until a difference or `cap` bytes (a result >= cap is
    // not exact: the caller only needs to know it reached cap)
    __device__ __forceinline__ uint32_t lane_lcp(uint32_t a, uint32_t b, uint32_t cap = MAX_MATCH, uint32_t from = 0)
    {
        uint32_t l = from;
        while (l < cap) {
#if VCF_ZLIB_PROF
            ++lcp_steps;
#endif
            const uint32_t x0 = ld4(a + l) ^ ld4(b + l), x1 = ld4(a + l + 4) ^ ld4(b + l + 4);
            const uint32_t x2 = ld4(a + l + 8) ^ ld4(b + l + 8), x3 = ld4(a + l + 12) ^ ld4(b + l + 12);
            if (x0 | x1 | x2 | x3) {
                l += x0 ? 0 : x1 ? 4 : x2 ? 8 : 12;
                l += (uint32_t)__builtin_ctz(x0 ? x0 : x1 ? x1 : x2 ? x2 : x3) >> 3;
                break;
            }
            l += 16;
        }
        return min(l, (uint32_t)MAX_MATCH);
    }
#if VCF_ZLIB_PROF
    unsigned long long t_longest = 0, t_flush = 0, n_longest = 0, n_rounds = 0, n_shift = 0;
    unsigned long long t_head = 0, n_lcp = 0, n_cand = 0, n_pf = 0, t_wait = 0, t_r0 = 0, t_r1 = 0, t_r2 = 0;
    unsigned long long n_headhit = 0, n_farround = 0, n_farlcp = 0, n_farwave = 0, n_farhead = 0, n_none = 0;
    __device__ __forceinline__ bool longest(uint32_t p, uint32_t hdp, uint32_t prev_len, uint32_t chain, uint32_t nice,
                            uint32_t limit, uint32_t &len, uint32_t &pos)
    {
        const unsigned long long t0 = clock64();
        const bool r = longest_impl(p, hdp, prev_len, chain, nice, limit, len, pos);
        t_longest += clock64() - t0;
        ++n_longest;
        return r;
    }
    __device__ __forceinline__ void flush(uint32_t stored_len, bool buf_ok, uint32_t block_start, bool last)
    {
        const unsigned long long t0 = clock64();
        flush_impl(stored_len, buf_ok, block_start, last);
        t_flush += clock64() - t0;
    }
#else
    __device__ __forceinline__ bool longest(uint32_t p, uint32_t hdp, uint32_t prev_len, uint32_t chain, uint32_t nice,
                            uint32_t limit, uint32_t &len, uint32_t &pos)
    {
        return longest_impl(p, hdp, prev_len, chain, nice, limit, len, pos);
    }
    __device__ __forceinline__ void flush(uint32_t stored_len, bool buf_ok, uint32_t block_start, bool last)
    {
        flush_impl(stored_len, buf_ok, block_start, last);
    }
#endif
    // candidates 0..127 of the chain of a position whose bucket slot is ip (both rounds,
    // whatever chain limit the call will have: the reduced limit of one call may be the
    // full limit of the next)
    __device__ __forceinline__ void fetch_cands(uint32_t ip, uint32_t &c0, uint32_t &c1)
    {
        const uint16_t *vs = sorted;
        const uint32_t g0 = lane_id(), g1 = 64 + lane_id();
        c0 = wload16(vs + (g0 < ip ? ip - 1 - g0 : 0u));
        c1 = wload16(vs + (g1 < ip ? ip - 1 - g1 : 0u));
    }
    __device__ __forceinline__ uint32_t idx_known(uint32_t q)   // idx[q] from the windows, or ~0 if outside them
    {
        constexpr uint32_t per = kLWin / 64;
        const uint32_t off = q - ibase;
        if (off >= 2 * kLWin) return 0xffffffffu;
        const uint32_t o = off & (kLWin - 1), e = o % per;
        return (pickL(off < kLWin ? liv : liv_n, o / per, e >> 1) >> ((e & 1) * 16)) & 0xffffu;
    }
    // VCF_ZX_PREDICT (A/B): the position deflate_slow calls longest_match at next follows
    // from this call's result and prev_length: with match_length ml (this call's length,
    // clamped to the lookahead, TOO_FAR applied; prev_length when nothing was found), the
    // previous match is emitted when prev_length >= MIN_MATCH and ml <= prev_length (next
    // call at p - 1 + prev_length), else a match of at least `lazy` is emitted at the next
    // step (next call at p + ml), else the parse moves to p + 1.  Slot a takes that
    // position; slot b (PREDICT 2) p + 1 as well, for the calls the hash head skips.
    __device__ __forceinline__ uint32_t predict_next(uint32_t p, bool found, uint32_t len, uint32_t pos,
                                                     uint32_t prev_len) const
    {
        const uint32_t look = n - p;
        uint32_t ml = found ? min(len, look) : min(prev_len, look);
        if (found && ml == (uint32_t)MIN_MATCH && p - pos > (uint32_t)TOO_FAR) ml = MIN_MATCH - 1;
        if (prev_len >= (uint32_t)MIN_MATCH && ml <= prev_len) return p - 1 + prev_len;
        if (ml >= lazy && ml >= (uint32_t)MIN_MATCH) return p + ml;
        return p + 1;
    }
    __device__ __forceinline__ void prefetch_next(uint32_t p, uint32_t len, bool found = false, uint32_t pos = 0,
                                                  uint32_t prev_len = 0)
    {
#if VCF_ZX_PREDICT
        const uint32_t qa = predict_next(p, found, len, pos, prev_len);
        const uint32_t qb = VCF_ZX_PREDICT == 2 ? p + 1 : qa;
#else
        const uint32_t qa = p + 1, qb = p + (len >= (uint32_t)MIN_MATCH ? len : 1u);
#endif
        const uint32_t ia = idx_known(qa);
        pfa_p = ia != 0xffffffffu && qa + MIN_MATCH <= n ? qa : 0xffffffffu;
        if (pfa_p != 0xffffffffu) fetch_cands(ia, pfa0, pfa1);
        if constexpr (VCF_ZX_PREDICT != 1) {   // (1: one exact slot; b unused)
            const uint32_t ib = qb != qa ? idx_known(qb) : 0xffffffffu;
            pfb_p = ib != 0xffffffffu && qb + MIN_MATCH <= n ? qb : 0xffffffffu;
            if (pfb_p != 0xffffffffu) fetch_cands(ib, pfb0, pfb1);
        }
    }
    __device__ __forceinline__ bool longest_impl(uint32_t p, uint32_t hdp, uint32_t prev_len, uint32_t chain,
                                                 uint32_t nice, uint32_t limit, uint32_t &len, uint32_t &pos)
    {
        if constexpr (LAZY) {
            const bool r = lazy_longest(p, hdp, prev_len, chain, nice, limit, len, pos);
            prefetch_next(p, r ? len : 0u, r, pos, prev_len);
            return r;
        }
        // the K2 results: the full chain's, or the reduced chain's once prev_len >= good
        window(p);
        const uint32_t r = prev_len >= good ? u32_at(rv0, rv1, p) : u32_at(fv0, fv1, p);
        len = r >> 16;
        pos = p - (r & 0xffffu);
        return len > prev_len;
    }
#if VCF_ZLIB_PROF
    uint32_t lcp_steps = 0;
#endif
    __device__ __forceinline__ bool lazy_longest(uint32_t p, uint32_t hdp, uint32_t prev_len, uint32_t chain,
                                                 uint32_t nice, uint32_t limit, uint32_t &len, uint32_t &pos)
    {
#if VCF_ZLIB_PROF
        const unsigned long long th0 = clock64();
        if (p == pfa_p || p == pfb_p) ++n_pf;
#endif
        {
            // the first candidate (chain order) reaching max(nice, prev_len+1), else the
            // first reaching the longest length found, if longer than prev_len
            ensure(p);
            // window offsets from here on: p's own bytes are in the window; a candidate below
            // wbase (at most MAX_DIST back, always c + 274 < p, so real strip bytes) is
            // read from HBM instead (the `far` lanes)
            const uint32_t wp = p - wbase;
#if VCF_ZX_WINCHECK
            cur_p = p;
            for (uint32_t P0 = (p > 128u + wbase ? p - 128u : wbase); P0 < p + 256u; P0 += 64) {
                const uint32_t P = P0 + lane_id();
                const uint32_t got = lwin[P - wbase], want = win_src(P);
                wincheck(2u, P, P < wbase + kLazyWin && got != want, got, want);
            }
#endif
            const uint32_t Tn = max(nice, prev_len + 1);
            lazy_windows(p);
            const uint32_t ip = idx_known(p);
            // the first two chain rounds' candidates: prefetched by the previous call, or
            // requested here before the head compare so their latency overlaps it
            uint32_t pre0, pre1;
            if (p == pfa_p) {
                pre0 = pfa0;
                pre1 = pfa1;
            } else if (p == pfb_p) {
                pre0 = pfb0;
                pre1 = pfb1;
            } else {
                fetch_cands(ip, pre0, pre1);
            }
            // a chain round's LDS reads that do not depend on the head's length: the
            // candidate's first four bytes (its hash) and the first 16 bytes of the
            // compare, on every lane (a lane off the chain reads p's own bytes)
            struct RoundRd {
                uint32_t c, wc, c4, x16[4];
                bool v, far;
            };
            auto rd = [&](uint32_t b) -> RoundRd {
                RoundRd r;
                const uint32_t gk = b + lane_id();
                r.v = gk < chain && gk < ip;
                r.c = !r.v ? 0u : b == 0 ? pre0 : b == 64 ? pre1 : wload16(sorted + ip - 1 - gk);
                // sorted[] runs on past the bucket: a candidate of another bucket can be any
                // position, so the bucket end must not be judged from bytes read at it before
                // it is known to be p's: p's own bucket holds only earlier positions, and those
                // past `limit` are real strip bytes (in the window, or in HBM when farther back
                // than the window reaches): c < p first, then the hash.
                r.v = r.v && r.c < p && (gk == 0 || r.c > limit);
                r.far = r.v && r.c < wbase;
                r.wc = r.v && !r.far ? r.c - wbase : wp;
                r.c4 = ld4(r.wc);
#pragma unroll
                for (int u = 0; u < 4; ++u) r.x16[u] = ld4(r.wc + 4 * u) ^ ld4(wp + 4 * u);
                if (__ballot(r.far)) {   // wave-uniform: this round reaches past the window
                    if (r.far) {
                        r.c4 = g4(r.c);
                        r.x16[0] = r.c4 ^ ld4(wp);
#pragma unroll
                        for (int u = 1; u < 4; ++u) r.x16[u] = g4(r.c + 4 * u) ^ ld4(wp + 4 * u);
                    }
                }
                return r;
            };
            // round 0's reads in the round (VCF_ZX_EARLY0 = 1: issued with the head compare's)
            RoundRd r0;
            if (VCF_ZX_EARLY0) r0 = rd(0);
            const uint32_t hp = hash_at(wp);
            const uint32_t l1 = wave_lcp_at(hdp, wp);
#if VCF_ZLIB_PROF
            if (hdp < wbase) ++n_farhead;
            {
                const unsigned long long th1 = clock64();
                t_head += th1 - th0;
                asm volatile("" ::"v"(pre0), "v"(pre1));   // (diagnostic) wait for the candidates here
                t_wait += clock64() - th1;
            }
#endif
            if (l1 >= Tn) {
                len = l1;
                pos = hdp;
#if VCF_ZLIB_PROF
                ++n_headhit;
#endif
                return true;
            }
            // only a candidate longer than F = max(prev_len, the head's length) can change the
            // result, and such a one matches at bytes F-1 and F (longest_match's scan_end test)
            const uint32_t F = max(prev_len, l1);
            uint32_t best = prev_len, bpos = 0;
            bool found = false;
            for (uint32_t b = 0; b < chain; b += 64) {
                VCF_ZPROF_COUNT(n_rounds);
#if VCF_ZLIB_PROF
                const unsigned long long tr0 = clock64();
#endif
                const uint32_t gk = b + lane_id();
                const RoundRd rr = VCF_ZX_EARLY0 && b == 0 ? r0 : rd(b);
                bool v = rr.v;
                const bool far = rr.far;
                const uint32_t c = rr.c, wc = rr.wc, c4 = rr.c4;
                const uint32_t *x16 = rr.x16;
                // zlib's scan_end bytes at F (known only after the head compare)
                uint32_t e0 = lwin[wc + F - 1], e1 = lwin[wc + F];
                if (__ballot(far)) {
                    if (far) {
                        e0 = src[c + F - 1];
                        e1 = src[c + F];
                    }
                }
                const bool se = e1 == lwin[wp + F] && e0 == lwin[wp + F - 1];
#if VCF_ZLIB_PROF
                if (__ballot(far)) ++n_farround;
#endif
#if VCF_ZX_WINCHECK
                {
                    const uint32_t want = v ? win_src(c) | win_src(c + 1) << 8 | win_src(c + 2) << 16 | win_src(c + 3) << 24 : c4;
                    wincheck(3u, c, v && c4 != want, c4, want);
                    wincheck(4u, c, v && !far && c < wbase, c, wbase);   // a near read below the window
                }
#endif
                v = v && hash3(c4 & 0xffu, (c4 >> 8) & 0xffu, (c4 >> 16) & 0xffu) == hp;
                const uint64_t stop = __ballot(!v);
#if VCF_ZLIB_PROF
                const unsigned long long tr1 = clock64();
                t_r0 += tr1 - tr0;
#endif
                const uint32_t nv = stop ? (uint32_t)__ffsll((unsigned long long)stop) - 1 : 64u;
                v = lane_id() < nv;
                const bool cand = v && gk != 0 && se;
#if VCF_ZLIB_PROF
                n_cand += (unsigned long long)__popcll(__ballot(cand));
                lcp_steps = 0;
#endif
                // compared up to Tn only: a candidate reaching Tn ends the call, and its
                // full length (zlib compares on to MAX_MATCH) comes from one wave compare
                uint32_t l = 0;
                if (v && gk == 0) l = l1;
                if (cand) {
                    const uint32_t x = x16[0] | x16[1] | x16[2] | x16[3];
                    if (x) {
                        const uint32_t q = x16[0] ? 0u : x16[1] ? 4u : x16[2] ? 8u : 12u;
                        l = q + ((uint32_t)__builtin_ctz(x16[0] ? x16[0] : x16[1] ? x16[1] : x16[2] ? x16[2] : x16[3]) >> 3);
                    } else if (!far) {
                        l = lane_lcp(wc, wp, VCF_ZX_NOCAP ? (uint32_t)MAX_MATCH : Tn, 16u);
                    } else {
                        l = far_lcp(c, wp, VCF_ZX_NOCAP ? (uint32_t)MAX_MATCH : Tn, 16u);
                    }
                }
#if VCF_ZLIB_PROF
                n_farlcp += (unsigned long long)__popcll(__ballot(cand && far && !(x16[0] | x16[1] | x16[2] | x16[3])));
#endif
#if VCF_ZLIB_PROF
                {
                    uint32_t ms = lcp_steps;
#pragma unroll
                    for (int d = 32; d >= 1; d >>= 1) ms = max(ms, (uint32_t)__shfl_xor(ms, d, 64));
                    n_lcp += uni(ms);
                }
#endif
                const uint64_t hit = __ballot(v && l >= Tn);
#if VCF_ZLIB_PROF
                const unsigned long long tr2 = clock64();
                t_r1 += tr2 - tr1;
#endif
                if (hit) {
                    const uint32_t k = (uint32_t)__ffsll((unsigned long long)hit) - 1;
                    pos = lane_val(c, k);
#if VCF_ZLIB_PROF
                    if (!(k == 0 && b == 0) && pos < wbase) ++n_farwave;
#endif
                    len = k == 0 && b == 0 ? l1 : wave_lcp_at(pos, wp);
                    return true;
                }
                // the first lane with the longest length beyond best: step from improvement
                // to improvement in lane order (few steps; no cross-lane max reduction)
                for (uint64_t better = __ballot(v && l > best); better; better = __ballot(v && l > best)) {
                    const uint32_t k = (uint32_t)__ffsll((unsigned long long)better) - 1;
                    best = lane_val(l, k);
                    bpos = lane_val(c, k);
                    found = true;
                }
#if VCF_ZLIB_PROF
                t_r2 += clock64() - tr2;
#endif
                if (nv < 64) break;
            }
            len = best;
            pos = bpos;
#if VCF_ZLIB_PROF
            if (!found) ++n_none;
#endif
            return found;
        }
    }
    __device__ __forceinline__ bool tally(uint32_t dist, uint32_t lc)
    {
        if (lane_id() == 0) st_l2(syms + nsym, dist << 8 | lc);   // counted at flush
        ++nsym;
        return nsym == (uint32_t)LIT_BUFSIZE - 1;
    }
    __device__ __forceinline__ void init_freqs()
    {
        for (uint32_t i = lane_id(); i < (uint32_t)L_CODES; i += 64) sm.lfreq[i] = 0;
        if (lane_id() < (uint32_t)D_CODES) sm.dfreq[lane_id()] = 0;
        if (lane_id() < (uint32_t)BL_CODES) sm.bfreq[lane_id()] = 0;
        wave_sync();
    }
    __device__ __forceinline__ static void add16(uint16_t *a, uint32_t i)   // a[i]++ as a packed 32-bit LDS add (no carry: < 65536)
    {
        atomicAdd(reinterpret_cast<uint32_t *>(a) + (i >> 1), 1u << ((i & 1) * 16));
    }
    // _tr_tally's counts for the whole block at once (LDS atomics), then init_block's END_BLOCK
    __device__ __forceinline__ void count_block()
    {
        for (uint32_t i = lane_id(); i < nsym; i += 64) {
            const uint32_t sy = ld_l2(syms + i), dist = sy >> 8, lc = sy & 0xff;
            if (dist == 0) {
                add16(sm.lfreq, lc);
            } else {
                add16(sm.lfreq, (uint32_t)length_code((int)lc) + 257);
                add16(sm.dfreq, (uint32_t)dist_code((int)(dist - 1)));
            }
        }
        wave_sync();
        if (lane_id() == 0) sm.lfreq[END_BLOCK] += 1;   // init_block's END_BLOCK count
        wave_sync();
    }
    __device__ __forceinline__ void flush_impl(uint32_t stored_len, bool buf_ok, uint32_t block_start, bool last)
    {
        __threadfence();   // the block's symbols (lane 0's stores) before the other lanes read them
        wave_sync();
        init_freqs();   // (here, not after the flush: the lazy window lies over these arrays in between)
        count_block();
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
                emit_par(q < stored_len ? (uint32_t)src[block_start + q] : 0u, q < stored_len ? 8u : 0u);
            }
        } else {
            if (kind == 1) {
                for (uint32_t i = lane_id(); i < (uint32_t)L_CODES; i += 64) {
                    sm.lfreq[i] = (uint16_t)static_lcode((int)i);   // (Code shares Freq's storage)
                    sm.llen[i] = (uint16_t)static_llen((int)i);
                }
                if (lane_id() < (uint32_t)D_CODES) {
                    sm.dfreq[lane_id()] = (uint16_t)static_dcode((int)lane_id());
                    sm.dlen[lane_id()] = 5;
                }
                wave_sync();
            }
            for (uint32_t i = 0; i < nsym; i += 64) {
                const uint32_t q = i + lane_id();
                uint64_t v = 0;
                int nb = 0;
                if (q < nsym) symbol_bits(ld_l2(syms + q), sm.lfreq, sm.llen, sm.dfreq, sm.dlen, v, nb);
                emit_par(v, (uint32_t)nb);
            }
            emit_par(lane_id() == 0 ? sm.lfreq[END_BLOCK] : 0u, lane_id() == 0 ? sm.llen[END_BLOCK] : 0u);
        }
        nsym = 0;
        if (last) windup();
        if constexpr (LAZY) {
            if (VCF_ZX_ALIAS && !last) reload();   // the flush used the window's LDS
        }
    }
};

template <bool LAZY>
struct ParseShared {
    ParseSmem sm;
};
template <>
#ifndef VCF_ZX_LDSPAD   // (diagnostic) extra LDS per lazy-parse workgroup: fewer strips per CU
#define VCF_ZX_LDSPAD 0
#endif
struct ParseShared<true> {
#if VCF_ZX_ALIAS
    union {
        ParseSmem sm;
        struct {
            uint32_t keep[offsetof(ParseSmem, lfreq) / 4];   // stg, bcast
            uint32_t win32[kLazyWin / 4];                    // the sliding window (Wave::ensure)
        } w;
    };
#else
    ParseSmem sm;
    struct {
        uint32_t win32[kLazyWin / 4];   // the sliding window of the strip (Wave::ensure)
    } w;
#endif
#if VCF_ZX_LDSPAD
    uint32_t pad[VCF_ZX_LDSPAD / 4];
#endif
};
static_assert(VCF_ZX_LDSPAD || VCF_ZX_WG != 1 || sizeof(ParseShared<true>) <= 10240 ||
                  (!VCF_ZX_ALIAS && VCF_ZX_LAZYWIN != 3840),
              "sixteen lazy-parse workgroups per CU");

#ifdef VCF_ZX_WPE   // A/B (diagnostic builds): registers capped for this many waves per SIMD
#define VCF_ZX_WPE_ATTR __attribute__((amdgpu_waves_per_eu(VCF_ZX_WPE, VCF_ZX_WPE)))
#else
#define VCF_ZX_WPE_ATTR
#endif
// The lazy parse's dispatch order: a strip's parse time grows with its literals and
// short matches, and the last workgroups dispatched form the kernel's tail on an
// otherwise idle GPU -- so the strips go out longest first (by K1's distinct-hash
// count, in 256 classes), the short ones last.  One workgroup: a counting sort of the
// round's strips by class, descending; position i of the order is stored in strip
// slot i's workspace (kSumOff + 28).  The order inside a class is whatever the
// atomics give: it changes only the schedule, never a strip's bytes.
#ifndef VCF_ZX_LPT   // A/B (diagnostic builds)
#define VCF_ZX_LPT 1
#endif
constexpr int kLptThreads = 1024;
__device__ __forceinline__ uint32_t lpt_class(uint32_t dsum) { return 255u - min(255u, dsum >> 7); }
__global__ __launch_bounds__(kLptThreads) void zlib_lpt_kernel(uint8_t *__restrict__ ws, uint32_t cnt)
{
    __shared__ uint32_t hist[256];
    const uint32_t tid = threadIdx.x;
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < cnt; i += kLptThreads)
        atomicAdd(&hist[lpt_class(*reinterpret_cast<const uint32_t *>(ws + i * kWsPerStrip + kSumOff + 24))], 1u);
    __syncthreads();
    if (tid < 64) {   // exclusive scan of the 256 classes, 4 per lane
        uint32_t c[4], t = 0;
        for (int k = 0; k < 4; ++k) t += (c[k] = hist[4 * tid + k]);
        uint32_t tot;
        uint32_t run = excl_scan(t, tot);
        for (int k = 0; k < 4; ++k) {
            hist[4 * tid + k] = run;
            run += c[k];
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < cnt; i += kLptThreads) {
        const uint32_t k = lpt_class(*reinterpret_cast<const uint32_t *>(ws + i * kWsPerStrip + kSumOff + 24));
        const uint32_t pos = atomicAdd(&hist[k], 1u);
        *reinterpret_cast<uint32_t *>(ws + (uint64_t)pos * kWsPerStrip + kSumOff + 28) = i;
    }
}
// one strip's deflate_slow, trees and bits by the calling wave
template <bool LAZY>
__device__ __forceinline__ void parse_strip(const uint8_t *__restrict__ in, int64_t frame_bytes, int32_t strip_bytes,
                                            int32_t spf, int32_t level, uint8_t *__restrict__ out, int64_t slot_bytes,
                                            int32_t *__restrict__ sizes, uint8_t *__restrict__ ws, int64_t s0,
                                            int64_t s, ParseShared<LAZY> &sh)
{
    ParseSmem &sm = sh.sm;
    const Strip S = strip_of(in, frame_bytes, strip_bytes, spf, ws, s0, s);
    const uint32_t lane = lane_id();
#ifndef VCF_ZX_PARSEPRIO   // the lazy parse at wave priority 3: beside the side stream's K2b waves on a CU it wins issue (-0.7 %)
#define VCF_ZX_PARSEPRIO 3
#endif
    if (LAZY && VCF_ZX_PARSEPRIO) __builtin_amdgcn_s_setprio(VCF_ZX_PARSEPRIO);
#if VCF_ZX_LDSZERO   // (diagnostic) LDS cleared first: a read of never-written LDS becomes deterministic
    for (uint32_t i = lane; i < sizeof(sh) / 4; i += 64) reinterpret_cast<uint32_t *>(&sh)[i] = 0;
    wave_sync();
#endif
    Config cfg;
    level_config(level, cfg);
    for (uint32_t i = lane; i < (uint32_t)kStgWords; i += 64) sm.stg[i] = 0;
    Wave<LAZY> wv(sm, S.src, S.n, S.ws, (uint32_t)cfg.good, reinterpret_cast<uint32_t *>(out + s * slot_bytes),
                  (uint32_t)(slot_bytes >> 2));
    wv.lazy = (uint32_t)cfg.lazy;
    if constexpr (LAZY) {
        // the window's first kLazyWin bytes: the strip, then zeros (fill_window's high_water zeroing)
        uint8_t *win = reinterpret_cast<uint8_t *>(sh.w.win32);
        if (((uintptr_t)S.src & 3) == 0) {
            const uint32_t *s32 = reinterpret_cast<const uint32_t *>(S.src);
            for (uint32_t q = lane; q < kLazyWin / 4; q += 64) sh.w.win32[q] = 4 * q + 4 <= S.n ? s32[q] : 0u;
            wave_sync();
            for (uint32_t p = (S.n & ~3u) + lane; p < min(S.n, kLazyWin); p += 64) win[p] = S.src[p];
        } else {
            for (uint32_t p = lane; p < kLazyWin; p += 64) win[p] = p < S.n ? S.src[p] : 0u;
        }
        wv.lwin = win;
#if VCF_ZX_WINCHECK
        wv.dbg_strip = (uint32_t)s;
#endif
        wv.idx = reinterpret_cast<const uint16_t *>(S.ws + kIdxOff);
        wv.sorted = reinterpret_cast<const uint16_t *>(S.ws + kSortOff);
    }
    if (!LAZY || !VCF_ZX_ALIAS) wv.init_freqs();   // (each flush zeroes them again first)
    wave_sync();   // the staging words and the window

    const uint32_t hdr = zlib_header(level);
    wv.emit_par(lane == 0 ? ((hdr >> 8) | ((hdr & 0xffu) << 8)) : 0u, lane == 0 ? 16u : 0u);
#if VCF_ZLIB_PROF
    const unsigned long long tp0 = clock64();
#endif
    deflate_slow(wv, S.n, cfg);
#if VCF_ZLIB_PROF
    if (lane == 0) {
        const unsigned long long tp = clock64() - tp0;
        if (LAZY) {
            atomicAdd(&g_zprof[0], tp);
            atomicAdd(&g_zprof[1], wv.t_longest);
            atomicAdd(&g_zprof[2], wv.t_flush);
            atomicAdd(&g_zprof[3], wv.n_longest);
            atomicAdd(&g_zprof[4], wv.n_rounds);
            atomicAdd(&g_zprof[5], wv.n_shift);
            atomicAdd(&g_zprof[6], 1ull);
            atomicAdd(&g_zprof[8], wv.t_head);
            atomicAdd(&g_zprof[9], wv.n_lcp);
            atomicAdd(&g_zprof[10], wv.n_cand);
            atomicAdd(&g_zprof[11], wv.n_pf);
            atomicAdd(&g_zprof[12], wv.t_wait);
            atomicAdd(&g_zprof[13], wv.t_r0);
            atomicAdd(&g_zprof[14], wv.t_r1);
            atomicAdd(&g_zprof[15], wv.t_r2);
            atomicAdd(&g_zprof[16], wv.n_headhit);
            atomicAdd(&g_zprof[17], wv.n_farround);
            atomicAdd(&g_zprof[18], wv.n_farlcp);
            atomicAdd(&g_zprof[19], wv.n_farwave);
            atomicAdd(&g_zprof[20], wv.n_farhead);
            atomicAdd(&g_zprof[21], wv.n_none);
        } else {
            atomicAdd(&g_zprof[7], tp);
        }
    }
#endif
    const uint64_t *sums = reinterpret_cast<const uint64_t *>(S.ws + kSumOff);
    const uint32_t ad = adler32_from_sums(sums[0], sums[1], S.n);
    const uint32_t be = (ad >> 24) | ((ad >> 8) & 0xff00u) | ((ad << 8) & 0xff0000u) | (ad << 24);
    wv.emit_par(lane == 0 ? be : 0u, lane == 0 ? 32u : 0u);
    if (wv.bitpos & 31) wv.store_words(wv.bitpos >> 5, 1);
    const bool ovf = __ballot(wv.overflow) != 0;
    if (lane == 0) sizes[s] = ovf ? -1 : (int32_t)(wv.bitpos >> 3);
}
// LAZY: one strip per wave of the round, in the longest-first order (zlib_lpt_kernel),
// non-lazy strips returning at once; K3 (!LAZY): the waves loop over K1's list of the
// round's non-lazy strips
template <bool LAZY>
__global__ __launch_bounds__(64 * kParseWG) VCF_ZX_WPE_ATTR void zlib_parse_kernel(
    const uint8_t *__restrict__ in, int64_t frame_bytes, int32_t strip_bytes, int32_t spf, int32_t level,
    uint8_t *__restrict__ out, int64_t slot_bytes, int32_t *__restrict__ sizes, uint8_t *__restrict__ ws, int64_t s0,
    int64_t s_end)
{
    __shared__ __attribute__((aligned(16))) ParseShared<LAZY> shs[kParseWG];
    const int wv_id = kParseWG == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    ParseShared<LAZY> &sh = shs[wv_id];
    if constexpr (LAZY) {
        int64_t s = s0 + (int64_t)blockIdx.x * kParseWG + wv_id;
        if (s >= s_end) return;
        if (VCF_ZX_LPT)   // the longest-first order (zlib_lpt_kernel)
            s = s0 + *reinterpret_cast<const uint32_t *>(ws + (s - s0) * kWsPerStrip + kSumOff + 28);
        if (!strip_lazy(strip_of(in, frame_bytes, strip_bytes, spf, ws, s0, s))) return;   // K3 codes this strip
        parse_strip<true>(in, frame_bytes, strip_bytes, spf, level, out, slot_bytes, sizes, ws, s0, s, sh);
    } else {
        const uint32_t cnt = side_count(ws);
        for (uint32_t i = blockIdx.x * kParseWG + wv_id; i < cnt; i += gridDim.x * kParseWG) {
            parse_strip<false>(in, frame_bytes, strip_bytes, spf, level, out, slot_bytes, sizes, ws, s0,
                               s0 + side_strip(ws, i), sh);
            wave_sync();   // the wave's LDS is reused for its next strip
        }
    }
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

int32_t vcf_zlib_max_strip(void) { return dfl::MAX_STRIP; }

#if VCF_ZX_WINCHECK
int vcf_zlib_dbg_read(unsigned int *host8)
{
    return hip_check(hipMemcpyFromSymbol(host8, HIP_SYMBOL(g_zdbg), sizeof(g_zdbg)), "hipMemcpyFromSymbol");
}
#endif
#if VCF_ZLIB_PROF
int vcf_zlib_prof_read(unsigned long long *host24, int reset)
{
    int rc = hip_check(hipMemcpyFromSymbol(host24, HIP_SYMBOL(g_zprof), sizeof(g_zprof)), "hipMemcpyFromSymbol");
    if (rc == VCF_OK && reset) {
        static const unsigned long long z[48] = {};
        rc = hip_check(hipMemcpyToSymbol(HIP_SYMBOL(g_zprof), z, sizeof(z)), "hipMemcpyToSymbol");
    }
    return rc;
}
#endif

int vcf_zlib_set_workspace_budget(int64_t bytes)
{
    if (bytes < 0) return set_error(VCF_ERR_INVALID, "negative workspace budget");
    if (bytes > 0 && bytes < kWsPerStrip)
        return set_error(VCF_ERR_INVALID, "workspace budget %lld below one strip's %lld bytes", (long long)bytes,
                         (long long)kWsPerStrip);
    g_ws_override[current_device()].store(bytes, std::memory_order_relaxed);
    return VCF_OK;
}

int64_t vcf_zlib_workspace(int64_t n_strips)
{
    if (n_strips < 0) return -1;
    const ZRounds zr(n_strips);
    return zr.per * kWsPerStrip;
}

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
    if (((uintptr_t)out_dev & 3) || ((uintptr_t)ws_dev & 15) || ((uintptr_t)sizes_dev & 3))
        return set_error(VCF_ERR_INVALID, "out_dev and sizes_dev must be 4-byte aligned, ws_dev 16-byte aligned");
    if (n_frames == 0 || frame_bytes == 0) return VCF_OK;
    const int64_t spf = vcf_zlib_strip_count(frame_bytes, strip_bytes);
    const int64_t total = spf * n_frames;
    hipStream_t st = (hipStream_t)stream;
    const int chunks = (int)((std::min<int64_t>(strip_bytes, frame_bytes) + kChunk - 1) / kChunk);
    // A round: K1 on the caller's stream; then the two kinds of
    // strips side by side -- the lazy parse of the repetitive strips on the caller's
    // stream, K2a/K2b and the register-window parse of the others on a library side
    // stream (forked by an event, joined back before the next round reuses the
    // workspace).  The two sides touch disjoint strips: their own output slots,
    // sizes and workspace regions; both only read K1's tables.
    // (Round 4's two workspace slots with rounds in flight are gone: with the
    // device-sized budget a call is one round up to ~30 000 strips.)
    AuxStreams &ax = aux_for_current_device();
    std::lock_guard<std::mutex> lock(ax.mu);
    int rc = ax.init();
    if (rc != VCF_OK) return rc;
    // the side stream at the highest priority: its strips are fewer but each takes
    // longer (K2b walks every listed position's chain), and as a normal-priority queue
    // its workgroups only got a CU when a lazy parse left one
    static hipStream_t side_hi[kMaxDevices] = {};
    const int dev = current_device();
    if (!VCF_ZX_NOPRIO && !side_hi[dev]) {
        int least = 0, greatest = 0;
        rc = hip_check(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
        if (rc == VCF_OK)
            rc = hip_check(hipStreamCreateWithPriority(&side_hi[dev], hipStreamNonBlocking, greatest),
                           "hipStreamCreateWithPriority");
        if (rc != VCF_OK) return rc;
    }
    const ZRounds zr(total);
    const hipStream_t ms = st, ss = VCF_ZX_SERIAL ? st : VCF_ZX_NOPRIO ? ax.s[2] : side_hi[dev];
    auto round = [&](int64_t s0, unsigned cnt, uint8_t *ws) -> int {
        int rc0 = hip_check(hipMemsetAsync(ws + kSumOff + 40, 0, 4, ms), "hipMemsetAsync");   // K1's list: empty
        if (rc0 != VCF_OK) return rc0;
        hipLaunchKernelGGL(zlib_sort_kernel, dim3(cnt), dim3(64 * kSortWaves), 0, ms, in_dev, frame_bytes, strip_bytes,
                           (int32_t)spf, ws, s0);
        int rc = hip_check(hipGetLastError(), "zlib_sort_kernel launch");
        if (rc != VCF_OK) return rc;
        if (ss != ms) {
            if ((rc = hip_check(hipEventRecord(ax.big[0], ms), "hipEventRecord")) != VCF_OK) return rc;
            if ((rc = hip_check(hipStreamWaitEvent(ss, ax.big[0], 0), "hipStreamWaitEvent")) != VCF_OK) return rc;
        }
#ifdef VCF_ZX_NOSIDE   // diagnostic builds only: no side kernels (wrong output for non-lazy strips)
        if (false)
#endif
        hipLaunchKernelGGL(zlib_match_kernel, dim3((unsigned)chunks, std::min(cnt, kSideK2a)), dim3(kK2Threads), 0, ss, in_dev,
                           frame_bytes, strip_bytes, (int32_t)spf, level, ws, s0);
        rc = hip_check(hipGetLastError(), "zlib_match_kernel launch");
#ifdef VCF_ZX_NOSIDE
        if (false)
#endif
        if (rc == VCF_OK) {
            hipLaunchKernelGGL(zlib_chain_kernel, dim3(std::min(cnt, kSideK2b), kK2bSplit), dim3(kK2bThreads), 0, ss, in_dev, frame_bytes,
                               strip_bytes, (int32_t)spf, level, ws, s0);
            rc = hip_check(hipGetLastError(), "zlib_chain_kernel launch");
        }
#ifdef VCF_ZX_NOSIDE
        if (false)
#endif
        if (rc == VCF_OK) {
            hipLaunchKernelGGL(zlib_parse_kernel<false>, dim3((std::min(cnt, kSideK3) + kParseWG - 1) / kParseWG),
                               dim3(64 * kParseWG),
                               0, ss, in_dev, frame_bytes, strip_bytes, (int32_t)spf, level, out_dev, slot_bytes,
                               sizes_dev, ws, s0, s0 + (int64_t)cnt);
            rc = hip_check(hipGetLastError(), "zlib_parse_kernel launch");
        }
        if (rc == VCF_OK && VCF_ZX_LPT) {
            hipLaunchKernelGGL(zlib_lpt_kernel, dim3(1), dim3(kLptThreads), 0, ms, ws, cnt);
            rc = hip_check(hipGetLastError(), "zlib_lpt_kernel launch");
        }
        if (rc == VCF_OK) {
            hipLaunchKernelGGL(zlib_parse_kernel<true>, dim3((cnt + kParseWG - 1) / kParseWG), dim3(64 * kParseWG),
                               0, ms, in_dev, frame_bytes, strip_bytes, (int32_t)spf, level, out_dev, slot_bytes,
                               sizes_dev, ws, s0, s0 + (int64_t)cnt);
            rc = hip_check(hipGetLastError(), "zlib_parse_kernel (lazy) launch");
        }
        // join the side stream even after an error, so the caller's stream never runs ahead
        if (ss != ms) {
            int r2 = hip_check(hipEventRecord(ax.join[0], ss), "hipEventRecord");
            if (r2 == VCF_OK) r2 = hip_check(hipStreamWaitEvent(ms, ax.join[0], 0), "hipStreamWaitEvent");
            if (rc == VCF_OK) rc = r2;
        }
        return rc;
    };
    for (int64_t s0 = 0; s0 < total && rc == VCF_OK; s0 += zr.per)
        rc = round(s0, (unsigned)std::min<int64_t>(zr.per, total - s0), (uint8_t *)ws_dev);
    return rc;
}

}  // extern "C"
