// vcf_dwt_band.h -- fused forward levels 1 + 2 of the 2D-DWT encode
// (src/2D-DWT.py:57-78: pywt.wavedec2(mode='per') per YCoCg channel, A6;
// the per-subband deadzone of :113-136), included by vcf_dwt.hip.
//
// Why: level 1's LL is a float64 plane of h/2 x w/2 per channel -- at 4K
// 49.8 MB per frame, twice the frame's bytes -- that the level-by-level
// kernels write to HBM and level 2 reads back.  Here a workgroup keeps it on
// chip: it owns a tile of level-2 output columns and a band of level-2 output
// rows of one (frame, channel) and slides down its band, one level-1 output
// row pair per step:
//   level-1 axis-0 pass: lane = two input columns, a register window of the
//     last F input rows of each, two new rows per step (pywt's tap order);
//   level-1 axis-1 pass: lane = one LL1 column of the A row (-> LL1 into LDS
//     and the HL1 byte) and of the D row (-> LH1, HH1 bytes);
//   level-2 axis-0 pass: lane = one LL1 column, a register window of the last
//     F LL1 rows, an output row pair every second step;
//   level-2 axis-1 pass: lane = one level-2 output of the A2 or the D2 row
//     (-> LL2 as float64 for level 3, or u16 when level 2 is the last; the
//     level-2 detail bytes).
// The four phases run as a software pipeline over double-buffered LDS rows:
// in step t the axis-0 pass of row t, the axis-1 pass of row t-1, the level-2
// axis-0 pass fed by row t-2 and the level-2 axis-1 pass of the level-2 row
// formed at t-1 -- one workgroup barrier per step.
//
// Geometry (F = 2P taps, both plane dimensions even at both levels, i.e.
// h % 4 == 0 and w % 4 == 0): a tile owns kBT2 level-2 output columns
// [c2, c2 + kBT2); they read LL1 columns [2 c2 - P + 1, 2 (c2 + kBT2) + P - 1)
// (2 kBT2 + F - 2 of them), which read input columns from 2 (2 c2 - P + 1) -
// P + 1 on (2 (2 kBT2 + F - 2) + F - 2 of them): ~5 % of level 1 is computed
// twice, in the neighbouring tile.  A band owns level-2 rows [r2, r2 + B) and
// computes LL1 rows [2 r2 - P + 1, 2 (r2 + B) + P - 1): F - 2 LL1 rows of
// halo per band.  Positions are logical (before the periodic wrap): an even
// plane wraps modulo its length, so the windows slide across the wrap; what
// pywt does differently there -- an output whose taps pass the END of the
// line (i = P + 2o >= N) sums the wrapped taps first (wrap_sum) -- is decided
// by the output's actual index, the rest is natural order (nat_sum).
// Zero taps and Z0 as in the strip kernels (bit-identical bytes).
#pragma once

constexpr int kBT2 = 120;   // level-2 output columns per tile
constexpr int kBNT = 512;   // threads per workgroup: one input column per lane

__host__ __device__ constexpr int band_l1c(int F) { return 2 * kBT2 + F - 2; }        // LL1 columns per tile
__host__ __device__ constexpr int band_l0c(int F) { return 2 * band_l1c(F) + F - 2; } // input columns per tile

__device__ __forceinline__ int wrap_once(int p, int N)   // p in (-N, 2N) -> [0, N)
{
    p = p < 0 ? p + N : p;
    return p >= N ? p - N : p;
}

// Block b -> (unit, channel): the three channels of a unit are blocks b,
// b + 8, b + 16 -- the same XCD under round-robin dispatch -- so the RGB
// bytes each of them reads come from one L2.
struct BandUnit {
    int unit, ch;
};
__device__ __forceinline__ BandUnit band_unit(int b)
{
    const int grp = b / 24, r = b - 24 * grp;
    return {grp * 8 + (r & 7), r >> 3};
}

// wrap_sum for an output whose centre passes the line end by K (i = N + K):
// taps K .. 0 first (descending), then K + 1 .. F - 1 -- straight-line code
template <int F, unsigned Z, int K>
__device__ __forceinline__ double wrap_sum_k(const double (&f)[F], const double (&v)[F])
{
    double s = 0.0;
#pragma unroll
    for (int m = K; m >= 0; --m)
        if (!((Z >> m) & 1u)) s = s + f[m] * v[F - 1 - m];
#pragma unroll
    for (int m = K + 1; m < F; ++m)
        if (!((Z >> m) & 1u)) s = s + f[m] * v[F - 1 - m];
    return s;
}

// The axis-1 outputs whose taps pass the end of an even line: i = P + 2o >=
// N happens for o = N/2 - 2 (K = 1) and N/2 - 1 (K = 3) when P = 5.  Lanes
// differ, so the sums are taken only in the waves holding such a lane (a
// wave-uniform branch) and selected per lane: no per-tap predication in the
// common path.
template <int F, unsigned Z>
__device__ __forceinline__ double tail_sum(const double (&f)[F], const double (&v)[F], int k, double nat)
{
    static_assert(F == 10, "tail K values of P = 5");
    const double s1 = wrap_sum_k<F, Z, 1>(f, v), s3 = wrap_sum_k<F, Z, 3>(f, v);
    return k == 1 ? s1 : k == 3 ? s3 : nat;
}

template <int F, unsigned ZLO, unsigned ZHI, int CT, bool LAST2, bool QP2>
__global__ __launch_bounds__(kBNT, 2) void dwt_band12_kernel(
    const uint8_t *__restrict__ rgb, long long rgb_stride, double *__restrict__ LLout, long long plane_stride,
    uint8_t *__restrict__ packed, long long packed_stride, long long ll_off, long long o1lh, long long o1hl,
    long long o1hh, long long o2lh, long long o2hl, long long o2hh, int h, int w, int Q, int n_tiles, int n_bands,
    int brows, int n_units, Taps<F> tp)
{
    constexpr int P = F / 2, L1C = band_l1c(F), L0C = band_l0c(F);
    constexpr int HALF = kBNT / 2;   // waves [0, 4): A roles, level-2 axis 0; [4, 8): D roles, level-2 axis 1
    static_assert(L0C <= kBNT && L1C <= HALF && kBT2 <= 128, "tile geometry");
    static_assert(F == 10, "band kernel: 10-tap filters");
    // The level-1 window has NW = F + 2 slots (logical offset k of step s in slot
    // (2 s + k) % NW: period NW / 2 steps) and the LDS ring RING = F + 2 rows
    // (LL1 row i in slot i % RING: the level-2 window plus the row being
    // written); an unrolled group of U = 12 steps makes every slot a constant.
    constexpr int NW = F + 2, RING = F + 2, U = 12;
    static_assert(U % (NW / 2) == 0 && U % RING == 0 && U % 2 == 0, "unroll");
    __shared__ __attribute__((aligned(16))) double ad1[2][2][kBNT];   // [buf][A|D][input column]
    __shared__ __attribute__((aligned(16))) double ll1[RING][HALF];   // LL1 row i in slot i % RING
    __shared__ __attribute__((aligned(16))) double ad2[2][HALF + 8];  // [A2|D2][LL1 column]

    const BandUnit bu = band_unit((int)blockIdx.x);
    if (bu.unit >= n_units) return;
    const int ch = bu.ch;
    const int tile = bu.unit % n_tiles, rest = bu.unit / n_tiles;
    const int band = rest % n_bands;
    const long long frame = rest / n_bands;
    const int lane = threadIdx.x;
    const bool hiwave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6) >= HALF / 64;   // wave-uniform
    const int hl = lane & (HALF - 1);                          // lane within its half
    const int h1 = h >> 1, w1 = w >> 1, h2 = h >> 2, w2 = w >> 2;
    const int c2 = tile * kBT2;
    const int a1 = 2 * c2 - P + 1, a0 = 2 * a1 - P + 1;   // first LL1 / input column (logical)
    const int r2_0 = band * brows, r2_1 = min(h2, r2_0 + brows);
    const int p0 = 2 * r2_0 - P + 1;                      // first LL1 row (logical)
    const int n_p = 2 * (r2_1 - r2_0) + F - 2;            // LL1 rows computed
    const int n_int = n_p + 3;                            // pipeline steps

    double flo[F], fhi[F];
#pragma unroll
    for (int m = 0; m < F; ++m) {
        flo[m] = CT ? ct_dec(CT, false, m) : tp.lo[m];
        fhi[m] = CT ? ct_dec(CT, true, m) : tp.hi[m];
    }
    const int qsh = __builtin_ctz((unsigned)Q);
    auto kq = [&](double v) -> int32_t { return (int32_t)(QP2 ? __builtin_ldexp(v, -qsh) : v / (double)Q); };

    // ---- level-1 input: the lane's column, one unaligned dword per pixel that
    // starts a byte early (at x = 0: at the pixel), so it never leaves the frame
    const uint8_t *const frgb = rgb + frame * rgb_stride;
    const int x = wrap_once(a0 + lane, w);
    const int xoff = x > 0 ? 3 * x - 1 : 0, xsh = x > 0 ? 8 : 0;
    const uint32_t row_bytes = 3u * (uint32_t)w, frame_bytes = row_bytes * (uint32_t)h;
    auto load_px = [&](int q) -> uint32_t {   // logical input row q
        uint32_t d;
        __builtin_memcpy(&d, frgb + (uint32_t)wrap_once(q, h) * row_bytes + xoff, 4);
        return d;
    };
    // the prefetch rows' byte offsets as running values in VGPRs (a uniform
    // value the compiler keeps in SGPRs costs the CU's one scalar unit, shared
    // by its 16 waves; the vector form costs each SIMD's 4): rows 2 p_s + P - 1
    // and 2 p_s + P of the step s whose rows the next prefetch loads (s = t + 2
    // at step t), advanced by two rows per prefetch, wrapped at the frame end
    uint32_t roffA = opaque_mov((uint32_t)wrap_once(2 * (p0 + 2) + P - 1, h) * row_bytes);
    uint32_t roffB = opaque_mov((uint32_t)wrap_once(2 * (p0 + 2) + P, h) * row_bytes);
    auto prefetch = [&](uint32_t (&r)[2]) {
        __builtin_memcpy(&r[0], frgb + (roffA + xoff), 4);
        __builtin_memcpy(&r[1], frgb + (roffB + xoff), 4);
        roffA += 2 * row_bytes;
        roffB += 2 * row_bytes;
        roffA = min(roffA, roffA - frame_bytes);   // unsigned: subtracts only past the end
        roffB = min(roffB, roffB - frame_bytes);
    };
    // (int16) YCoCg sample (A4) without a branch on the channel: Y = (R + 2G +
    // B) / 4, Co = (R - B) / 2, Cg = (2G - R - B) / 4, each truncated toward
    // zero (the float terms are multiples of 1/4 below 2^9: exact), as
    // c_R R + c_G G + c_B B over 2^dsh
    const int cR = ch == 2 ? -1 : 1, cG = ch == 1 ? 0 : 2, cB = ch == 0 ? 1 : -1, dsh = ch == 1 ? 1 : 2;
    const int dmask = (1 << dsh) - 1;
    auto sample = [&](uint32_t d) -> double {
        const uint32_t px = d >> xsh;
        const int R = px & 0xFF, G = (px >> 8) & 0xFF, B = (px >> 16) & 0xFF;
        const int v = cR * R + cG * G + cB * B;
        return (double)((v + ((v >> 31) & dmask)) >> dsh);
    };

    // ---- stores: buffer stores issued unconditionally, dropped past the buffer
    constexpr uint32_t kDrop = 0x80000000u;
    typedef unsigned int U32x2 __attribute__((__vector_size__(8)));
    uint8_t *const pk = packed + frame * packed_stride;
    const __amdgpu_buffer_rsrc_t rs_pk = __builtin_amdgcn_make_buffer_rsrc(pk, 0, (int)packed_stride, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_ll = __builtin_amdgcn_make_buffer_rsrc(
        LLout + (frame * 3 + ch) * plane_stride, 0, LAST2 ? 0 : (int)((long long)h2 * w2 * 8), 0x00020000);
    auto q8 = [&](double v) -> uint8_t { return (uint8_t)(uint32_t)(kq(v) + 128); };

    // level-1 axis-1 roles: lane hl = LL1 column a1 + hl of the A row (low
    // waves: LL1 into the ring, HL1) or the D row (high waves: LH1, HH1)
    const int ac1 = wrap_once(a1 + hl, w1);                              // actual LL1 column
    const bool own1c = hl >= P - 1 && hl < P - 1 + 2 * kBT2 && 2 * c2 + (hl - (P - 1)) < w1;
    const int ic1 = P + 2 * ac1;                                         // its centre on the input line
    const bool tail1 = ic1 >= w && hl < L1C;                             // taps wrap past the line end
    const int jr1 = min(hl, L1C - 1);                                    // reads stay inside the row
    const uint32_t e1_lane = (uint32_t)(ac1 * 3 + ch);
    const uint32_t drop1 = own1c ? 0u : kDrop;
    // level-2 axis-1 roles (high waves): A2 item o = hl (< kBT2), D2 item o = hl - 128
    const int src2 = hl >= 128 ? 1 : 0, o2 = hl - 128 * src2;
    const int oc2 = c2 + o2;
    const bool own2c = o2 < kBT2 && oc2 < w2;
    const int ic2 = P + 2 * min(oc2, w2 - 1);
    const bool tail2 = ic2 >= w1 && o2 < kBT2;
    const int or2 = min(o2, kBT2 - 1);
    const uint32_t drop2 = own2c ? 0u : kDrop, drop2a = own2c && !src2 ? 0u : kDrop;
    const uint32_t e2_lane = (uint32_t)(oc2 * 3 + ch);
    // wave-uniform: does this wave hold a lane whose axis-1 taps pass the line end?
    const bool tailw1 = __builtin_amdgcn_ballot_w64(tail1) != 0, tailw2 = __builtin_amdgcn_ballot_w64(tail2) != 0;

    double win[NW];    // level-1 window: slot (2 s + k) % NW holds logical row 2 p_s - P + 1 + k
    uint32_t e1row = 0, e2row = 0, e2ll = 0;   // steady groups: running store offsets (set per group)
    uint32_t raw[2][2];   // prefetched input rows: [step parity][row]
#pragma unroll
    for (int k = 0; k < F - 2; ++k) win[k] = sample(load_px(2 * p0 - P + 1 + k));
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        if (s < n_p) {
            raw[s][0] = load_px(2 * (p0 + s) + P - 1);
            raw[s][1] = load_px(2 * (p0 + s) + P);
        }
    }

    // STEADY (every phase active, no prefetch past the band, no output row
    // whose axis-0 taps wrap past the plane's bottom): the phases' guards drop
    // out, so the stores and loads between a prefetch and its use are the
    // same on every path and the compiler's vmcnt waits count exactly (with
    // guarded stores it must assume the fewest and waits for the loads issued
    // this step), and the scalar work per step is a few row offsets
    auto step = [&](int t, auto uc, auto steady) {
        constexpr int u = decltype(uc)::value;   // t % U
        constexpr int b = u & 1;                 // this step's write buffer
        constexpr bool ST = decltype(steady)::value;
        // the axis-1 pass's inputs (the other buffer) are read first: their LDS
        // latency hides behind the axis-0 arithmetic
        const bool do_row1 = ST || (t >= 1 && t - 1 < n_p);
        double va[F];
        if (do_row1) {
            const double *row = &ad1[b ^ 1][hiwave ? 1 : 0][2 * jr1];
#pragma unroll
            for (int k = 0; k < F; k += 2) {
                const double2 xx = *(const double2 *)(row + k);
                va[k] = xx.x;
                va[k + 1] = xx.y;
            }
        }
        // ---- level-1 axis-0 pass of LL1 row p0 + t (every lane: its column)
        if (ST || t < n_p) {
            win[(2 * u + F - 2) % NW] = sample(raw[b][0]);
            win[(2 * u + F - 1) % NW] = sample(raw[b][1]);
            if (ST || t + 2 < n_p) prefetch(raw[b]);   // two steps ahead
            double v[F];
#pragma unroll
            for (int q = 0; q < F; ++q) v[q] = win[(2 * u + q) % NW];
            double lo, hi;
            const int ia = ST ? 0 : P + 2 * wrap_once(p0 + t, h1);   // centre of the actual LL1 row
            if (!ST && ia >= h) {   // block-uniform: the bottom rows take pywt's wrapped order
                lo = wrap_sum<F, ZLO>(flo, v, ia, h);
                hi = wrap_sum<F, ZHI>(fhi, v, ia, h);
            } else {
                lo = nat_sum<F, ZLO, true>(flo, v);
                hi = nat_sum<F, ZHI, true>(fhi, v);
            }
            ad1[b][0][lane] = lo;
            ad1[b][1][lane] = hi;
        }
        // ---- level-1 axis-1 pass of LL1 row p0 + t - 1 (written in the previous step)
        if (do_row1) {
            const int p = p0 + t - 1;
            const bool own_r = ST || (p >= 2 * r2_0 && p < 2 * r2_1);   // steady rows are owned
            double lo = nat_sum<F, ZLO, true>(flo, va), hi = nat_sum<F, ZHI, true>(fhi, va);
            if (tailw1) {   // only the waves holding the line end
                const int k = tail1 ? ic1 - w : 0;
                lo = tail_sum<F, ZLO>(flo, va, k, lo);
                hi = tail_sum<F, ZHI>(fhi, va, k, hi);
            }
            // steady: a running row offset (VGPR); else from the actual row
            const uint32_t e = (ST ? e1row : (uint32_t)wrap_once(p, h1) * (uint32_t)(3 * w1)) + e1_lane;
            if (ST) e1row += (uint32_t)(3 * w1);
            const uint32_t dr = own_r ? drop1 : kDrop;
            if (!hiwave) {   // A row: aa -> LL1 (ring), ad = cV -> HL
                ll1[(u + U - 1) % RING][hl] = lo;   // LL1 row t - 1
                __builtin_amdgcn_raw_buffer_store_b8(q8(hi), rs_pk, ((uint32_t)o1hl + e) | dr, 0, 0);
            } else {         // D row: da = cH -> LH, dd = cD -> HH
                __builtin_amdgcn_raw_buffer_store_b8(q8(lo), rs_pk, ((uint32_t)o1lh + e) | dr, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b8(q8(hi), rs_pk, ((uint32_t)o1hh + e) | dr, 0, 0);
            }
        }
        // ---- level-2 axis-0 pass (low waves): LL1 rows i - F + 1 .. i (i = t - 2,
        // odd) from the LDS ring complete a level-2 output row every second step
        // (splitting the level-2 work between the halves by filter measured 3 %
        // slower: twice the LDS reads)
        if constexpr ((u & 1) == 1) {
            const int i = t - 2;
            if (!hiwave && (ST || (i >= F - 1 && i < n_p))) {
                const int r2 = r2_0 + (i - (F - 1)) / 2;
                const int ia = P + 2 * r2;
                const int j = min(hl, L1C - 1);
                double v[F];
#pragma unroll
                for (int q = 0; q < F; ++q) v[q] = ll1[(u + U - 2 - (F - 1) + q) % RING][j];   // LL1 row i - F + 1 + q
                double lo, hi;
                if (!ST && ia >= h1) {
                    lo = wrap_sum<F, ZLO>(flo, v, ia, h1);
                    hi = wrap_sum<F, ZHI>(fhi, v, ia, h1);
                } else {
                    lo = nat_sum<F, ZLO, true>(flo, v);
                    hi = nat_sum<F, ZHI, true>(fhi, v);
                }
                ad2[0][hl] = lo;
                ad2[1][hl] = hi;
            }
        }
        // ---- level-2 axis-1 pass (high waves) of the level-2 row formed in the previous step
        if constexpr ((u & 1) == 0) {
            const int i = t - 3;
            if (hiwave && (ST || (i >= F - 1 && i < n_p))) {
                const int r2 = r2_0 + (i - (F - 1)) / 2;
                double v[F];
                const double *row = &ad2[src2][2 * or2];
#pragma unroll
                for (int k = 0; k < F; k += 2) {
                    const double2 xx = *(const double2 *)(row + k);
                    v[k] = xx.x;
                    v[k + 1] = xx.y;
                }
                double lo = nat_sum<F, ZLO, true>(flo, v), hi = nat_sum<F, ZHI, true>(fhi, v);
                if (tailw2) {
                    const int k = tail2 ? ic2 - w1 : 0;
                    lo = tail_sum<F, ZLO>(flo, v, k, lo);
                    hi = tail_sum<F, ZHI>(fhi, v, k, hi);
                }
                const uint32_t e = (ST ? e2row : (uint32_t)r2 * (uint32_t)(3 * w2)) + e2_lane;
                const uint32_t ell = (ST ? e2ll : (uint32_t)r2 * (uint32_t)(8 * w2)) + (uint32_t)(8 * oc2);
                if (ST) {
                    e2row += (uint32_t)(3 * w2);
                    e2ll += (uint32_t)(8 * w2);
                }
                // A2 lanes: ad -> HL2, aa -> LL2; D2 lanes: da -> LH2, dd -> HH2
                __builtin_amdgcn_raw_buffer_store_b8(q8(src2 ? lo : hi), rs_pk,
                                                     ((uint32_t)(src2 ? o2lh : o2hl) + e) | drop2, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b8(q8(hi), rs_pk, ((uint32_t)o2hh + e) | (src2 ? drop2 : kDrop), 0,
                                                     0);
                if constexpr (LAST2)
                    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(uint32_t)(kq(lo) + 128), rs_pk,
                                                          ((uint32_t)ll_off + 2 * e) | drop2a, 0, 0);
                else
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(U32x2, lo), rs_ll, ell | drop2a, 0, 0);
            }
        }
        __syncthreads();
    };

    // steady groups: t in [t_s, t_e), every phase active there (t - 3 >= F - 1,
    // t + 2 < n_p) and no level-1 row with wrapped axis-0 taps (actual LL1 rows
    // h1 - 2, h1 - 1: steps h1 - 2 - p0 .. in the band holding the bottom; the
    // level-2 rows with wrapped taps come after n_p - 2); the rest through the
    // guarded steps
    // (and t - 1 < n_p - 4: the LL1 rows of the axis-1 pass are the band's own)
    const int t_s = U;
    int t_lim = n_p - 4;
    if (h1 - 2 - p0 >= 0 && h1 - 2 - p0 < t_lim) t_lim = h1 - 2 - p0;
    const int t_e = t_lim > t_s ? t_s + (t_lim - t_s) / U * U : t_s;
    for (int t0 = 0; t0 < n_int; t0 += U) {
        if (t0 >= t_s && t0 < t_e) {
            // running offsets: LL1 row p0 + t0 - 1 (axis-1 pass of step t0), level-2 row of step t0
            // (u = 0: i = t0 - 3, r2 = r2_0 + (i - F + 1) / 2)
            e1row = opaque_mov((uint32_t)(p0 + t0 - 1) * (uint32_t)(3 * w1));
            const uint32_t r2g = (uint32_t)(r2_0 + (t0 - 3 - (F - 1)) / 2);
            e2row = opaque_mov(r2g * (uint32_t)(3 * w2));
            e2ll = opaque_mov(r2g * (uint32_t)(8 * w2));
#define VCF_BAND_STEP(k) step(t0 + k, std::integral_constant<int, k>(), std::true_type());
            VCF_BAND_STEP(0)
            VCF_BAND_STEP(1)
            VCF_BAND_STEP(2)
            VCF_BAND_STEP(3)
            VCF_BAND_STEP(4)
            VCF_BAND_STEP(5)
            VCF_BAND_STEP(6)
            VCF_BAND_STEP(7)
            VCF_BAND_STEP(8)
            VCF_BAND_STEP(9)
            VCF_BAND_STEP(10)
            VCF_BAND_STEP(11)
#undef VCF_BAND_STEP
        } else {
#define VCF_BAND_STEP(k)                                                                                           \
    if (t0 + k < n_int) step(t0 + k, std::integral_constant<int, k>(), std::false_type());
            VCF_BAND_STEP(0)
            VCF_BAND_STEP(1)
            VCF_BAND_STEP(2)
            VCF_BAND_STEP(3)
            VCF_BAND_STEP(4)
            VCF_BAND_STEP(5)
            VCF_BAND_STEP(6)
            VCF_BAND_STEP(7)
            VCF_BAND_STEP(8)
            VCF_BAND_STEP(9)
            VCF_BAND_STEP(10)
            VCF_BAND_STEP(11)
#undef VCF_BAND_STEP
        }
    }
}
