// vcf_idwt_band21.h -- inverse levels 2 and 1 of the 2D-DWT in one launch,
// bit-exact (src/2D-DWT.py:80-101: pywt.waverec2(mode='per') per YCoCg
// channel, A6; to_RGB + clip + u8), included by vcf_dwt.hip.
//
// Why: as two idwt_line_kernel launches, level 2 writes LL1 as a float64 plane
// (49.8 MB per 4K frame) that level 1 reads back: 0.8 GB of HBM traffic per
// 8-frame C3 call, and level 2 ran memory-bound (25 % float64 issue, round-5
// counters).  Here LL1 never leaves the chip: a workgroup owns kB21C level-1
// subband columns (2 kB21C RGB columns) and a band of level-1 rows of one
// frame, one wave per YCoCg channel, and slides down the band one level-1 row
// per step (the line kernel's schedule, vcf_idwt_line.h), producing the LL1
// row each step consumes with a level-2 line pipeline of its own: every
// second step, one level-2 row (LDS) -> row pass -> a register window of five
// 'a'/'d' rows -> column pass -> two LL1 rows.
//
// Lanes.  Level 1: lane L is LL1 column c = P0 - 2 + L (two halo columns each
// side; lanes 2 .. 61 own outputs).  Level 2: the 64 LL1 columns are the
// pairs p = P0/2 - 1 + (L & 31); lanes 0..31 run the row pass of 'a' (LL2,
// HL2) for their pair, lanes 32..63 that of 'd' (LH2, HH2), both parities;
// then lane L keeps the value of its own column (2p for L < 32, 2p + 1 for
// L >= 32) and trades the other with lane L ^ 32 (one cross-lane move), so
// each lane runs the column pass of one LL1 column and writes it to its LDS
// slot.  Per level-1 step that is 2 inv_pair of level-2 work against level 1's
// 8: the work of the two launches, without the plane.
//
// Arithmetic: every output is the line kernel's (inv_pair: the same products
// and sums in the same order, zero taps skipped, sums from the first
// product), so the bytes equal the two launches' (tested) and the oracle's.
// Planes that halve evenly (h1 = 2 h2, w1 = 2 w2: the wrap of LL1 is then the
// wrap of level 2's output) with subbands of at least 5 x 5.
#pragma once

constexpr int kB21C = 60;            // owned level-1 subband columns per tile (64 lanes, 2 halo each side)
constexpr int kB21S2 = 36;           // staged level-2 subband columns per row
constexpr int kB21NT = 192;          // one wave per YCoCg channel
#ifndef VCF_B21_SPLIT   // (A/B) the level-1 row pass's two halves kept apart: fewer live VGPRs
#define VCF_B21_SPLIT 1
#endif

template <bool FROM_PACKED_LL2, unsigned ZLO, unsigned ZHI, int CT, bool QS>
__global__ __launch_bounds__(kB21NT) void idwt_band21_kernel(
    const uint8_t *__restrict__ packed, long long packed_stride, long long ll_off, long long off2_lh,
    long long off2_hl, long long off2_hh, long long off1_lh, long long off1_hl, long long off1_hh,
    const double *__restrict__ prev, long long plane_stride, int lda, uint8_t *__restrict__ rgb, int h2, int w2,
    int h1, int w1, int Q, int n_tiles, int n_bands, int brows)
{
    __shared__ __attribute__((aligned(16))) double s1[2][3][4][64];           // level-1 rows [buf][ch][LL|HL|LH|HH][slot]
    __shared__ __attribute__((aligned(16))) double s2[2][3][4][kB21S2 + 4];   // level-2 rows, per wave
    __shared__ __attribute__((aligned(16))) double sout[2][2][3][2 * kB21C];  // output pairs for the RGB stage

    const int tile = blockIdx.x % n_tiles, rest = blockIdx.x / n_tiles;
    const int band = rest % n_bands;
    const long long frame = rest / n_bands;
    const int tid = threadIdx.x;
    const int ch = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int P0 = tile * kB21C;                      // first owned level-1 column (even)
    const int m0 = band * brows, m1 = min(h1, m0 + brows);   // level-1 rows [m0, m1) -> RGB rows [2 m0, 2 m1)
    const int nsteps = m1 - m0 + 4;                   // level-1 rows m0 - 2 .. m1 + 1
    const double qd = (double)Q;
    const uint8_t *pk = packed + frame * packed_stride;
    const double *pv = FROM_PACKED_LL2 ? nullptr : prev + (frame * 3 + ch) * plane_stride;
    const int ow = 2 * w1, oh = 2 * h1;

    // ---- level 1: lane = LL1 column P0 - 2 + lane (its detail bytes) ----
    const uint32_t b1 = 3u * (uint32_t)mod_n(P0 - 2 + lane, w1) + ch;
    struct Det {
        uint32_t hl, lh, hh;
    };
    auto load1 = [&](int rw) -> Det {   // level-1 row rw (already wrapped)
        const uint8_t *row = pk + (long long)rw * w1 * 3;
        return Det{(row + off1_hl)[b1], (row + off1_lh)[b1], (row + off1_hh)[b1]};
    };
    // LL1 value slot of this lane's level-2 column: pair L & 31, parity L >> 5
    const int pi = lane & 31, part = lane >> 5;
    const int ll_slot = 2 * pi + part;
    auto put1 = [&](int buf, double ll, const Det &d) {
        s1[buf][ch][0][ll_slot] = ll;
        s1[buf][ch][1][lane] = dequant_b<QS>(d.hl, Q, qd);
        s1[buf][ch][2][lane] = dequant_b<QS>(d.lh, Q, qd);
        s1[buf][ch][3][lane] = dequant_b<QS>(d.hh, Q, qd);
    };

    // ---- level 2: lanes 0 .. kB21S2 - 1 stage level-2 columns P0/2 - 3 + lane ----
    const int l2 = min(lane, kB21S2 - 1);
    const int c2 = mod_n(P0 / 2 - 3 + l2, w2);
    const uint32_t b2 = 3u * (uint32_t)c2 + ch;
    struct Row2 {
        double ll;
        uint32_t hl, lh, hh;
    };
    auto load2 = [&](int y) -> Row2 {   // level-2 row y (already wrapped)
        const long long rb = (long long)y * w2 * 3;
        Row2 v;
        if (FROM_PACKED_LL2) v.ll = dequant((int16_t)*reinterpret_cast<const uint16_t *>(pk + ll_off + 2 * (rb + b2)), Q);
        else v.ll = (pv + (long long)y * lda)[c2];
        const uint8_t *row = pk + rb;
        v.hl = (row + off2_hl)[b2];
        v.lh = (row + off2_lh)[b2];
        v.hh = (row + off2_hh)[b2];
        return v;
    };
    auto put2 = [&](int buf, const Row2 &v) {
        if (lane < kB21S2) {
            double *s = &s2[buf][ch][0][lane];
            s[0] = v.ll;
            s[kB21S2 + 4] = dequant_b<QS>(v.hl, Q, qd);
            s[2 * (kB21S2 + 4)] = dequant_b<QS>(v.lh, Q, qd);
            s[3 * (kB21S2 + 4)] = dequant_b<QS>(v.hh, Q, qd);
        }
    };
    // the level-2 window: the row pass values of this lane's own LL1 column (wk)
    // and the partner's (wr), oldest first
    double wk[5], wr[5];
    // level-2 row pass of the staged row in s2[buf] -> push into the window
    auto row2 = [&](int buf) {
        const double *S = &s2[buf][ch][2 * part][pi];
        double x[5], y[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            x[j] = S[4 - j];                      // column p + 2 - j of LL2 / LH2
            y[j] = S[(kB21S2 + 4) + 4 - j];       // ... of HL2 / HH2
        }
        const double v0 = inv_pair<ZLO, ZHI, CT, 0>(x, y), v1 = inv_pair<ZLO, ZHI, CT, 1>(x, y);
        const double keep = part ? v1 : v0, send = part ? v0 : v1;
        const double got = __shfl_xor(send, 32, 64);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            wk[j] = wk[j + 1];
            wr[j] = wr[j + 1];
        }
        wk[4] = keep;
        wr[4] = got;
    };
    // level-2 column pass over the window -> LL1 rows 2 m2, 2 m2 + 1 of this lane's column
    auto col2 = [&](double &r0, double &r1) {
        double xa[5], xd[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) {   // x[j] = row m2 + 2 - j: newest first
            xa[j] = part ? wr[4 - j] : wk[4 - j];
            xd[j] = part ? wk[4 - j] : wr[4 - j];
        }
        r0 = inv_pair<ZLO, ZHI, CT, 0>(xa, xd);
        r1 = inv_pair<ZLO, ZHI, CT, 1>(xa, xd);
    };

    // RGB stage of output pair m from sout[buf] by one channel wave: lane = (row
    // lane / 32, pixels 4q .. 4q + 3 of the tile row) -> three dwords of bytes
    const int npx = min(2 * kB21C, ow - 2 * P0);
    auto to_rgb = [&](int buf, int m) {
        const int r = lane >> 5, q = lane & 31;
        const int n = 2 * m + r;
        if (n >= oh || 4 * q >= npx) return;
        const double2 *Yp = reinterpret_cast<const double2 *>(&sout[buf][r][0][4 * q]);
        const double2 *Op = reinterpret_cast<const double2 *>(&sout[buf][r][1][4 * q]);
        const double2 *Gp = reinterpret_cast<const double2 *>(&sout[buf][r][2][4 * q]);
        const double2 y01 = Yp[0], y23 = Yp[1], o01 = Op[0], o23 = Op[1], g01 = Gp[0], g23 = Gp[1];
        const double Y[4] = {y01.x, y01.y, y23.x, y23.y}, Co[4] = {o01.x, o01.y, o23.x, o23.y},
                     Cg[4] = {g01.x, g01.y, g23.x, g23.y};
        uint32_t b[12];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            b[3 * i] = rgb_u8(Y[i] + Co[i] - Cg[i]);
            b[3 * i + 1] = rgb_u8(Y[i] + Cg[i]);
            b[3 * i + 2] = rgb_u8(Y[i] - Co[i] - Cg[i]);
        }
        uint8_t *o = rgb + frame * ((long long)oh * ow * 3) + ((long long)n * ow + 2 * P0) * 3 + 12 * q;
        if (4 * q + 4 <= npx && (reinterpret_cast<uintptr_t>(o) & 3) == 0) {
            uint32_t *o4 = reinterpret_cast<uint32_t *>(o);
#pragma unroll
            for (int k = 0; k < 3; ++k)
                o4[k] = b[4 * k] | (b[4 * k + 1] << 8) | (b[4 * k + 2] << 16) | (b[4 * k + 3] << 24);
        } else {
            const int nb = 3 * min(4, npx - 4 * q);
            for (int k = 0; k < nb; ++k) o[k] = (uint8_t)b[k];
        }
    };

    // ---- prologue: the level-2 window up to m2 = m0/2 - 1, LL1 rows m0 - 2, m0 - 1 ----
    const int m2f = m0 / 2 - 1;     // (brows and m0 even)
    // the next level-2 row to stage, wrapped (advanced by one: no division per step)
    int y2 = mod_n(m2f - 2, h2);
    auto next_y2 = [&]() { y2 = y2 + 1 == h2 ? 0 : y2 + 1; };
#pragma unroll
    for (int j = 0; j < 5; ++j) wk[j] = wr[j] = 0.0;
    for (int u = 0; u < 5; ++u) {   // rows m2f - 2 .. m2f + 2
        put2(u & 1, load2(y2));
        next_y2();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        row2(u & 1);
    }
    double ll_a, ll_b;              // LL1 rows 2 m2f = m0 - 2 and m0 - 1
    col2(ll_a, ll_b);
    int b2buf = 1;                  // the s2 buffer the next staged row goes to
    Row2 pre2;                      // loaded at an even step, staged at the next (odd) one
    int r1w = mod_n(m0 - 2, h1);   // the wrapped level-1 row of the next detail load
    put1(0, ll_a, load1(r1w));
    r1w = r1w + 1 == h1 ? 0 : r1w + 1;
    double ll_hold = ll_b;          // LL1 row r + 1 when r is even
    __syncthreads();

    const int lc = min(max(lane, 2), 2 + kB21C - 1);   // level-1 lane for the LDS reads (halo lanes: clamped)
    double wa[5][2], wd[5][2];      // level-1 'a' / 'd' rows, slot t % 5
    for (int t0 = 0; t0 < nsteps; t0 += 5) {
#pragma unroll
        for (int u = 0; u < 5; ++u) {
            const int t = t0 + u;
            if (t >= nsteps) break;
            // this step's level-1 row is r = m0 - 2 + t
            const bool odd = (t & 1) != 0;             // r odd: a level-2 step makes LL1 rows r + 1, r + 2
            // prefetch: level-1 details of row r + 1; at even steps the level-2 row the
            // next (odd) step stages (issued a step ahead of its LDS store)
            const Det d1 = load1(r1w);   // row r + 1
            r1w = r1w + 1 == h1 ? 0 : r1w + 1;
            if (!odd) {
                pre2 = load2(y2);
                next_y2();
            }
            // level-1 row pass of row r
            {
                const double *S = &s1[t & 1][ch][0][lc - 2];
#pragma unroll
                for (int half = 0; half < 2; ++half) {   // 'a' (LL, HL), then 'd' (LH, HH)
                    double x[5], y[5];
#pragma unroll
                    for (int j = 0; j < 5; ++j) {
                        x[j] = S[2 * half * 64 + 4 - j];
                        y[j] = S[(2 * half + 1) * 64 + 4 - j];
                    }
                    double(&o)[5][2] = half ? wd : wa;
                    o[u][0] = inv_pair<ZLO, ZHI, CT, 0>(x, y);
                    o[u][1] = inv_pair<ZLO, ZHI, CT, 1>(x, y);
                    if (VCF_B21_SPLIT) asm volatile("" ::: "memory");   // the 'd' loads after the 'a' sums
                }
            }
            // level-1 column pass: output pair m = r - 2 from rows r - 4 .. r
            if (t >= 4) {
                double o[2][2];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    double xa[5], xd[5];
#pragma unroll
                    for (int j = 0; j < 5; ++j) {
                        xa[j] = wa[(u + 5 - j) % 5][e];
                        xd[j] = wd[(u + 5 - j) % 5][e];
                    }
                    o[0][e] = inv_pair<ZLO, ZHI, CT, 0>(xa, xd);
                    o[1][e] = inv_pair<ZLO, ZHI, CT, 1>(xa, xd);
                }
                if (lane >= 2 && lane < 2 + kB21C) {
#pragma unroll
                    for (int rr = 0; rr < 2; ++rr)
                        *reinterpret_cast<double2 *>(&sout[t & 1][rr][ch][2 * (lane - 2)]) =
                            make_double2(o[rr][0], o[rr][1]);
                }
            }
            // the LL1 value of row r + 1
            double ll_next;
            if (odd) {   // level-2 step: stage the prefetched row, row pass, column pass
                put2(b2buf, pre2);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                row2(b2buf);
                b2buf ^= 1;
                double ra, rb;
                col2(ra, rb);
                ll_next = ra;
                ll_hold = rb;
            } else {
                ll_next = ll_hold;
            }
            put1((t + 1) & 1, ll_next, d1);
            if (t >= 5 && ch == t % 3) to_rgb((t - 1) & 1, m0 - 5 + t);
            __syncthreads();
        }
    }
    if (ch == nsteps % 3) to_rgb((nsteps - 1) & 1, m1 - 1);
}
