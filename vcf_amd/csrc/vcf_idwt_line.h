// vcf_idwt_line.h -- one level of the inverse 2D-DWT (src/2D-DWT.py:80-101:
// pywt.waverec2(mode='per') per YCoCg channel, A6; to_RGB + clip + u8 at
// level 1) as a line-based kernel, included by vcf_dwt.hip.
//
// Why: the tiled level kernel (idwt_level_kernel) stages a 2-D block of the
// four subbands per channel, runs the row pass over the block's halo rows
// (1.6x the outputs at 64 x 16) and the three channels one after another
// behind barriers; at 4K its level 1 took 0.66 ms of the C3 decode's 0.94.
// Here a workgroup owns a tile of kILC subband columns (2 kILC output
// columns) and a band of output row pairs of one frame, one channel group of
// kILC lanes per YCoCg channel, and slides down the band one subband row per
// step:
//   row pass (axis 1): lane = subband column p, from the double-buffered LDS
//     row of the four subbands (columns p - 2 .. p + 2): 'a' = idwt(LL, HL)
//     and 'd' = idwt(LH, HH) at output columns 2p, 2p + 1;
//   column pass (axis 0): a register window of the last five 'a' and 'd'
//     rows of the lane's two columns gives output rows 2m, 2m + 1;
//   level 1: the three channels' outputs meet in LDS and every thread turns
//     one dword of the two RGB output rows into bytes (coalesced stores);
//     other levels store their float64 plane directly.
// One barrier per step: step t issues the HBM loads of row t + 1, runs row t's
// row pass from LDS and the column pass over window rows t - 4 .. t, stores
// row t + 1 into the other LDS buffer (the loads' only wait), and one channel
// wave's RGB stage converts step t - 1's outputs.  (A/B on C3 level 1, scripts/
// micro/idwt_line_exp.py: 64-lane channel groups 0.469 ms vs 128 lanes 0.518;
// the column pass before the row pass -- LDS reads in flight over it -- 0.71,
// its 40 more live VGPRs cost a wave per SIMD; halo lanes' loads under a
// branch 0.56: the compiler consumed them right after issue)
//
// Arithmetic (bit-exact): output n of idwt(x, y) over a line
// of N is sum_j lo[2j + e] x[(i - j) mod N] then sum_j hi[2j + e] y[(i - j)
// mod N], j = 0..F/2 - 1 ascending, i = (n + F/2 - 1) / 2, e = n & 1, one
// product at a time (-ffp-contract=off).  pywt's reordered first F/4 pair
// indices only swap the first two products of the sum (idwt_top with N >=
// F/4), and a + b == b + a, so every output takes the plain order; the sums
// start at the first product (Z0) and skip zero taps -- the same bytes.
#pragma once

constexpr int kILC = 64;             // subband columns per tile = lanes per channel group (one wave)
constexpr int kINT = 3 * kILC;       // threads per workgroup: one channel group per YCoCg channel
constexpr int kINC = kILC + 4;       // LDS columns per subband row: two halo columns each side

// sum over the five pair taps of parity E: x[j] / y[j] = approximation /
// detail input i - j
template <unsigned ZLO, unsigned ZHI, int CT, int E>
__device__ __forceinline__ double inv_pair(const double (&x)[5], const double (&y)[5])
{
    double s = 0.0;
    bool first = true;   // resolved at compile time (unrolled, constant masks)
#pragma unroll
    for (int j = 0; j < 5; ++j)
        if (!((ZLO >> (2 * j + E)) & 1u)) {
            const double p = ct_rec(CT, false, 2 * j + E) * x[j];
            s = first ? p : s + p;
            first = false;
        }
#pragma unroll
    for (int j = 0; j < 5; ++j)
        if (!((ZHI >> (2 * j + E)) & 1u)) {
            const double p = ct_rec(CT, true, 2 * j + E) * y[j];
            s = first ? p : s + p;
            first = false;
        }
    return s;
}

__device__ __forceinline__ int mod_n(int p, int N)
{
    p %= N;
    return p < 0 ? p + N : p;
}

// one subband column of one row: LL (float64) and the three detail bytes
struct InvCol {
    double ll;
    uint32_t hl, lh, hh;
};

// dequant of a detail byte (2D-DWT.py:88-93): (b - 128) * Q in int16; for
// Q <= 256 the product never wraps and is b * Q - 128 Q exactly (QS)
template <bool QS>
__device__ __forceinline__ double dequant_b(uint32_t b, int Q, double qd)
{
    if constexpr (QS) return __builtin_fma((double)b, qd, -128.0 * qd);
    return dequant((int16_t)b, Q);
}

// clip to [0, 255] and astype(uint8) (2D-DWT.py:96-101)
__device__ __forceinline__ uint32_t rgb_u8(double v)
{
    return (uint32_t)__builtin_fmin(__builtin_fmax(v, 0.0), 255.0);
}

template <bool FROM_PACKED_LL, bool TO_RGB, unsigned ZLO, unsigned ZHI, int CT, bool QS>
__global__ __launch_bounds__(kINT) void idwt_line_kernel(const uint8_t *__restrict__ packed, long long packed_stride,
                                                         long long ll_off, long long off_lh, long long off_hl,
                                                         long long off_hh, const double *__restrict__ prev,
                                                         long long plane_stride, int lda, double *__restrict__ out,
                                                         uint8_t *__restrict__ rgb, int h, int w, int oh, int ow,
                                                         int Q, int n_tiles, int n_bands, int brows)
{
    __shared__ __attribute__((aligned(16))) double sin[2][3][4][kINC];   // [buf][ch][LL|HL|LH|HH][column]
    __shared__ __attribute__((aligned(16))) double sout[TO_RGB ? 2 : 1][2][3][TO_RGB ? 2 * kILC : 2];

    const int tile = blockIdx.x % n_tiles, rest = blockIdx.x / n_tiles;
    const int band = rest % n_bands;
    const long long frame = rest / n_bands;
    const int tid = threadIdx.x;
    const int ch = __builtin_amdgcn_readfirstlane(tid / kILC);   // wave-uniform: kILC % 64 == 0
    const int lane = tid - ch * kILC;
    const int P0 = tile * kILC;
    const int ohp = (oh + 1) >> 1;
    const int m0 = band * brows, m1 = min(ohp, m0 + brows);
    const int nsteps = m1 - m0 + 4;   // subband rows m0 - 2 .. m1 + 1
    const double qd = (double)Q;
    const uint8_t *pk = packed + frame * packed_stride;
    const double *pv = FROM_PACKED_LL ? nullptr : prev + (frame * 3 + ch) * plane_stride;

    // this lane's LDS columns: slot lane + 2 (subband column P0 + lane) and, for
    // lanes 0..3, one halo slot (0, 1, kILC + 2, kILC + 3); slot c holds column
    // (P0 - 2 + c) mod w.  Loads: a row base in SGPRs + a 32-bit lane offset.
    // (every lane loads a halo column -- its own again unless it is a halo lane
    // -- so the loads stay unconditional and in flight until the step's end)
    const bool has_halo = lane < 4;
    const int hslot = lane < 2 ? lane : kILC + lane;
    const uint32_t x_main = (uint32_t)mod_n(P0 + lane, w);
    const uint32_t x_halo = has_halo ? (uint32_t)mod_n(P0 - 2 + hslot, w) : x_main;
    const uint32_t b_main = 3 * x_main + ch, b_halo = 3 * x_halo + ch;
    auto load = [&](int y, uint32_t x, uint32_t bo) -> InvCol {
        InvCol c;
        const long long rb = (long long)y * w * 3;
        const uint8_t *row = pk + rb;
        if (FROM_PACKED_LL) {
            const uint16_t v = *reinterpret_cast<const uint16_t *>(pk + ll_off + 2 * (rb + bo));
            c.ll = dequant((int16_t)v, Q);
        } else {
            c.ll = (pv + (long long)y * lda)[x];
        }
        c.hl = (row + off_hl)[bo];   // 'ad' = cV = HL
        c.lh = (row + off_lh)[bo];   // 'da' = cH = LH
        c.hh = (row + off_hh)[bo];   // 'dd' = cD = HH
        return c;
    };
    auto store = [&](int buf, int slot, const InvCol &c) {
        double *s = &sin[buf][ch][0][slot];
        s[0] = c.ll;
        s[kINC] = dequant_b<QS>(c.hl, Q, qd);
        s[2 * kINC] = dequant_b<QS>(c.lh, Q, qd);
        s[3 * kINC] = dequant_b<QS>(c.hh, Q, qd);
    };

    // RGB stage of output pair m from sout[buf], by channel group g (a
    // different one each step): lane = (row lane / 64, pixels 4q .. 4q + 3 of
    // the tile row, q = lane % 64) -> three dwords of bytes
    const int npx = min(2 * kILC, ow - 2 * P0);   // valid pixels of a tile row
    auto to_rgb = [&](int buf, int m) {
        const int r = lane / (kILC / 2), q = lane % (kILC / 2);
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

    // prologue: row 0 of the band (subband row m0 - 2) into buffer 0
    {
        const int y = wrap_once(m0 - 2, h);
        store(0, lane + 2, load(y, x_main, b_main));
        store(0, has_halo ? hslot : lane + 2, load(y, x_halo, b_halo));
    }
    __syncthreads();

    const bool lane_ok = P0 + lane < w;
    const int xo = 2 * (P0 + lane);
    double wa[5][2], wd[5][2];   // 'a' / 'd' row of step t (columns 2p, 2p + 1) in slot t % 5
    for (int t0 = 0; t0 < nsteps; t0 += 5) {
#pragma unroll
        for (int u = 0; u < 5; ++u) {
            const int t = t0 + u;
            if (t >= nsteps) break;
            // prefetch row t + 1 (past the band's last row: a row nobody reads)
            const int yn = wrap_once(m0 - 1 + t, h);   // h >= 5: one wrap at most
            const InvCol nm = load(yn, x_main, b_main), nh = load(yn, x_halo, b_halo);
            // row pass of row t (subband row m0 - 2 + t) into window slot t % 5
            {
                const double *S = &sin[t & 1][ch][0][lane];
                double xl[5], xh[5], yl[5], yh[5];
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    xl[j] = S[4 - j];
                    xh[j] = S[kINC + 4 - j];
                    yl[j] = S[2 * kINC + 4 - j];
                    yh[j] = S[3 * kINC + 4 - j];
                }
                wa[u][0] = inv_pair<ZLO, ZHI, CT, 0>(xl, xh);
                wa[u][1] = inv_pair<ZLO, ZHI, CT, 1>(xl, xh);
                wd[u][0] = inv_pair<ZLO, ZHI, CT, 0>(yl, yh);
                wd[u][1] = inv_pair<ZLO, ZHI, CT, 1>(yl, yh);
            }
            // column pass: output pair m = m0 - 4 + t from rows m - 2 .. m + 2 (steps t - 4 .. t)
            if (t >= 4) {
                const int m = m0 - 4 + t;
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
                if constexpr (TO_RGB) {
#pragma unroll
                    for (int r = 0; r < 2; ++r)
                        *reinterpret_cast<double2 *>(&sout[t & 1][r][ch][2 * lane]) = make_double2(o[r][0], o[r][1]);
                } else if (lane_ok) {
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        const int n = 2 * m + r;
                        if (n >= oh) continue;
                        double *q = out + (frame * 3 + ch) * plane_stride + (long long)n * ow;
                        if (xo + 1 < ow && (((reinterpret_cast<uintptr_t>(q) >> 3) + xo) & 1) == 0)
                            *reinterpret_cast<double2 *>(q + xo) = make_double2(o[r][0], o[r][1]);
                        else {
                            q[xo] = o[r][0];
                            if (xo + 1 < ow) q[xo + 1] = o[r][1];
                        }
                    }
                }
            }
            // row t + 1 into LDS; a non-halo lane's "halo" is its own column again
            // (the same bytes to the same slot: no branch, so the loads stay in
            // flight until here)
            store((t + 1) & 1, lane + 2, nm);
            store((t + 1) & 1, has_halo ? hslot : lane + 2, nh);
            // the RGB bytes of step t - 1 (after the prefetch has landed: its wait
            // does not cover these stores)
            if constexpr (TO_RGB) {
                if (t >= 5 && ch == t % 3) to_rgb((t - 1) & 1, m0 - 5 + t);
            }
            __syncthreads();
        }
    }
    if constexpr (TO_RGB) {
        if (ch == nsteps % 3) to_rgb((nsteps - 1) & 1, m1 - 1);
    }
}
