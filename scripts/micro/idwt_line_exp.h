#pragma once
template <bool FROM_PACKED_LL, bool TO_RGB, unsigned ZLO, unsigned ZHI, int CT, bool QS, bool REORDER, bool HALO_BR, int NL, int WPE>
__global__ __launch_bounds__(3 * NL) __attribute__((amdgpu_waves_per_eu(WPE))) void idwt_line_exp_kernel(const uint8_t *__restrict__ packed, long long packed_stride,
                                                         long long ll_off, long long off_lh, long long off_hl,
                                                         long long off_hh, const double *__restrict__ prev,
                                                         long long plane_stride, int lda, double *__restrict__ out,
                                                         uint8_t *__restrict__ rgb, int h, int w, int oh, int ow,
                                                         int Q, int n_tiles, int n_bands, int brows)
{
    constexpr int XNC = NL + 4;
    __shared__ __attribute__((aligned(16))) double sin[2][3][4][XNC];   // [buf][ch][LL|HL|LH|HH][column]
    __shared__ __attribute__((aligned(16))) double sout[TO_RGB ? 2 : 1][2][3][TO_RGB ? 2 * NL : 2];

    const int tile = blockIdx.x % n_tiles, rest = blockIdx.x / n_tiles;
    const int band = rest % n_bands;
    const long long frame = rest / n_bands;
    const int tid = threadIdx.x;
    const int ch = __builtin_amdgcn_readfirstlane(tid / NL);   // wave-uniform: NL % 64 == 0
    const int lane = tid - ch * NL;
    const int P0 = tile * NL;
    const int ohp = (oh + 1) >> 1;
    const int m0 = band * brows, m1 = min(ohp, m0 + brows);
    const int nsteps = m1 - m0 + (REORDER ? 5 : 4);
    const double qd = (double)Q;
    const uint8_t *pk = packed + frame * packed_stride;
    const double *pv = FROM_PACKED_LL ? nullptr : prev + (frame * 3 + ch) * plane_stride;

    // this lane's LDS columns: slot lane + 2 (subband column P0 + lane) and, for
    // lanes 0..3, one halo slot (0, 1, NL + 2, NL + 3); slot c holds column
    // (P0 - 2 + c) mod w.  Loads: a row base in SGPRs + a 32-bit lane offset.
    // (every lane loads a halo column -- its own again unless it is a halo lane
    // -- so the loads stay unconditional and in flight until the step's end)
    const bool has_halo = lane < 4;
    const int hslot = lane < 2 ? lane : NL + lane;
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
        s[XNC] = dequant_b<QS>(c.hl, Q, qd);
        s[2 * XNC] = dequant_b<QS>(c.lh, Q, qd);
        s[3 * XNC] = dequant_b<QS>(c.hh, Q, qd);
    };

    // RGB stage of output pair m from sout[buf], by channel group g (a
    // different one each step): lane = (row lane / 64, pixels 4q .. 4q + 3 of
    // the tile row, q = lane % 64) -> three dwords of bytes
    const int npx = min(2 * NL, ow - 2 * P0);   // valid pixels of a tile row
    auto to_rgb = [&](int buf, int m) {
        const int r = lane / (NL / 2), q = lane % (NL / 2);
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
            const int yn = wrap_once(m0 - 1 + t, h);
            InvCol nm{}, nh{};
            nm = load(yn, x_main, b_main);
            if (HALO_BR) { if (has_halo) nh = load(yn, x_halo, b_halo); }
            else nh = load(yn, x_halo, b_halo);
            const double *S = &sin[t & 1][ch][0][lane];
            double xl[5], xh[5], yl[5], yh[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                xl[j] = S[4 - j];
                xh[j] = S[XNC + 4 - j];
                yl[j] = S[2 * XNC + 4 - j];
                yh[j] = S[3 * XNC + 4 - j];
            }
            auto rowpass = [&]() {
                wa[u][0] = inv_pair<ZLO, ZHI, CT, 0>(xl, xh);
                wa[u][1] = inv_pair<ZLO, ZHI, CT, 1>(xl, xh);
                wd[u][0] = inv_pair<ZLO, ZHI, CT, 0>(yl, yh);
                wd[u][1] = inv_pair<ZLO, ZHI, CT, 1>(yl, yh);
            };
            if (!REORDER) rowpass();
            // REORDER: pair m0 - 5 + t from slots of steps t-5..t-1; else pair m0 - 4 + t from t-4..t
            constexpr int LAG = REORDER ? 5 : 4;
            if (t >= LAG) {
                const int m = m0 - LAG + t;
                double o[2][2];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    double xa[5], xd[5];
#pragma unroll
                    for (int j = 0; j < 5; ++j) {
                        xa[j] = wa[(u + (REORDER ? 4 : 5) - j) % 5][e];
                        xd[j] = wd[(u + (REORDER ? 4 : 5) - j) % 5][e];
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
                        q[xo] = o[r][0];
                        if (xo + 1 < ow) q[xo + 1] = o[r][1];
                    }
                }
            }
            if (REORDER) rowpass();
            store((t + 1) & 1, lane + 2, nm);
            if (HALO_BR) { if (has_halo) store((t + 1) & 1, hslot, nh); }
            else store((t + 1) & 1, has_halo ? hslot : lane + 2, nh);
            if constexpr (TO_RGB) {
                if (t >= LAG + 1 && ch == t % 3) to_rgb((t - 1) & 1, m0 - LAG - 1 + t);
            }
            __syncthreads();
        }
    }
    if constexpr (TO_RGB) {
        if (ch == nsteps % 3) to_rgb((nsteps - 1) & 1, m1 - 1);
    }
}
