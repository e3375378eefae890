// vcf_dwt_lift.h -- the opt-in lifting form of the bior4.4 (CDF 9/7) 2D-DWT
// + deadzone encode and decode (vcf_dwt_dz_encode_lift / _decode_lift),
// included by vcf_dwt.hip.
//
// NOT bit-exact.  The product entry points (vcf_dwt_dz_encode / _decode)
// compute pywt's 'per' convolution tap by tap in pywt's order, which costs
// 16 float64 products + 16 sums per sample and axis (the C3 decode's level 1
// alone sits on the fp64 issue rate).  The same biorthogonal
// transform factors into four lifting steps and a scaling (Daubechies &
// Sweldens; the constants below):
//   forward, pairs (s_n, e_n) = (x[2n], x[2n+1]) of the periodic line:
//     e += a (s_n + s_n+1);  s += b (e_n-1 + e_n);  e += g (s_n + s_n+1);
//     s += d (e_n-1 + e_n);  cA = K s,  cD = -e / K
//   inverse: the same steps undone in reverse order.
// pywt's 'per' mode pads an odd line with a copy of its last sample (the
// forward here does the same); the phase of the pairs matches pywt's
// periodized bior4.4 exactly.  4 fused multiply-adds per sample and axis in
// place of 32 operations, but different roundings: an index or an output byte
// can land one step off the bit-exact path where a value sits on a
// quantization (or the final truncation) boundary.  Measured tolerance
// (tests/test_dwt_lift_gpu.py): every index and every decoded byte within +-1
// of the bit-exact path; no differences on the C3 synthetic 4K frame or on
// uniform-noise frames, a few 1e-4 of the indices and up to half of the
// decoded bytes of a flat white frame (255.0 reconstructed as 254.99999...).
//
// Kernels: one wave per (frame, YCoCg channel, strip of 124 coefficient
// columns, band of rows); a workgroup = the three channel waves of one strip
// and band.  Lane l holds coefficient columns j, j + 1 (j = strip * 124 - 2 +
// 2 l), i.e. the four sample columns 2j .. 2j + 3, so the horizontal lifting
// runs across the wave with one DPP lane shift per step (no LDS, no barrier)
// and coefficient pairs 2..125 of the wave come out exact (4 steps reach +-2
// pairs).  The vertical lifting streams down the band one row pair per step
// with the pipeline state in registers (5 doubles per column forward, 4
// inverse); a band of B output row pairs reads B + 4.  Pairs of levels run
// as one launch where the planes halve evenly (lift_fwd12_kernel /
// lift_inv21_kernel below: C3's levels 1 + 2 and 3 + 4), single levels on
// lift_fwd_kernel / lift_inv_kernel; LL planes between launches are float64
// in the caller's workspace (the product path's workspace layout is big
// enough), details and the last LL go straight into the packed layout.
// Level 1 of the encode stages its RGB rows through LDS (two dwords per
// thread), detail bytes leave through LDS as dwords, and level 1 of the
// decode meets the three channels in LDS to form RGB.
#pragma once

namespace lift {

// CDF 9/7 lifting constants (bior4.4)
constexpr double kA = -1.586134342059924;
constexpr double kB = -0.052980118572961;
constexpr double kG = 0.882911075530934;
constexpr double kD = 0.443506852043971;
constexpr double kK = 1.149604398860241;
constexpr double kIK = 1.0 / 1.149604398860241;

constexpr int kP = 2;                   // coefficient pairs per lane (4 sample columns)
constexpr int kValid = 64 * kP - 4;     // exact coefficient columns per wave: pairs 2 .. 64 kP - 3
constexpr int kNT = 192;                // threads per workgroup: one wave per YCoCg channel

// lane i <- lane i + 1 / i - 1 across the whole wave: DPP wave_shl:1 / wave_shr:1,
// one VALU move per dword (the end lanes read 0: halo lanes, their values unused)
template <int CTRL>
__device__ __forceinline__ double dpp_move(double v)
{
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)u, CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, true);
    return __builtin_bit_cast(double, (unsigned long long)(unsigned)lo | ((unsigned long long)(unsigned)hi << 32));
}
__device__ __forceinline__ double from_next(double v) { return dpp_move<0x130>(v); }   // wave_shl:1
__device__ __forceinline__ double from_prev(double v) { return dpp_move<0x138>(v); }   // wave_shr:1

// forward lifting of one row: the lane's two pairs (s[k], e[k]) = samples
// (x[2j+2k], x[2j+2k+1]) -> (cA, cD) = (K s, -e / K); one lane shift per step
__device__ __forceinline__ void fwd_row(double (&s)[2], double (&e)[2])
{
    e[0] = __builtin_fma(kA, s[0] + s[1], e[0]);
    e[1] = __builtin_fma(kA, s[1] + from_next(s[0]), e[1]);
    s[0] = __builtin_fma(kB, from_prev(e[1]) + e[0], s[0]);
    s[1] = __builtin_fma(kB, e[0] + e[1], s[1]);
    e[0] = __builtin_fma(kG, s[0] + s[1], e[0]);
    e[1] = __builtin_fma(kG, s[1] + from_next(s[0]), e[1]);
    s[0] = __builtin_fma(kD, from_prev(e[1]) + e[0], s[0]);
    s[1] = __builtin_fma(kD, e[0] + e[1], s[1]);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        s[k] = kK * s[k];
        e[k] = -e[k] * kIK;
    }
}

// inverse lifting of one row: (a[k], d[k]) = (cA, cD) of the lane's two
// pairs -> samples (x[2j+2k], x[2j+2k+1])
__device__ __forceinline__ void inv_row(double (&a)[2], double (&d)[2])
{
    double s[2] = {a[0] * kIK, a[1] * kIK}, e[2] = {-d[0] * kK, -d[1] * kK};
    s[0] = __builtin_fma(-kD, from_prev(e[1]) + e[0], s[0]);
    s[1] = __builtin_fma(-kD, e[0] + e[1], s[1]);
    e[0] = __builtin_fma(-kG, s[0] + s[1], e[0]);
    e[1] = __builtin_fma(-kG, s[1] + from_next(s[0]), e[1]);
    s[0] = __builtin_fma(-kB, from_prev(e[1]) + e[0], s[0]);
    s[1] = __builtin_fma(-kB, e[0] + e[1], s[1]);
    e[0] = __builtin_fma(-kA, s[0] + s[1], e[0]);
    e[1] = __builtin_fma(-kA, s[1] + from_next(s[0]), e[1]);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        a[k] = s[k];
        d[k] = e[k];
    }
}

__device__ __forceinline__ int wrap(int i, int n)
{
    i %= n;
    return i < 0 ? i + n : i;
}

// the int16 YCoCg sample (A4): R/4 + G/2 + B/4, R/2 - B/2, -R/4 + G/2 - B/4
// are exact in float64 and truncated toward zero -- integer division here.
// ch must be wave-uniform (a scalar branch).
__device__ __forceinline__ double ycocg(int R, int G, int B, int ch)
{
    const int v = ch == 0 ? (R + 2 * G + B) >> 2 : (ch == 1 ? (R - B) / 2 : (2 * G - R - B) / 4);
    return (double)v;
}

__device__ __forceinline__ double ycocg(const uint8_t *px, int ch) { return ycocg(px[0], px[1], px[2], ch); }

// the same for a compile-time channel, truncating divisions as shifts:
// t / 2 = (t + (t < 0)) >> 1, t / 4 = (t + 3 (t < 0)) >> 2
template <int CH>
__device__ __forceinline__ double ycocg_c(int R, int G, int B)
{
    if constexpr (CH == 0) {
        return (double)((R + 2 * G + B) >> 2);
    } else if constexpr (CH == 1) {
        const int t = R - B;
        return (double)((t + (int)((unsigned)t >> 31)) >> 1);
    } else {
        const int t = 2 * G - R - B;
        return (double)((t + ((t >> 31) & 3)) >> 2);
    }
}

// deadzone index + 128 as the packed byte / halfword (A5): a power-of-two Q
// (QP2) is an exact scaling by 2^-qsh, else numpy's correctly rounded x / Q
template <bool QP2>
__device__ __forceinline__ int32_t qk(double x, int Q, int qsh)
{
    return (int32_t)(QP2 ? __builtin_ldexp(x, -qsh) : x / (double)Q);
}

// Two bodies.  Planes whose rows are whole dwords and whose pairs never
// straddle the periodic wrap (w = 2 hw, hw % 4 == 0 forward; w even inverse:
// every C3 level) run a branch-free body (EDGE = false): every global load
// and store is issued unconditionally -- halo lanes' and past-the-row stores
// are buffer stores dropped past the buffer, the wrap is modular addressing
// -- so the compiler's wait counts stay exact and one step's stores stay in
// flight over the next step's loads (gfx950 counts both in vmcnt; a store
// under a lane branch made it wait for everything: 460 -> 234 us on C3's
// level 1).  Other shapes take the general body (EDGE = true).
__device__ __forceinline__ int strip_of(bool, int idx, int) { return idx; }

constexpr uint32_t kDrop = 0x80000000u;   // a buffer offset past any buffer: the store is dropped
typedef unsigned int U32x2 __attribute__((__vector_size__(8)));
typedef unsigned int U32x4 __attribute__((__vector_size__(16)));

__device__ __forceinline__ U32x4 pack2(double a, double b)
{
    const U32x2 x = __builtin_bit_cast(U32x2, a), y = __builtin_bit_cast(U32x2, b);
    return U32x4{x[0], x[1], y[0], y[1]};
}

// one forward level: plane h x w (level 1: the RGB frame) -> LL hh x hw
// (float64 plane, or u16 packed at the last level) and the three detail
// subbands (u8 packed)
constexpr int kRowDw = 64 * kP * 2 * 3 / 4;            // dwords of one staged RGB row
constexpr int kSbB = kValid * 3, kSbDw = 3 * kSbB / 4;  // bytes of one subband row, dwords of three

// RAW (diagnostic, vcf_dwt_lift_analyze_f64 only): the general body also stores the
// three detail subbands' float64 coefficients before quantization, raw[(sb * 3 +
// ch) * hh * hw + row * hw + col] for sb = LH, HL, HH of a single frame
template <bool FIRST, bool LAST, bool EDGE, bool QP2, bool RAW = false>
__device__ __forceinline__ void lift_fwd_body(const uint8_t *__restrict__ rgb, long long rgb_stride,
                                              const double *__restrict__ in, long long plane_stride,
                                              double *__restrict__ LLout, uint8_t *__restrict__ packed,
                                              long long packed_stride, long long ll_off, long long off_lh,
                                              long long off_hl, long long off_hh, int h, int w, int hh, int hw, int Q,
                                              int n_int, int n_set, int n_bands, int brows, int bid,
                                              uint32_t *px_lds, uint32_t *sb_lds, double *raw = nullptr)
{
    const int qsh = QP2 ? __builtin_ctz((unsigned)Q) : 0;
    // byte staging through LDS (interior strips; double-buffered, one barrier
    // each): level 1's two RGB rows of 256 pixels come in as two dwords per
    // thread, and the three detail subbands' kValid x 3 interleaved bytes
    // leave as dwords (+ one dummy dword for the halo lanes' bytes)
    const int t = threadIdx.x, lane = t & 63, ch = __builtin_amdgcn_readfirstlane(t >> 6);
    int b = bid;
    const int strip = strip_of(EDGE, b % n_set, n_int);
    b /= n_set;
    const int band = b % n_bands;
    const long long frame = b / n_bands;
    const long long plane = frame * 3 + ch;
    const int jl = strip * kValid - 2 + kP * lane;             // the lane's first coefficient column
    int col[2 * kP];                                           // its sample columns
    uint32_t drop[kP];
#pragma unroll
    for (int k = 0; k < kP; ++k) {
        if (EDGE) {
            col[2 * k] = 2 * wrap(jl + k, hw);
            col[2 * k + 1] = min(col[2 * k] + 1, w - 1);       // odd width: the last sample repeats
        } else {
            col[2 * k] = 2 * (wrap(jl, hw) + k);
            col[2 * k + 1] = 2 * (wrap(jl, hw) + k) + 1;
        }
        const int p = kP * lane + k;
        drop[k] = p >= 2 && p < 2 + kValid && jl + k < hw ? 0u : kDrop;
    }
    const int m0 = band * brows, m1 = min(m0 + brows, hh);
    const uint8_t *src8 = FIRST ? rgb + frame * rgb_stride : nullptr;
    const double *src = FIRST ? nullptr : in + plane * plane_stride;
    uint8_t *pk = packed + frame * packed_stride;
    const __amdgpu_buffer_rsrc_t rs_pk = __builtin_amdgcn_make_buffer_rsrc(pk, 0, (int)packed_stride, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_ll = __builtin_amdgcn_make_buffer_rsrc(
        LAST ? (void *)pk : (void *)(LLout + plane * plane_stride), 0, LAST ? 0 : (int)((long long)hh * hw * 8),
        0x00020000);
    const int x0 = strip * 2 * kValid - 4;                     // first staged pixel (level 1)
    // this thread's staged dword of a row, wrapped modulo the row's 3w bytes
    // (w % 4 == 0: the wrapped dword stays aligned and on the same byte phase)
    const int boff = wrap(3 * x0 + 4 * t, 3 * w);
    // row pairs are read ahead of the one in use (wrapped index nf)
    const int n_last = m1 + 1;
    int nf = wrap(m0 - 2, hh);
    auto next_pair = [&]() { nf = nf + 1 == hh ? 0 : nf + 1; };
    auto fetch = [&]() -> uint2 {
        const uint8_t *ra = src8 + (long long)(2 * nf) * w * 3 + boff;
        const uint8_t *rb = src8 + (long long)min(2 * nf + 1, h - 1) * w * 3 + boff;
        return make_uint2(*(const uint32_t *)ra, *(const uint32_t *)rb);
    };
    auto load = [&](double (&s2)[2 * kP], double (&e2)[2 * kP]) {
        const int ra = 2 * nf, rb = min(2 * nf + 1, h - 1);     // odd height: the last row repeats
        if (FIRST) {
            const uint8_t *pa = src8 + (long long)ra * w * 3, *pb = src8 + (long long)rb * w * 3;
#pragma unroll
            for (int k = 0; k < 2 * kP; ++k) {
                s2[k] = ycocg(pa + 3 * col[k], ch);
                e2[k] = ycocg(pb + 3 * col[k], ch);
            }
        } else if (EDGE) {
            const double *pa = src + (long long)ra * w, *pb = src + (long long)rb * w;
#pragma unroll
            for (int k = 0; k < 2 * kP; ++k) {
                s2[k] = pa[col[k]];
                e2[k] = pb[col[k]];
            }
        } else {
            const double2 *qa = (const double2 *)(src + (long long)ra * w + col[0]);
            const double2 *qb = (const double2 *)(src + (long long)rb * w + col[0]);
#pragma unroll
            for (int k = 0; k < kP; ++k) {
                const double2 va = qa[k], vb = qb[k];
                s2[2 * k] = va.x;
                s2[2 * k + 1] = va.y;
                e2[2 * k] = vb.x;
                e2[2 * k + 1] = vb.y;
            }
        }
    };
    constexpr bool kStaged = FIRST && !EDGE;
    uint2 q0 = make_uint2(0, 0), q1 = make_uint2(0, 0);
    double ns[2 * kP], ne[2 * kP];
    if (kStaged) {
        q0 = fetch();
        next_pair();
        q1 = fetch();
        next_pair();
    } else {
        load(ns, ne);
        next_pair();
    }
    int buf = 0;

    // the column pipelines: s_{n-1}, e_{n-1}, e1_{n-2}, s1_{n-2}, e2_{n-3} per sample column
    double sp[2 * kP], ep[2 * kP], e1p[2 * kP], s1p[2 * kP], e2p[2 * kP];
#pragma unroll
    for (int k = 0; k < 2 * kP; ++k) sp[k] = ep[k] = e1p[k] = s1p[k] = e2p[k] = 0.0;
    for (int n = m0 - 2; n <= n_last; ++n, buf ^= 1) {
        double s[2 * kP], e[2 * kP];
        if (kStaged) {
            uint32_t *st = px_lds + 2 * kRowDw * buf;
            st[t] = q0.x;
            st[kRowDw + t] = q0.y;
            q0 = q1;
            q1 = fetch();      // (unconditional: a branch around it would cost exact wait counts;
            next_pair();       // past the band it reads a wrapped row it does not use)
            asm volatile("" ::: "memory");   // (a compiler barrier: issued here, not sunk past the stores)
            __syncthreads();
            // the lane's four pixels of each row: 12 bytes at 12 * lane; one
            // scalar branch on the wave's channel around all eight samples
            auto unpack = [&](auto chc) {
                constexpr int C = decltype(chc)::value;
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const uint32_t *d = st + r * kRowDw + 3 * lane;
                    const int d0 = (int)d[0], d1 = (int)d[1], d2 = (int)d[2];
                    double *o = r ? e : s;
                    o[0] = ycocg_c<C>(d0 & 255, (d0 >> 8) & 255, (d0 >> 16) & 255);
                    o[1] = ycocg_c<C>((unsigned)d0 >> 24, d1 & 255, (d1 >> 8) & 255);
                    o[2] = ycocg_c<C>((d1 >> 16) & 255, (unsigned)d1 >> 24, d2 & 255);
                    o[3] = ycocg_c<C>((d2 >> 8) & 255, (d2 >> 16) & 255, (unsigned)d2 >> 24);
                }
            };
            if (ch == 0) unpack(std::integral_constant<int, 0>{});
            else if (ch == 1) unpack(std::integral_constant<int, 1>{});
            else unpack(std::integral_constant<int, 2>{});
        } else {
#pragma unroll
            for (int k = 0; k < 2 * kP; ++k) {
                s[k] = ns[k];
                e[k] = ne[k];
            }
            load(ns, ne);      // (unconditional, as above)
            next_pair();
            asm volatile("" ::: "memory");
        }
        double L[2 * kP], D[2 * kP];
#pragma unroll
        for (int k = 0; k < 2 * kP; ++k) {
            const double e1 = __builtin_fma(kA, sp[k] + s[k], ep[k]);    // e1_{n-1}
            const double s1 = __builtin_fma(kB, e1p[k] + e1, sp[k]);     // s1_{n-1}
            const double e2 = __builtin_fma(kG, s1p[k] + s1, e1p[k]);    // e2_{n-2}
            const double s2 = __builtin_fma(kD, e2p[k] + e2, s1p[k]);    // s2_{n-2}
            L[k] = kK * s2;
            D[k] = -e2 * kIK;
            sp[k] = s[k];
            ep[k] = e[k];
            e1p[k] = e1;
            s1p[k] = s1;
            e2p[k] = e2;
        }
        const int m = n - 2;                                       // output row pair (uniform)
        if (m < m0) continue;
        double ll[2] = {L[0], L[2]}, hl[2] = {L[1], L[3]}, lh[2] = {D[0], D[2]}, hhv[2] = {D[1], D[3]};
        fwd_row(ll, hl);    // (aa, ad) = (LL, HL)
        fwd_row(lh, hhv);   // (da, dd) = (LH, HH)
        const long long orow = (long long)m * hw;
        uint8_t q[3][kP];
#pragma unroll
        for (int k = 0; k < kP; ++k) {
            q[0][k] = (uint8_t)(uint32_t)(qk<QP2>(lh[k], Q, qsh) + 128);   // += 128, astype(uint8): wraps
            q[1][k] = (uint8_t)(uint32_t)(qk<QP2>(hl[k], Q, qsh) + 128);
            q[2][k] = (uint8_t)(uint32_t)(qk<QP2>(hhv[k], Q, qsh) + 128);
            const uint32_t o = (uint32_t)(orow + jl + k);          // (a halo lane's may be junk: dropped)
            if (LAST)
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(uint32_t)(qk<QP2>(ll[k], Q, qsh) + 128), rs_pk,
                                                      ((uint32_t)ll_off + 2 * (3 * o + ch)) | drop[k], 0, 0);
            else if (EDGE)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(U32x2, ll[k]), rs_ll, (8 * o) | drop[k], 0,
                                                      0);
        }
        if (!LAST && !EDGE)   // both pairs of a lane are in or out together (even jl, even hw): one 16-byte store
            __builtin_amdgcn_raw_buffer_store_b128(pack2(ll[0], ll[1]), rs_ll, (8 * (uint32_t)(orow + jl)) | drop[0],
                                                   0, 0);
        if (!EDGE) {
            uint8_t *so = (uint8_t *)(sb_lds + (kSbDw + 1) * buf);
#pragma unroll
            for (int k = 0; k < kP; ++k) {
                const int p = drop[k] ? 3 * kSbB : 3 * (kP * lane + k - 2) + ch;   // halo lanes: the dummy dword
                const int dsb = drop[k] ? 0 : kSbB;
                so[p] = q[0][k];
                so[p + dsb] = q[1][k];
                so[p + 2 * dsb] = q[2][k];
            }
            __syncthreads();
            const uint32_t base = (uint32_t)off_lh + 3 * (uint32_t)(orow + strip * kValid);
            const int row_b = 3 * (hw - strip * kValid);            // the strip's bytes in the row
            const uint32_t sstep = (uint32_t)(off_hl - off_lh);
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int i = t + r * kNT;
                const int ic = min(i, kSbDw - 1);
                const int sub = ic / (kSbB / 4), d = ic - (kSbB / 4) * sub;
                __builtin_amdgcn_raw_buffer_store_b32(sb_lds[(kSbDw + 1) * buf + ic], rs_pk,
                                                      (base + sub * sstep + 4 * d) |
                                                          (i < kSbDw && 4 * d < row_b ? 0u : kDrop),
                                                      0, 0);
            }
        } else {
#pragma unroll
            for (int k = 0; k < kP; ++k) {
                const uint32_t o = 3 * (uint32_t)(orow + jl + k) + ch;
                __builtin_amdgcn_raw_buffer_store_b8(q[0][k], rs_pk, ((uint32_t)off_lh + o) | drop[k], 0, 0);
                __builtin_amdgcn_raw_buffer_store_b8(q[1][k], rs_pk, ((uint32_t)off_hl + o) | drop[k], 0, 0);
                __builtin_amdgcn_raw_buffer_store_b8(q[2][k], rs_pk, ((uint32_t)off_hh + o) | drop[k], 0, 0);
                if (RAW && !drop[k]) {
                    const long long at = orow + jl + k, sbp = (long long)hh * hw;
                    raw[(0 * 3 + ch) * sbp + at] = lh[k];
                    raw[(1 * 3 + ch) * sbp + at] = hl[k];
                    raw[(2 * 3 + ch) * sbp + at] = hhv[k];
                }
            }
        }
    }
}

// the diagnostic launch: every workgroup on the general body, details also as float64
template <bool FIRST>
__global__ __launch_bounds__(kNT) void lift_fwd_raw_kernel(const uint8_t *__restrict__ rgb, const double *__restrict__ in,
                                                           long long plane_stride, double *__restrict__ LLout,
                                                           uint8_t *__restrict__ packed, long long packed_stride,
                                                           long long off_lh, long long off_hl, long long off_hh, int h,
                                                           int w, int hh, int hw, int n_strips, int n_bands, int brows,
                                                           double *__restrict__ raw)
{
    __shared__ uint32_t px_lds[1];
    __shared__ uint32_t sb_lds[2 * (kSbDw + 1)];
    lift_fwd_body<FIRST, false, true, false, true>(rgb, 0, in, plane_stride, LLout, packed, packed_stride, 0, off_lh,
                                                   off_hl, off_hh, h, w, hh, hw, 1, 0, n_strips, n_bands, brows,
                                                   blockIdx.x, px_lds, sb_lds, raw);
}

// one launch per level: the general body's workgroups first (odd shapes: all
// of them), then the branch-free body's (QP2: a power-of-two Q)
template <bool FIRST, bool LAST, bool QP2>
__global__ __launch_bounds__(kNT) void lift_fwd_kernel(const uint8_t *__restrict__ rgb, long long rgb_stride,
                                                       const double *__restrict__ in, long long plane_stride,
                                                       double *__restrict__ LLout, uint8_t *__restrict__ packed,
                                                       long long packed_stride, long long ll_off, long long off_lh,
                                                       long long off_hl, long long off_hh, int h, int w, int hh,
                                                       int hw, int Q, int n_int, int n_edge, int n_bands, int brows,
                                                       int n_bands_e, int brows_e, int edge_blocks)
{
    __shared__ uint32_t px_lds[FIRST ? 2 * 2 * kRowDw : 1];
    __shared__ uint32_t sb_lds[2 * (kSbDw + 1)];
    const int bid = blockIdx.x;
    if (bid < edge_blocks)
        lift_fwd_body<FIRST, LAST, true, QP2>(rgb, rgb_stride, in, plane_stride, LLout, packed, packed_stride, ll_off,
                                         off_lh, off_hl, off_hh, h, w, hh, hw, Q, n_int, n_edge, n_bands_e, brows_e,
                                         bid, px_lds, sb_lds);
    else
        lift_fwd_body<FIRST, LAST, false, QP2>(rgb, rgb_stride, in, plane_stride, LLout, packed, packed_stride, ll_off,
                                          off_lh, off_hl, off_hh, h, w, hh, hw, Q, n_int, n_int, n_bands, brows,
                                          bid - edge_blocks, px_lds, sb_lds);
}

// one inverse level: subbands h x w (LL float64 with row stride lda, or u16
// packed at the coarsest level) -> plane oh x ow (<= 2h x 2w; float64), or
// at level 1 RGB u8 (2h x 2w)
constexpr int kOut = 4 * kP;                      // outputs per lane and step: 2 rows x 2 kP columns
constexpr int kRgbRow = 2 * kValid * 3;           // bytes of one RGB output row of the strip
constexpr int kRgbDw = 2 * kRgbRow / 4;

template <bool FROM_PACKED, bool TO_RGB, bool EDGE>
__device__ __forceinline__ void lift_inv_body(const uint8_t *__restrict__ packed, long long packed_stride,
                                              long long ll_off, long long off_lh, long long off_hl, long long off_hh,
                                              const double *__restrict__ in, long long plane_stride, int lda,
                                              double *__restrict__ out, uint8_t *__restrict__ rgb_out,
                                              long long rgb_stride, int h, int w, int oh, int ow, int Q, int n_int,
                                              int n_set, int n_bands, int brows, int bid, double *xch,
                                              uint32_t *rgb_lds)
{
    const int t = threadIdx.x, lane = t & 63, ch = __builtin_amdgcn_readfirstlane(t >> 6);
    int b = bid;
    const int strip = strip_of(EDGE, b % n_set, n_int);
    b /= n_set;
    const int band = b % n_bands;
    const long long frame = b / n_bands;
    const long long plane = frame * 3 + ch;
    const int jl = strip * kValid - 2 + kP * lane;
    int j[kP];
    uint32_t drop[kP];
#pragma unroll
    for (int k = 0; k < kP; ++k) {
        j[k] = wrap(jl + k, w);
        const int p = kP * lane + k;
        drop[k] = p >= 2 && p < 2 + kValid && jl + k < w ? 0u : kDrop;
    }
    const int m0 = band * brows, m1 = min(m0 + brows, h);
    const uint8_t *pk = packed + frame * packed_stride;
    const double *src = FROM_PACKED ? nullptr : in + plane * plane_stride;
    const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(
        TO_RGB ? (void *)(rgb_out + frame * rgb_stride) : (void *)(out + plane * plane_stride), 0,
        TO_RGB ? (int)rgb_stride : (int)((long long)oh * ow * 8), 0x00020000);

    // the column pipelines: e_{q-1}, s1_{q-1}, e1_{q-2}, s2_{q-2} per output column
    double ep[2 * kP], s1p[2 * kP], e1pp[2 * kP], s2pp[2 * kP];
#pragma unroll
    for (int k = 0; k < 2 * kP; ++k) ep[k] = s1p[k] = e1pp[k] = s2pp[k] = 0.0;
    // the coefficients of row q + 1 are in flight over row q's lifting
    int qf = wrap(m0 - 2, h);
    double nA[kP];
    int nb[3][kP];
    auto load = [&]() {
        const long long row = (long long)qf * w;
        if (!FROM_PACKED && !EDGE) {
            const double2 v = *(const double2 *)(src + (long long)qf * lda + j[0]);
            nA[0] = v.x;
            nA[1] = v.y;
        }
#pragma unroll
        for (int k = 0; k < kP; ++k) {
            const long long idx = row + j[k];
            if (FROM_PACKED) nA[k] = dequant((int16_t)*(const uint16_t *)(pk + ll_off + 2 * (3 * idx + ch)), Q);
            else if (EDGE) nA[k] = src[(long long)qf * lda + j[k]];
            nb[0][k] = pk[off_hl + 3 * idx + ch];
            nb[1][k] = pk[off_lh + 3 * idx + ch];
            nb[2][k] = pk[off_hh + 3 * idx + ch];
        }
        qf = qf + 1 == h ? 0 : qf + 1;
    };
    load();
    for (int q = m0 - 2; q <= m1 + 1; ++q) {
        double a[kP], hl[kP], lh[kP], hhv[kP];
#pragma unroll
        for (int k = 0; k < kP; ++k) {
            a[k] = nA[k];
            hl[k] = dequant((int16_t)nb[0][k], Q);
            lh[k] = dequant((int16_t)nb[1][k], Q);
            hhv[k] = dequant((int16_t)nb[2][k], Q);
        }
        load();                // (unconditional: exact wait counts; past the band a wrapped row)
        asm volatile("" ::: "memory");   // (a compiler barrier: issued here, not sunk past the stores)
        inv_row(a, hl);     // row 'a' of the vertical pair: columns 2j .. 2j + 3
        inv_row(lh, hhv);   // row 'd'
        const double A[2 * kP] = {a[0], hl[0], a[1], hl[1]}, Dd[2 * kP] = {lh[0], hhv[0], lh[1], hhv[1]};
        double o0[2 * kP], o1[2 * kP];
#pragma unroll
        for (int k = 0; k < 2 * kP; ++k) {
            const double s = A[k] * kIK, e = -Dd[k] * kK;
            const double s1 = __builtin_fma(-kD, ep[k] + e, s);          // s1_q
            const double e1 = __builtin_fma(-kG, s1p[k] + s1, ep[k]);    // e1_{q-1}
            const double s2 = __builtin_fma(-kB, e1pp[k] + e1, s1p[k]);  // s2_{q-1}
            const double e2 = __builtin_fma(-kA, s2pp[k] + s2, e1pp[k]); // e2_{q-2}
            o0[k] = s2pp[k];                                             // row 2(q-2)
            o1[k] = e2;                                                  // row 2(q-2) + 1
            ep[k] = e;
            s1p[k] = s1;
            e1pp[k] = e1;
            s2pp[k] = s2;
        }
        const int m = q - 2;
        if (m < m0) continue;
        const int r0 = 2 * m, cc = 2 * jl;
        if (TO_RGB) {
            double *x = xch + ch * kOut * 64;
#pragma unroll
            for (int k = 0; k < 2 * kP; ++k) {
                x[k * 64 + lane] = o0[k];
                x[(2 * kP + k) * 64 + lane] = o1[k];
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kOut; ++k) {
                const int r = k / (2 * kP), c = k % (2 * kP);     // output row r0 + r, column cc + c
                const uint32_t dk = drop[c >> 1];
                const double Y = xch[k * 64 + lane], Co = xch[(kOut + k) * 64 + lane],
                             Cg = xch[(2 * kOut + k) * 64 + lane];
                const double v = ch == 0 ? Y + Co - Cg : (ch == 1 ? Y + Cg : Y - Co - Cg);
                const uint8_t u = (uint8_t)(v < 0.0 ? 0.0 : (v > 255.0 ? 255.0 : v));
                if (!EDGE) {
                    const int pos = dk ? kRgbDw * 4 : kRgbRow * r + 3 * (cc + c - 2 * strip * kValid) + ch;
                    ((uint8_t *)rgb_lds)[pos] = u;
                } else {
                    const uint32_t o = 3 * (uint32_t)((long long)(r0 + r) * ow + cc + c) + ch;
                    __builtin_amdgcn_raw_buffer_store_b8(u, rs_out, o | dk, 0, 0);
                }
            }
            __syncthreads();
            if (!EDGE) {
#pragma unroll
                for (int rr = 0; rr < 2; ++rr) {
                    const int i = t + rr * kNT;
                    const int ic = min(i, kRgbDw - 1);
                    const int row = ic >= kRgbRow / 4, d = ic - (kRgbRow / 4) * row;
                    const uint32_t o = 3 * (uint32_t)((long long)(r0 + row) * ow + 2 * strip * kValid) + 4 * d;
                    const uint32_t ok = i < kRgbDw && 4 * d < 3 * (ow - 2 * strip * kValid) ? 0u : kDrop;
                    __builtin_amdgcn_raw_buffer_store_b32(rgb_lds[ic], rs_out, o | ok, 0, 0);
                }
            }
        } else if (EDGE) {
#pragma unroll
            for (int k = 0; k < kOut; ++k) {
                const int r = r0 + k / (2 * kP), c = cc + k % (2 * kP);
                const uint32_t dk = (r < oh && c < ow) ? drop[(k % (2 * kP)) >> 1] : kDrop;
                const double v = k < 2 * kP ? o0[k] : o1[k - 2 * kP];
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(U32x2, v), rs_out,
                                                      (8 * (uint32_t)((long long)r * ow + c)) | dk, 0, 0);
            }
        } else {   // (ow even here: a pair's two columns are in or out together) 16-byte stores
#pragma unroll
            for (int k = 0; k < 2 * kP; ++k) {
                const int r = r0 + k / kP, c = cc + 2 * (k % kP);
                const uint32_t dk = r < oh ? drop[k % kP] : kDrop;
                const double *v = k < kP ? o0 : o1;
                __builtin_amdgcn_raw_buffer_store_b128(pack2(v[2 * (k % kP)], v[2 * (k % kP) + 1]), rs_out,
                                                       (8 * (uint32_t)((long long)r * ow + c)) | dk, 0, 0);
            }
        }
    }
}

template <bool FROM_PACKED, bool TO_RGB>
__global__ __launch_bounds__(kNT) void lift_inv_kernel(const uint8_t *__restrict__ packed, long long packed_stride,
                                                       long long ll_off, long long off_lh, long long off_hl,
                                                       long long off_hh, const double *__restrict__ in,
                                                       long long plane_stride, int lda, double *__restrict__ out,
                                                       uint8_t *__restrict__ rgb_out, long long rgb_stride, int h,
                                                       int w, int oh, int ow, int Q, int n_int, int n_edge,
                                                       int n_bands, int brows, int n_bands_e, int brows_e,
                                                       int edge_blocks)
{
    __shared__ double xch[TO_RGB ? 3 * kOut * 64 : 1];
    __shared__ uint32_t rgb_lds[TO_RGB ? kRgbDw + 1 : 1];
    const int bid = blockIdx.x;
    if (bid < edge_blocks)
        lift_inv_body<FROM_PACKED, TO_RGB, true>(packed, packed_stride, ll_off, off_lh, off_hl, off_hh, in,
                                                 plane_stride, lda, out, rgb_out, rgb_stride, h, w, oh, ow, Q, n_int,
                                                 n_edge, n_bands_e, brows_e, bid, xch, rgb_lds);
    else
        lift_inv_body<FROM_PACKED, TO_RGB, false>(packed, packed_stride, ll_off, off_lh, off_hl, off_hh, in,
                                                  plane_stride, lda, out, rgb_out, rgb_stride, h, w, oh, ow, Q, n_int,
                                                  n_int, n_bands, brows, bid - edge_blocks, xch, rgb_lds);
}

// ---- levels 1 and 2 in one launch (forward) ---------------------------------
// LL1 (49.8 MB of float64 per 4K frame) never leaves the chip.  A lane's two
// level-1 coefficient columns are one level-2 pair, so after each level-1 step
// the lane holds its pair of the new LL1 row; every two LL1 rows feed one step
// of a second column pipeline (level 2, 5 doubles per column) and a one-pair-
// per-lane horizontal lifting across the wave.  Exact lanes: level 1 pairs
// 2..125 of the wave, level 2 lanes 3..60, so a strip owns 58 level-2 columns
// (116 LL1 columns, 232 input columns) and a band of level-2 rows [M0, M1)
// runs 2 (M1 - M0) + 12 level-1 steps.  Even planes only (W % 4 == 0,
// W / 2 % 8 == 0, H % 4 == 0: no repeated LL1 row or column); level-1 detail
// bytes leave as dwords through LDS, level-2 ones as bytes (58 x 3 per row is
// not a whole number of dwords), LL2 as float64 (or u16 at levels == 2).
constexpr int kV2 = 58;                                   // owned level-2 columns per wave (lanes 3..60)
constexpr int kV1 = 2 * kV2;                              // owned level-1 columns (116)
constexpr int kSb1B = kV1 * 3, kSb1Dw = 3 * kSb1B / 4;    // 348 bytes per level-1 subband row, 261 dwords

// forward lifting of one row when each lane holds one pair (s, e) -> (K s, -e / K)
__device__ __forceinline__ void fwd_row1(double &s, double &e)
{
    e = __builtin_fma(kA, s + from_next(s), e);
    s = __builtin_fma(kB, from_prev(e) + e, s);
    e = __builtin_fma(kG, s + from_next(s), e);
    s = __builtin_fma(kD, from_prev(e) + e, s);
    s = kK * s;
    e = -e * kIK;
}

// FIRST = false: the same pair of levels l, l + 1 over a float64 LL plane
// (C3's levels 3 + 4), four input columns per lane as two 16-byte loads per row
template <bool QP2, bool LAST2, bool FIRST = true>
__global__ __launch_bounds__(kNT) void lift_fwd12_kernel(const uint8_t *__restrict__ rgb, long long rgb_stride,
                                                         const double *__restrict__ in,
                                                         double *__restrict__ LL2out, long long plane_stride,
                                                         uint8_t *__restrict__ packed, long long packed_stride,
                                                         long long ll_off, long long off1_lh, long long off1_hl,
                                                         long long off2_lh, long long off2_hl, long long off2_hh,
                                                         int h, int w, int hh, int hw, int hh2, int hw2, int Q,
                                                         int n_strips, int n_bands, int brows)
{
    __shared__ uint32_t px_lds[FIRST ? 2 * 2 * kRowDw : 1];
    __shared__ uint32_t sb_lds[2 * (kSb1Dw + 1)];
    const int qsh = QP2 ? __builtin_ctz((unsigned)Q) : 0;
    const int t = threadIdx.x, lane = t & 63, ch = __builtin_amdgcn_readfirstlane(t >> 6);
    int b = blockIdx.x;
    const int strip = b % n_strips;
    b /= n_strips;
    const int band = b % n_bands;
    const long long frame = b / n_bands;
    const long long plane = frame * 3 + ch;
    const int jl = strip * kV1 - 6 + 2 * lane;                 // the lane's level-1 columns jl, jl + 1
    const int j2 = strip * kV2 - 3 + lane;                     // = its level-2 column
    const bool own = lane >= 3 && lane < 3 + kV2;
    const uint32_t drop1 = own && jl < hw ? 0u : kDrop;        // (jl even, hw even: both columns)
    const uint32_t drop2 = own && j2 < hw2 ? 0u : kDrop;
    const int M0 = band * brows, M1 = min(M0 + brows, hh2);
    const uint8_t *src8 = FIRST ? rgb + frame * rgb_stride : nullptr;
    const double *src = FIRST ? nullptr : in + plane * plane_stride;
    const int cw = 2 * wrap(jl, hw);                           // float64 input: the lane's four columns
    uint8_t *pk = packed + frame * packed_stride;
    const __amdgpu_buffer_rsrc_t rs_pk = __builtin_amdgcn_make_buffer_rsrc(pk, 0, (int)packed_stride, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_ll = __builtin_amdgcn_make_buffer_rsrc(
        LAST2 ? (void *)pk : (void *)(LL2out + plane * plane_stride), 0,
        LAST2 ? 0 : (int)((long long)hh2 * hw2 * 8), 0x00020000);
    const int x0 = 2 * (strip * kV1 - 6);                      // first staged pixel
    const int boff = wrap(3 * x0 + 4 * t, 3 * w);
    int nf = wrap(2 * M0 - 6, hh);                             // the next input row pair to fetch
    auto next_pair = [&]() { nf = nf + 1 == hh ? 0 : nf + 1; };
    auto fetch = [&]() -> uint2 {
        if constexpr (!FIRST) return make_uint2(0, 0);
        const uint8_t *ra = src8 + (long long)(2 * nf) * w * 3 + boff;
        const uint8_t *rb = src8 + (long long)(2 * nf + 1) * w * 3 + boff;
        return make_uint2(*(const uint32_t *)ra, *(const uint32_t *)rb);
    };
    double ns[4] = {0, 0, 0, 0}, ne[4] = {0, 0, 0, 0};
    auto dload = [&]() {
        const double2 *qa = (const double2 *)(src + (long long)(2 * nf) * w + cw);
        const double2 *qb = (const double2 *)(src + (long long)(2 * nf + 1) * w + cw);
        const double2 a0 = qa[0], a1 = qa[1], b0 = qb[0], b1 = qb[1];
        ns[0] = a0.x;
        ns[1] = a0.y;
        ns[2] = a1.x;
        ns[3] = a1.y;
        ne[0] = b0.x;
        ne[1] = b0.y;
        ne[2] = b1.x;
        ne[3] = b1.y;
    };
    uint2 q0 = make_uint2(0, 0), q1 = make_uint2(0, 0);
    if (FIRST) {
        q0 = fetch();
        next_pair();
        q1 = fetch();
        next_pair();
    } else {
        dload();
        next_pair();
    }
    int buf = 0;
    double sp[4], ep[4], e1p[4], s1p[4], e2p[4];               // level-1 column pipelines
#pragma unroll
    for (int k = 0; k < 4; ++k) sp[k] = ep[k] = e1p[k] = s1p[k] = e2p[k] = 0.0;
    double tp[2], fp[2], f1p[2], t1p[2], f2p[2];               // level-2 column pipelines
#pragma unroll
    for (int k = 0; k < 2; ++k) tp[k] = fp[k] = f1p[k] = t1p[k] = f2p[k] = 0.0;
    const uint32_t sstep1 = (uint32_t)(off1_hl - off1_lh);
    const int row_b1 = 3 * (hw - strip * kV1);                 // the strip's bytes in a level-1 row

    // one level-1 step: ingests the next input row pair, returns the lane's
    // pair of LL1 row m and stores row m's level-1 details when the band owns it
    auto l1_step = [&](int m, bool row_own, double (&ll)[2]) {
        double s[4], e[4];
        uint32_t *st = px_lds + 2 * kRowDw * buf;
        if constexpr (!FIRST) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                s[k] = ns[k];
                e[k] = ne[k];
            }
            dload();
            next_pair();
            asm volatile("" ::: "memory");
        } else {
        st[t] = q0.x;
        st[kRowDw + t] = q0.y;
        q0 = q1;
        q1 = fetch();
        next_pair();
        asm volatile("" ::: "memory");
        __syncthreads();
        auto unpack = [&](auto chc) {
            constexpr int C = decltype(chc)::value;
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const uint32_t *d = st + r * kRowDw + 3 * lane;
                const int d0 = (int)d[0], d1 = (int)d[1], d2 = (int)d[2];
                double *o = r ? e : s;
                o[0] = ycocg_c<C>(d0 & 255, (d0 >> 8) & 255, (d0 >> 16) & 255);
                o[1] = ycocg_c<C>((unsigned)d0 >> 24, d1 & 255, (d1 >> 8) & 255);
                o[2] = ycocg_c<C>((d1 >> 16) & 255, (unsigned)d1 >> 24, d2 & 255);
                o[3] = ycocg_c<C>((d2 >> 8) & 255, (d2 >> 16) & 255, (unsigned)d2 >> 24);
            }
        };
        if (ch == 0) unpack(std::integral_constant<int, 0>{});
        else if (ch == 1) unpack(std::integral_constant<int, 1>{});
        else unpack(std::integral_constant<int, 2>{});
        }
        double L[4], D[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double e1 = __builtin_fma(kA, sp[k] + s[k], ep[k]);
            const double s1 = __builtin_fma(kB, e1p[k] + e1, sp[k]);
            const double e2 = __builtin_fma(kG, s1p[k] + s1, e1p[k]);
            const double s2 = __builtin_fma(kD, e2p[k] + e2, s1p[k]);
            L[k] = kK * s2;
            D[k] = -e2 * kIK;
            sp[k] = s[k];
            ep[k] = e[k];
            e1p[k] = e1;
            s1p[k] = s1;
            e2p[k] = e2;
        }
        double a[2] = {L[0], L[2]}, hl[2] = {L[1], L[3]}, lh[2] = {D[0], D[2]}, hhv[2] = {D[1], D[3]};
        fwd_row(a, hl);
        fwd_row(lh, hhv);
        ll[0] = a[0];
        ll[1] = a[1];
        uint8_t *so = (uint8_t *)(sb_lds + (kSb1Dw + 1) * buf);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int p = drop1 ? 3 * kSb1B : 3 * (2 * (lane - 3) + k) + ch;   // others: the dummy dword
            const int dsb = drop1 ? 0 : kSb1B;
            so[p] = (uint8_t)(uint32_t)(qk<QP2>(lh[k], Q, qsh) + 128);
            so[p + dsb] = (uint8_t)(uint32_t)(qk<QP2>(hl[k], Q, qsh) + 128);
            so[p + 2 * dsb] = (uint8_t)(uint32_t)(qk<QP2>(hhv[k], Q, qsh) + 128);
        }
        __syncthreads();
        const uint32_t base = (uint32_t)off1_lh + 3 * (uint32_t)(m * hw + strip * kV1);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int i = t + r * kNT;
            const int ic = min(i, kSb1Dw - 1);
            const int sub = ic / (kSb1B / 4), d = ic - (kSb1B / 4) * sub;
            const uint32_t ok = row_own && i < kSb1Dw && 4 * d < row_b1 ? 0u : kDrop;
            __builtin_amdgcn_raw_buffer_store_b32(sb_lds[(kSb1Dw + 1) * buf + ic], rs_pk,
                                                  (base + sub * sstep1 + 4 * d) | ok, 0, 0);
        }
        buf ^= 1;
    };

    double ll_e[2], ll_o[2];
    // level-1 warm-up: input pairs 2 M0 - 6 .. 2 M0 - 3 (no LL1 row yet)
    for (int u = 0; u < 4; ++u) l1_step(0, false, ll_e);
    for (int k = M0 - 2; k <= M1 + 1; ++k) {
        // LL1 rows 2k, 2k + 1 (owned: 2 M0 <= row < 2 M1)
        l1_step(2 * k, k >= M0 && k < M1, ll_e);
        l1_step(2 * k + 1, k >= M0 && k < M1, ll_o);
        double L2[2], D2[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const double e1 = __builtin_fma(kA, tp[c] + ll_e[c], fp[c]);    // e1_{k-1}
            const double s1 = __builtin_fma(kB, f1p[c] + e1, tp[c]);        // s1_{k-1}
            const double e2 = __builtin_fma(kG, t1p[c] + s1, f1p[c]);       // e2_{k-2}
            const double s2 = __builtin_fma(kD, f2p[c] + e2, t1p[c]);       // s2_{k-2}
            L2[c] = kK * s2;
            D2[c] = -e2 * kIK;
            tp[c] = ll_e[c];
            fp[c] = ll_o[c];
            f1p[c] = e1;
            t1p[c] = s1;
            f2p[c] = e2;
        }
        fwd_row1(L2[0], L2[1]);   // (LL2, HL2)
        fwd_row1(D2[0], D2[1]);   // (LH2, HH2)
        const int m2 = k - 2;
        const uint32_t d2 = m2 >= M0 ? drop2 : kDrop;          // level-2 row m2 once the pipeline is full
        const uint32_t o2 = (uint32_t)(m2 * hw2 + j2);
        if (LAST2)
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(uint32_t)(qk<QP2>(L2[0], Q, qsh) + 128), rs_pk,
                                                  ((uint32_t)ll_off + 2 * (3 * o2 + ch)) | d2, 0, 0);
        else
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(U32x2, L2[0]), rs_ll, (8 * o2) | d2, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(uint32_t)(qk<QP2>(D2[0], Q, qsh) + 128), rs_pk,
                                             ((uint32_t)off2_lh + 3 * o2 + ch) | d2, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(uint32_t)(qk<QP2>(L2[1], Q, qsh) + 128), rs_pk,
                                             ((uint32_t)off2_hl + 3 * o2 + ch) | d2, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(uint32_t)(qk<QP2>(D2[1], Q, qsh) + 128), rs_pk,
                                             ((uint32_t)off2_hh + 3 * o2 + ch) | d2, 0, 0);
    }
}

// ---- levels 2 and 1 in one launch (inverse) ---------------------------------
// The mirror of lift_fwd12_kernel: a lane's level-2 pair, inverted across the
// wave (one pair per lane), is the lane's two LL1 columns; a level-2 column
// pipeline turns each level-2 row into two LL1 rows, each of which is one step
// of the level-1 inverse (two pairs per lane) down to RGB.  LL1 never reaches
// HBM.  Exact lanes 3..60 (level 2 leaves lanes 2..61, level 1 narrows by
// one); a band of level-2 rows [B0, B1) owns RGB rows [4 B0, 4 B1) and runs
// B1 - B0 + 6 level-2 steps.  Planes that halve evenly (LL1 = 2x LL2 both
// ways).
constexpr int kRgbRow12 = 2 * kV1 * 3;                    // bytes of one owned RGB row (232 pixels)
constexpr int kRgbDw12 = 2 * kRgbRow12 / 4;               // both rows, dwords (348)

// inverse lifting of one row when each lane holds one pair (cA, cD) -> (x[2j], x[2j+1])
__device__ __forceinline__ void inv_row1(double &a, double &d)
{
    double s = a * kIK, e = -d * kK;
    s = __builtin_fma(-kD, from_prev(e) + e, s);
    e = __builtin_fma(-kG, s + from_next(s), e);
    s = __builtin_fma(-kB, from_prev(e) + e, s);
    e = __builtin_fma(-kA, s + from_next(s), e);
    a = s;
    d = e;
}

// TO_RGB = false: the same pair of levels l + 1, l down to level l - 1's
// float64 LL plane (2 h1 x 2 w1; C3's levels 4 + 3), 16-byte stores
template <bool FROM_PACKED2, bool TO_RGB = true>
__global__ __launch_bounds__(kNT) void lift_inv21_kernel(const uint8_t *__restrict__ packed, long long packed_stride,
                                                         long long ll_off, long long off2_lh, long long off2_hl,
                                                         long long off2_hh, long long off1_lh, long long off1_hl,
                                                         long long off1_hh, const double *__restrict__ in,
                                                         long long plane_stride, double *__restrict__ out,
                                                         uint8_t *__restrict__ rgb_out, long long rgb_stride, int h2,
                                                         int w2, int h1, int w1, int Q, int n_strips, int n_bands,
                                                         int brows)
{
    __shared__ double xch[TO_RGB ? 3 * kOut * 64 : 1];
    __shared__ uint32_t rgb_lds[TO_RGB ? kRgbDw12 + 1 : 1];
    const int t = threadIdx.x, lane = t & 63, ch = __builtin_amdgcn_readfirstlane(t >> 6);
    int b = blockIdx.x;
    const int strip = b % n_strips;
    b /= n_strips;
    const int band = b % n_bands;
    const long long frame = b / n_bands;
    const long long plane = frame * 3 + ch;
    const int j2o = strip * kV2 - 3 + lane;                    // the lane's level-2 column (unwrapped)
    const int j2 = wrap(j2o, w2);
    const int jl = 2 * j2;                                     // its level-1 columns jl, jl + 1 (even w1)
    const bool own = lane >= 3 && lane < 3 + kV2 && j2o < w2;
    const int B0 = band * brows, B1 = min(B0 + brows, h2);
    const int ow = 2 * w1;                                     // RGB width
    const uint8_t *pk = packed + frame * packed_stride;
    const double *src = FROM_PACKED2 ? nullptr : in + plane * plane_stride;
    const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(
        TO_RGB ? (void *)(rgb_out + frame * rgb_stride) : (void *)(out + plane * plane_stride), 0,
        TO_RGB ? (int)rgb_stride : (int)((long long)ow * (2 * h1) * 8), 0x00020000);
    const int row_b = 3 * (ow - 2 * strip * kV1);              // the strip's bytes in an RGB row

    // prefetch: level-2 row q2f (LL2 and its three detail bytes), and the level-1
    // detail bytes of the two LL1 rows the next step produces
    int q2f = wrap(B0 - 3, h2);
    double nA2;
    int n2[3], n1[2][3][2];
    auto load2 = [&]() {
        const long long idx = (long long)q2f * w2 + j2;
        nA2 = FROM_PACKED2 ? dequant((int16_t)*(const uint16_t *)(pk + ll_off + 2 * (3 * idx + ch)), Q)
                           : src[(long long)q2f * w2 + j2];
        n2[0] = pk[off2_hl + 3 * idx + ch];
        n2[1] = pk[off2_lh + 3 * idx + ch];
        n2[2] = pk[off2_hh + 3 * idx + ch];
        q2f = q2f + 1 == h2 ? 0 : q2f + 1;
    };
    auto load1 = [&](int m2) {   // LL1 rows 2 m2, 2 m2 + 1 (wrapped)
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const long long row = (long long)wrap(2 * m2 + r, h1) * w1;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const long long idx = row + jl + k;
                n1[r][0][k] = pk[off1_hl + 3 * idx + ch];
                n1[r][1][k] = pk[off1_lh + 3 * idx + ch];
                n1[r][2][k] = pk[off1_hh + 3 * idx + ch];
            }
        }
    };
    // level-2 column pipelines (the lane's two LL1 columns), level-1 ones (its four output columns)
    double ep2[2], s1p2[2], e1pp2[2], s2pp2[2], ep[4], s1p[4], e1pp[4], s2pp[4];
#pragma unroll
    for (int k = 0; k < 2; ++k) ep2[k] = s1p2[k] = e1pp2[k] = s2pp2[k] = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) ep[k] = s1p[k] = e1pp[k] = s2pp[k] = 0.0;

    // one level-2 step: the prefetched row -> the lane's LL1 values of rows 2(q2-2), 2(q2-2)+1
    auto l2_step = [&](double (&r0)[2], double (&r1)[2]) {
        double a = nA2, hl = dequant((int16_t)n2[0], Q), lh = dequant((int16_t)n2[1], Q),
               hh = dequant((int16_t)n2[2], Q);
        load2();
        asm volatile("" ::: "memory");
        inv_row1(a, hl);   // 'a' row: LL1 columns jl, jl + 1 of the vertical low band
        inv_row1(lh, hh);  // 'd' row
        const double A[2] = {a, hl}, Dd[2] = {lh, hh};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const double s = A[k] * kIK, e = -Dd[k] * kK;
            const double s1 = __builtin_fma(-kD, ep2[k] + e, s);
            const double e1 = __builtin_fma(-kG, s1p2[k] + s1, ep2[k]);
            const double s2 = __builtin_fma(-kB, e1pp2[k] + e1, s1p2[k]);
            const double e2 = __builtin_fma(-kA, s2pp2[k] + s2, e1pp2[k]);
            r0[k] = s2pp2[k];
            r1[k] = e2;
            ep2[k] = e;
            s1p2[k] = s1;
            e1pp2[k] = e1;
            s2pp2[k] = s2;
        }
    };
    // one level-1 step: LL1 row q (the lane's two values, the details in n1[r]) ->
    // RGB rows 2(q-2), 2(q-2)+1, stored when `emit`
    auto l1_step = [&](const double (&x)[2], const int (&db)[3][2], int q, bool emit) {
        double a[2] = {x[0], x[1]}, hl[2], lh[2], hhv[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            hl[k] = dequant((int16_t)db[0][k], Q);
            lh[k] = dequant((int16_t)db[1][k], Q);
            hhv[k] = dequant((int16_t)db[2][k], Q);
        }
        inv_row(a, hl);
        inv_row(lh, hhv);
        const double A[4] = {a[0], hl[0], a[1], hl[1]}, Dd[4] = {lh[0], hhv[0], lh[1], hhv[1]};
        double o0[4], o1[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double s = A[k] * kIK, e = -Dd[k] * kK;
            const double s1 = __builtin_fma(-kD, ep[k] + e, s);
            const double e1 = __builtin_fma(-kG, s1p[k] + s1, ep[k]);
            const double s2 = __builtin_fma(-kB, e1pp[k] + e1, s1p[k]);
            const double e2 = __builtin_fma(-kA, s2pp[k] + s2, e1pp[k]);
            o0[k] = s2pp[k];
            o1[k] = e2;
            ep[k] = e;
            s1p[k] = s1;
            e1pp[k] = e1;
            s2pp[k] = s2;
        }
        if constexpr (!TO_RGB) {   // two 16-byte stores per output row (a pair's columns: in or out together)
            const int r0 = 2 * (q - 2);
#pragma unroll
            for (int rr = 0; rr < 2; ++rr)
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const double *v = rr ? o1 : o0;
                    const uint32_t ok = emit && own ? 0u : kDrop;
                    const uint32_t o = 8 * (uint32_t)((r0 + rr) * ow + 2 * jl + 2 * k);
                    __builtin_amdgcn_raw_buffer_store_b128(pack2(v[2 * k], v[2 * k + 1]), rs_out, o | ok, 0, 0);
                }
        } else {
        double *xo = xch + ch * kOut * 64;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            xo[k * 64 + lane] = o0[k];
            xo[(4 + k) * 64 + lane] = o1[k];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kOut; ++k) {
            const int rr = k / 4, c = k % 4;
            const double Y = xch[k * 64 + lane], Co = xch[(kOut + k) * 64 + lane], Cg = xch[(2 * kOut + k) * 64 + lane];
            const double v = ch == 0 ? Y + Co - Cg : (ch == 1 ? Y + Cg : Y - Co - Cg);
            const uint8_t u = (uint8_t)(v < 0.0 ? 0.0 : (v > 255.0 ? 255.0 : v));
            const int pos = own ? kRgbRow12 * rr + 3 * (4 * (lane - 3) + c) + ch : kRgbDw12 * 4;   // others: dummy
            ((uint8_t *)rgb_lds)[pos] = u;
        }
        __syncthreads();
        const int r0 = 2 * (q - 2);
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2) {
            const int i = t + i2 * kNT;
            const int ic = min(i, kRgbDw12 - 1);
            const int row = ic >= kRgbRow12 / 4, d = ic - (kRgbRow12 / 4) * row;
            const uint32_t o = 3 * (uint32_t)((r0 + row) * ow + 2 * strip * kV1) + 4 * d;
            const uint32_t ok = emit && i < kRgbDw12 && 4 * d < row_b ? 0u : kDrop;
            __builtin_amdgcn_raw_buffer_store_b32(rgb_lds[ic], rs_out, o | ok, 0, 0);
        }
        }
    };

    load2();
    // level-2 warm-up: rows B0 - 3 .. B0 (no LL1 row yet)
    double r0[2], r1[2];
    for (int u = 0; u < 4; ++u) l2_step(r0, r1);
    load1(B0 - 1);
    for (int q2 = B0 + 1; q2 <= B1 + 2; ++q2) {
        const int m2 = q2 - 2;                                 // this step's LL1 rows 2 m2, 2 m2 + 1
        l2_step(r0, r1);
        int cur[2][3][2];
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int u = 0; u < 3; ++u)
#pragma unroll
                for (int k = 0; k < 2; ++k) cur[r][u][k] = n1[r][u][k];
        load1(m2 + 1);                                         // the next step's level-1 details
        asm volatile("" ::: "memory");
        // level-1 rows 2 m2, 2 m2 + 1: RGB row pairs 2 m2 - 2, 2 m2 - 1 (owned from 2 B0 on)
        l1_step(r0, cur[0], 2 * m2, m2 >= B0 + 1);
        l1_step(r1, cur[1], 2 * m2 + 1, m2 >= B0 + 1);
    }
}

}  // namespace lift
