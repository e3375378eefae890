// vcf_pocketfft_blue.h -- the block sizes pocketfft_r plans with Bluestein
// (the first is 191; 67 of the lengths up to 600): its fftblue<T0> over a
// complex cfftp<T0> of length n2 = good_size_cmplx(2n - 1), in pocketfft's
// exact operation order, with the length known only at run time.
//
//   cfftp: factors 8s, then 4s, then one 2 swapped to the front, then odd
//     factors; good_size_cmplx lengths are 11-smooth, so only the hard-coded
//     pass2/3/4/5/7/8/11 occur (never the generic passg);
//   fftblue::fft<fwd>: a_k = c_k (*) bk_k, zero-pad to n2, forward cfftp,
//     pointwise (*) bkf, backward cfftp, (*) bk_k, * fct;
//   fftblue::exec_r: real input as complex (r2hc, the forward real FFT) or
//     the halfcomplex input mirrored into a Hermitian array (backward).
// bk, bkf and the cfftp twiddles are built on the host (vcf_dct_any.hip
// rt_fill) by the same code: every function here is __host__ __device__, so
// the host's bkf FFT is the one the GPU would compute.
//
// The arrays are a thread's slices of global scratch, as in
// vcf_pocketfft_rt.h: complex element i of thread t sits at base[(2i) *
// stride + t] (re) and base[(2i + 1) * stride + t] (im), so a wave whose
// threads run the same length touches consecutive addresses at every step.
// Checked bit for bit against oracle/vcf_dct_general_oracle.cpp (itself
// pinned to scipy 1.7.1's pocketfft at every Bluestein length <= 600).
// Build with -ffp-contract=off.
// Restates pocketfft (BSD-3-Clause, Copyright (C) 2010-2019 Max-Planck-Society);
// license text in THIRD_PARTY_NOTICES.md.
#pragma once
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define VCF_HD __host__ __device__ __forceinline__
#else   // g++ build of the CPU harness (tests/cpu/blue_harness.cpp)
#define VCF_HD inline
#endif

#include <cstddef>
#include <vector>

#include "vcf_sincos.h"

namespace vcf {
namespace pfft {

template <typename T>
struct Cx {
    T r, i;
};

template <typename T> VCF_HD Cx<T> cx_add(Cx<T> a, Cx<T> b) { return {a.r + b.r, a.i + b.i}; }
template <typename T> VCF_HD Cx<T> cx_sub(Cx<T> a, Cx<T> b) { return {a.r - b.r, a.i - b.i}; }
template <typename T> VCF_HD Cx<T> cx_scale(Cx<T> a, T f) { return {a.r * f, a.i * f}; }
// special_mul<fwd>: a * conj(w) forward, a * w backward
template <bool FWD, typename T> VCF_HD Cx<T> cx_spec(Cx<T> a, Cx<T> w)
{
    return FWD ? Cx<T>{a.r * w.r + a.i * w.i, a.i * w.r - a.r * w.i}
               : Cx<T>{a.r * w.r - a.i * w.i, a.r * w.i + a.i * w.r};
}
template <bool FWD, typename T> VCF_HD Cx<T> cx_rot90(Cx<T> a)
{
    return FWD ? Cx<T>{a.i, -a.r} : Cx<T>{-a.i, a.r};
}
template <bool FWD, typename T> VCF_HD Cx<T> cx_rot45(Cx<T> a)
{
    const T h = T(0.707106781186547524400844362104849L);
    return FWD ? Cx<T>{h * (a.r + a.i), h * (a.i - a.r)} : Cx<T>{h * (a.r - a.i), h * (a.i + a.r)};
}
template <bool FWD, typename T> VCF_HD Cx<T> cx_rot135(Cx<T> a)
{
    const T h = T(0.707106781186547524400844362104849L);
    return FWD ? Cx<T>{h * (a.i - a.r), h * (-a.r - a.i)} : Cx<T>{h * (-a.r - a.i), h * (a.r - a.i)};
}

// a complex array in strided scratch (stride 1 on the host)
template <typename T>
struct CLine {
    T *p;
    int stride;
    VCF_HD Cx<T> get(size_t i) const { return {p[2 * i * (size_t)stride], p[(2 * i + 1) * (size_t)stride]}; }
    VCF_HD void set(size_t i, Cx<T> v) const
    {
        p[2 * i * (size_t)stride] = v.r;
        p[(2 * i + 1) * (size_t)stride] = v.i;
    }
    // the interleaved real view (pocketfft's reinterpret_cast<T *>)
    VCF_HD T &re(size_t q) const { return p[q * (size_t)stride]; }
};

constexpr int kCfMaxFactors = 24;

// cfftp factors of n2 and their twiddle offsets (in reals) into the plan memory
struct CfPlan {
    int n, nf;
    int fct[kCfMaxFactors], tw[kCfMaxFactors];
};

// cfftp<T0>::factorize
inline void cf_factorize(int n, CfPlan &P)
{
    P.n = n;
    P.nf = 0;
    if (n == 1) return;
    int l = n;
    while ((l & 7) == 0) { P.fct[P.nf++] = 8; l >>= 3; }
    while ((l & 3) == 0) { P.fct[P.nf++] = 4; l >>= 2; }
    if ((l & 1) == 0) {
        l >>= 1;
        P.fct[P.nf++] = 2;
        const int t = P.fct[0]; P.fct[0] = P.fct[P.nf - 1]; P.fct[P.nf - 1] = t;
    }
    for (int d = 3; d * d <= l; d += 2)
        while (l % d == 0) { P.fct[P.nf++] = d; l /= d; }
    if (l > 1) P.fct[P.nf++] = l;
}

template <typename T>
struct RtCfft {
    const T *mem;   // twiddles (re, im pairs)

    VCF_HD Cx<T> twd(const T *wa, size_t ido, size_t x, size_t i) const
    {
        const size_t o = 2 * (i - 1 + x * (ido - 1));
        return {wa[o], wa[o + 1]};
    }

    template <bool FWD>
    VCF_HD void pass2(size_t ido, size_t l1, CLine<T> cc, CLine<T> ch, const T *wa) const
    {
        for (size_t k = 0; k < l1; ++k)
            for (size_t i = 0; i < ido; ++i) {
                const Cx<T> a = cc.get(i + ido * (0 + 2 * k)), b = cc.get(i + ido * (1 + 2 * k));
                ch.set(i + ido * (k + l1 * 0), cx_add(a, b));
                ch.set(i + ido * (k + l1 * 1), i == 0 ? cx_sub(a, b) : cx_spec<FWD>(cx_sub(a, b), twd(wa, ido, 0, i)));
            }
    }

    template <bool FWD>
    VCF_HD void pass3(size_t ido, size_t l1, CLine<T> cc, CLine<T> ch, const T *wa) const
    {
        const T tw1r = T(-0.5), tw1i = (FWD ? -1 : 1) * T(0.8660254037844386467637231707529362L);
        for (size_t k = 0; k < l1; ++k)
            for (size_t i = 0; i < ido; ++i) {
                const Cx<T> t0 = cc.get(i + ido * (0 + 3 * k)), c1 = cc.get(i + ido * (1 + 3 * k)),
                            c2 = cc.get(i + ido * (2 + 3 * k));
                const Cx<T> t1 = cx_add(c1, c2), t2 = cx_sub(c1, c2);
                ch.set(i + ido * k, cx_add(t0, t1));
                const Cx<T> ca = cx_add(t0, cx_scale(t1, tw1r));
                const Cx<T> cb{-(t2.i * tw1i), t2.r * tw1i};
                if (i == 0) {
                    ch.set(ido * (k + l1), cx_add(ca, cb));
                    ch.set(ido * (k + 2 * l1), cx_sub(ca, cb));
                } else {
                    ch.set(i + ido * (k + l1), cx_spec<FWD>(cx_add(ca, cb), twd(wa, ido, 0, i)));
                    ch.set(i + ido * (k + 2 * l1), cx_spec<FWD>(cx_sub(ca, cb), twd(wa, ido, 1, i)));
                }
            }
    }

    template <bool FWD>
    VCF_HD void pass4(size_t ido, size_t l1, CLine<T> cc, CLine<T> ch, const T *wa) const
    {
        for (size_t k = 0; k < l1; ++k)
            for (size_t i = 0; i < ido; ++i) {
                const Cx<T> c0 = cc.get(i + ido * (0 + 4 * k)), c1 = cc.get(i + ido * (1 + 4 * k)),
                            c2 = cc.get(i + ido * (2 + 4 * k)), c3 = cc.get(i + ido * (3 + 4 * k));
                const Cx<T> t2 = cx_add(c0, c2), t1 = cx_sub(c0, c2);
                const Cx<T> t3 = cx_add(c1, c3), t4 = cx_rot90<FWD>(cx_sub(c1, c3));
                auto CH = [&](size_t u) { return i + ido * (k + l1 * u); };
                if (i == 0) {
                    ch.set(CH(0), cx_add(t2, t3));
                    ch.set(CH(2), cx_sub(t2, t3));
                    ch.set(CH(1), cx_add(t1, t4));
                    ch.set(CH(3), cx_sub(t1, t4));
                } else {
                    ch.set(CH(0), cx_add(t2, t3));
                    ch.set(CH(1), cx_spec<FWD>(cx_add(t1, t4), twd(wa, ido, 0, i)));
                    ch.set(CH(2), cx_spec<FWD>(cx_sub(t2, t3), twd(wa, ido, 1, i)));
                    ch.set(CH(3), cx_spec<FWD>(cx_sub(t1, t4), twd(wa, ido, 2, i)));
                }
            }
    }

    template <bool FWD>
    VCF_HD void pass8(size_t ido, size_t l1, CLine<T> cc, CLine<T> ch, const T *wa) const
    {
        for (size_t k = 0; k < l1; ++k)
            for (size_t i = 0; i < ido; ++i) {
                auto CC = [&](size_t j) { return cc.get(i + ido * (j + 8 * k)); };
                auto CH = [&](size_t u) { return i + ido * (k + l1 * u); };
                Cx<T> a1 = cx_add(CC(1), CC(5)), a5 = cx_sub(CC(1), CC(5));
                Cx<T> a3 = cx_add(CC(3), CC(7)), a7 = cx_sub(CC(3), CC(7));
                { const Cx<T> t = a1; a1 = cx_add(t, a3); a3 = cx_sub(t, a3); }
                a3 = cx_rot90<FWD>(a3);
                a7 = cx_rot90<FWD>(a7);
                { const Cx<T> t = a5; a5 = cx_add(t, a7); a7 = cx_sub(t, a7); }
                a5 = cx_rot45<FWD>(a5);
                a7 = cx_rot135<FWD>(a7);
                Cx<T> a0 = cx_add(CC(0), CC(4)), a4 = cx_sub(CC(0), CC(4));
                Cx<T> a2 = cx_add(CC(2), CC(6)), a6 = cx_sub(CC(2), CC(6));
                if (i == 0) {
                    const Cx<T> s02 = cx_add(a0, a2), d02 = cx_sub(a0, a2);
                    ch.set(CH(0), cx_add(s02, a1));
                    ch.set(CH(4), cx_sub(s02, a1));
                    ch.set(CH(2), cx_add(d02, a3));
                    ch.set(CH(6), cx_sub(d02, a3));
                    a6 = cx_rot90<FWD>(a6);
                    const Cx<T> s46 = cx_add(a4, a6), d46 = cx_sub(a4, a6);
                    ch.set(CH(1), cx_add(s46, a5));
                    ch.set(CH(5), cx_sub(s46, a5));
                    ch.set(CH(3), cx_add(d46, a7));
                    ch.set(CH(7), cx_sub(d46, a7));
                } else {
                    { const Cx<T> t = a0; a0 = cx_add(t, a2); a2 = cx_sub(t, a2); }
                    ch.set(CH(0), cx_add(a0, a1));
                    ch.set(CH(4), cx_spec<FWD>(cx_sub(a0, a1), twd(wa, ido, 3, i)));
                    ch.set(CH(2), cx_spec<FWD>(cx_add(a2, a3), twd(wa, ido, 1, i)));
                    ch.set(CH(6), cx_spec<FWD>(cx_sub(a2, a3), twd(wa, ido, 5, i)));
                    a6 = cx_rot90<FWD>(a6);
                    { const Cx<T> t = a4; a4 = cx_add(t, a6); a6 = cx_sub(t, a6); }
                    ch.set(CH(1), cx_spec<FWD>(cx_add(a4, a5), twd(wa, ido, 0, i)));
                    ch.set(CH(5), cx_spec<FWD>(cx_sub(a4, a5), twd(wa, ido, 4, i)));
                    ch.set(CH(3), cx_spec<FWD>(cx_add(a6, a7), twd(wa, ido, 2, i)));
                    ch.set(CH(7), cx_spec<FWD>(cx_sub(a6, a7), twd(wa, ido, 6, i)));
                }
            }
    }

    // pass5 / pass7 / pass11: the output pair (u, P - u) sums x_j = cos(2 pi
    // u j / P) (twr[m], m the folded multiple) times the PM sums and y_j =
    // +-sin times the PM differences, left to right, as pocketfft's
    // hard-coded PARTSTEP macros do
    template <bool FWD, int P>
    VCF_HD void passp(size_t ido, size_t l1, CLine<T> cc, CLine<T> ch, const T *wa, const T *twr,
                      const T *twi0) const
    {
        constexpr int H = (P - 1) / 2;
        T twi[H + 1];
        for (int m = 1; m <= H; ++m) twi[m] = (FWD ? -1 : 1) * twi0[m];
        for (size_t k = 0; k < l1; ++k)
            for (size_t i = 0; i < ido; ++i) {
                Cx<T> t[P + 1];
                t[1] = cc.get(i + ido * (0 + P * k));
                for (int j = 1; j <= H; ++j) {
                    const Cx<T> a = cc.get(i + ido * (j + P * k)), b = cc.get(i + ido * ((P - j) + P * k));
                    t[j + 1] = cx_add(a, b);
                    t[P + 1 - j] = cx_sub(a, b);
                }
                Cx<T> s0 = t[1];
                for (int j = 1; j <= H; ++j) s0.r = s0.r + t[j + 1].r;
                for (int j = 1; j <= H; ++j) s0.i = s0.i + t[j + 1].i;
                ch.set(i + ido * k, s0);
                for (int u = 1; u <= H; ++u) {
                    Cx<T> ca = t[1];
                    T cbi = T(0), cbr = T(0);
                    for (int j = 1; j <= H; ++j) {
                        const int mm = (u * j) % P, m = mm <= H ? mm : P - mm;
                        const T x = twr[m], y = mm <= H ? twi[m] : -twi[m];
                        ca.r = ca.r + x * t[j + 1].r;
                        ca.i = ca.i + x * t[j + 1].i;
                        if (j == 1) { cbi = y * t[P + 1 - j].r; cbr = y * t[P + 1 - j].i; }
                        else { cbi = cbi + y * t[P + 1 - j].r; cbr = cbr + y * t[P + 1 - j].i; }
                    }
                    const Cx<T> cb{-cbr, cbi};
                    if (i == 0) {
                        ch.set(ido * (k + l1 * u), cx_add(ca, cb));
                        ch.set(ido * (k + l1 * (P - u)), cx_sub(ca, cb));
                    } else {
                        ch.set(i + ido * (k + l1 * u), cx_spec<FWD>(cx_add(ca, cb), twd(wa, ido, u - 1, i)));
                        ch.set(i + ido * (k + l1 * (P - u)), cx_spec<FWD>(cx_sub(ca, cb), twd(wa, ido, P - u - 1, i)));
                    }
                }
            }
    }

    // cfftp::pass_all<fwd>(c, fct) with fct == 1 (all fftblue uses); ch is scratch
    template <bool FWD>
    VCF_HD void pass_all(CLine<T> c, CLine<T> ch, const CfPlan &P) const
    {
        const T tw5r[3] = {T(0), T(0.3090169943749474241022934171828191L), T(-0.8090169943749474241022934171828191L)};
        const T tw5i[3] = {T(0), T(0.9510565162951535721164393333793821L), T(0.5877852522924731291687059546390728L)};
        const T tw7r[4] = {T(0), T(0.6234898018587335305250048840042398L), T(-0.2225209339563144042889025644967948L),
                           T(-0.9009688679024191262361023195074451L)};
        const T tw7i[4] = {T(0), T(0.7818314824680298087084445266740578L), T(0.9749279121818236070181316829939312L),
                           T(0.4338837391175581204757683328483588L)};
        const T tw11r[6] = {T(0), T(0.8412535328311811688618116489193677L), T(0.4154150130018864255292741492296232L),
                            T(-0.1423148382732851404437926686163697L), T(-0.6548607339452850640569250724662936L),
                            T(-0.9594929736144973898903680570663277L)};
        const T tw11i[6] = {T(0), T(0.5406408174555975821076359543186917L), T(0.9096319953545183714117153830790285L),
                            T(0.9898214418809327323760920377767188L), T(0.7557495743542582837740358439723444L),
                            T(0.2817325568414296977114179153466169L)};
        if (P.n == 1) return;
        CLine<T> p1 = c, p2 = ch;
        size_t l1 = 1;
        const size_t n = (size_t)P.n;
        for (int k = 0; k < P.nf; ++k) {
            const size_t ip = (size_t)P.fct[k], ido = n / (l1 * ip);
            const T *tw = mem + P.tw[k];
            if (ip == 4) pass4<FWD>(ido, l1, p1, p2, tw);
            else if (ip == 8) pass8<FWD>(ido, l1, p1, p2, tw);
            else if (ip == 2) pass2<FWD>(ido, l1, p1, p2, tw);
            else if (ip == 3) pass3<FWD>(ido, l1, p1, p2, tw);
            else if (ip == 5) passp<FWD, 5>(ido, l1, p1, p2, tw, tw5r, tw5i);
            else if (ip == 7) passp<FWD, 7>(ido, l1, p1, p2, tw, tw7r, tw7i);
            else passp<FWD, 11>(ido, l1, p1, p2, tw, tw11r, tw11i);   // (the plan holds 11-smooth lengths only)
            const CLine<T> t = p1; p1 = p2; p2 = t;
            l1 *= ip;
        }
        if (p1.p != c.p)
            for (size_t i = 0; i < n; ++i) c.set(i, p1.get(i));
    }
};

// the Bluestein plan of one length n (offsets in reals into the plan memory)
struct BluePlan {
    int n, n2;
    int bk, bkf;   // bk: n complex chirp values; bkf: n2/2 + 1 of its transform
    CfPlan cf;
};

// fftblue<T0>::fft<fwd>(c, fct) on the complex array c of length n; akf and ch
// are n2-element scratch
template <bool FWD, typename T>
VCF_HD void blue_fft(const T *mem, const BluePlan &B, CLine<T> c, CLine<T> akf, CLine<T> ch, T fct)
{
    const RtCfft<T> F{mem};
    const size_t n = (size_t)B.n, n2 = (size_t)B.n2;
    auto bk = [&](size_t m) { return Cx<T>{mem[B.bk + 2 * m], mem[B.bk + 2 * m + 1]}; };
    auto bkf = [&](size_t m) { return Cx<T>{mem[B.bkf + 2 * m], mem[B.bkf + 2 * m + 1]}; };
    for (size_t m = 0; m < n; ++m) akf.set(m, cx_spec<FWD>(c.get(m), bk(m)));
    const Cx<T> zero = cx_scale(akf.get(0), T(0));
    for (size_t m = n; m < n2; ++m) akf.set(m, zero);
    F.template pass_all<true>(akf, ch, B.cf);
    akf.set(0, cx_spec<!FWD>(akf.get(0), bkf(0)));
    for (size_t m = 1; m < (n2 + 1) / 2; ++m) {
        akf.set(m, cx_spec<!FWD>(akf.get(m), bkf(m)));
        akf.set(n2 - m, cx_spec<!FWD>(akf.get(n2 - m), bkf(m)));
    }
    if ((n2 & 1) == 0) akf.set(n2 / 2, cx_spec<!FWD>(akf.get(n2 / 2), bkf(n2 / 2)));
    F.template pass_all<false>(akf, ch, B.cf);
    for (size_t m = 0; m < n; ++m) c.set(m, cx_scale(cx_spec<FWD>(akf.get(m), bk(m)), fct));
}

// fftblue<T0>::exec_r(c, fct, fwd) on the real array c (any accessor with
// operator[]); tmp is n-element, akf and ch n2-element complex scratch
template <typename T, typename A>
VCF_HD void blue_exec_r(const T *mem, const BluePlan &B, A c, CLine<T> tmp, CLine<T> akf, CLine<T> ch, T fct,
                        bool fwd)
{
    const size_t n = (size_t)B.n;
    if (fwd) {
        const T zero = T(0) * c[0];
        for (size_t m = 0; m < n; ++m) tmp.set(m, Cx<T>{c[m], zero});
        blue_fft<true>(mem, B, tmp, akf, ch, fct);
        c[0] = tmp.get(0).r;
        for (size_t q = 0; q + 1 < n; ++q) c[1 + q] = tmp.re(2 + q);
    } else {
        tmp.set(0, Cx<T>{c[0], c[0] * T(0)});
        for (size_t q = 0; q + 1 < n; ++q) tmp.re(2 + q) = c[1 + q];
        if ((n & 1) == 0) tmp.re(n + 1) = T(0) * c[0];
        for (size_t m = 1; 2 * m < n; ++m) {
            const Cx<T> v = tmp.get(m);
            tmp.set(n - m, Cx<T>{v.r, -v.i});
        }
        blue_fft<false>(mem, B, tmp, akf, ch, fct);
        for (size_t m = 0; m < n; ++m) c[m] = tmp.get(m).r;
    }
}

// host: fftblue<T0>(n)'s plan: cfftp(n2) factorize + comp_twiddle, the chirp
// bk from sincos_2pibyn(2n), and bkf = the forward cfftp of bk / n2
// (zero-padded, mirrored), computed by the pass code above; appended to mem
template <typename T>
inline void blue_fill(int n, int n2, BluePlan &B, std::vector<T> &mem)
{
    B.n = n;
    B.n2 = n2;
    cf_factorize(n2, B.cf);
    size_t l1 = 1;
    for (int k = 0; k < B.cf.nf; ++k) {
        const size_t ip = (size_t)B.cf.fct[k], ido = (size_t)n2 / (l1 * ip);
        B.cf.tw[k] = (int)mem.size();
        for (size_t j = 1; j < ip; ++j)
            for (size_t i = 1; i < ido; ++i) {
                T re, im;
                sincos_2pibyn<T>((size_t)n2, j * l1 * i, re, im);
                mem.push_back(re);
                mem.push_back(im);
            }
        l1 *= ip;
    }
    B.bk = (int)mem.size();
    std::vector<Cx<T>> bk((size_t)n);
    bk[0] = {T(1), T(0)};
    size_t coeff = 0;
    for (size_t m = 1; m < (size_t)n; ++m) {
        coeff += 2 * m - 1;
        if (coeff >= 2 * (size_t)n) coeff -= 2 * (size_t)n;
        sincos_2pibyn<T>(2 * (size_t)n, coeff, bk[m].r, bk[m].i);
    }
    for (const auto &v : bk) { mem.push_back(v.r); mem.push_back(v.i); }
    const size_t N2 = (size_t)n2;
    std::vector<T> tbkf(2 * N2, T(0)), scr(2 * N2);
    const CLine<T> tb{tbkf.data(), 1};
    const T xn2 = T(1) / T(N2);
    tb.set(0, cx_scale(bk[0], xn2));
    for (size_t m = 1; m < (size_t)n; ++m) {
        tb.set(m, cx_scale(bk[m], xn2));
        tb.set(N2 - m, cx_scale(bk[m], xn2));
    }
    const RtCfft<T> F{mem.data()};
    F.template pass_all<true>(tb, CLine<T>{scr.data(), 1}, B.cf);
    B.bkf = (int)mem.size();
    mem.insert(mem.end(), tbkf.begin(), tbkf.begin() + 2 * (N2 / 2 + 1));
}

#undef VCF_HD

}  // namespace pfft
}  // namespace vcf
