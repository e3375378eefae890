// vcf_pocketfft_rt.h -- run-time-length DCT-II / DCT-III in pocketfft's exact
// operation order: the block transforms for the -B sizes vcf_pocketfft.h does
// not compile in: any length pocketfft plans with rfftp, including its
// generic radfg/radbg passes for prime factors above 5, and the lengths
// pocketfft_r's cost model plans with Bluestein (vcf_pocketfft_blue.h).
//
// Same restatement as vcf_pocketfft.h (rfftp factorisation, radf/radb passes,
// copy_and_norm, T_dcst23's twiddle loops and ortho scalings), with the length
// and the factor list known only at run time: the passes loop over ido / l1
// and read their twiddles from a plan array (RtPlan offsets into `mem`).  The
// working arrays are a thread's slices of global scratch, reached through
// Line: element i of thread t sits at base[i * stride + t], so a wave whose
// threads run the same length touches consecutive addresses at every step.
// Build with -ffp-contract=off.
// Restates pocketfft (BSD-3-Clause, Copyright (C) 2010-2019 Max-Planck-Society);
// license text in THIRD_PARTY_NOTICES.md.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#include "vcf_pocketfft.h"
#include "vcf_pocketfft_blue.h"
#include "vcf_sincos.h"

#include <algorithm>
#include <cmath>
#include <vector>

// host and device: the CPU harness (tests/cpu/rt_harness.hip) runs these
// functions on the host against the oracle
#define VCF_RT_HD __host__ __device__ __forceinline__

namespace vcf {
namespace pfft {

constexpr int kRtMaxFactors = 24;

// the plan of one length: rfftp's factors and the offsets of their twiddles
// (tw: (ip-1)(ido-1) values for all but the last factor; tws: radfg/radbg's 2 ip
// values for factors above 5), T_dcst23's N twiddles, the norm factor; or,
// when blue is set, the Bluestein plan (nf = 0)
struct RtPlan {
    int n, nf;
    int fct[kRtMaxFactors], tw[kRtMaxFactors], tws[kRtMaxFactors];
    int dct_tw, norm;
    int blue;
    BluePlan bl;
};

// per-thread scratch reals of a plan: the two lines c, ch of n, and for
// Bluestein its n-element and two n2-element complex arrays
__host__ __device__ inline long long rt_line_reals(const RtPlan &P)
{
    return 2LL * P.n + (P.blue ? 2LL * P.n + 4LL * P.bl.n2 : 0);
}

template <typename T>
struct Line {
    T *p;
    int stride;
    VCF_RT_HD T &operator[](size_t i) const { return p[i * (size_t)stride]; }
};

template <typename T>
VCF_RT_HD bool same_line(const Line<T> &a, const Line<T> &b) { return a.p == b.p; }

template <typename T>
struct RtFft {
    const T *mem;       // the plan's twiddle values
    T *bw = nullptr;    // Bluestein scratch of this thread (rt_line_reals beyond c, ch)
    int bstride = 1;

    template <typename A>
    VCF_RT_HD void blue(A c, const RtPlan &P, T fct, bool fwd) const
    {
        const size_t n = (size_t)P.n, n2 = (size_t)P.bl.n2, s = (size_t)bstride;
        const CLine<T> tmp{bw, bstride}, akf{bw + 2 * n * s, bstride}, ch{bw + (2 * n + 2 * n2) * s, bstride};
        blue_exec_r(mem, P.bl, c, tmp, akf, ch, fct, fwd);
    }

    /* radfg: any odd factor ip > 5 (pocketfft rfftp::radfg); input in cc as
     * (ido, l1, ip), result back in cc as (ido, ip, l1), ch is scratch */
    template <typename A>
    VCF_RT_HD void radfg(size_t ido, size_t ip, size_t l1, A cc, A ch, const T *wa, const T *csarr) const
    {
        const size_t cdim = ip, ipph = (ip + 1) / 2, idl1 = ido * l1;
        auto CC = [&](size_t a, size_t b, size_t c) -> T & { return cc[a + ido * (b + cdim * c)]; };
        auto CH = [&](size_t a, size_t b, size_t c) -> T & { return ch[a + ido * (b + l1 * c)]; };
        auto C1 = [&](size_t a, size_t b, size_t c) -> T & { return cc[a + ido * (b + l1 * c)]; };
        auto C2 = [&](size_t a, size_t b) -> T & { return cc[a + idl1 * b]; };
        auto CH2 = [&](size_t a, size_t b) -> T & { return ch[a + idl1 * b]; };
        if (ido > 1) {
            for (size_t j = 1, jc = ip - 1; j < ipph; ++j, --jc) {
                size_t is = (j - 1) * (ido - 1), is2 = (jc - 1) * (ido - 1);
                for (size_t k = 0; k < l1; ++k) {
                    size_t idij = is, idij2 = is2;
                    for (size_t i = 1; i <= ido - 2; i += 2) {
                        T t1 = C1(i, k, j), t2 = C1(i + 1, k, j), t3 = C1(i, k, jc), t4 = C1(i + 1, k, jc);
                        T x1 = wa[idij] * t1 + wa[idij + 1] * t2, x2 = wa[idij] * t2 - wa[idij + 1] * t1,
                          x3 = wa[idij2] * t3 + wa[idij2 + 1] * t4, x4 = wa[idij2] * t4 - wa[idij2 + 1] * t3;
                        PM(C1(i, k, j), C1(i + 1, k, jc), x3, x1);
                        PM(C1(i + 1, k, j), C1(i, k, jc), x2, x4);
                        idij += 2;
                        idij2 += 2;
                    }
                }
            }
        }
        for (size_t j = 1, jc = ip - 1; j < ipph; ++j, --jc)
            for (size_t k = 0; k < l1; ++k) {
                T t1 = C1(0, k, j), t2 = C1(0, k, jc);
                PM(C1(0, k, j), C1(0, k, jc), t2, t1);
            }
        for (size_t l = 1, lc = ip - 1; l < ipph; ++l, --lc) {
            for (size_t ik = 0; ik < idl1; ++ik) {
                CH2(ik, l) = C2(ik, 0) + csarr[2 * l] * C2(ik, 1) + csarr[4 * l] * C2(ik, 2);
                CH2(ik, lc) = csarr[2 * l + 1] * C2(ik, ip - 1) + csarr[4 * l + 1] * C2(ik, ip - 2);
            }
            size_t iang = 2 * l, j = 3, jc = ip - 3;
            for (; j < ipph - 3; j += 4, jc -= 4) {
                iang += l; if (iang > ip) iang -= ip;
                T ar1 = csarr[2 * iang], ai1 = csarr[2 * iang + 1];
                iang += l; if (iang > ip) iang -= ip;
                T ar2 = csarr[2 * iang], ai2 = csarr[2 * iang + 1];
                iang += l; if (iang > ip) iang -= ip;
                T ar3 = csarr[2 * iang], ai3 = csarr[2 * iang + 1];
                iang += l; if (iang > ip) iang -= ip;
                T ar4 = csarr[2 * iang], ai4 = csarr[2 * iang + 1];
                for (size_t ik = 0; ik < idl1; ++ik) {
                    CH2(ik, l) += ar1 * C2(ik, j) + ar2 * C2(ik, j + 1) + ar3 * C2(ik, j + 2) + ar4 * C2(ik, j + 3);
                    CH2(ik, lc) += ai1 * C2(ik, jc) + ai2 * C2(ik, jc - 1) + ai3 * C2(ik, jc - 2) + ai4 * C2(ik, jc - 3);
                }
            }
            for (; j < ipph - 1; j += 2, jc -= 2) {
                iang += l; if (iang > ip) iang -= ip;
                T ar1 = csarr[2 * iang], ai1 = csarr[2 * iang + 1];
                iang += l; if (iang > ip) iang -= ip;
                T ar2 = csarr[2 * iang], ai2 = csarr[2 * iang + 1];
                for (size_t ik = 0; ik < idl1; ++ik) {
                    CH2(ik, l) += ar1 * C2(ik, j) + ar2 * C2(ik, j + 1);
                    CH2(ik, lc) += ai1 * C2(ik, jc) + ai2 * C2(ik, jc - 1);
                }
            }
            for (; j < ipph; ++j, --jc) {
                iang += l; if (iang > ip) iang -= ip;
                T ar = csarr[2 * iang], ai = csarr[2 * iang + 1];
                for (size_t ik = 0; ik < idl1; ++ik) {
                    CH2(ik, l) += ar * C2(ik, j);
                    CH2(ik, lc) += ai * C2(ik, jc);
                }
            }
        }
        for (size_t ik = 0; ik < idl1; ++ik) CH2(ik, 0) = C2(ik, 0);
        for (size_t j = 1; j < ipph; ++j)
            for (size_t ik = 0; ik < idl1; ++ik) CH2(ik, 0) += C2(ik, j);
        for (size_t k = 0; k < l1; ++k)
            for (size_t i = 0; i < ido; ++i) CC(i, 0, k) = CH(i, k, 0);
        for (size_t j = 1, jc = ip - 1; j < ipph; ++j, --jc) {
            size_t j2 = 2 * j - 1;
            for (size_t k = 0; k < l1; ++k) {
                CC(ido - 1, j2, k) = CH(0, k, j);
                CC(0, j2 + 1, k) = CH(0, k, jc);
            }
        }
        if (ido == 1) return;
        for (size_t j = 1, jc = ip - 1; j < ipph; ++j, --jc) {
            size_t j2 = 2 * j - 1;
            for (size_t k = 0; k < l1; ++k)
                for (size_t i = 1, ic = ido - i - 2; i <= ido - 2; i += 2, ic -= 2) {
                    CC(i, j2 + 1, k) = CH(i, k, j) + CH(i, k, jc);
                    CC(ic, j2, k) = CH(i, k, j) - CH(i, k, jc);
                    CC(i + 1, j2 + 1, k) = CH(i + 1, k, j) + CH(i + 1, k, jc);
                    CC(ic + 1, j2, k) = CH(i + 1, k, jc) - CH(i + 1, k, j);
                }
        }
    }

    /* radbg: any odd factor ip > 5 (pocketfft rfftp::radbg); input in cc as
     * (ido, ip, l1), result in ch as (ido, l1, ip) */
    template <typename A>
    VCF_RT_HD void radbg(size_t ido, size_t ip, size_t l1, A cc, A ch, const T *wa, const T *csarr) const
    {
        const size_t cdim = ip, ipph = (ip + 1) / 2, idl1 = ido * l1;
        auto CC = [&](size_t a, size_t b, size_t c) -> T & { return cc[a + ido * (b + cdim * c)]; };
        auto CH = [&](size_t a, size_t b, size_t c) -> T & { return ch[a + ido * (b + l1 * c)]; };
        auto C1 = [&](size_t a, size_t b, size_t c) -> T & { return cc[a + ido * (b + l1 * c)]; };
        auto C2 = [&](size_t a, size_t b) -> T & { return cc[a + idl1 * b]; };
        auto CH2 = [&](size_t a, size_t b) -> T & { return ch[a + idl1 * b]; };
        for (size_t k = 0; k < l1; ++k)
            for (size_t i = 0; i < ido; ++i) CH(i, k, 0) = CC(i, 0, k);
        for (size_t j = 1, jc = ip - 1; j < ipph; ++j, --jc) {
            size_t j2 = 2 * j - 1;
            for (size_t k = 0; k < l1; ++k) {
                CH(0, k, j) = T(2) * CC(ido - 1, j2, k);
                CH(0, k, jc) = T(2) * CC(0, j2 + 1, k);
            }
        }
        if (ido != 1) {
            for (size_t j = 1, jc = ip - 1; j < ipph; ++j, --jc) {
                size_t j2 = 2 * j - 1;
                for (size_t k = 0; k < l1; ++k)
                    for (size_t i = 1, ic = ido - i - 2; i <= ido - 2; i += 2, ic -= 2) {
                        CH(i, k, j) = CC(i, j2 + 1, k) + CC(ic, j2, k);
                        CH(i, k, jc) = CC(i, j2 + 1, k) - CC(ic, j2, k);
                        CH(i + 1, k, j) = CC(i + 1, j2 + 1, k) - CC(ic + 1, j2, k);
                        CH(i + 1, k, jc) = CC(i + 1, j2 + 1, k) + CC(ic + 1, j2, k);
                    }
            }
        }
        for (size_t l = 1, lc = ip - 1; l < ipph; ++l, --lc) {
            for (size_t ik = 0; ik < idl1; ++ik) {
                C2(ik, l) = CH2(ik, 0) + csarr[2 * l] * CH2(ik, 1) + csarr[4 * l] * CH2(ik, 2);
                C2(ik, lc) = csarr[2 * l + 1] * CH2(ik, ip - 1) + csarr[4 * l + 1] * CH2(ik, ip - 2);
            }
            size_t iang = 2 * l, j = 3, jc = ip - 3;
            for (; j < ipph - 3; j += 4, jc -= 4) {
                iang += l; if (iang > ip) iang -= ip;
                T ar1 = csarr[2 * iang], ai1 = csarr[2 * iang + 1];
                iang += l; if (iang > ip) iang -= ip;
                T ar2 = csarr[2 * iang], ai2 = csarr[2 * iang + 1];
                iang += l; if (iang > ip) iang -= ip;
                T ar3 = csarr[2 * iang], ai3 = csarr[2 * iang + 1];
                iang += l; if (iang > ip) iang -= ip;
                T ar4 = csarr[2 * iang], ai4 = csarr[2 * iang + 1];
                for (size_t ik = 0; ik < idl1; ++ik) {
                    C2(ik, l) += ar1 * CH2(ik, j) + ar2 * CH2(ik, j + 1) + ar3 * CH2(ik, j + 2) + ar4 * CH2(ik, j + 3);
                    C2(ik, lc) += ai1 * CH2(ik, jc) + ai2 * CH2(ik, jc - 1) + ai3 * CH2(ik, jc - 2) + ai4 * CH2(ik, jc - 3);
                }
            }
            for (; j < ipph - 1; j += 2, jc -= 2) {
                iang += l; if (iang > ip) iang -= ip;
                T ar1 = csarr[2 * iang], ai1 = csarr[2 * iang + 1];
                iang += l; if (iang > ip) iang -= ip;
                T ar2 = csarr[2 * iang], ai2 = csarr[2 * iang + 1];
                for (size_t ik = 0; ik < idl1; ++ik) {
                    C2(ik, l) += ar1 * CH2(ik, j) + ar2 * CH2(ik, j + 1);
                    C2(ik, lc) += ai1 * CH2(ik, jc) + ai2 * CH2(ik, jc - 1);
                }
            }
            for (; j < ipph; ++j, --jc) {
                iang += l; if (iang > ip) iang -= ip;
                T war = csarr[2 * iang], wai = csarr[2 * iang + 1];
                for (size_t ik = 0; ik < idl1; ++ik) {
                    C2(ik, l) += war * CH2(ik, j);
                    C2(ik, lc) += wai * CH2(ik, jc);
                }
            }
        }
        for (size_t j = 1; j < ipph; ++j)
            for (size_t ik = 0; ik < idl1; ++ik) CH2(ik, 0) += CH2(ik, j);
        for (size_t j = 1, jc = ip - 1; j < ipph; ++j, --jc)
            for (size_t k = 0; k < l1; ++k) {
                CH(0, k, j) = C1(0, k, j) - C1(0, k, jc);
                CH(0, k, jc) = C1(0, k, j) + C1(0, k, jc);
            }
        if (ido == 1) return;
        for (size_t j = 1, jc = ip - 1; j < ipph; ++j, --jc)
            for (size_t k = 0; k < l1; ++k)
                for (size_t i = 1; i <= ido - 2; i += 2) {
                    CH(i, k, j) = C1(i, k, j) - C1(i + 1, k, jc);
                    CH(i, k, jc) = C1(i, k, j) + C1(i + 1, k, jc);
                    CH(i + 1, k, j) = C1(i + 1, k, j) + C1(i, k, jc);
                    CH(i + 1, k, jc) = C1(i + 1, k, j) - C1(i, k, jc);
                }
        for (size_t j = 1; j < ip; ++j) {
            size_t is = (j - 1) * (ido - 1);
            for (size_t k = 0; k < l1; ++k) {
                size_t idij = is;
                for (size_t i = 1; i <= ido - 2; i += 2) {
                    T t1 = CH(i, k, j), t2 = CH(i + 1, k, j);
                    CH(i, k, j) = wa[idij] * t1 - wa[idij + 1] * t2;
                    CH(i + 1, k, j) = wa[idij] * t2 + wa[idij + 1] * t1;
                    idij += 2;
                }
            }
        }
    }

    template <typename A>
    VCF_RT_HD void radf2(size_t ido, size_t l1, A cc, A ch, const T *wa) const
    {
        auto WA = [&](size_t x, size_t i) { return wa[i + x * (ido - 1)]; };
        auto CC = [&](size_t a, size_t b, size_t c) -> T & { return cc[a + ido * (b + l1 * c)]; };
        auto CH = [&](size_t a, size_t b, size_t c) -> T & { return ch[a + ido * (b + 2 * c)]; };
        for (size_t k = 0; k < l1; k++) PM(CH(0, 0, k), CH(ido - 1, 1, k), CC(0, k, 0), CC(0, k, 1));
        if ((ido & 1) == 0)
            for (size_t k = 0; k < l1; k++) {
                CH(0, 1, k) = -CC(ido - 1, k, 1);
                CH(ido - 1, 0, k) = CC(ido - 1, k, 0);
            }
        if (ido <= 2) return;
        for (size_t k = 0; k < l1; k++)
            for (size_t i = 2; i < ido; i += 2) {
                size_t ic = ido - i;
                T tr2, ti2;
                MULPM(tr2, ti2, WA(0, i - 2), WA(0, i - 1), CC(i - 1, k, 1), CC(i, k, 1));
                PM(CH(i - 1, 0, k), CH(ic - 1, 1, k), CC(i - 1, k, 0), tr2);
                PM(CH(i, 0, k), CH(ic, 1, k), ti2, CC(i, k, 0));
            }
    }

    template <typename A>
    VCF_RT_HD void radf3(size_t ido, size_t l1, A cc, A ch, const T *wa) const
    {
        const T taur = T(-0.5), taui = T(0.8660254037844386467637231707529362L);
        auto WA = [&](size_t x, size_t i) { return wa[i + x * (ido - 1)]; };
        auto CC = [&](size_t a, size_t b, size_t c) -> T & { return cc[a + ido * (b + l1 * c)]; };
        auto CH = [&](size_t a, size_t b, size_t c) -> T & { return ch[a + ido * (b + 3 * c)]; };
        for (size_t k = 0; k < l1; k++) {
            T cr2 = CC(0, k, 1) + CC(0, k, 2);
            CH(0, 0, k) = CC(0, k, 0) + cr2;
            CH(0, 2, k) = taui * (CC(0, k, 2) - CC(0, k, 1));
            CH(ido - 1, 1, k) = CC(0, k, 0) + taur * cr2;
        }
        if (ido == 1) return;
        for (size_t k = 0; k < l1; k++)
            for (size_t i = 2; i < ido; i += 2) {
                size_t ic = ido - i;
                T di2, di3, dr2, dr3;
                MULPM(dr2, di2, WA(0, i - 2), WA(0, i - 1), CC(i - 1, k, 1), CC(i, k, 1));
                MULPM(dr3, di3, WA(1, i - 2), WA(1, i - 1), CC(i - 1, k, 2), CC(i, k, 2));
                T cr2 = dr2 + dr3, ci2 = di2 + di3;
                CH(i - 1, 0, k) = CC(i - 1, k, 0) + cr2;
                CH(i, 0, k) = CC(i, k, 0) + ci2;
                T tr2 = CC(i - 1, k, 0) + taur * cr2;
                T ti2 = CC(i, k, 0) + taur * ci2;
                T tr3 = taui * (di2 - di3);
                T ti3 = taui * (dr3 - dr2);
                PM(CH(i - 1, 2, k), CH(ic - 1, 1, k), tr2, tr3);
                PM(CH(i, 2, k), CH(ic, 1, k), ti3, ti2);
            }
    }

    template <typename A>
    VCF_RT_HD void radf4(size_t ido, size_t l1, A cc, A ch, const T *wa) const
    {
        const T hsqt2 = T(0.707106781186547524400844362104849L);
        auto WA = [&](size_t x, size_t i) { return wa[i + x * (ido - 1)]; };
        auto CC = [&](size_t a, size_t b, size_t c) -> T & { return cc[a + ido * (b + l1 * c)]; };
        auto CH = [&](size_t a, size_t b, size_t c) -> T & { return ch[a + ido * (b + 4 * c)]; };
        for (size_t k = 0; k < l1; k++) {
            T tr1, tr2;
            PM(tr1, CH(0, 2, k), CC(0, k, 3), CC(0, k, 1));
            PM(tr2, CH(ido - 1, 1, k), CC(0, k, 0), CC(0, k, 2));
            PM(CH(0, 0, k), CH(ido - 1, 3, k), tr2, tr1);
        }
        if ((ido & 1) == 0)
            for (size_t k = 0; k < l1; k++) {
                T ti1 = -hsqt2 * (CC(ido - 1, k, 1) + CC(ido - 1, k, 3));
                T tr1 = hsqt2 * (CC(ido - 1, k, 1) - CC(ido - 1, k, 3));
                PM(CH(ido - 1, 0, k), CH(ido - 1, 2, k), CC(ido - 1, k, 0), tr1);
                PM(CH(0, 3, k), CH(0, 1, k), ti1, CC(ido - 1, k, 2));
            }
        if (ido <= 2) return;
        for (size_t k = 0; k < l1; k++)
            for (size_t i = 2; i < ido; i += 2) {
                size_t ic = ido - i;
                T ci2, ci3, ci4, cr2, cr3, cr4, ti1, ti2, ti3, ti4, tr1, tr2, tr3, tr4;
                MULPM(cr2, ci2, WA(0, i - 2), WA(0, i - 1), CC(i - 1, k, 1), CC(i, k, 1));
                MULPM(cr3, ci3, WA(1, i - 2), WA(1, i - 1), CC(i - 1, k, 2), CC(i, k, 2));
                MULPM(cr4, ci4, WA(2, i - 2), WA(2, i - 1), CC(i - 1, k, 3), CC(i, k, 3));
                PM(tr1, tr4, cr4, cr2);
                PM(ti1, ti4, ci2, ci4);
                PM(tr2, tr3, CC(i - 1, k, 0), cr3);
                PM(ti2, ti3, CC(i, k, 0), ci3);
                PM(CH(i - 1, 0, k), CH(ic - 1, 3, k), tr2, tr1);
                PM(CH(i, 0, k), CH(ic, 3, k), ti1, ti2);
                PM(CH(i - 1, 2, k), CH(ic - 1, 1, k), tr3, ti4);
                PM(CH(i, 2, k), CH(ic, 1, k), tr4, ti3);
            }
    }

    template <typename A>
    VCF_RT_HD void radf5(size_t ido, size_t l1, A cc, A ch, const T *wa) const
    {
        const T tr11 = T(0.3090169943749474241022934171828191L), ti11 = T(0.9510565162951535721164393333793821L),
                tr12 = T(-0.8090169943749474241022934171828191L), ti12 = T(0.5877852522924731291687059546390728L);
        auto WA = [&](size_t x, size_t i) { return wa[i + x * (ido - 1)]; };
        auto CC = [&](size_t a, size_t b, size_t c) -> T & { return cc[a + ido * (b + l1 * c)]; };
        auto CH = [&](size_t a, size_t b, size_t c) -> T & { return ch[a + ido * (b + 5 * c)]; };
        for (size_t k = 0; k < l1; k++) {
            T cr2, cr3, ci4, ci5;
            PM(cr2, ci5, CC(0, k, 4), CC(0, k, 1));
            PM(cr3, ci4, CC(0, k, 3), CC(0, k, 2));
            CH(0, 0, k) = CC(0, k, 0) + cr2 + cr3;
            CH(ido - 1, 1, k) = CC(0, k, 0) + tr11 * cr2 + tr12 * cr3;
            CH(0, 2, k) = ti11 * ci5 + ti12 * ci4;
            CH(ido - 1, 3, k) = CC(0, k, 0) + tr12 * cr2 + tr11 * cr3;
            CH(0, 4, k) = ti12 * ci5 - ti11 * ci4;
        }
        if (ido == 1) return;
        for (size_t k = 0; k < l1; ++k)
            for (size_t i = 2, ic = ido - 2; i < ido; i += 2, ic -= 2) {
                T di2, di3, di4, di5, dr2, dr3, dr4, dr5;
                MULPM(dr2, di2, WA(0, i - 2), WA(0, i - 1), CC(i - 1, k, 1), CC(i, k, 1));
                MULPM(dr3, di3, WA(1, i - 2), WA(1, i - 1), CC(i - 1, k, 2), CC(i, k, 2));
                MULPM(dr4, di4, WA(2, i - 2), WA(2, i - 1), CC(i - 1, k, 3), CC(i, k, 3));
                MULPM(dr5, di5, WA(3, i - 2), WA(3, i - 1), CC(i - 1, k, 4), CC(i, k, 4));
                rearrange(dr2, di2, dr5, di5);
                rearrange(dr3, di3, dr4, di4);
                CH(i - 1, 0, k) = CC(i - 1, k, 0) + dr2 + dr3;
                CH(i, 0, k) = CC(i, k, 0) + di2 + di3;
                T tr2 = CC(i - 1, k, 0) + tr11 * dr2 + tr12 * dr3;
                T ti2 = CC(i, k, 0) + tr11 * di2 + tr12 * di3;
                T tr3 = CC(i - 1, k, 0) + tr12 * dr2 + tr11 * dr3;
                T ti3 = CC(i, k, 0) + tr12 * di2 + tr11 * di3;
                T tr5, tr4, ti5, ti4;
                MULPM(tr5, tr4, dr5, dr4, ti11, ti12);
                MULPM(ti5, ti4, di5, di4, ti11, ti12);
                PM(CH(i - 1, 2, k), CH(ic - 1, 1, k), tr2, tr5);
                PM(CH(i, 2, k), CH(ic, 1, k), ti5, ti2);
                PM(CH(i - 1, 4, k), CH(ic - 1, 3, k), tr3, tr4);
                PM(CH(i, 4, k), CH(ic, 3, k), ti4, ti3);
            }
    }

    VCF_RT_HD static void rearrange(T &rx, T &ix, T &ry, T &iy)
    {
        T t1 = rx + ry, t2 = ry - rx, t3 = ix + iy, t4 = ix - iy;
        rx = t1; ix = t3; ry = t4; iy = t2;
    }

    template <typename A>
    VCF_RT_HD void radb5(size_t ido, size_t l1, A cc, A ch, const T *wa) const
    {
        const T tr11 = T(0.3090169943749474241022934171828191L), ti11 = T(0.9510565162951535721164393333793821L),
                tr12 = T(-0.8090169943749474241022934171828191L), ti12 = T(0.5877852522924731291687059546390728L);
        auto WA = [&](size_t x, size_t i) { return wa[i + x * (ido - 1)]; };
        auto CC = [&](size_t a, size_t b, size_t c) -> T & { return cc[a + ido * (b + 5 * c)]; };
        auto CH = [&](size_t a, size_t b, size_t c) -> T & { return ch[a + ido * (b + l1 * c)]; };
        for (size_t k = 0; k < l1; k++) {
            T ti5 = CC(0, 2, k) + CC(0, 2, k);
            T ti4 = CC(0, 4, k) + CC(0, 4, k);
            T tr2 = CC(ido - 1, 1, k) + CC(ido - 1, 1, k);
            T tr3 = CC(ido - 1, 3, k) + CC(ido - 1, 3, k);
            CH(0, k, 0) = CC(0, 0, k) + tr2 + tr3;
            T cr2 = CC(0, 0, k) + tr11 * tr2 + tr12 * tr3;
            T cr3 = CC(0, 0, k) + tr12 * tr2 + tr11 * tr3;
            T ci4, ci5;
            MULPM(ci5, ci4, ti5, ti4, ti11, ti12);
            PM(CH(0, k, 4), CH(0, k, 1), cr2, ci5);
            PM(CH(0, k, 3), CH(0, k, 2), cr3, ci4);
        }
        if (ido == 1) return;
        for (size_t k = 0; k < l1; ++k)
            for (size_t i = 2, ic = ido - 2; i < ido; i += 2, ic -= 2) {
                T tr2, tr3, tr4, tr5, ti2, ti3, ti4, ti5;
                PM(tr2, tr5, CC(i - 1, 2, k), CC(ic - 1, 1, k));
                PM(ti5, ti2, CC(i, 2, k), CC(ic, 1, k));
                PM(tr3, tr4, CC(i - 1, 4, k), CC(ic - 1, 3, k));
                PM(ti4, ti3, CC(i, 4, k), CC(ic, 3, k));
                CH(i - 1, k, 0) = CC(i - 1, 0, k) + tr2 + tr3;
                CH(i, k, 0) = CC(i, 0, k) + ti2 + ti3;
                T cr2 = CC(i - 1, 0, k) + tr11 * tr2 + tr12 * tr3;
                T ci2 = CC(i, 0, k) + tr11 * ti2 + tr12 * ti3;
                T cr3 = CC(i - 1, 0, k) + tr12 * tr2 + tr11 * tr3;
                T ci3 = CC(i, 0, k) + tr12 * ti2 + tr11 * ti3;
                T ci4, ci5, cr5, cr4;
                MULPM(cr5, cr4, tr5, tr4, ti11, ti12);
                MULPM(ci5, ci4, ti5, ti4, ti11, ti12);
                T dr2, dr3, dr4, dr5, di2, di3, di4, di5;
                PM(dr4, dr3, cr3, ci4);
                PM(di3, di4, ci3, cr4);
                PM(dr5, dr2, cr2, ci5);
                PM(di2, di5, ci2, cr5);
                MULPM(CH(i, k, 1), CH(i - 1, k, 1), WA(0, i - 2), WA(0, i - 1), di2, dr2);
                MULPM(CH(i, k, 2), CH(i - 1, k, 2), WA(1, i - 2), WA(1, i - 1), di3, dr3);
                MULPM(CH(i, k, 3), CH(i - 1, k, 3), WA(2, i - 2), WA(2, i - 1), di4, dr4);
                MULPM(CH(i, k, 4), CH(i - 1, k, 4), WA(3, i - 2), WA(3, i - 1), di5, dr5);
            }
    }

    template <typename A>
    VCF_RT_HD void radb2(size_t ido, size_t l1, A cc, A ch, const T *wa) const
    {
        auto WA = [&](size_t x, size_t i) { return wa[i + x * (ido - 1)]; };
        auto CC = [&](size_t a, size_t b, size_t c) -> T & { return cc[a + ido * (b + 2 * c)]; };
        auto CH = [&](size_t a, size_t b, size_t c) -> T & { return ch[a + ido * (b + l1 * c)]; };
        for (size_t k = 0; k < l1; k++) PM(CH(0, k, 0), CH(0, k, 1), CC(0, 0, k), CC(ido - 1, 1, k));
        if ((ido & 1) == 0)
            for (size_t k = 0; k < l1; k++) {
                CH(ido - 1, k, 0) = T(2) * CC(ido - 1, 0, k);
                CH(ido - 1, k, 1) = T(-2) * CC(0, 1, k);
            }
        if (ido <= 2) return;
        for (size_t k = 0; k < l1; ++k)
            for (size_t i = 2; i < ido; i += 2) {
                size_t ic = ido - i;
                T ti2, tr2;
                PM(CH(i - 1, k, 0), tr2, CC(i - 1, 0, k), CC(ic - 1, 1, k));
                PM(ti2, CH(i, k, 0), CC(i, 0, k), CC(ic, 1, k));
                MULPM(CH(i, k, 1), CH(i - 1, k, 1), WA(0, i - 2), WA(0, i - 1), ti2, tr2);
            }
    }

    template <typename A>
    VCF_RT_HD void radb3(size_t ido, size_t l1, A cc, A ch, const T *wa) const
    {
        const T taur = T(-0.5), taui = T(0.8660254037844386467637231707529362L);
        auto WA = [&](size_t x, size_t i) { return wa[i + x * (ido - 1)]; };
        auto CC = [&](size_t a, size_t b, size_t c) -> T & { return cc[a + ido * (b + 3 * c)]; };
        auto CH = [&](size_t a, size_t b, size_t c) -> T & { return ch[a + ido * (b + l1 * c)]; };
        for (size_t k = 0; k < l1; k++) {
            T tr2 = T(2) * CC(ido - 1, 1, k);
            T cr2 = CC(0, 0, k) + taur * tr2;
            CH(0, k, 0) = CC(0, 0, k) + tr2;
            T ci3 = (T(2) * taui) * CC(0, 2, k);
            PM(CH(0, k, 2), CH(0, k, 1), cr2, ci3);
        }
        if (ido == 1) return;
        for (size_t k = 0; k < l1; k++)
            for (size_t i = 2, ic = ido - 2; i < ido; i += 2, ic -= 2) {
                T tr2 = CC(i - 1, 2, k) + CC(ic - 1, 1, k);
                T ti2 = CC(i, 2, k) - CC(ic, 1, k);
                T cr2 = CC(i - 1, 0, k) + taur * tr2;
                T ci2 = CC(i, 0, k) + taur * ti2;
                CH(i - 1, k, 0) = CC(i - 1, 0, k) + tr2;
                CH(i, k, 0) = CC(i, 0, k) + ti2;
                T cr3 = taui * (CC(i - 1, 2, k) - CC(ic - 1, 1, k));
                T ci3 = taui * (CC(i, 2, k) + CC(ic, 1, k));
                T di2, di3, dr2, dr3;
                PM(dr3, dr2, cr2, ci3);
                PM(di2, di3, ci2, cr3);
                MULPM(CH(i, k, 1), CH(i - 1, k, 1), WA(0, i - 2), WA(0, i - 1), di2, dr2);
                MULPM(CH(i, k, 2), CH(i - 1, k, 2), WA(1, i - 2), WA(1, i - 1), di3, dr3);
            }
    }

    template <typename A>
    VCF_RT_HD void radb4(size_t ido, size_t l1, A cc, A ch, const T *wa) const
    {
        const T sqrt2 = T(1.414213562373095048801688724209698L);
        auto WA = [&](size_t x, size_t i) { return wa[i + x * (ido - 1)]; };
        auto CC = [&](size_t a, size_t b, size_t c) -> T & { return cc[a + ido * (b + 4 * c)]; };
        auto CH = [&](size_t a, size_t b, size_t c) -> T & { return ch[a + ido * (b + l1 * c)]; };
        for (size_t k = 0; k < l1; k++) {
            T tr1, tr2;
            PM(tr2, tr1, CC(0, 0, k), CC(ido - 1, 3, k));
            T tr3 = T(2) * CC(ido - 1, 1, k);
            T tr4 = T(2) * CC(0, 2, k);
            PM(CH(0, k, 0), CH(0, k, 2), tr2, tr3);
            PM(CH(0, k, 3), CH(0, k, 1), tr1, tr4);
        }
        if ((ido & 1) == 0)
            for (size_t k = 0; k < l1; k++) {
                T tr1, tr2, ti1, ti2;
                PM(ti1, ti2, CC(0, 3, k), CC(0, 1, k));
                PM(tr2, tr1, CC(ido - 1, 0, k), CC(ido - 1, 2, k));
                CH(ido - 1, k, 0) = tr2 + tr2;
                CH(ido - 1, k, 1) = sqrt2 * (tr1 - ti1);
                CH(ido - 1, k, 2) = ti2 + ti2;
                CH(ido - 1, k, 3) = -sqrt2 * (tr1 + ti1);
            }
        if (ido <= 2) return;
        for (size_t k = 0; k < l1; ++k)
            for (size_t i = 2; i < ido; i += 2) {
                T ci2, ci3, ci4, cr2, cr3, cr4, ti1, ti2, ti3, ti4, tr1, tr2, tr3, tr4;
                size_t ic = ido - i;
                PM(tr2, tr1, CC(i - 1, 0, k), CC(ic - 1, 3, k));
                PM(ti1, ti2, CC(i, 0, k), CC(ic, 3, k));
                PM(tr4, ti3, CC(i, 2, k), CC(ic, 1, k));
                PM(tr3, ti4, CC(i - 1, 2, k), CC(ic - 1, 1, k));
                PM(CH(i - 1, k, 0), cr3, tr2, tr3);
                PM(CH(i, k, 0), ci3, ti2, ti3);
                PM(cr4, cr2, tr1, tr4);
                PM(ci2, ci4, ti1, ti4);
                MULPM(CH(i, k, 1), CH(i - 1, k, 1), WA(0, i - 2), WA(0, i - 1), ci2, cr2);
                MULPM(CH(i, k, 2), CH(i - 1, k, 2), WA(1, i - 2), WA(1, i - 1), ci3, cr3);
                MULPM(CH(i, k, 3), CH(i - 1, k, 3), WA(2, i - 2), WA(2, i - 1), ci4, cr4);
            }
    }


    template <typename A>
    VCF_RT_HD void copy_and_norm(A c, A p1, size_t len, T fct) const
    {
        if (!same_line(p1, c)) {
            if (fct != T(1)) for (size_t i = 0; i < len; ++i) c[i] = fct * p1[i];
            else for (size_t i = 0; i < len; ++i) c[i] = p1[i];
        } else if (fct != T(1)) {
            for (size_t i = 0; i < len; ++i) c[i] *= fct;
        }
    }

    // rfftp::forward: radf passes in reverse factor order (radfg leaves its
    // result in place, hence the extra swap)
    template <typename A>
    VCF_RT_HD void forward(A c, A ch, const RtPlan &P, T fct) const
    {
        if (P.blue) { blue(c, P, fct, true); return; }   // pocketfft_r::forward -> fftblue::exec_r
        if (P.n == 1) { c[0] *= fct; return; }
        A p1 = c, p2 = ch;
        size_t n = (size_t)P.n, nf = (size_t)P.nf, l1 = n;
        for (size_t k1 = 0; k1 < nf; ++k1) {
            size_t k = nf - k1 - 1, ip = (size_t)P.fct[k], ido = n / l1;
            l1 /= ip;
            const T *tw = mem + P.tw[k];
            if (ip == 4) radf4(ido, l1, p1, p2, tw);
            else if (ip == 2) radf2(ido, l1, p1, p2, tw);
            else if (ip == 3) radf3(ido, l1, p1, p2, tw);
            else if (ip == 5) radf5(ido, l1, p1, p2, tw);
            else {
                radfg(ido, ip, l1, p1, p2, tw, mem + P.tws[k]);
                A t = p1; p1 = p2; p2 = t;
            }
            A t = p1; p1 = p2; p2 = t;
        }
        copy_and_norm(c, p1, n, fct);
    }

    // rfftp::backward: radb passes in factor order
    template <typename A>
    VCF_RT_HD void backward(A c, A ch, const RtPlan &P, T fct) const
    {
        if (P.blue) { blue(c, P, fct, false); return; }
        if (P.n == 1) { c[0] *= fct; return; }
        A p1 = c, p2 = ch;
        size_t n = (size_t)P.n, nf = (size_t)P.nf, l1 = 1;
        for (size_t k = 0; k < nf; k++) {
            size_t ip = (size_t)P.fct[k], ido = n / (ip * l1);
            const T *tw = mem + P.tw[k];
            if (ip == 4) radb4(ido, l1, p1, p2, tw);
            else if (ip == 2) radb2(ido, l1, p1, p2, tw);
            else if (ip == 3) radb3(ido, l1, p1, p2, tw);
            else if (ip == 5) radb5(ido, l1, p1, p2, tw);
            else radbg(ido, ip, l1, p1, p2, tw, mem + P.tws[k]);
            A t = p1; p1 = p2; p2 = t;
            l1 *= ip;
        }
        copy_and_norm(c, p1, n, fct);
    }

    // T_dcst23::exec(type 2, ortho, cosine): scipy.fftpack.dct(x, norm='ortho')
    template <typename A>
    VCF_RT_HD void dct2(A c, A ch, const RtPlan &P) const
    {
        const T sqrt2 = T(1.414213562373095048801688724209698L);
        const T *twiddle = mem + P.dct_tw;
        const size_t N = (size_t)P.n, NS2 = (N + 1) / 2;
        c[0] *= T(2);
        if ((N & 1) == 0) c[N - 1] *= T(2);
        for (size_t k = 1; k + 1 < N; k += 2) { T t = c[k + 1]; c[k + 1] = t - c[k]; c[k] = c[k] + t; }
        backward(c, ch, P, mem[P.norm]);
        for (size_t k = 1, kc = N - 1; k < NS2; ++k, --kc) {
            T t1 = twiddle[k - 1] * c[kc] + twiddle[kc - 1] * c[k];
            T t2 = twiddle[k - 1] * c[k] - twiddle[kc - 1] * c[kc];
            c[k] = T(0.5) * (t1 + t2);
            c[kc] = T(0.5) * (t1 - t2);
        }
        if ((N & 1) == 0) c[NS2] *= twiddle[NS2 - 1];
        c[0] *= sqrt2 * T(0.5);
    }

    // T_dcst23::exec(type 3, ortho, cosine): scipy.fftpack.idct(x, norm='ortho')
    template <typename A>
    VCF_RT_HD void dct3(A c, A ch, const RtPlan &P) const
    {
        const T sqrt2 = T(1.414213562373095048801688724209698L);
        const T *twiddle = mem + P.dct_tw;
        const size_t N = (size_t)P.n, NS2 = (N + 1) / 2;
        c[0] *= sqrt2;
        for (size_t k = 1, kc = N - 1; k < NS2; ++k, --kc) {
            T t1 = c[k] + c[kc], t2 = c[k] - c[kc];
            c[k] = twiddle[k - 1] * t2 + twiddle[kc - 1] * t1;
            c[kc] = twiddle[k - 1] * t1 - twiddle[kc - 1] * t2;
        }
        if ((N & 1) == 0) c[NS2] *= T(2) * twiddle[NS2 - 1];
        forward(c, ch, P, mem[P.norm]);
        for (size_t k = 1; k + 1 < N; k += 2) { T t = c[k]; c[k] = t - c[k + 1]; c[k + 1] = c[k + 1] + t; }
    }
};

// ---- host: run-time plans (pocketfft rfftp or fftblue + T_dcst23 setup) ---
// pocketfft_r<T0>(length)'s plan choice: Bluestein only for lengths >= 50
// whose largest prime factor p has p*p > length, when its cost guess wins
// (util::largest_prime_factor, cost_guess, good_size_cmplx)
inline size_t rt_largest_prime_factor(size_t n)
{
    size_t res = 1;
    while ((n & 1) == 0) { res = 2; n >>= 1; }
    for (size_t x = 3; x * x <= n; x += 2)
        while (n % x == 0) { res = x; n /= x; }
    if (n > 1) res = n;
    return res;
}
inline double rt_cost_guess(size_t n)
{
    const double lfp = 1.1;   // penalty for non-hardcoded larger factors
    const size_t ni = n;
    double result = 0.;
    while ((n & 1) == 0) { result += 2; n >>= 1; }
    for (size_t x = 3; x * x <= n; x += 2)
        while (n % x == 0) { result += (x <= 5) ? double(x) : lfp * double(x); n /= x; }
    if (n > 1) result += (n <= 5) ? double(n) : lfp * double(n);
    return result * double(ni);
}
inline size_t rt_good_size_cmplx(size_t n)
{
    if (n <= 12) return n;
    size_t bestfac = 2 * n;
    for (size_t f11 = 1; f11 < bestfac; f11 *= 11)
        for (size_t f117 = f11; f117 < bestfac; f117 *= 7)
            for (size_t f1175 = f117; f1175 < bestfac; f1175 *= 5) {
                size_t x = f1175;
                while (x < n) x *= 2;
                for (;;) {
                    if (x < n) x *= 3;
                    else if (x > n) {
                        if (x < bestfac) bestfac = x;
                        if (x & 1) break;
                        x >>= 1;
                    } else return n;
                }
            }
    return bestfac;
}
inline bool rt_uses_bluestein(size_t n)
{
    const size_t tmp = (n < 50) ? 0 : rt_largest_prime_factor(n);
    if (tmp * tmp <= n) return false;
    const double comp1 = 0.5 * rt_cost_guess(n);
    const double comp2 = 2 * rt_cost_guess(rt_good_size_cmplx(2 * n - 1)) * 1.5;   // pocketfft's fudge factor
    return comp2 < comp1;
}

// rfftp factorize + comp_twiddle (or the Bluestein plan), T_dcst23's
// twiddle, pypocketfft's norm_fct
template <typename T>
inline void rt_fill(int n, RtPlan &P, std::vector<T> &mem)
{
    P.n = n;
    P.nf = 0;
    P.blue = rt_uses_bluestein((size_t)n) ? 1 : 0;
    P.bl = BluePlan{};
    mem.clear();
    if (P.blue) blue_fill<T>(n, (int)rt_good_size_cmplx(2 * (size_t)n - 1), P.bl, mem);
    int l = n;
    if (n > 1 && !P.blue) {
        while (l % 4 == 0) { P.fct[P.nf++] = 4; l >>= 2; }
        if (l % 2 == 0) {
            l >>= 1;
            P.fct[P.nf++] = 2;
            std::swap(P.fct[0], P.fct[P.nf - 1]);
        }
        for (int d = 3; d * d <= l; d += 2)
            while (l % d == 0) { P.fct[P.nf++] = d; l /= d; }
        if (l > 1) P.fct[P.nf++] = l;
    }
    size_t l1 = 1;
    for (int k = 0; k < P.nf; ++k) {
        const size_t ip = (size_t)P.fct[k], ido = (size_t)n / (l1 * ip);
        P.tw[k] = (int)mem.size();
        if (k < P.nf - 1) {
            const size_t off = mem.size();
            mem.resize(off + (ip - 1) * (ido - 1));
            for (size_t j = 1; j < ip; ++j)
                for (size_t i = 1; i <= (ido - 1) / 2; ++i) {
                    T re, im;
                    sincos_2pibyn<T>((size_t)n, j * l1 * i, re, im);
                    mem[off + (j - 1) * (ido - 1) + 2 * i - 2] = re;
                    mem[off + (j - 1) * (ido - 1) + 2 * i - 1] = im;
                }
        }
        P.tws[k] = (int)mem.size();
        if (ip > 5) {
            const size_t off = mem.size();
            mem.resize(off + 2 * ip);
            mem[off] = T(1);
            mem[off + 1] = T(0);
            for (size_t i = 2, ic = 2 * ip - 2; i <= ic; i += 2, ic -= 2) {
                T re, im;
                sincos_2pibyn<T>((size_t)n, i / 2 * ((size_t)n / ip), re, im);
                mem[off + i] = re;
                mem[off + i + 1] = im;
                mem[off + ic] = re;
                mem[off + ic + 1] = -im;
            }
        }
        l1 *= ip;
    }
    P.dct_tw = (int)mem.size();
    for (int i = 0; i < n; ++i) {
        T re, im;
        sincos_2pibyn<T>(4 * (size_t)n, (size_t)i + 1, re, im);
        mem.push_back(re);
    }
    P.norm = (int)mem.size();
    mem.push_back(T(1 / std::sqrt((long double)(2 * n))));
}

}  // namespace pfft
}  // namespace vcf
