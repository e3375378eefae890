// vcf_pocketfft.h -- compile-time-length DCT-II / DCT-III in pocketfft's
// exact operation order, for the block transforms of any -B block size
// (src/2D-DCT.py:29 -B, :303 analyze_image, :440 synthesize_image, and the
// 2..128 sweep of optimize_block_size :533-579).
//
// The reference's block DCT is scipy.fftpack's dct/idct with norm='ortho'
// (assumptions A1/A2, idiom at src/IPP_DCT.py:257-259), i.e. pocketfft's
// T_dcst23<T>::exec over rfftp<T>.  Bit-exactness needs the same float
// operations in the same order, so this restates that code path:
//   - rfftp factorisation: 4s first, then a 2 swapped to the front, then 3s
//     and 5s;
//   - backward (DCT-II) runs radb2/3/4/5 in factor order, forward (DCT-III)
//     runs radf4/2/3/5 in reverse factor order, each pass
//     reading one register array and writing the other;
//   - the final multiplication by fct = 1/sqrt(2N) (copy_and_norm);
//   - T_dcst23's pre/post twiddle loops and the ortho sqrt2 scalings.
// Every length is a template parameter: all loops unroll and both arrays
// live in VGPRs.  The twiddles (pocketfft's sincos_2pibyn values, computed in
// double on the host, vcf_dct_any.hip) are read from a __constant__ table at
// compile-time offsets, i.e. with scalar loads.  Build with -ffp-contract=off.
// Restates pocketfft (BSD-3-Clause, Copyright (C) 2010-2019 Max-Planck-Society);
// license text in THIRD_PARTY_NOTICES.md.
#pragma once
#include <hip/hip_runtime.h>

namespace vcf {
namespace pfft {

struct Factors {
    int n = 0;
    int f[12] = {};
    int tw_off[12] = {};   // offset of factor k's rfftp twiddles in the slot
    int tw_len = 0;        // total rfftp twiddles (the DCT twiddles follow)
    bool ok = true;
};

// rfftp<T>::factorize + comp_twiddle's layout (sizes only)
constexpr Factors factorize(int len)
{
    Factors r{};
    if (len <= 1) return r;
    int l = len;
    while (l % 4 == 0) { r.f[r.n++] = 4; l >>= 2; }
    if (l % 2 == 0) {
        l >>= 1;
        r.f[r.n++] = 2;
        int t = r.f[0]; r.f[0] = r.f[r.n - 1]; r.f[r.n - 1] = t;
    }
    for (int d = 3; d * d <= l; d += 2)
        while (l % d == 0) { r.f[r.n++] = d; l /= d; }
    if (l > 1) r.f[r.n++] = l;
    int l1 = 1, off = 0;
    for (int k = 0; k < r.n; ++k) {
        if (r.f[k] != 2 && r.f[k] != 3 && r.f[k] != 4 && r.f[k] != 5) r.ok = false;
        int ip = r.f[k], ido = len / (l1 * ip);
        r.tw_off[k] = off;
        if (k < r.n - 1) off += (ip - 1) * (ido - 1);
        l1 *= ip;
    }
    r.tw_len = off;
    return r;
}

template <typename T> __host__ __device__ __forceinline__ void PM(T &a, T &b, T c, T d) { a = c + d; b = c - d; }
template <typename T> __host__ __device__ __forceinline__ void MULPM(T &a, T &b, T c, T d, T e, T f)
{
    a = c * e + d * f;
    b = c * f - d * e;
}

// ---- forward passes (real -> halfcomplex) --------------------------------
template <typename T, int IDO, int L1>
__device__ __forceinline__ void radf2(const T *cc, T *ch, const T *wa)
{
#define CC(a, b, c) cc[(a) + IDO * ((b) + L1 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + 2 * (c))]
#define WA(x, i) wa[(i) + (x) * (IDO - 1)]
#pragma unroll
    for (int k = 0; k < L1; k++) PM(CH(0, 0, k), CH(IDO - 1, 1, k), CC(0, k, 0), CC(0, k, 1));
    if constexpr ((IDO & 1) == 0) {
#pragma unroll
        for (int k = 0; k < L1; k++) {
            CH(0, 1, k) = -CC(IDO - 1, k, 1);
            CH(IDO - 1, 0, k) = CC(IDO - 1, k, 0);
        }
    }
    if constexpr (IDO > 2) {
#pragma unroll
        for (int k = 0; k < L1; k++)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
                T tr2, ti2;
                MULPM(tr2, ti2, WA(0, i - 2), WA(0, i - 1), CC(i - 1, k, 1), CC(i, k, 1));
                PM(CH(i - 1, 0, k), CH(ic - 1, 1, k), CC(i - 1, k, 0), tr2);
                PM(CH(i, 0, k), CH(ic, 1, k), ti2, CC(i, k, 0));
            }
    }
#undef CC
#undef CH
#undef WA
}

template <typename T, int IDO, int L1>
__device__ __forceinline__ void radf3(const T *cc, T *ch, const T *wa)
{
    const T taur = T(-0.5), taui = T(0.8660254037844386467637231707529362L);
#define CC(a, b, c) cc[(a) + IDO * ((b) + L1 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + 3 * (c))]
#define WA(x, i) wa[(i) + (x) * (IDO - 1)]
#pragma unroll
    for (int k = 0; k < L1; k++) {
        T cr2 = CC(0, k, 1) + CC(0, k, 2);
        CH(0, 0, k) = CC(0, k, 0) + cr2;
        CH(0, 2, k) = taui * (CC(0, k, 2) - CC(0, k, 1));
        CH(IDO - 1, 1, k) = CC(0, k, 0) + taur * cr2;
    }
    if constexpr (IDO > 1) {
#pragma unroll
        for (int k = 0; k < L1; k++)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
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
#undef CC
#undef CH
#undef WA
}

template <typename T, int IDO, int L1>
__device__ __forceinline__ void radf4(const T *cc, T *ch, const T *wa)
{
    const T hsqt2 = T(0.707106781186547524400844362104849L);
#define CC(a, b, c) cc[(a) + IDO * ((b) + L1 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + 4 * (c))]
#define WA(x, i) wa[(i) + (x) * (IDO - 1)]
#pragma unroll
    for (int k = 0; k < L1; k++) {
        T tr1, tr2;
        PM(tr1, CH(0, 2, k), CC(0, k, 3), CC(0, k, 1));
        PM(tr2, CH(IDO - 1, 1, k), CC(0, k, 0), CC(0, k, 2));
        PM(CH(0, 0, k), CH(IDO - 1, 3, k), tr2, tr1);
    }
    if constexpr ((IDO & 1) == 0) {
#pragma unroll
        for (int k = 0; k < L1; k++) {
            T ti1 = -hsqt2 * (CC(IDO - 1, k, 1) + CC(IDO - 1, k, 3));
            T tr1 = hsqt2 * (CC(IDO - 1, k, 1) - CC(IDO - 1, k, 3));
            PM(CH(IDO - 1, 0, k), CH(IDO - 1, 2, k), CC(IDO - 1, k, 0), tr1);
            PM(CH(0, 3, k), CH(0, 1, k), ti1, CC(IDO - 1, k, 2));
        }
    }
    if constexpr (IDO > 2) {
#pragma unroll
        for (int k = 0; k < L1; k++)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
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
#undef CC
#undef CH
#undef WA
}

template <typename T>
__device__ __forceinline__ void rearrange(T &rx, T &ix, T &ry, T &iy)   // POCKETFFT_REARRANGE
{
    const T t1 = rx + ry, t2 = ry - rx, t3 = ix + iy, t4 = ix - iy;
    rx = t1; ix = t3; ry = t4; iy = t2;
}

template <typename T, int IDO, int L1>
__device__ __forceinline__ void radf5(const T *cc, T *ch, const T *wa)
{
    const T tr11 = T(0.3090169943749474241022934171828191L), ti11 = T(0.9510565162951535721164393333793821L),
            tr12 = T(-0.8090169943749474241022934171828191L), ti12 = T(0.5877852522924731291687059546390728L);
#define CC(a, b, c) cc[(a) + IDO * ((b) + L1 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + 5 * (c))]
#define WA(x, i) wa[(i) + (x) * (IDO - 1)]
#pragma unroll
    for (int k = 0; k < L1; k++) {
        T cr2, cr3, ci4, ci5;
        PM(cr2, ci5, CC(0, k, 4), CC(0, k, 1));
        PM(cr3, ci4, CC(0, k, 3), CC(0, k, 2));
        CH(0, 0, k) = CC(0, k, 0) + cr2 + cr3;
        CH(IDO - 1, 1, k) = CC(0, k, 0) + tr11 * cr2 + tr12 * cr3;
        CH(0, 2, k) = ti11 * ci5 + ti12 * ci4;
        CH(IDO - 1, 3, k) = CC(0, k, 0) + tr12 * cr2 + tr11 * cr3;
        CH(0, 4, k) = ti12 * ci5 - ti11 * ci4;
    }
    if constexpr (IDO > 1) {
#pragma unroll
        for (int k = 0; k < L1; ++k)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
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
#undef CC
#undef CH
#undef WA
}

// ---- backward passes (halfcomplex -> real) -------------------------------
template <typename T, int IDO, int L1>
__device__ __forceinline__ void radb2(const T *cc, T *ch, const T *wa)
{
#define CC(a, b, c) cc[(a) + IDO * ((b) + 2 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + L1 * (c))]
#define WA(x, i) wa[(i) + (x) * (IDO - 1)]
#pragma unroll
    for (int k = 0; k < L1; k++) PM(CH(0, k, 0), CH(0, k, 1), CC(0, 0, k), CC(IDO - 1, 1, k));
    if constexpr ((IDO & 1) == 0) {
#pragma unroll
        for (int k = 0; k < L1; k++) {
            CH(IDO - 1, k, 0) = T(2) * CC(IDO - 1, 0, k);
            CH(IDO - 1, k, 1) = T(-2) * CC(0, 1, k);
        }
    }
    if constexpr (IDO > 2) {
#pragma unroll
        for (int k = 0; k < L1; ++k)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
                T ti2, tr2;
                PM(CH(i - 1, k, 0), tr2, CC(i - 1, 0, k), CC(ic - 1, 1, k));
                PM(ti2, CH(i, k, 0), CC(i, 0, k), CC(ic, 1, k));
                MULPM(CH(i, k, 1), CH(i - 1, k, 1), WA(0, i - 2), WA(0, i - 1), ti2, tr2);
            }
    }
#undef CC
#undef CH
#undef WA
}

template <typename T, int IDO, int L1>
__device__ __forceinline__ void radb3(const T *cc, T *ch, const T *wa)
{
    const T taur = T(-0.5), taui = T(0.8660254037844386467637231707529362L);
#define CC(a, b, c) cc[(a) + IDO * ((b) + 3 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + L1 * (c))]
#define WA(x, i) wa[(i) + (x) * (IDO - 1)]
#pragma unroll
    for (int k = 0; k < L1; k++) {
        T tr2 = T(2) * CC(IDO - 1, 1, k);
        T cr2 = CC(0, 0, k) + taur * tr2;
        CH(0, k, 0) = CC(0, 0, k) + tr2;
        T ci3 = (T(2) * taui) * CC(0, 2, k);
        PM(CH(0, k, 2), CH(0, k, 1), cr2, ci3);
    }
    if constexpr (IDO > 1) {
#pragma unroll
        for (int k = 0; k < L1; k++)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
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
#undef CC
#undef CH
#undef WA
}

template <typename T, int IDO, int L1>
__device__ __forceinline__ void radb4(const T *cc, T *ch, const T *wa)
{
    const T sqrt2 = T(1.414213562373095048801688724209698L);
#define CC(a, b, c) cc[(a) + IDO * ((b) + 4 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + L1 * (c))]
#define WA(x, i) wa[(i) + (x) * (IDO - 1)]
#pragma unroll
    for (int k = 0; k < L1; k++) {
        T tr1, tr2;
        PM(tr2, tr1, CC(0, 0, k), CC(IDO - 1, 3, k));
        T tr3 = T(2) * CC(IDO - 1, 1, k);
        T tr4 = T(2) * CC(0, 2, k);
        PM(CH(0, k, 0), CH(0, k, 2), tr2, tr3);
        PM(CH(0, k, 3), CH(0, k, 1), tr1, tr4);
    }
    if constexpr ((IDO & 1) == 0) {
#pragma unroll
        for (int k = 0; k < L1; k++) {
            T tr1, tr2, ti1, ti2;
            PM(ti1, ti2, CC(0, 3, k), CC(0, 1, k));
            PM(tr2, tr1, CC(IDO - 1, 0, k), CC(IDO - 1, 2, k));
            CH(IDO - 1, k, 0) = tr2 + tr2;
            CH(IDO - 1, k, 1) = sqrt2 * (tr1 - ti1);
            CH(IDO - 1, k, 2) = ti2 + ti2;
            CH(IDO - 1, k, 3) = -sqrt2 * (tr1 + ti1);
        }
    }
    if constexpr (IDO > 2) {
#pragma unroll
        for (int k = 0; k < L1; ++k)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
                T ci2, ci3, ci4, cr2, cr3, cr4, ti1, ti2, ti3, ti4, tr1, tr2, tr3, tr4;
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
#undef CC
#undef CH
#undef WA
}

template <typename T, int IDO, int L1>
__device__ __forceinline__ void radb5(const T *cc, T *ch, const T *wa)
{
    const T tr11 = T(0.3090169943749474241022934171828191L), ti11 = T(0.9510565162951535721164393333793821L),
            tr12 = T(-0.8090169943749474241022934171828191L), ti12 = T(0.5877852522924731291687059546390728L);
#define CC(a, b, c) cc[(a) + IDO * ((b) + 5 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + L1 * (c))]
#define WA(x, i) wa[(i) + (x) * (IDO - 1)]
#pragma unroll
    for (int k = 0; k < L1; k++) {
        T ti5 = CC(0, 2, k) + CC(0, 2, k);
        T ti4 = CC(0, 4, k) + CC(0, 4, k);
        T tr2 = CC(IDO - 1, 1, k) + CC(IDO - 1, 1, k);
        T tr3 = CC(IDO - 1, 3, k) + CC(IDO - 1, 3, k);
        CH(0, k, 0) = CC(0, 0, k) + tr2 + tr3;
        T cr2 = CC(0, 0, k) + tr11 * tr2 + tr12 * tr3;
        T cr3 = CC(0, 0, k) + tr12 * tr2 + tr11 * tr3;
        T ci4, ci5;
        MULPM(ci5, ci4, ti5, ti4, ti11, ti12);
        PM(CH(0, k, 4), CH(0, k, 1), cr2, ci5);
        PM(CH(0, k, 3), CH(0, k, 2), cr3, ci4);
    }
    if constexpr (IDO > 1) {
#pragma unroll
        for (int k = 0; k < L1; ++k)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
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
#undef CC
#undef CH
#undef WA
}

// ---- rfftp backward()/forward() over the whole factor list ----------------
// p1 holds the data; each pass writes the other array.  Returns (statically)
// which array holds the result: true = p1.
template <typename T, int N, int K, int L1>
__device__ __forceinline__ void backward_passes(T *p1, T *p2, const T *tw)
{
    constexpr Factors F = factorize(N);
    if constexpr (K < F.n) {
        constexpr int ip = F.f[K], ido = N / (ip * L1);
        if constexpr (ip == 4) radb4<T, ido, L1>(p1, p2, tw + F.tw_off[K]);
        else if constexpr (ip == 2) radb2<T, ido, L1>(p1, p2, tw + F.tw_off[K]);
        else if constexpr (ip == 3) radb3<T, ido, L1>(p1, p2, tw + F.tw_off[K]);
        else radb5<T, ido, L1>(p1, p2, tw + F.tw_off[K]);
        backward_passes<T, N, K + 1, L1 * ip>(p2, p1, tw);
    }
}

template <typename T, int N, int K1, int L1>
__device__ __forceinline__ void forward_passes(T *p1, T *p2, const T *tw)
{
    constexpr Factors F = factorize(N);
    if constexpr (K1 < F.n) {
        constexpr int k = F.n - K1 - 1, ip = F.f[k], ido = N / L1, l1 = L1 / ip;
        if constexpr (ip == 4) radf4<T, ido, l1>(p1, p2, tw + F.tw_off[k]);
        else if constexpr (ip == 2) radf2<T, ido, l1>(p1, p2, tw + F.tw_off[k]);
        else if constexpr (ip == 3) radf3<T, ido, l1>(p1, p2, tw + F.tw_off[k]);
        else radf5<T, ido, l1>(p1, p2, tw + F.tw_off[k]);
        forward_passes<T, N, K1 + 1, l1>(p2, p1, tw);
    }
}

// ---- T_dcst23<T>::exec, cosine, ortho ------------------------------------
// tw: this length's slot: rfftp twiddles (F.tw_len), then the N DCT twiddles
// (sincos_2pibyn(4N)[i+1].r), then fct = 1/sqrt(2N).
template <typename T, int N>
__device__ __forceinline__ void dct2(T (&c)[N], const T *tw)   // scipy dct(x, 2, norm='ortho')
{
    constexpr Factors F = factorize(N);
    const T *dtw = tw + F.tw_len;
    const T fct = dtw[N];
    const T sqrt2 = T(1.414213562373095048801688724209698L);
    constexpr int NS2 = (N + 1) / 2;
    c[0] *= T(2);
    if constexpr ((N & 1) == 0) c[N - 1] *= T(2);
#pragma unroll
    for (int k = 1; k + 1 < N; k += 2) {
        T t = c[k + 1];
        c[k + 1] = t - c[k];
        c[k] = c[k] + t;
    }
    if constexpr (N == 1) {
        c[0] *= fct;
    } else {
        T ch[N];
        backward_passes<T, N, 0, 1>(c, ch, tw);
        if constexpr (F.n & 1) {
#pragma unroll
            for (int i = 0; i < N; ++i) c[i] = fct * ch[i];
        } else {
#pragma unroll
            for (int i = 0; i < N; ++i) c[i] *= fct;
        }
    }
#pragma unroll
    for (int k = 1, kc = N - 1; k < NS2; ++k, --kc) {
        T t1 = dtw[k - 1] * c[kc] + dtw[kc - 1] * c[k];
        T t2 = dtw[k - 1] * c[k] - dtw[kc - 1] * c[kc];
        c[k] = T(0.5) * (t1 + t2);
        c[kc] = T(0.5) * (t1 - t2);
    }
    if constexpr ((N & 1) == 0) c[NS2] *= dtw[NS2 - 1];
    c[0] *= sqrt2 * T(0.5);
}

template <typename T, int N>
__device__ __forceinline__ void dct3(T (&c)[N], const T *tw)   // scipy idct(x, 2, norm='ortho')
{
    constexpr Factors F = factorize(N);
    const T *dtw = tw + F.tw_len;
    const T fct = dtw[N];
    const T sqrt2 = T(1.414213562373095048801688724209698L);
    constexpr int NS2 = (N + 1) / 2;
    c[0] *= sqrt2;
#pragma unroll
    for (int k = 1, kc = N - 1; k < NS2; ++k, --kc) {
        T t1 = c[k] + c[kc], t2 = c[k] - c[kc];
        c[k] = dtw[k - 1] * t2 + dtw[kc - 1] * t1;
        c[kc] = dtw[k - 1] * t1 - dtw[kc - 1] * t2;
    }
    if constexpr ((N & 1) == 0) c[NS2] *= T(2) * dtw[NS2 - 1];
    if constexpr (N == 1) {
        c[0] *= fct;
    } else {
        T ch[N];
        forward_passes<T, N, 0, N>(c, ch, tw);
        if constexpr (F.n & 1) {
#pragma unroll
            for (int i = 0; i < N; ++i) c[i] = fct * ch[i];
        } else {
#pragma unroll
            for (int i = 0; i < N; ++i) c[i] *= fct;
        }
    }
#pragma unroll
    for (int k = 1; k + 1 < N; k += 2) {
        T t = c[k];
        c[k] = t - c[k + 1];
        c[k + 1] = c[k + 1] + t;
    }
}

}  // namespace pfft
}  // namespace vcf
