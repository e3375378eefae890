// vcf_sincos.h -- host: pocketfft's sincos_2pibyn<T>(n)[idx] (values computed
// in double exactly as pocketfft computes them, cast to T on use), the source of
// every twiddle the DCT transforms read (vcf_pocketfft_tables.h,
// vcf_dct_any.hip, vcf_pocketfft_blue.h).  Plain C++: also built by g++ for the
// CPU harness tests.
// Restates pocketfft (BSD-3-Clause, Copyright (C) 2010-2019 Max-Planck-Society);
// license text in THIRD_PARTY_NOTICES.md.
#pragma once
#include <cmath>
#include <cstddef>

namespace vcf {

// ---- host: pocketfft sincos_2pibyn<T>(n)[idx].{r,i} (values in double) ----
inline void sc_calc(size_t x, size_t n, double ang, double &re, double &im)
{
    /* pocketfft takes cos and sin of the same angle; gcc -O2 (the build of
     * scipy's pocketfft the fixtures pin) fuses each pair into one glibc
     * sincos() call, which differs from separate sin/cos in the last bit for
     * some angles, so call it explicitly */
    double s, c;
    x <<= 3;
    if (x < 4 * n) {
        if (x < 2 * n) {
            if (x < n) { sincos(double(x) * ang, &s, &c); re = c; im = s; return; }
            sincos(double(2 * n - x) * ang, &s, &c); re = s; im = c; return;
        }
        x -= 2 * n;
        if (x < n) { sincos(double(x) * ang, &s, &c); re = -s; im = c; return; }
        sincos(double(2 * n - x) * ang, &s, &c); re = -c; im = s; return;
    }
    x = 8 * n - x;
    if (x < 2 * n) {
        if (x < n) { sincos(double(x) * ang, &s, &c); re = c; im = -s; return; }
        sincos(double(2 * n - x) * ang, &s, &c); re = s; im = -c; return;
    }
    x -= 2 * n;   /* the third quadrant: x in [2n, 4n] */
    if (x < n) { sincos(double(x) * ang, &s, &c); re = -s; im = -c; return; }
    sincos(double(2 * n - x) * ang, &s, &c); re = -c; im = -s;
}

// value pocketfft hands out for index idx of a table of length n (cast to T)
template <typename T> inline void sincos_2pibyn(size_t n, size_t idx, T &re_out, T &im_out)
{
    const long double pi = 3.141592653589793238462643383279502884197L;
    const double ang = double(0.25L * pi / (long double)n);
    const size_t nval = (n + 2) / 2;
    size_t shift = 1;
    while ((size_t(1) << shift) * (size_t(1) << shift) < nval) ++shift;
    const size_t mask = (size_t(1) << shift) - 1;
    bool conj = false;
    if (2 * idx > n) { idx = n - idx; conj = true; }
    double r1 = 1.0, i1 = 0.0, r2 = 1.0, i2 = 0.0;
    if (idx & mask) sc_calc(idx & mask, n, ang, r1, i1);
    if (idx >> shift) sc_calc((idx >> shift) * (mask + 1), n, ang, r2, i2);
    re_out = T(r1 * r2 - i1 * i2);
    T im = T(r1 * i2 + i1 * r2);
    im_out = conj ? -im : im;
}

}  // namespace vcf
