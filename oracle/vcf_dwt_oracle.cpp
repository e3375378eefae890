/*
  * vcf_dwt_oracle.cpp -- CPU restatement of VCF's 2D-DWT + deadzone path.
 *
 * TEST INFRASTRUCTURE ONLY (like vcf_oracle.c): the checker tests/ and
 * bench.py compare the HIP path with; nothing under vcf_amd/ uses it.
 *
 * Restates (reference = /root/reference, Sistemas-Multimedia/VCF):
 *   encode src/2D-DWT.py:57-78 encode_fn
 *     :59      img.astype(int16) (no offset)
 *     :62      color_transforms.YCoCg.from_RGB into empty_like(int16)  (A4):
 *              Y = R/4 + G/2 + B/4, Co = R/2 - B/2, Cg = -R/4 + G/2 - B/4
 *              in float64, truncated toward zero by the int16 store
 *     :64      DWT2D.color_dyadic_DWT.analyze (A6): per channel
 *              pywt.wavedec2(mode='per') in float64
 *     :67      quantize_decom_fn (:113-136) -> deadzone (x/Q).astype(int32) (A5)
 *     :68      write_decom_fn (:162-200): LL + 128 -> uint16, details + 128
 *              -> uint8 (both wrap), one TIFF each, LL_{l}, {LH,HL,HH}_{l..1}
 *   decode src/2D-DWT.py:80-101 decode_fn
 *     :82      read_decom_fn (:202-228): astype(int16) - 128
 *     :84      dequantize_decom_fn (:138-160): Q * k in int16 (A5)
 *     :85      synthesize: pywt.waverec2(mode='per') per channel (float64)
 *     :94-97   to_RGB (float64), clip(0, 255).astype(uint8)
 *
 * pywt 1.1.1's C convolution (not vendored; pinned here against pywt itself
 * by tests/golden/make_golden_dwt.py -> dwt_pywt.npz and the reference runs):
 *   dwt 'per' (downsampling_convolution_periodization): odd N is extended by
 *     its last sample; out[o] = sum_j f[j] * x[(F/2 + 2o - j) mod N'] with j
 *     ascending -- except outputs i = F/2 + 2o >= N, which first add the taps
 *     that run past the end (i - j >= N) in descending j, then the others in
 *     ascending j.
 *   idwt 'per' (upsampling_convolution_valid_sf_periodization, called for
 *     cA with rec_lo and then cD with rec_hi, both accumulating into a
 *     zeroed output): out[(2i + p + 1 - F/2) mod 2N] += f[2j + p] * c[(i - j)
 *     mod N], one product at a time, j ascending; for the first
 *     ceil((F/2 - 1) / 2) values of i (whose outputs wrap to the end) the
 *     taps j <= top come first in descending j, then j > top ascending
 *     (top = i for lines of at least F/2 samples).
 *   For lines shorter than the taps (pywt's short-input branch, which wraps
 *   the coefficients around more than once) the reordered indices are
 *   i < ceil((F/2 - 1) / 2) still, with top = the largest i + kN below that
 *   bound instead of i (found against pywt 1.1.1 for all 106 discrete wavelets,
 *   N = 1 .. F/2 + 3, make_golden_dwt_short.py).
 *   2D: wavedec2 = per level dwt along axis 0 then axis 1 (keys aa, da, ad,
 *   dd -> cA, (cH, cV, cD)); waverec2 = per level trim cA to the detail
 *   shape, idwt along axis 1 (aa+ad -> a, da+dd -> d), then along axis 0.
 *
 * Build with -ffp-contract=off (no FMA: pywt's x86-64 build has none).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../vcf_amd/csrc/vcf_wavelets.h"

using vcf::kNumWavelets;
using vcf::kWavelets;

extern "C" {

int vcfo_wavelet_index(const char *name)
{
    for (int i = 0; i < kNumWavelets; ++i)
        if (strcmp(kWavelets[i].name, name) == 0) return i;
    return -1;
}

int vcfo_wavelet_len(int id) { return (id >= 0 && id < kNumWavelets) ? kWavelets[id].len : -1; }

/* 1-D forward, mode 'per'.  x[k*xs], k < N -> out[o*os], o < (N+1)/2 */
void vcfo_dwt1_per(const double *x, int N, int xs, const double *f, int F, double *out, int os)
{
    const int pad = N & 1, Ne = N + pad;
    int o = 0;
    for (int i = F / 2; i < Ne + F / 2; i += 2, ++o) {
        double s = 0.0;
        if (i >= N) {
            for (int m = F - 1; m >= 0; --m) {          /* taps past the end, descending */
                if (i - m < N) continue;
                const int p = ((i - m) % Ne + Ne) % Ne;
                s = s + f[m] * (p < N ? x[(long)p * xs] : x[(long)(N - 1) * xs]);
            }
            for (int m = 0; m < F; ++m) {               /* the rest, ascending */
                if (i - m >= N) continue;
                const int p = ((i - m) % Ne + Ne) % Ne;
                s = s + f[m] * (p < N ? x[(long)p * xs] : x[(long)(N - 1) * xs]);
            }
        } else {
            for (int m = 0; m < F; ++m) {
                const int p = ((i - m) % Ne + Ne) % Ne;
                s = s + f[m] * (p < N ? x[(long)p * xs] : x[(long)(N - 1) * xs]);
            }
        }
        out[(long)o * os] = s;
    }
}

/* 1-D inverse, mode 'per': a, d (N each) -> out (2N) */
void vcfo_idwt1_per(const double *a, const double *d, int N, int cs, const double *lo, const double *hi,
                    int F, double *out, int os)
{
    const int F2 = F / 2, shift = 1 - F2;
    const int T = (F2 - 1 + 1) / 2;   /* ceil((F/2 - 1) / 2) */
    for (int n = 0; n < 2 * N; ++n) out[(long)n * os] = 0.0;
    for (int pass = 0; pass < 2; ++pass) {
        const double *c = pass ? d : a;
        const double *f = pass ? hi : lo;
        for (int i = 0; i < N; ++i) {
            const long oe = (long)(((2 * i + shift) % (2 * N) + 2 * N) % (2 * N)) * os;
            const long oo = (long)(((2 * i + 1 + shift) % (2 * N) + 2 * N) % (2 * N)) * os;
            for (int t = 0; t < F2; ++t) {
                int j;
                if (i < T) {
                    /* the largest i + kN below T: i itself unless N < T (pywt's short-input branch) */
                    const int top = i + N * ((T - 1 - i) / N);
                    j = t <= top ? top - t : t;   /* top..0, then top+1.. */
                } else {
                    j = t;
                }
                const double cv = c[(long)(((i - j) % N + N) % N) * cs];
                out[oe] += f[2 * j] * cv;
                out[oo] += f[2 * j + 1] * cv;
            }
        }
    }
}

/* 1-D lines by wavelet id (pywt.dwt / pywt.idwt, mode 'periodization') */
int vcfo_dwt1_per_w(const double *x, int N, int wavelet, double *cA, double *cD)
{
    if (wavelet < 0 || wavelet >= kNumWavelets || N < 1) return -1;
    const vcf::WaveletDef &wd = kWavelets[wavelet];
    vcfo_dwt1_per(x, N, 1, wd.dec_lo, wd.len, cA, 1);
    vcfo_dwt1_per(x, N, 1, wd.dec_hi, wd.len, cD, 1);
    return 0;
}

int vcfo_idwt1_per_w(const double *a, const double *d, int N, int wavelet, double *out)
{
    if (wavelet < 0 || wavelet >= kNumWavelets || N < 1) return -1;
    const vcf::WaveletDef &wd = kWavelets[wavelet];
    vcfo_idwt1_per(a, d, N, 1, wd.rec_lo, wd.rec_hi, wd.len, out, 1);
    return 0;
}

static int half(int n) { return (n + 1) / 2; }

/* subband shapes: hs[l], ws[l] for l = 1..levels (level 1 = finest) */
int vcfo_dwt_shapes(int H, int W, int levels, int *hs, int *ws)
{
    int h = H, w = W;
    for (int l = 1; l <= levels; ++l) {
        h = half(h);
        w = half(w);
        hs[l - 1] = h;
        ws[l - 1] = w;
    }
    return 0;
}

/* one 2-D level on a plane (h x w, row stride ld): aa (hh x hw), da, ad, dd */
static void dwt2_level(const double *x, int h, int w, const double *lo, const double *hi, int F, double *aa,
                       double *da, double *ad, double *dd)
{
    const int hh = half(h), hw = half(w);
    double *A = (double *)malloc(sizeof(double) * hh * w), *D = (double *)malloc(sizeof(double) * hh * w);
    for (int c = 0; c < w; ++c) {
        vcfo_dwt1_per(x + c, h, w, lo, F, A + c, w);
        vcfo_dwt1_per(x + c, h, w, hi, F, D + c, w);
    }
    for (int r = 0; r < hh; ++r) {
        vcfo_dwt1_per(A + (long)r * w, w, 1, lo, F, aa + (long)r * hw, 1);
        vcfo_dwt1_per(A + (long)r * w, w, 1, hi, F, ad + (long)r * hw, 1);
        vcfo_dwt1_per(D + (long)r * w, w, 1, lo, F, da + (long)r * hw, 1);
        vcfo_dwt1_per(D + (long)r * w, w, 1, hi, F, dd + (long)r * hw, 1);
    }
    free(A);
    free(D);
}

/* one inverse level: aa (trimmed to h x w), da, ad, dd (h x w) -> out (2h x 2w) */
static void idwt2_level(const double *aa, int lda, const double *da, const double *ad, const double *dd, int h,
                        int w, const double *lo, const double *hi, int F, double *out)
{
    double *A = (double *)malloc(sizeof(double) * h * 2 * w), *D = (double *)malloc(sizeof(double) * h * 2 * w);
    for (int r = 0; r < h; ++r) {
        vcfo_idwt1_per(aa + (long)r * lda, ad + (long)r * w, w, 1, lo, hi, F, A + (long)r * 2 * w, 1);
        vcfo_idwt1_per(da + (long)r * w, dd + (long)r * w, w, 1, lo, hi, F, D + (long)r * 2 * w, 1);
    }
    for (int c = 0; c < 2 * w; ++c)
        vcfo_idwt1_per(A + c, D + c, h, 2 * w, lo, hi, F, out + c, 2 * w);
    free(A);
    free(D);
}

/* pywt.wavedec2 of one float64 plane: coefficients laid out as the codec
 * files: [LL_L] then for r = L..1: LH_r, HL_r, HH_r (each hs[r-1] x ws[r-1]) */
int vcfo_wavedec2(const double *x, int H, int W, int wavelet, int levels, double *coeffs)
{
    if (wavelet < 0 || wavelet >= kNumWavelets || levels < 1) return -1;
    const vcf::WaveletDef &wd = kWavelets[wavelet];
    int hs[32], ws[32];
    vcfo_dwt_shapes(H, W, levels, hs, ws);
    /* offsets of each subband in the output */
    long off = (long)hs[levels - 1] * ws[levels - 1];
    long det_off[32];
    for (int r = levels; r >= 1; --r) {
        det_off[r - 1] = off;
        off += 3L * hs[r - 1] * ws[r - 1];
    }
    double *cur = (double *)malloc(sizeof(double) * H * W);
    memcpy(cur, x, sizeof(double) * H * W);
    int h = H, w = W;
    for (int l = 1; l <= levels; ++l) {
        const int hh = hs[l - 1], hw = ws[l - 1];
        double *aa = (double *)malloc(sizeof(double) * hh * hw);
        double *base = coeffs + det_off[l - 1];
        dwt2_level(cur, h, w, wd.dec_lo, wd.dec_hi, wd.len, aa, base, base + (long)hh * hw,
                   base + 2L * hh * hw);
        free(cur);
        cur = aa;
        h = hh;
        w = hw;
    }
    memcpy(coeffs, cur, sizeof(double) * h * w);
    free(cur);
    return 0;
}

/* pywt.waverec2 of coefficients in the vcfo_wavedec2 layout -> out
 * (2*hs[0] x 2*ws[0]) */
int vcfo_waverec2(const double *coeffs, int H, int W, int wavelet, int levels, double *out)
{
    if (wavelet < 0 || wavelet >= kNumWavelets || levels < 1) return -1;
    const vcf::WaveletDef &wd = kWavelets[wavelet];
    int hs[32], ws[32];
    vcfo_dwt_shapes(H, W, levels, hs, ws);
    long off = (long)hs[levels - 1] * ws[levels - 1];
    long det_off[32];
    for (int r = levels; r >= 1; --r) {
        det_off[r - 1] = off;
        off += 3L * hs[r - 1] * ws[r - 1];
    }
    int ah = hs[levels - 1], aw = ws[levels - 1];
    double *a = (double *)malloc(sizeof(double) * ah * aw);
    memcpy(a, coeffs, sizeof(double) * ah * aw);
    for (int r = levels; r >= 1; --r) {
        const int h = hs[r - 1], w = ws[r - 1];   /* detail shape; a is trimmed to it */
        const double *base = coeffs + det_off[r - 1];
        double *y = (double *)malloc(sizeof(double) * 4L * h * w);
        idwt2_level(a, aw, base, base + (long)h * w, base + 2L * h * w, h, w, wd.rec_lo, wd.rec_hi, wd.len, y);
        free(a);
        a = y;
        ah = 2 * h;
        aw = 2 * w;
    }
    memcpy(out, a, sizeof(double) * ah * aw);
    free(a);
    return 0;
}

static long total_coeffs(int H, int W, int levels)
{
    int hs[32], ws[32];
    vcfo_dwt_shapes(H, W, levels, hs, ws);
    long n = (long)hs[levels - 1] * ws[levels - 1];
    for (int r = 1; r <= levels; ++r) n += 3L * hs[r - 1] * ws[r - 1];
    return n;
}

/* 2D-DWT.py encode_fn up to the TIFF writer.  LL: hs[L-1] x ws[L-1] x 3 u16;
 * details: for r = L..1, LH_r, HL_r, HH_r, each hs[r-1] x ws[r-1] x 3 u8 */
int vcfo_dwt_dz_encode(const uint8_t *rgb, int H, int W, int wavelet, int levels, int Q, uint16_t *LL,
                       uint8_t *details)
{
    if (wavelet < 0 || wavelet >= kNumWavelets || levels < 1 || levels > 30 || Q < 1) return -1;
    const long n = (long)H * W, nc = total_coeffs(H, W, levels);
    double *plane = (double *)malloc(sizeof(double) * n);
    double *co[3];
    for (int ch = 0; ch < 3; ++ch) {
        for (long p = 0; p < n; ++p) {
            const double R = rgb[3 * p], G = rgb[3 * p + 1], B = rgb[3 * p + 2];
            double v;
            if (ch == 0) v = R / 4 + G / 2 + B / 4;
            else if (ch == 1) v = R / 2 - B / 2;
            else v = -R / 4 + G / 2 - B / 4;
            plane[p] = (double)(int16_t)v;   /* empty_like(int16) store: truncation */
        }
        co[ch] = (double *)malloc(sizeof(double) * nc);
        vcfo_wavedec2(plane, H, W, wavelet, levels, co[ch]);
    }
    int hs[32], ws[32];
    vcfo_dwt_shapes(H, W, levels, hs, ws);
    const long nll = (long)hs[levels - 1] * ws[levels - 1];
    for (long p = 0; p < nll; ++p)
        for (int ch = 0; ch < 3; ++ch) {
            const int32_t k = (int32_t)(co[ch][p] / (double)Q);
            LL[3 * p + ch] = (uint16_t)(uint32_t)(k + 128);
        }
    for (long p = nll; p < nc; ++p)
        for (int ch = 0; ch < 3; ++ch) {
            const int32_t k = (int32_t)(co[ch][p] / (double)Q);
            details[3 * (p - nll) + ch] = (uint8_t)(uint32_t)(k + 128);
        }
    for (int ch = 0; ch < 3; ++ch) free(co[ch]);
    free(plane);
    return 0;
}

/* 2D-DWT.py decode_fn after the TIFF reader -> out (2*ceil(H/2) x 2*ceil(W/2) x 3) */
int vcfo_dwt_dz_decode(const uint16_t *LL, const uint8_t *details, int H, int W, int wavelet, int levels, int Q,
                       uint8_t *out)
{
    if (wavelet < 0 || wavelet >= kNumWavelets || levels < 1 || levels > 30 || Q < 1 || Q > 32767) return -1;
    const long nc = total_coeffs(H, W, levels);
    int hs[32], ws[32];
    vcfo_dwt_shapes(H, W, levels, hs, ws);
    const long nll = (long)hs[levels - 1] * ws[levels - 1];
    const int Ho = 2 * hs[0], Wo = 2 * ws[0];
    double *co = (double *)malloc(sizeof(double) * nc);
    double *y[3];
    for (int ch = 0; ch < 3; ++ch) {
        for (long p = 0; p < nc; ++p) {
            int16_t k = p < nll ? (int16_t)(uint16_t)LL[3 * p + ch] : (int16_t)details[3 * (p - nll) + ch];
            k = (int16_t)(k - 128);
            co[p] = (double)(int16_t)(uint16_t)((uint32_t)Q * (uint32_t)(int32_t)k);   /* Q*k in int16 */
        }
        y[ch] = (double *)malloc(sizeof(double) * Ho * Wo);
        vcfo_waverec2(co, H, W, wavelet, levels, y[ch]);
    }
    for (long p = 0; p < (long)Ho * Wo; ++p) {
        const double Y = y[0][p], Co = y[1][p], Cg = y[2][p];
        const double v[3] = {Y + Co - Cg, Y + Cg, Y - Co - Cg};
        for (int ch = 0; ch < 3; ++ch) {
            double c = v[ch] < 0.0 ? 0.0 : (v[ch] > 255.0 ? 255.0 : v[ch]);
            out[3 * p + ch] = (uint8_t)c;   /* clip then astype(uint8): truncation */
        }
    }
    for (int ch = 0; ch < 3; ++ch) free(y[ch]);
    free(co);
    return 0;
}

}  /* extern "C" */
