/*
 * vcf_oracle.c -- CPU restatement of VCF's per-frame DCT + deadzone path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under vcf_amd/ links, loads or calls
 * this file.  It is the checker that tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py compare the HIP path against.
 *
 * What it restates (reference = /root/reference, Sistemas-Multimedia/VCF):
 *   encode: src/2D-DCT.py:268-372 (encode_fn)
 *     :276      u8 RGB -> float32
 *     :281-287  pad_and_center_to_multiple_of_block_size (:187-229), zeros,
 *               centred, extra row/col bottom/right
 *     :292      img -= 128        (offset, :107-110, quantizer == deadzone)
 *     :298      color_transforms.YCoCg.from_RGB          (assumption A4)
 *     :303      DCT2D.block_DCT.analyze_image             (assumption A1)
 *     :313-327  -p perceptual weighting (Y_QSSs/121, C_QSSs/99, :63-90)
 *     :333-336  DCT2D.block_DCT.get_subbands (or -x)      (assumption A3)
 *     :343      deadzone.quantize_fn (deadzone.py:95-102) -> Deadzone_Quantizer
 *               .encode                                    (assumption A5)
 *     :348,361  += 128, astype(uint8) (wraps modulo 256)
 *   decode: src/2D-DCT.py:377-468 (decode_fn)
 *     :399-403  astype(int16) - 128
 *     :411      dequantize -> Deadzone_Quantizer.decode = Q*k in int16 (A5)
 *     :416      get_blocks (or -x)
 *     :421-435  -p perceptual de-weighting (float32, stored back into int16)
 *     :440      DCT2D.block_DCT.synthesize_image           (assumption A2)
 *     :444      remove_padding (:231-266)
 *     :449      to_RGB (int16 arithmetic)                  (assumption A4)
 *     :454,466  += 128, clip(0,255).astype(uint8)
 *
 * The block DCT of DCT2D (not vendored, requirements.txt:11) is assumed to be
 * the in-tree idiom dct(dct(b.T, norm='ortho').T, norm='ortho')
 * (src/IPP_DCT.py:257-259) over scipy.fftpack, i.e. pocketfft.  The 8-point
 * DCT-II / DCT-III below restate pocketfft's T_dcst23::exec + rfftp
 * radf4/radf2/radb4/radb2 operation by operation (no FMA contraction: build
 * with -ffp-contract=off), including pocketfft's sincos_2pibyn twiddle
 * construction, so results are bitwise equal to scipy (checked in
 * tests/test_oracle.py against tests/golden fixtures made by the reference's
 * own glue; see tests/golden/make_golden.py).
  *
 * Restates pocketfft (BSD-3-Clause, Copyright (C) 2010-2019 Max-Planck-Society);
 * license text in THIRD_PARTY_NOTICES.md.
 */
#define _GNU_SOURCE   /* sincos */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define VCFO_FLAG_NO_SUBBANDS 1u  /* -x, 2D-DCT.py:40 */
#define VCFO_FLAG_PERCEPTUAL  2u  /* -p, 2D-DCT.py:38 */

/* ------------------------------------------------------------------------ */
/* pocketfft sincos_2pibyn<double> (Thigh = double for both float and double) */
/* ------------------------------------------------------------------------ */
static void sc_calc(size_t x, size_t n, double ang, double *re, double *im)
{
    /* pocketfft takes cos and sin of the same angle; gcc -O2 (the build of
     * scipy's pocketfft the fixtures pin) fuses each pair into one glibc
     * sincos() call, which differs from separate sin/cos in the last bit for
     * some angles, so call it explicitly */
    double s, c;
    x <<= 3;
    if (x < 4 * n) {
        if (x < 2 * n) {
            if (x < n) { sincos((double)x * ang, &s, &c); *re = c; *im = s; return; }
            sincos((double)(2 * n - x) * ang, &s, &c); *re = s; *im = c; return;
        }
        x -= 2 * n;
        if (x < n) { sincos((double)x * ang, &s, &c); *re = -s; *im = c; return; }
        sincos((double)(2 * n - x) * ang, &s, &c); *re = -c; *im = s; return;
    }
    x = 8 * n - x;
    if (x < 2 * n) {
        if (x < n) { sincos((double)x * ang, &s, &c); *re = c; *im = -s; return; }
        sincos((double)(2 * n - x) * ang, &s, &c); *re = s; *im = -c; return;
    }
    x -= 2 * n;   /* the third quadrant: x in [2n, 4n] */
    if (x < n) { sincos((double)x * ang, &s, &c); *re = -s; *im = -c; return; }
    sincos((double)(2 * n - x) * ang, &s, &c); *re = -c; *im = -s;
}

/* value of sincos_2pibyn(n)[idx] in double (before the cast to T) */
static void sincos_2pibyn(size_t n, size_t idx, double *re, double *im)
{
    const long double pi = 3.141592653589793238462643383279502884197L;
    double ang = (double)(0.25L * pi / (long double)n);
    size_t nval = (n + 2) / 2, shift = 1;
    while (((size_t)1 << shift) * ((size_t)1 << shift) < nval) ++shift;
    size_t mask = ((size_t)1 << shift) - 1;
    int conj = 0;
    if (2 * idx > n) { idx = n - idx; conj = 1; }
    double r1 = 1.0, i1 = 0.0, r2 = 1.0, i2 = 0.0;
    if (idx & mask) sc_calc(idx & mask, n, ang, &r1, &i1);
    if (idx >> shift) sc_calc((idx >> shift) * (mask + 1), n, ang, &r2, &i2);
    *re = r1 * r2 - i1 * i2;
    *im = r1 * i2 + i1 * r2;
    if (conj) *im = -*im;
}

typedef struct {
    float  tw_f[8];   /* T_dcst23 twiddle, N=8: sincos_2pibyn(32)[i+1].r */
    double tw_d[8];
    float  wr_f, wi_f; /* rfftp N=8 twiddle: sincos_2pibyn(8)[1] */
    double wr_d, wi_d;
    float  sqrt2_f;
    double sqrt2_d;
} pf_consts;

static pf_consts PF;
static int pf_ready = 0;

static void pf_init(void)
{
    if (pf_ready) return;
    for (size_t i = 0; i < 8; ++i) {
        double re, im;
        sincos_2pibyn(32, i + 1, &re, &im);
        PF.tw_d[i] = re;
        PF.tw_f[i] = (float)re;
    }
    double re, im;
    sincos_2pibyn(8, 1, &re, &im);
    PF.wr_d = re; PF.wi_d = im;
    PF.wr_f = (float)re; PF.wi_f = (float)im;
    PF.sqrt2_d = (double)1.414213562373095048801688724209698L;
    PF.sqrt2_f = (float)1.414213562373095048801688724209698L;
    pf_ready = 1;
}

/* ------------------------------------------------------------------------ */
/* pocketfft rfftp<T>, length 8 = factors {2,4}                              */
/* ------------------------------------------------------------------------ */
#define DEF_RFFT8(T, SFX, WR, WI)                                              \
/* backward (halfcomplex -> real): radb2(ido=4,l1=1) then radb4(ido=1,l1=2) */ \
static void rfftb8_##SFX(T c[8])                                               \
{                                                                              \
    T ch[8], t[8];                                                             \
    /* radb2: CC(a,b,0)=c[a+4b], CH(a,0,k)=ch[a+4k] */                         \
    ch[0] = c[0] + c[7];                                                       \
    ch[4] = c[0] - c[7];                                                       \
    ch[3] = (T)2 * c[3];                                                       \
    ch[7] = (T)(-2) * c[4];                                                    \
    {                                                                          \
        T tr2, ti2;                                                            \
        ch[1] = c[1] + c[5]; tr2 = c[1] - c[5];                                \
        ti2 = c[2] + c[6];   ch[2] = c[2] - c[6];                              \
        ch[6] = WR * ti2 + WI * tr2;                                           \
        ch[5] = WR * tr2 - WI * ti2;                                           \
    }                                                                          \
    /* radb4: CC(0,b,k)=ch[b+4k], CH(0,k,c)=t[k+2c] */                         \
    for (int k = 0; k < 2; ++k) {                                              \
        const T *cc = ch + 4 * k;                                              \
        T tr2 = cc[0] + cc[3], tr1 = cc[0] - cc[3];                            \
        T tr3 = (T)2 * cc[1], tr4 = (T)2 * cc[2];                              \
        t[k + 0] = tr2 + tr3; t[k + 4] = tr2 - tr3;                            \
        t[k + 6] = tr1 + tr4; t[k + 2] = tr1 - tr4;                            \
    }                                                                          \
    memcpy(c, t, sizeof(t));                                                   \
}                                                                              \
/* forward (real -> halfcomplex): radf4(ido=1,l1=2) then radf2(ido=4,l1=1) */  \
static void rfftf8_##SFX(T c[8])                                               \
{                                                                              \
    T ch[8], t[8];                                                             \
    /* radf4: CC(0,k,c)=c[k+2c], CH(0,b,k)=ch[b+4k] */                         \
    for (int k = 0; k < 2; ++k) {                                              \
        T tr1 = c[k + 6] + c[k + 2]; ch[4 * k + 2] = c[k + 6] - c[k + 2];      \
        T tr2 = c[k + 0] + c[k + 4]; ch[4 * k + 1] = c[k + 0] - c[k + 4];      \
        ch[4 * k + 0] = tr2 + tr1;   ch[4 * k + 3] = tr2 - tr1;                \
    }                                                                          \
    /* radf2: CC(a,0,c)=ch[a+4c], CH(a,b,0)=t[a+4b] */                         \
    t[0] = ch[0] + ch[4]; t[7] = ch[0] - ch[4];                                \
    t[4] = -ch[7];        t[3] = ch[3];                                        \
    {                                                                          \
        T e = ch[5], f = ch[6];                                                \
        T tr2 = WR * e + WI * f, ti2 = WR * f - WI * e;                        \
        t[1] = ch[1] + tr2; t[5] = ch[1] - tr2;                                \
        t[2] = ti2 + ch[2]; t[6] = ti2 - ch[2];                                \
    }                                                                          \
    memcpy(c, t, sizeof(t));                                                   \
}

DEF_RFFT8(float, f32, PF.wr_f, PF.wi_f)
DEF_RFFT8(double, f64, PF.wr_d, PF.wi_d)

/* ------------------------------------------------------------------------ */
/* pocketfft T_dcst23<T>::exec, N=8, cosine, ortho, fct = 1/sqrt(2N) = 0.25  */
/* ------------------------------------------------------------------------ */
#define DEF_DCST23(T, SFX)                                                     \
void vcfo_dct2_8_##SFX(T c[8])   /* scipy.fftpack.dct(x, 2, norm='ortho') */   \
{                                                                              \
    pf_init();                                                                 \
    const T *tw = (const T *)PF.tw_##SFX##_arr;                                \
    c[0] *= (T)2;                                                              \
    c[7] *= (T)2;                                                              \
    for (int k = 1; k < 7; k += 2) { T t = c[k + 1]; c[k + 1] -= c[k]; c[k] += t; } \
    rfftb8_##SFX(c);                                                           \
    for (int k = 0; k < 8; ++k) c[k] = (T)0.25 * c[k];                         \
    for (int k = 1, kc = 7; k < 4; ++k, --kc) {                                \
        T t1 = tw[k - 1] * c[kc] + tw[kc - 1] * c[k];                          \
        T t2 = tw[k - 1] * c[k] - tw[kc - 1] * c[kc];                          \
        c[k] = (T)0.5 * (t1 + t2); c[kc] = (T)0.5 * (t1 - t2);                 \
    }                                                                          \
    c[4] *= tw[3];                                                             \
    c[0] *= PF.sqrt2_##SFX##_v * (T)0.5;                                       \
}                                                                              \
void vcfo_dct3_8_##SFX(T c[8])   /* scipy.fftpack.idct(x, 2, norm='ortho') */  \
{                                                                              \
    pf_init();                                                                 \
    const T *tw = (const T *)PF.tw_##SFX##_arr;                                \
    c[0] *= PF.sqrt2_##SFX##_v;                                                \
    for (int k = 1, kc = 7; k < 4; ++k, --kc) {                                \
        T t1 = c[k] + c[kc], t2 = c[k] - c[kc];                                \
        c[k] = tw[k - 1] * t2 + tw[kc - 1] * t1;                               \
        c[kc] = tw[k - 1] * t1 - tw[kc - 1] * t2;                              \
    }                                                                          \
    c[4] *= (T)2 * tw[3];                                                      \
    rfftf8_##SFX(c);                                                           \
    for (int k = 0; k < 8; ++k) c[k] = (T)0.25 * c[k];                         \
    for (int k = 1; k < 7; k += 2) { T t = c[k]; c[k] -= c[k + 1]; c[k + 1] += t; } \
}

#define tw_f32_arr tw_f
#define tw_f64_arr tw_d
#define sqrt2_f32_v sqrt2_f
#define sqrt2_f64_v sqrt2_d
DEF_DCST23(float, f32)
DEF_DCST23(double, f64)

/* exported for tests: the constants the restatement uses */
void vcfo_pocketfft_consts(float *tw_f, double *tw_d, float *rf, double *rd,
                           float *sqrt2_f, double *sqrt2_d)
{
    pf_init();
    memcpy(tw_f, PF.tw_f, sizeof(PF.tw_f));
    memcpy(tw_d, PF.tw_d, sizeof(PF.tw_d));
    rf[0] = PF.wr_f; rf[1] = PF.wi_f;
    rd[0] = PF.wr_d; rd[1] = PF.wi_d;
    *sqrt2_f = PF.sqrt2_f; *sqrt2_d = PF.sqrt2_d;
}

/* ------------------------------------------------------------------------ */
/* JPEG tables used by -p (2D-DCT.py:66-82), B = 8 only                      */
/* ------------------------------------------------------------------------ */
static const uint8_t Y_QSS[64] = {
    16, 11, 10, 16, 24, 40, 51, 61,   12, 12, 14, 19, 26, 58, 60, 55,
    14, 13, 16, 24, 40, 57, 69, 56,   14, 17, 22, 29, 51, 87, 80, 62,
    18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
static const uint8_t C_QSS[64] = {
    17, 18, 24, 47, 99, 99, 99, 99,   18, 21, 26, 66, 99, 99, 99, 99,
    24, 26, 56, 99, 99, 99, 99, 99,   47, 66, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99,   99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99,   99, 99, 99, 99, 99, 99, 99, 99};

/* numpy: uint8_table / 121 -> float64 (true_divide) */
static double pweight(int ch, int i, int j)
{
    return ch == 0 ? (double)Y_QSS[i * 8 + j] / 121.0 : (double)C_QSS[i * 8 + j] / 99.0;
}

void vcfo_perceptual_weights(double *w /* [3][8][8] */)
{
    for (int c = 0; c < 3; ++c)
        for (int i = 0; i < 64; ++i) w[c * 64 + i] = pweight(c, i / 8, i % 8);
}

/* numpy float64 -> int16 cast of an in-range-or-not value (x86: cvttsd2si to
 * int32, then keep the low 16 bits). */
static int16_t f64_to_i16(double v)
{
    int32_t i;
    if (v != v || v >= 2147483648.0 || v < -2147483648.0) i = INT32_MIN;
    else i = (int32_t)v;
    return (int16_t)i;
}

static int16_t f32_to_i16(float v) { return f64_to_i16((double)v); }

/* ------------------------------------------------------------------------ */
/* Frame encode: 2D-DCT.py:268-361 (everything up to the entropy codec)      */
/* ------------------------------------------------------------------------ */
int vcfo_dct_dz_encode(const uint8_t *rgb, int H, int W, int Q, unsigned flags,
                       uint8_t *k_out /* Hp x Wp x 3 */)
{
    const int Bs = 8;
    if (H <= 0 || W <= 0 || Q <= 0) return -1;
    pf_init();
    const int Hp = (H + Bs - 1) / Bs * Bs, Wp = (W + Bs - 1) / Bs * Bs;
    const int top = (Hp - H) / 2, left = (Wp - W) / 2;
    const size_t npx = (size_t)Hp * Wp;
    float *img = (float *)malloc(npx * 3 * sizeof(float));
    float *dct = (float *)malloc(npx * 3 * sizeof(float));
    if (!img || !dct) { free(img); free(dct); return -2; }

    /* :276 astype(float32); :282 zero pad; :292 -= 128; :298 from_RGB (A4):
     * o0 = R/4 + G/2 + B/4 ; o1 = R/2 - B/2 ; o2 = -R/4 + G/2 - B/4 */
    for (int y = 0; y < Hp; ++y)
        for (int x = 0; x < Wp; ++x) {
            int sy = y - top, sx = x - left;
            float p[3] = {0.f, 0.f, 0.f};
            if (sy >= 0 && sy < H && sx >= 0 && sx < W)
                for (int c = 0; c < 3; ++c) p[c] = (float)rgb[((size_t)sy * W + sx) * 3 + c];
            float R = p[0] - 128.f, G = p[1] - 128.f, B = p[2] - 128.f;
            float *o = img + ((size_t)y * Wp + x) * 3;
            o[0] = (R / 4.f + G / 2.f) + B / 4.f;
            o[1] = R / 2.f - B / 2.f;
            o[2] = ((-R) / 4.f + G / 2.f) - B / 4.f;
        }

    /* :303 analyze_image (A1): per block, per channel, axis 0 then axis 1 */
    for (int by = 0; by < Hp; by += Bs)
        for (int bx = 0; bx < Wp; bx += Bs)
            for (int c = 0; c < 3; ++c) {
                float b[8][8];
                for (int y = 0; y < 8; ++y)
                    for (int x = 0; x < 8; ++x) b[y][x] = img[((size_t)(by + y) * Wp + bx + x) * 3 + c];
                for (int x = 0; x < 8; ++x) {
                    float v[8];
                    for (int y = 0; y < 8; ++y) v[y] = b[y][x];
                    vcfo_dct2_8_f32(v);
                    for (int y = 0; y < 8; ++y) b[y][x] = v[y];
                }
                for (int y = 0; y < 8; ++y) vcfo_dct2_8_f32(b[y]);
                /* :313-327 -p: block[..., c] *= table/121|99 (float32 *= float64) */
                for (int y = 0; y < 8; ++y)
                    for (int x = 0; x < 8; ++x) {
                        float v = b[y][x];
                        if (flags & VCFO_FLAG_PERCEPTUAL) v = (float)((double)v * pweight(c, y, x));
                        dct[((size_t)(by + y) * Wp + bx + x) * 3 + c] = v;
                    }
            }

    /* :333-336 get_subbands (A3), :343 quantize (A5), :348 +128, :361 uint8 */
    const int sy = Hp / Bs, sx = Wp / Bs;
    for (int y = 0; y < Hp; ++y)
        for (int x = 0; x < Wp; ++x) {
            int dy = y, dx = x;   /* destination of coefficient at (y, x) */
            if (!(flags & VCFO_FLAG_NO_SUBBANDS)) {
                int i = y % Bs, by = y / Bs, j = x % Bs, bx = x / Bs;
                dy = i * sy + by; dx = j * sx + bx;
            }
            for (int c = 0; c < 3; ++c) {
                float v = dct[((size_t)y * Wp + x) * 3 + c];
                float q = v / (float)Q;               /* float32 / int -> float32 */
                int32_t k = (int32_t)q;               /* astype(int32): trunc    */
                k += 128;
                k_out[((size_t)dy * Wp + dx) * 3 + c] = (uint8_t)(k & 0xff);
            }
        }
    free(img); free(dct);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Frame decode: 2D-DCT.py:377-466 (everything after the entropy decoder)    */
/* ------------------------------------------------------------------------ */
int vcfo_dct_dz_decode(const uint8_t *k_in /* Hp x Wp x 3 */, int H, int W, int Q,
                       unsigned flags, uint8_t *rgb_out /* H x W x 3 */)
{
    const int Bs = 8;
    if (H <= 0 || W <= 0 || Q <= 0 || Q > 32767) return -1;
    pf_init();
    const int Hp = (H + Bs - 1) / Bs * Bs, Wp = (W + Bs - 1) / Bs * Bs;
    const int top = (Hp - H) / 2, left = (Wp - W) / 2;
    const size_t npx = (size_t)Hp * Wp;
    int16_t *blk = (int16_t *)malloc(npx * 3 * sizeof(int16_t));
    int16_t *ct = (int16_t *)malloc(npx * 3 * sizeof(int16_t));
    if (!blk || !ct) { free(blk); free(ct); return -2; }

    /* :399 astype(int16); :403 -= 128; :411 Q*k (int16, wraps); :416 get_blocks */
    const int sy = Hp / Bs, sx = Wp / Bs;
    for (int y = 0; y < Hp; ++y)
        for (int x = 0; x < Wp; ++x) {
            int dy = y, dx = x;   /* block-domain destination of subband sample (y, x) */
            if (!(flags & VCFO_FLAG_NO_SUBBANDS)) {
                int i = y / sy, by = y % sy, j = x / sx, bx = x % sx;
                dy = by * Bs + i; dx = bx * Bs + j;
            }
            for (int c = 0; c < 3; ++c) {
                int16_t k = (int16_t)((int16_t)k_in[((size_t)y * Wp + x) * 3 + c] - 128);
                int16_t v = (int16_t)(Q * (int32_t)k);
                blk[((size_t)dy * Wp + dx) * 3 + c] = v;
            }
        }

    /* :421-435 -p: float32 block /= table (float64), stored back into int16;
     * :440 synthesize_image (A2): idct on int16 -> float64, stored into int16 */
    for (int by = 0; by < Hp; by += Bs)
        for (int bx = 0; bx < Wp; bx += Bs)
            for (int c = 0; c < 3; ++c) {
                double b[8][8];
                for (int y = 0; y < 8; ++y)
                    for (int x = 0; x < 8; ++x) {
                        int16_t v = blk[((size_t)(by + y) * Wp + bx + x) * 3 + c];
                        if (flags & VCFO_FLAG_PERCEPTUAL)
                            v = f32_to_i16((float)((double)(float)v / pweight(c, y, x)));
                        b[y][x] = (double)v;
                    }
                for (int x = 0; x < 8; ++x) {
                    double v[8];
                    for (int y = 0; y < 8; ++y) v[y] = b[y][x];
                    vcfo_dct3_8_f64(v);
                    for (int y = 0; y < 8; ++y) b[y][x] = v[y];
                }
                for (int y = 0; y < 8; ++y) vcfo_dct3_8_f64(b[y]);
                for (int y = 0; y < 8; ++y)
                    for (int x = 0; x < 8; ++x)
                        ct[((size_t)(by + y) * Wp + bx + x) * 3 + c] = f64_to_i16(b[y][x]);
            }

    /* :444 remove_padding; :449 to_RGB (A4, int16); :454 += 128; :466 clip, u8 */
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const int16_t *p = ct + ((size_t)(y + top) * Wp + x + left) * 3;
            int16_t Y = p[0], Co = p[1], Cg = p[2];
            int16_t r = (int16_t)((int16_t)(Y + Co) - Cg);
            int16_t g = (int16_t)(Y + Cg);
            int16_t b = (int16_t)((int16_t)(Y - Co) - Cg);
            int16_t o[3] = {(int16_t)(r + 128), (int16_t)(g + 128), (int16_t)(b + 128)};
            for (int c = 0; c < 3; ++c) {
                int v = o[c] < 0 ? 0 : (o[c] > 255 ? 255 : o[c]);
                rgb_out[((size_t)y * W + x) * 3 + c] = (uint8_t)v;
            }
        }
    free(blk); free(ct);
    return 0;
}
