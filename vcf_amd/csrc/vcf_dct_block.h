// vcf_dct_block.h -- per-8x8-block arithmetic of the DCT+deadzone kernels.
//
// Host+device so that tests/cpu can compile exactly this code with g++ and
// check it against the oracle on a CPU-only machine; the kernels in
// vcf_dct_dz.hip only add the memory movement around it.
//
// encode (one channel C of one block; src/2D-DCT.py:276-361):
//   u8 RGB -> (R-128, G-128, B-128) -> YCoCg (A4, scaled to integers)
//   -> dct2_8r on columns then rows (A1) -> [-p weight] -> / (Q * 2^e)
//   -> trunc -> +128 -> u8 (wraps)
// decode (src/2D-DCT.py:399-454):
//   u8 -> int16 - 128 -> Q*k in int16 (A5) -> [-p de-weight] -> float64
//   -> dct3_8r on columns then rows (A2) -> * 1/16 -> trunc -> int16
//   -> to_RGB in int16 (A4) -> +128 -> clip to u8
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "vcf_dct8.h"

#if defined(__HIP_DEVICE_COMPILE__)
// An empty asm that makes `x` look redefined: blocks CSE / sinking across it.
#define VCF_OPAQUE(x) asm volatile("" : "+v"(x))
// Keep the machine scheduler from interleaving independent phases (it
// otherwise overlaps all eight column transforms and spills).
#define VCF_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define VCF_OPAQUE(x) ((void)0)
#define VCF_SCHED_FENCE() ((void)0)
#endif

#if defined(__HIPCC__)
#define VCF_HD_HOST __host__
#else
#define VCF_HD_HOST
#endif

namespace vcf {

// JPEG tables of -p (2D-DCT.py:66-82)
constexpr unsigned char kYQ[64] = {
    16, 11, 10, 16, 24, 40, 51, 61,   12, 12, 14, 19, 26, 58, 60, 55,
    14, 13, 16, 24, 40, 57, 69, 56,   14, 17, 22, 29, 51, 87, 80, 62,
    18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
constexpr unsigned char kCQ[64] = {
    17, 18, 24, 47, 99, 99, 99, 99,   18, 21, 26, 66, 99, 99, 99, 99,
    24, 26, 56, 99, 99, 99, 99, 99,   47, 66, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99,   99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99,   99, 99, 99, 99, 99, 99, 99, 99};

// numpy: uint8 table / 121 (or 99) -> float64
template <int C>
VCF_HD double pweight(int n)
{
    return C == 0 ? (double)kYQ[n] / 121.0 : (double)kCQ[n] / 99.0;
}

VCF_HD uint32_t byte_of(const uint32_t (&row)[6], int n)
{
    return (row[n >> 2] >> ((n & 3) * 8)) & 0xffu;
}

// YCoCg of (R-128, G-128, B-128) scaled to integers: 4Y, 2Co, 4Cg (exact)
template <int C>
VCF_HD float ycocg_scaled(uint32_t r, uint32_t g, uint32_t b)
{
    if (C == 0) return (float)((int)r + 2 * (int)g + (int)b - 512);
    if (C == 1) return (float)((int)r - (int)b);
    return (float)(2 * (int)g - (int)r - (int)b);
}

// log2 of the quantizer divisor's power of two: channel scale (4, 2, 4) times
// 1/(s_i s_j) of the reduced DCT-II.  Ranges over 3..6.
template <int C>
VCF_HD constexpr int qexp(int i, int j)
{
    return (C == 1 ? 1 : 2) + dct2_inv_scale_log2(i) + dct2_inv_scale_log2(j);
}

// qd[e-3] = Q*2^e (general Q, correctly rounded division) or 2^-e/Q (power-of-two Q)
template <bool POW2>
VCF_HD float quant_div(float t, float d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return POW2 ? t * d : __fdiv_rn(t, d);
#else
    return POW2 ? t * d : t / d;
#endif
}

// Order the eight 1-D transforms of a pass one after another: `dep` is an
// output of the previous transform, and the empty asm makes this transform's
// inputs depend on it.  Without it the compiler overlaps all eight (plus the
// other channels) for ILP and spills; with it a block channel needs about
// 64 + 16 registers and the wave scheduler supplies the overlap instead.
template <typename T>
VCF_HD void chain8(T (&c)[8], T dep)
{
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]),
                 "+v"(c[6]), "+v"(c[7]) : "v"(dep));
#else
    (void)c;
    (void)dep;
#endif
}

// Order groups of ILP 1-D transforms one after another (see chain8); within
// a group the ILP transforms are independent, so the compiler interleaves them.
template <int ILP>
VCF_HD void chain_group(float (*cols)[8], float dep)
{
    if (ILP == 1) {
        chain8(cols[0], dep);
    } else {
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+v"(cols[0][0]), "+v"(cols[0][1]), "+v"(cols[0][2]), "+v"(cols[0][3]),
                     "+v"(cols[0][4]), "+v"(cols[0][5]), "+v"(cols[0][6]), "+v"(cols[0][7]),
                     "+v"(cols[1][0]), "+v"(cols[1][1]), "+v"(cols[1][2]), "+v"(cols[1][3]),
                     "+v"(cols[1][4]), "+v"(cols[1][5]), "+v"(cols[1][6]), "+v"(cols[1][7])
                     : "v"(dep));
#endif
        if (ILP == 4) chain_group<2>(cols + 2, cols[1][0]);
    }
}

// One channel of one block -> 64 index bytes (k + 128) in (i*8 + j) order,
// packed four per word (byte n in bits 8*(n&3) of K[n>>2]).
template <int C, bool POW2, bool PERC, int ILP = 1>
VCF_HD void encode_block_channel(const uint32_t (&raw)[8][6], const float (&qd)[4], uint32_t (&K)[16])
{
    float v[8][8];   // v[y][x]; after the column pass row i holds coefficient row i
    float dep = qd[0];
    // axis 0 (columns) first, then axis 1 (rows): dct(dct(b.T).T)
#pragma unroll
    for (int x0 = 0; x0 < 8; x0 += ILP) {
        float col[ILP][8];
#pragma unroll
        for (int u = 0; u < ILP; ++u)
#pragma unroll
            for (int y = 0; y < 8; ++y)
                col[u][y] = ycocg_scaled<C>(byte_of(raw[y], 3 * (x0 + u)), byte_of(raw[y], 3 * (x0 + u) + 1),
                                            byte_of(raw[y], 3 * (x0 + u) + 2));
        // (the asm also hides that these are small integers: LLVM would
        // otherwise turn the first butterflies into integer adds across columns)
        chain_group<ILP>(col, dep);
#pragma unroll
        for (int u = 0; u < ILP; ++u) dct2_8r(col[u]);
#pragma unroll
        for (int u = 0; u < ILP; ++u)
#pragma unroll
            for (int y = 0; y < 8; ++y) v[y][x0 + u] = col[u][y];
        dep = col[ILP - 1][0];
    }
#pragma unroll
    for (int i0 = 0; i0 < 8; i0 += ILP) {
        chain_group<ILP>(&v[i0], dep);
#pragma unroll
        for (int u = 0; u < ILP; ++u) dct2_8r(v[i0 + u]);
        dep = v[i0 + ILP - 1][0];
#pragma unroll
        for (int i = i0; i < i0 + ILP; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float t = v[i][j];
                if (PERC) t = (float)((double)t * pweight<C>(i * 8 + j));
                const float q = quant_div<POW2>(t, qd[qexp<C>(i, j) - 3]);
                const int k = (int)q;   // astype(int32): truncation toward zero
                const uint32_t b = (uint32_t)(k + 128) & 0xffu;   // += 128, astype(uint8)
                const int n = i * 8 + j;
                K[n >> 2] = (n & 3) ? (K[n >> 2] | (b << (8 * (n & 3)))) : b;
                // pin the finished word here (volatile asms keep program order):
                // otherwise the quantization is sunk to the word's far-away use
                // and 64 coefficients stay live through the next channels
                if ((n & 3) == 3) VCF_OPAQUE(K[n >> 2]);
            }
    }
}

// ---------------------------------------------------------------------------
// Conversion-free variant (the float<->int conversions are quarter-rate on
// gfx950 and were ~15% of the block's VALU time):
//   * int -> float: the float with bits 0x4B000000 + n is 2^23 + n exactly,
//     so (bits(n + magic) - (2^23 + bias)) is n - bias in one full-rate sub;
//   * float -> byte: trunc(q) + (3*2^22 + 128) lies in [2^23, 2^24) for
//     |q| < 2^22, where the float's bit pattern is 0x4B000000 + 2^22 + 128 +
//     trunc(q): its low byte is (trunc(q) + 128) mod 256, exactly
//     astype(int32) + 128 -> astype(uint8).  The byte is stored straight from
//     that register.
// ---------------------------------------------------------------------------
VCF_HD float bits_as_float(uint32_t u)
{
#if defined(__HIPCC__)
    return __uint_as_float(u);
#else
    float f;
    memcpy(&f, &u, 4);
    return f;
#endif
}

VCF_HD uint32_t float_bits(float f)
{
#if defined(__HIPCC__)
    return __float_as_uint(f);
#else
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
#endif
}

constexpr uint32_t kMagicI = 0x4B000000u;      // bits of 2^23
constexpr float kQuantMagic = 12583040.0f;     // 3*2^22 + 128

// 4Y, 2Co, 4Cg of (R-128, G-128, B-128) as floats, without a conversion
template <int C>
VCF_HD float ycocg_magic(uint32_t r, uint32_t g, uint32_t b)
{
    if (C == 0) return bits_as_float(kMagicI + r + 2 * g + b) - (8388608.0f + 512.0f);
    if (C == 1) return bits_as_float(kMagicI + 256u + r - b) - (8388608.0f + 256.0f);
    return bits_as_float(kMagicI + 512u + 2 * g - r - b) - (8388608.0f + 512.0f);
}

VCF_HD float trunc_f(float x)
{
#if defined(__HIPCC__)
    return __builtin_truncf(x);
#else
    return truncf(x);
#endif
}

// One channel of one block; sink(i, j, word) receives each coefficient's
// index byte in the low 8 bits of `word`, row by row as the rows finish.
// ILP transforms of a pass are issued as one group (see chain_group): enough
// independent work per wave to cover the VALU dependency latency.
template <int C, bool POW2, bool PERC, int ILP = 1, typename Sink>
VCF_HD void encode_block_channel_bytes(const uint32_t (&raw)[8][6], const float (&qd)[4], Sink &&sink)
{
    float v[8][8];
    float dep = qd[0];
#pragma unroll
    for (int x0 = 0; x0 < 8; x0 += ILP) {
        float col[ILP][8];
#pragma unroll
        for (int u = 0; u < ILP; ++u)
#pragma unroll
            for (int y = 0; y < 8; ++y)
                col[u][y] = ycocg_magic<C>(byte_of(raw[y], 3 * (x0 + u)), byte_of(raw[y], 3 * (x0 + u) + 1),
                                           byte_of(raw[y], 3 * (x0 + u) + 2));
        chain_group<ILP>(col, dep);
#pragma unroll
        for (int u = 0; u < ILP; ++u) dct2_8r(col[u]);
#pragma unroll
        for (int u = 0; u < ILP; ++u)
#pragma unroll
            for (int y = 0; y < 8; ++y) v[y][x0 + u] = col[u][y];
        dep = col[ILP - 1][0];
    }
#pragma unroll
    for (int i0 = 0; i0 < 8; i0 += ILP) {
        chain_group<ILP>(&v[i0], dep);
#pragma unroll
        for (int u = 0; u < ILP; ++u) dct2_8r(v[i0 + u]);
        dep = v[i0 + ILP - 1][0];
#pragma unroll
        for (int i = i0; i < i0 + ILP; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float t = v[i][j];
                if (PERC) t = (float)((double)t * pweight<C>(i * 8 + j));
                const float q = quant_div<POW2>(t, qd[qexp<C>(i, j) - 3]);
                sink(i, j, float_bits(trunc_f(q) + kQuantMagic));
            }
    }
}

// ---------------------------------------------------------------------------
// Fetch-lean encode body (v6).  The tile kernel is bound by instruction fetch
// (SQC busy ~100 %, no misses) at ~5.7 code bytes per instruction, so:
//   * every constant (pocketfft twiddles, quantizer multipliers, magics, dot
//     weights) comes from a kernel-argument struct, i.e. an SGPR operand
//     instead of a 32-bit literal: the DCT's multiplies stay 4-byte VOP2;
//   * YCoCg is one or two v_dot4 of the signed bytes (RGB - 128) per sample
//     (the raw words are XORed with 0x80808080 once), accumulated onto
//     2^23 + bias and turned into a float by one subtraction (see above).
// ---------------------------------------------------------------------------
struct EncConsts {
    float tw[7];      // pocketfft DCT-II twiddles (fp32)
    float hf;         // rfft8 twiddle = sqrt2/2 (fp32)
    float hfx2, tw3x2; // 2*hf, 2*tw[3] (exact): column pass of the column-per-lane kernel
    float qd[4];      // quantizer divisors Q*2^e or, for power-of-two Q, 2^-e/Q
    float qmagic;     // 3*2^22 + 128
    float csub[3];    // 2^23 + 1024 per channel (what the dot accumulator's float is offset by)
    uint32_t cinit;   // bits of 2^23 + 1024: the dot accumulator's start value
    uint32_t w[3][6]; // per channel: dot weights of the six byte patterns of a 24-byte row
};

#define VCF_K_TW(k, i) (k).tw[i]

// DCT-II of dct2_8r with the constants taken from K (bit-identical ops)
VCF_HD void dct2_8k(float (&c)[8], const EncConsts &K)
{
    const float x1 = c[1] + c[2], x2 = c[2] - c[1];
    const float x3 = c[3] + c[4], x7 = c[3] - c[4];
    const float x5 = c[5] + c[6], x6 = c[6] - c[5];
    const float a0 = c[0] + c[7], a4 = c[0] - c[7];
    const float a1 = x1 + x5, tr2 = x1 - x5;
    const float ti2 = x2 + x6, a2 = x2 - x6;
    const float a6 = K.hf * ti2 + K.hf * tr2;
    const float a5 = K.hf * tr2 - K.hf * ti2;
    const float T2 = a0 + x3, T1 = a0 - x3;
    const float r0 = T2 + a1, r4 = T2 - a1, r6 = T1 + a2, r2 = T1 - a2;
    const float U2 = a4 + x7, U1 = a4 - x7;
    const float r1 = U2 + a5, r5 = U2 - a5, r7 = U1 + a6, r3 = U1 - a6;
    float t1, t2;
    t1 = K.tw[0] * r7 + K.tw[6] * r1; t2 = K.tw[0] * r1 - K.tw[6] * r7;
    c[1] = t1 + t2; c[7] = t1 - t2;
    t1 = K.tw[1] * r6 + K.tw[5] * r2; t2 = K.tw[1] * r2 - K.tw[5] * r6;
    c[2] = t1 + t2; c[6] = t1 - t2;
    t1 = K.tw[2] * r5 + K.tw[4] * r3; t2 = K.tw[2] * r3 - K.tw[4] * r5;
    c[3] = t1 + t2; c[5] = t1 - t2;
    c[4] = r4 * K.tw[3];
    c[0] = r0 * K.hf;
}

// Column pass of the column-per-lane kernel: dct2_8k with outputs 0 and 4
// doubled (2*hf, 2*tw3 are exact), so all eight outputs carry the scale 1/4.
VCF_HD void dct2_8k_colpass(float (&c)[8], const EncConsts &K)
{
    const float x1 = c[1] + c[2], x2 = c[2] - c[1];
    const float x3 = c[3] + c[4], x7 = c[3] - c[4];
    const float x5 = c[5] + c[6], x6 = c[6] - c[5];
    const float a0 = c[0] + c[7], a4 = c[0] - c[7];
    const float a1 = x1 + x5, tr2 = x1 - x5;
    const float ti2 = x2 + x6, a2 = x2 - x6;
    const float a6 = K.hf * ti2 + K.hf * tr2;
    const float a5 = K.hf * tr2 - K.hf * ti2;
    const float T2 = a0 + x3, T1 = a0 - x3;
    const float r0 = T2 + a1, r4 = T2 - a1, r6 = T1 + a2, r2 = T1 - a2;
    const float U2 = a4 + x7, U1 = a4 - x7;
    const float r1 = U2 + a5, r5 = U2 - a5, r7 = U1 + a6, r3 = U1 - a6;
    float t1, t2;
    t1 = K.tw[0] * r7 + K.tw[6] * r1; t2 = K.tw[0] * r1 - K.tw[6] * r7;
    c[1] = t1 + t2; c[7] = t1 - t2;
    t1 = K.tw[1] * r6 + K.tw[5] * r2; t2 = K.tw[1] * r2 - K.tw[5] * r6;
    c[2] = t1 + t2; c[6] = t1 - t2;
    t1 = K.tw[2] * r5 + K.tw[4] * r3; t2 = K.tw[2] * r3 - K.tw[4] * r5;
    c[3] = t1 + t2; c[5] = t1 - t2;
    c[4] = r4 * K.tw3x2;
    c[0] = r0 * K.hfx2;
}

// -p weight with a runtime table index (column-per-lane kernel: row = lane)
VCF_HD double pweight_rt(int C, int n)
{
    return C == 0 ? (double)kYQ[n] / 121.0 : (double)kCQ[n] / 99.0;
}

VCF_HD int sdot4(uint32_t a, uint32_t b, int c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
#else
    int s = c;
    for (int k = 0; k < 4; ++k) s += (int)(int8_t)(a >> (8 * k)) * (int)(int8_t)(b >> (8 * k));
    return s;
#endif
}

// Weights of channel C (4Y = R'+2G'+B', 2Co = R'-B', 4Cg = -R'+2G'-B') laid
// on the six byte patterns of a row: pixel p occupies bytes 3p..3p+2.
VCF_HD_HOST inline void make_enc_consts(EncConsts &K, int Q)
{
    K.tw[0] = VCF_TWF0; K.tw[1] = VCF_TWF1; K.tw[2] = VCF_TWF2; K.tw[3] = VCF_TWF3;
    K.tw[4] = VCF_TWF4; K.tw[5] = VCF_TWF5; K.tw[6] = VCF_TWF6; K.hf = VCF_HF;
    K.hfx2 = 2.0f * VCF_HF;
    K.tw3x2 = 2.0f * VCF_TWF3;
    const bool pow2 = (Q & (Q - 1)) == 0;
    for (int e = 0; e < 4; ++e) {
        const double D = (double)Q * (double)(1 << (e + 3));
        K.qd[e] = pow2 ? (float)(1.0 / D) : (float)D;
    }
    K.qmagic = 12583040.0f;
    K.cinit = 0x4B000000u + 1024u;
    for (int c = 0; c < 3; ++c) K.csub[c] = 8388608.0f + 1024.0f;
    const int wt[3][3] = {{1, 2, 1}, {1, 0, -1}, {-1, 2, -1}};
    for (int c = 0; c < 3; ++c) {
        auto wb = [&](int comp) { return (uint32_t)(uint8_t)(int8_t)wt[c][comp]; };
        // A=[R,G,B,0] B1=[0,0,0,R] B2=[G,B,0,0] C1=[0,0,R,G] C2=[B,0,0,0] D=[0,R,G,B]
        K.w[c][0] = wb(0) | (wb(1) << 8) | (wb(2) << 16);
        K.w[c][1] = wb(0) << 24;
        K.w[c][2] = wb(1) | (wb(2) << 8);
        K.w[c][3] = (wb(0) << 16) | (wb(1) << 24);
        K.w[c][4] = wb(2);
        K.w[c][5] = (wb(0) << 8) | (wb(1) << 16) | (wb(2) << 24);
    }
}

// channel-C value of pixel x of a row whose six words hold the signed bytes
// (R-128, G-128, B-128): 4Y, 2Co or 4Cg as an exact float
template <int C>
VCF_HD float ycocg_dot(const uint32_t (&row)[6], int x, const EncConsts &K)
{
    const int q = x >> 2, p = x & 3;   // pixels 4q..4q+3 live in words 3q..3q+2
    int acc;
    if (p == 0) acc = sdot4(row[3 * q], K.w[C][0], (int)K.cinit);
    else if (p == 1) acc = sdot4(row[3 * q + 1], K.w[C][2], sdot4(row[3 * q], K.w[C][1], (int)K.cinit));
    else if (p == 2) acc = sdot4(row[3 * q + 2], K.w[C][4], sdot4(row[3 * q + 1], K.w[C][3], (int)K.cinit));
    else acc = sdot4(row[3 * q + 2], K.w[C][5], (int)K.cinit);
    return bits_as_float((uint32_t)acc) - K.csub[C];
}

// v6 channel body: columns then rows, sink(i, j, word) as in
// encode_block_channel_bytes; raw holds the signed bytes (raw ^ 0x80808080).
template <int C, bool POW2, bool PERC, typename Sink>
VCF_HD void encode_block_channel_v6(const uint32_t (&raw)[8][6], const EncConsts &K, Sink &&sink)
{
    float v[8][8];
    float dep = K.qd[0];
#pragma unroll
    for (int x = 0; x < 8; ++x) {
        float col[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) col[y] = ycocg_dot<C>(raw[y], x, K);
        chain8(col, dep);
        dct2_8k(col, K);
#pragma unroll
        for (int y = 0; y < 8; ++y) v[y][x] = col[y];
        dep = col[0];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        chain8(v[i], dep);
        dct2_8k(v[i], K);
        dep = v[i][0];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float t = v[i][j];
            if (PERC) t = (float)((double)t * pweight<C>(i * 8 + j));
            const float q = quant_div<POW2>(t, K.qd[qexp<C>(i, j) - 3]);
            sink(i, j, float_bits(trunc_f(q) + K.qmagic));
        }
    }
}

// ---------------------------------------------------------------------------
// "Folded" channel body (encode variants 1 and 2).  For a power-of-two Q the
// quantizer divisor Q * 2^e, e = chs + inv(i) + inv(j), is a power of two,
// and every DCT output leaves its pass through one final multiplication
// (t1 +- t2 with t = tw*r +- tw*r, or r*tw3, r*hf), so the division folds
// into those final constants exactly: the column pass's by 2^-(chs+inv(i))
// (compile-time literals), the row pass's by 2^-(inv(j)+log2 Q) (kernel
// arguments -> SGPR operands).  The row pass then yields x / Q / 2^e itself;
// one v_cvt_i32_f32 (truncation toward zero = astype(int32)) gives k, whose
// low byte goes to the sink; the +128 of 2D-DCT.py:348 is applied later to
// whole words (XOR 0x80 per byte == +128 mod 256).  Non-power-of-two Q keeps
// the unscaled transforms and a correctly rounded division.
// ---------------------------------------------------------------------------
struct FinalK {
    float p0a, p0b;   // tw0, tw6 -> outputs 1, 7
    float p1a, p1b;   // tw1, tw5 -> outputs 2, 6
    float p2a, p2b;   // tw2, tw4 -> outputs 3, 5
    float s4, s0;     // tw3 -> output 4, hf -> output 0
};

VCF_HD constexpr FinalK final_k(float pair_scale, float single_scale)
{
    return FinalK{VCF_TWF0 * pair_scale, VCF_TWF6 * pair_scale, VCF_TWF1 * pair_scale, VCF_TWF5 * pair_scale,
                  VCF_TWF2 * pair_scale, VCF_TWF4 * pair_scale, VCF_TWF3 * single_scale, VCF_HF * single_scale};
}

// dct2_8r with caller-chosen final multipliers (see above).  T = float, or
// (device) a 2-vector of floats: two independent transforms in lock step,
// which clang issues as packed v_pk_add_f32 / v_pk_mul_f32 -- each element
// sees the same IEEE operations in the same order, so the results are the
// scalar ones bit for bit.
template <typename T>
VCF_HD void dct2_8f(T (&c)[8], const FinalK &k)
{
    const T x1 = c[1] + c[2], x2 = c[2] - c[1];
    const T x3 = c[3] + c[4], x7 = c[3] - c[4];
    const T x5 = c[5] + c[6], x6 = c[6] - c[5];
    const T a0 = c[0] + c[7], a4 = c[0] - c[7];
    const T a1 = x1 + x5, tr2 = x1 - x5;
    const T ti2 = x2 + x6, a2 = x2 - x6;
    const T a6 = VCF_HF * ti2 + VCF_HF * tr2;
    const T a5 = VCF_HF * tr2 - VCF_HF * ti2;
    const T T2 = a0 + x3, T1 = a0 - x3;
    const T r0 = T2 + a1, r4 = T2 - a1, r6 = T1 + a2, r2 = T1 - a2;
    const T U2 = a4 + x7, U1 = a4 - x7;
    const T r1 = U2 + a5, r5 = U2 - a5, r7 = U1 + a6, r3 = U1 - a6;
    T t1, t2;
    t1 = k.p0a * r7 + k.p0b * r1; t2 = k.p0a * r1 - k.p0b * r7;
    c[1] = t1 + t2; c[7] = t1 - t2;
    t1 = k.p1a * r6 + k.p1b * r2; t2 = k.p1a * r2 - k.p1b * r6;
    c[2] = t1 + t2; c[6] = t1 - t2;
    t1 = k.p2a * r5 + k.p2b * r3; t2 = k.p2a * r3 - k.p2b * r5;
    c[3] = t1 + t2; c[5] = t1 - t2;
    c[4] = r4 * k.s4;
    c[0] = r0 * k.s0;
}

VCF_HD int cvt_trunc_i32(float q)
{
    return (int)q;   // v_cvt_i32_f32: rounds toward zero, like astype(int32)
}

// Row-pass final constants for a power-of-two Q (kernel argument).
VCF_HD_HOST inline FinalK row_final_k(int Q)
{
    int l = 0;
    while ((1 << l) < Q) ++l;
    const float s = 1.0f / (float)(1u << l);   // exact
    return final_k(0.25f * s, 0.5f * s);       // 2^-(inv(j) + log2 Q)
}

// ---- YCoCg straight from the packed bytes with SDWA byte operands --------
// A VOP2 SDWA instruction reads any byte of either source register as a
// zero-extended operand, so byte extraction costs nothing:
//   4Y  bits = magic + r + b + 2g : lshl_sdwa(2g), add_sdwa(r + b), add3  (3)
//   2Co bits = magic + r - b      : add_sdwa(magic + r), sub_sdwa(.. - b) (2)
//   4Cg bits = magic - (r+b) + 2g : add_sdwa(r + b), sub, add_sdwa(+g) x2 (4)
// each followed by one float subtraction of the magic (2^23 + centring),
// 12 VALU per pixel where the generic byte code needs about 17.
template <int SEL>
VCF_HD uint32_t byte_sel(uint32_t w)
{
    return (w >> (8 * SEL)) & 0xffu;
}

// VCF_SDWA_ASM (default 1): the byte-operand adds as inline SDWA asm; 0 leaves them to the
// compiler's SDWA peephole (A/B, DESIGN.md §6: the asm form costs a hazard s_nop after
// each block, the compiler's form more plain adds)
#ifndef VCF_SDWA_ASM
#define VCF_SDWA_ASM 1
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define VCF_SDWA_BODY(OP, S0, S1)                                                                    \
    asm(OP " %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:" S0 " src1_sel:" S1          \
        : "=v"(r) : "v"(a), "v"(b))
#define VCF_SDWA_SEL(OP, S0)                                                                         \
    if (B1 == 0) VCF_SDWA_BODY(OP, S0, "BYTE_0");                                                    \
    else if (B1 == 1) VCF_SDWA_BODY(OP, S0, "BYTE_1");                                               \
    else if (B1 == 2) VCF_SDWA_BODY(OP, S0, "BYTE_2");                                               \
    else VCF_SDWA_BODY(OP, S0, "BYTE_3");
#define VCF_SDWA_FN(OP)                                                                              \
    uint32_t r;                                                                                      \
    if (B0 < 0) { VCF_SDWA_SEL(OP, "DWORD") }                                                        \
    else if (B0 == 0) { VCF_SDWA_SEL(OP, "BYTE_0") }                                                 \
    else if (B0 == 1) { VCF_SDWA_SEL(OP, "BYTE_1") }                                                 \
    else if (B0 == 2) { VCF_SDWA_SEL(OP, "BYTE_2") }                                                 \
    else { VCF_SDWA_SEL(OP, "BYTE_3") }                                                              \
    return r;
#endif

// a[B0] + b[B1]; B0 < 0 takes all of a
template <int B0, int B1>
VCF_HD uint32_t add_sdwa(uint32_t a, uint32_t b)
{
#if defined(__HIP_DEVICE_COMPILE__) && VCF_SDWA_ASM
    VCF_SDWA_FN("v_add_u32_sdwa")
#else
    return (B0 < 0 ? a : byte_sel<(B0 < 0 ? 0 : B0)>(a)) + byte_sel<B1>(b);
#endif
}

// a[B0] - b[B1]
template <int B0, int B1>
VCF_HD uint32_t sub_sdwa(uint32_t a, uint32_t b)
{
#if defined(__HIP_DEVICE_COMPILE__) && VCF_SDWA_ASM
    VCF_SDWA_FN("v_sub_u32_sdwa")
#else
    return (B0 < 0 ? a : byte_sel<(B0 < 0 ? 0 : B0)>(a)) - byte_sel<B1>(b);
#endif
}

// b[B1] << 1  (src0 is the shift count)
template <int B1>
VCF_HD uint32_t twice_byte(uint32_t b)
{
#if defined(__HIP_DEVICE_COMPILE__) && VCF_SDWA_ASM
    constexpr int B0 = -1;
    const uint32_t a = 1;
    VCF_SDWA_FN("v_lshlrev_b32_sdwa")
#else
    return byte_sel<B1>(b) << 1;
#endif
}

// channel C of pixel x of a 24-byte row, scaled (4Y, 2Co, 4Cg) and centred
template <int C, int X>
VCF_HD float ycocg_sdwa(const uint32_t (&row)[6], uint32_t magic)
{
    constexpr int nr = 3 * X, ng = 3 * X + 1, nb = 3 * X + 2;
    const uint32_t wr = row[nr >> 2], wg = row[ng >> 2], wb = row[nb >> 2];
    if (C == 0) {
        const uint32_t rb = add_sdwa<nr & 3, nb & 3>(wr, wb);
        return bits_as_float(rb + twice_byte<ng & 3>(wg) + magic) - (8388608.0f + 512.0f);
    }
    if (C == 1) {
        const uint32_t t = add_sdwa<-1, nr & 3>(magic, wr);
        return bits_as_float(sub_sdwa<-1, nb & 3>(t, wb)) - (8388608.0f + 256.0f);
    }
    const uint32_t rb = add_sdwa<nr & 3, nb & 3>(wr, wb);
    const uint32_t t = add_sdwa<-1, ng & 3>(magic - rb, wg);
    return bits_as_float(add_sdwa<-1, ng & 3>(t, wg)) - (8388608.0f + 512.0f);
}

// the per-channel magic word: 2^23's bits plus the offset that keeps the
// integer non-negative (Co: r - b >= -255; Cg: 2g - r - b >= -510)
template <int C>
VCF_HD constexpr uint32_t ycocg_magic_word()
{
    return C == 0 ? kMagicI : C == 1 ? kMagicI + 256u : kMagicI + 512u;
}

template <int C, int X, bool SDWA>
VCF_HD void fold_columns(const uint32_t (&raw)[8][6], uint32_t magic, const FinalK &colk, float (&v)[8][8],
                         float &dep)
{
    if constexpr (X < 8) {
        float col[8];
#pragma unroll
        for (int y = 0; y < 8; ++y)
            col[y] = SDWA ? ycocg_sdwa<C, X>(raw[y], magic)
                          : ycocg_magic<C>(byte_of(raw[y], 3 * X), byte_of(raw[y], 3 * X + 1),
                                           byte_of(raw[y], 3 * X + 2));
        chain8(col, dep);
        dct2_8f(col, colk);
#pragma unroll
        for (int y = 0; y < 8; ++y) v[y][X] = col[y];
        dep = col[0];
        fold_columns<C, X + 1, SDWA>(raw, magic, colk, v, dep);
    }
}

template <int C, bool POW2, bool PERC, bool SDWA = false, typename Sink>
VCF_HD void encode_block_channel_fold(const uint32_t (&raw)[8][6], const FinalK &rowk, const float (&qd)[4],
                                      Sink &&sink)
{
    // column pass: 2^-(chs + inv(i)), chs = log2 of the channel scale (4Y, 2Co, 4Cg)
    constexpr float cs = C == 1 ? 0.5f : 0.25f;
    constexpr FinalK colk = POW2 ? final_k(cs * 0.25f, cs * 0.5f) : final_k(1.0f, 1.0f);
    float v[8][8];
    float dep = qd[0];
    uint32_t magic = ycocg_magic_word<C>();
    VCF_OPAQUE(magic);   // one VGPR, not a literal per use
    fold_columns<C, 0, SDWA>(raw, magic, colk, v, dep);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        chain8(v[i], dep);
        if (POW2) dct2_8f(v[i], rowk);
        else dct2_8r(v[i]);
        dep = v[i][0];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float t = v[i][j];
            if (PERC) t = (float)((double)t * pweight<C>(i * 8 + j));
            const float q = POW2 ? t : quant_div<false>(t, qd[qexp<C>(i, j) - 3]);
            sink(i, j, (uint32_t)cvt_trunc_i32(q));
        }
    }
}

#if defined(__HIPCC__)
// ---- packed-fp32 channel encoder (POW2 Q, no -p) --------------------------
// The same arithmetic as encode_block_channel_fold<C, true, false, true>, two
// 1-D transforms per instruction: the column pass runs pixel columns (x, x+1)
// as one float2 transform, a 2x2 transpose per (row pair, column pair)
// regroups the results as rows (i, i+1), and the row pass runs those row
// pairs.  Element for element the IEEE operations and their order are those
// of the scalar path (tests/test_dct_gpu.py checks every variant against the
// oracle), at about half the VALU instructions for the transforms.
typedef float vcf_f2 __attribute__((ext_vector_type(2)));
typedef uint32_t vcf_u2 __attribute__((ext_vector_type(2)));

// bits of (channel C of pixel X) + magic, before the float subtraction
template <int C, int X>
VCF_HD uint32_t ycocg_bits_sdwa(const uint32_t (&row)[6], uint32_t magic)
{
    constexpr int nr = 3 * X, ng = 3 * X + 1, nb = 3 * X + 2;
    const uint32_t wr = row[nr >> 2], wg = row[ng >> 2], wb = row[nb >> 2];
    if (C == 0) return add_sdwa<nr & 3, nb & 3>(wr, wb) + twice_byte<ng & 3>(wg) + magic;
    if (C == 1) return sub_sdwa<-1, nb & 3>(add_sdwa<-1, nr & 3>(magic, wr), wb);
    const uint32_t rb = add_sdwa<nr & 3, nb & 3>(wr, wb);
    return add_sdwa<-1, ng & 3>(add_sdwa<-1, ng & 3>(magic - rb, wg), wg);
}

template <int C, int XP>
VCF_HD void fold_columns_pk(const uint32_t (&raw)[8][6], uint32_t magic, const FinalK &colk,
                            vcf_f2 (&v)[8][4], vcf_f2 &dep)
{
    if constexpr (XP < 4) {
        constexpr float centre = C == 1 ? 8388608.0f + 256.0f : 8388608.0f + 512.0f;
        vcf_f2 col[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) {
            const vcf_u2 b = {ycocg_bits_sdwa<C, 2 * XP>(raw[y], magic),
                              ycocg_bits_sdwa<C, 2 * XP + 1>(raw[y], magic)};
            col[y] = __builtin_bit_cast(vcf_f2, b) - centre;
        }
        chain8(col, dep);
        dct2_8f(col, colk);
#pragma unroll
        for (int y = 0; y < 8; ++y) v[y][XP] = col[y];
        dep = col[0];
        fold_columns_pk<C, XP + 1>(raw, magic, colk, v, dep);
    }
}

template <int C, typename Sink>
VCF_HD void encode_block_channel_pk(const uint32_t (&raw)[8][6], const FinalK &rowk, float dep0, Sink &&sink)
{
    constexpr float cs = C == 1 ? 0.5f : 0.25f;
    constexpr FinalK colk = final_k(cs * 0.25f, cs * 0.5f);
    vcf_f2 v[8][4];
    vcf_f2 dep = {dep0, dep0};
    uint32_t magic = ycocg_magic_word<C>();
    VCF_OPAQUE(magic);
    fold_columns_pk<C, 0>(raw, magic, colk, v, dep);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        vcf_f2 r[8];
#pragma unroll
        for (int xp = 0; xp < 4; ++xp) {
            r[2 * xp] = __builtin_shufflevector(v[2 * p][xp], v[2 * p + 1][xp], 0, 2);
            r[2 * xp + 1] = __builtin_shufflevector(v[2 * p][xp], v[2 * p + 1][xp], 1, 3);
        }
        chain8(r, dep);
        dct2_8f(r, rowk);
        dep = r[0];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            sink(2 * p, j, (uint32_t)cvt_trunc_i32(r[j].x));
            sink(2 * p + 1, j, (uint32_t)cvt_trunc_i32(r[j].y));
        }
    }
}
#endif

VCF_HD uint32_t byte_at(const uint32_t (&K)[16], int n)
{
    return (K[n >> 2] >> (8 * (n & 3))) & 0xffu;
}

// One channel of one block: 64 index bytes in (i*8 + j) order -> 64 int16
// samples packed two per word (sample n in bits 16*(n&1) of word n>>1).
template <int C, bool PERC>
VCF_HD void decode_block_channel(const uint8_t (&kb)[64], int Q, uint32_t (&res)[32])
{
    double v[8][8];
#pragma unroll
    for (int n = 0; n < 64; ++n) {
        int16_t y = (int16_t)(Q * ((int)kb[n] - 128));   // int16(k) - 128, Q*k in int16
        if (PERC) {
            const float f = (float)((double)(float)y / pweight<C>(n));
            y = (int16_t)(int)f;
        }
        v[n >> 3][n & 7] = (double)y;
    }
#pragma unroll
    for (int x = 0; x < 8; ++x) {
        double col[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) col[y] = v[y][x];
        dct3_8r(col);
#pragma unroll
        for (int y = 0; y < 8; ++y) v[y][x] = col[y];
    }
#pragma unroll
    for (int y = 0; y < 8; ++y) dct3_8r(v[y]);
#pragma unroll
    for (int n = 0; n < 32; ++n) {
        // * 1/16 restores pocketfft's fct = 1/4 of both passes; float64 -> int16 truncates
        const uint32_t lo = (uint16_t)(int16_t)(int)(v[(2 * n) >> 3][(2 * n) & 7] * 0.0625);
        const uint32_t hi = (uint16_t)(int16_t)(int)(v[(2 * n + 1) >> 3][(2 * n + 1) & 7] * 0.0625);
        res[n] = lo | (hi << 16);
    }
    // materialise the packed samples here: otherwise the conversions are sunk
    // into the to_RGB stage and all 3 x 64 doubles stay live (spills)
#pragma unroll
    for (int n = 0; n < 32; ++n) VCF_OPAQUE(res[n]);
}

VCF_HD uint32_t clip_u8(int v)
{
    v = (int16_t)(v + 128);   // y += 128 in int16
    return (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

VCF_HD int sample_of(const uint32_t (&p)[32], int n)
{
    return (int16_t)(uint16_t)(p[n >> 1] >> ((n & 1) * 16));
}

// Pixel row y (0..7) of a decoded block -> 24 RGB bytes (as u32 values 0..255).
VCF_HD void to_rgb_row(const uint32_t (&Yv)[32], const uint32_t (&Co)[32], const uint32_t (&Cg)[32],
                       int y, uint32_t (&px)[24])
{
#pragma unroll
    for (int x = 0; x < 8; ++x) {
        const int n = y * 8 + x;
        const int yv = sample_of(Yv, n), co = sample_of(Co, n), cg = sample_of(Cg, n);
        // to_RGB (A4) in int16: R = Y + Co - Cg, G = Y + Cg, B = Y - Co - Cg
        px[3 * x + 0] = clip_u8((int16_t)(yv + co - cg));
        px[3 * x + 1] = clip_u8((int16_t)(yv + cg));
        px[3 * x + 2] = clip_u8((int16_t)(yv - co - cg));
    }
    // ROCm 7.2 / gfx950 miscompile: clamp-to-u8 of two values followed by the
    // byte packing in the caller is selected as v_ashr_pk_u8_i32 and the
    // packed word's upper half leaks into byte 2 (wrong pixels at every 4th
    // byte, found by tests/test_dct_gpu.py).  Hiding the clamped values from
    // the combiner avoids that pattern; the asm emits no instruction.
#pragma unroll
    for (int q = 0; q < 24; ++q) VCF_OPAQUE(px[q]);
}

}  // namespace vcf
