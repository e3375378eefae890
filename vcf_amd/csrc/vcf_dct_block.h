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
#include <stdint.h>

#include "vcf_dct8.h"

#if defined(__HIP_DEVICE_COMPILE__)
// An empty asm that makes `x` look redefined: blocks CSE / sinking across it.
#define VCF_OPAQUE(x) asm volatile("" : "+v"(x))
#else
#define VCF_OPAQUE(x) ((void)0)
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

// One channel of one block -> 64 index bytes (k + 128) in (i*8 + j) order.
template <int C, bool POW2, bool PERC>
VCF_HD void encode_block_channel(const uint32_t (&raw)[8][6], const float (&qd)[4], uint8_t (&kb)[64])
{
    float v[8][8];
#pragma unroll
    for (int y = 0; y < 8; ++y)
#pragma unroll
        for (int x = 0; x < 8; ++x)
            v[y][x] = ycocg_scaled<C>(byte_of(raw[y], 3 * x), byte_of(raw[y], 3 * x + 1),
                                      byte_of(raw[y], 3 * x + 2));
    // axis 0 (columns) first, then axis 1 (rows): dct(dct(b.T).T)
#pragma unroll
    for (int x = 0; x < 8; ++x) {
        float col[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) col[y] = v[y][x];
        dct2_8r(col);
#pragma unroll
        for (int y = 0; y < 8; ++y) v[y][x] = col[y];
    }
#pragma unroll
    for (int y = 0; y < 8; ++y) dct2_8r(v[y]);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float t = v[i][j];
            if (PERC) t = (float)((double)t * pweight<C>(i * 8 + j));
            const float q = quant_div<POW2>(t, qd[qexp<C>(i, j) - 3]);
            const int k = (int)q;   // astype(int32): truncation toward zero
            kb[i * 8 + j] = (uint8_t)(k + 128);
        }
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
