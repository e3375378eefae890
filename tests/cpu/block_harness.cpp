// Host build of the kernels' per-block arithmetic (vcf_amd/csrc/vcf_dct_block.h)
// for CPU-only parity tests against the oracle (tests/test_block_math.py).
#include <string.h>

#include <type_traits>

#include "vcf_dct_block.h"

using namespace vcf;

template <bool POW2, bool PERC>
static void enc(const uint32_t (&raw)[8][6], const float (&qd)[4], uint8_t *k)
{
    uint32_t K[3][16];
    encode_block_channel<0, POW2, PERC>(raw, qd, K[0]);
    encode_block_channel<1, POW2, PERC>(raw, qd, K[1]);
    encode_block_channel<2, POW2, PERC>(raw, qd, K[2]);
    for (int n = 0; n < 64; ++n)
        for (int c = 0; c < 3; ++c) k[n * 3 + c] = (uint8_t)byte_at(K[c], n);
}

extern "C" void hb_encode_block(const uint8_t *rgb, int Q, unsigned flags, uint8_t *k)
{
    uint32_t raw[8][6];
    memcpy(raw, rgb, 192);   // little-endian byte order, as the kernel's loads
    const bool pow2 = (Q & (Q - 1)) == 0;
    float qd[4];
    for (int e = 0; e < 4; ++e) {
        const double D = (double)Q * (double)(1 << (e + 3));
        qd[e] = pow2 ? (float)(1.0 / D) : (float)D;
    }
    const bool perc = flags & 2;
    if (pow2) perc ? enc<true, true>(raw, qd, k) : enc<true, false>(raw, qd, k);
    else perc ? enc<false, true>(raw, qd, k) : enc<false, false>(raw, qd, k);
}

extern "C" void hb_decode_block(const uint8_t *k, int Q, unsigned flags, uint8_t *rgb)
{
    uint8_t kb[3][64];
    for (int n = 0; n < 64; ++n)
        for (int c = 0; c < 3; ++c) kb[c][n] = k[n * 3 + c];
    uint32_t Y[32], Co[32], Cg[32];
    if (flags & 2) {
        decode_block_channel<0, true>(kb[0], Q, Y);
        decode_block_channel<1, true>(kb[1], Q, Co);
        decode_block_channel<2, true>(kb[2], Q, Cg);
    } else {
        decode_block_channel<0, false>(kb[0], Q, Y);
        decode_block_channel<1, false>(kb[1], Q, Co);
        decode_block_channel<2, false>(kb[2], Q, Cg);
    }
    for (int y = 0; y < 8; ++y) {
        uint32_t px[24];
        to_rgb_row(Y, Co, Cg, y, px);
        for (int q = 0; q < 24; ++q) rgb[y * 24 + q] = (uint8_t)px[q];
    }
}

template <bool POW2, bool PERC>
static void enc_bytes(const uint32_t (&raw)[8][6], const float (&qd)[4], uint8_t *k)
{
    auto s0 = [&](int i, int j, uint32_t w) { k[(i * 8 + j) * 3 + 0] = (uint8_t)w; };
    auto s1 = [&](int i, int j, uint32_t w) { k[(i * 8 + j) * 3 + 1] = (uint8_t)w; };
    auto s2 = [&](int i, int j, uint32_t w) { k[(i * 8 + j) * 3 + 2] = (uint8_t)w; };
    encode_block_channel_bytes<0, POW2, PERC>(raw, qd, s0);
    encode_block_channel_bytes<1, POW2, PERC>(raw, qd, s1);
    encode_block_channel_bytes<2, POW2, PERC>(raw, qd, s2);
}

extern "C" void hb_encode_block_bytes(const uint8_t *rgb, int Q, unsigned flags, uint8_t *k)
{
    uint32_t raw[8][6];
    memcpy(raw, rgb, 192);
    const bool pow2 = (Q & (Q - 1)) == 0;
    float qd[4];
    for (int e = 0; e < 4; ++e) {
        const double D = (double)Q * (double)(1 << (e + 3));
        qd[e] = pow2 ? (float)(1.0 / D) : (float)D;
    }
    const bool perc = flags & 2;
    if (pow2) perc ? enc_bytes<true, true>(raw, qd, k) : enc_bytes<true, false>(raw, qd, k);
    else perc ? enc_bytes<false, true>(raw, qd, k) : enc_bytes<false, false>(raw, qd, k);
}

// Column-per-lane schedule of dct_dz_encode_cols (vcf_dct_dz.hip): lane x
// transforms pixel column x (outputs 0 and 4 doubled), the block transposes
// through a tile, lane x transforms coefficient row x and quantizes it.
template <bool POW2, bool PERC>
static void enc_cols(const uint8_t *rgb, const EncConsts &K, uint8_t *k)
{
    uint32_t px[8][8];   // [lane x][row y]: signed R', G', B' bytes of pixel (y, x)
    for (int x = 0; x < 8; ++x)
        for (int y = 0; y < 8; ++y) {
            const uint8_t *p = rgb + (y * 8 + x) * 3;
            px[x][y] = ((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16)) ^ 0x80808080u;
        }
    for (int C = 0; C < 3; ++C) {
        float tr[8][8];
        for (int x = 0; x < 8; ++x) {
            float col[8];
            for (int y = 0; y < 8; ++y)
                col[y] = bits_as_float((uint32_t)sdot4(px[x][y], K.w[C][0], (int)K.cinit)) - K.csub[C];
            dct2_8k_colpass(col, K);
            for (int i = 0; i < 8; ++i) tr[i][x] = col[i];
        }
        for (int x = 0; x < 8; ++x) {
            float row[8];
            for (int j = 0; j < 8; ++j) row[j] = tr[x][j];
            dct2_8k(row, K);
            for (int j = 0; j < 8; ++j) {
                float t = row[j];
                if (PERC) t = (float)((double)t * pweight_rt(C, x * 8 + j));
                const int e = (C == 1 ? 1 : 2) + 2 + dct2_inv_scale_log2(j);
                const float q = quant_div<POW2>(t, K.qd[e - 3]);
                k[(x * 8 + j) * 3 + C] = (uint8_t)float_bits(trunc_f(q) + K.qmagic);
            }
        }
    }
}

extern "C" void hb_encode_block_cols(const uint8_t *rgb, int Q, unsigned flags, uint8_t *k)
{
    EncConsts K;
    make_enc_consts(K, Q);
    const bool pow2 = (Q & (Q - 1)) == 0;
    const bool perc = flags & 2;
    if (pow2) perc ? enc_cols<true, true>(rgb, K, k) : enc_cols<true, false>(rgb, K, k);
    else perc ? enc_cols<false, true>(rgb, K, k) : enc_cols<false, false>(rgb, K, k);
}

// Folded-quantizer body of encode variants 1/2: the sink gets the low byte of
// k; the kernel's copy-out adds 128 by XOR 0x80.
extern "C" void hb_encode_block_fold(const uint8_t *rgb, int Q, unsigned flags, uint8_t *k)
{
    uint32_t raw[8][6];
    memcpy(raw, rgb, 192);
    EncConsts K;
    make_enc_consts(K, Q);
    const bool pow2 = (Q & (Q - 1)) == 0;
    const FinalK rowk = pow2 ? row_final_k(Q) : final_k(1.0f, 1.0f);
    const bool perc = flags & 2;
    auto run = [&](auto pw2, auto pc) {
        constexpr bool P2 = decltype(pw2)::value, PC = decltype(pc)::value;
        auto s0 = [&](int i, int j, uint32_t w) { k[(i * 8 + j) * 3 + 0] = (uint8_t)(w ^ 0x80u); };
        auto s1 = [&](int i, int j, uint32_t w) { k[(i * 8 + j) * 3 + 1] = (uint8_t)(w ^ 0x80u); };
        auto s2 = [&](int i, int j, uint32_t w) { k[(i * 8 + j) * 3 + 2] = (uint8_t)(w ^ 0x80u); };
        encode_block_channel_fold<0, P2, PC>(raw, rowk, K.qd, s0);
        encode_block_channel_fold<1, P2, PC>(raw, rowk, K.qd, s1);
        encode_block_channel_fold<2, P2, PC>(raw, rowk, K.qd, s2);
    };
    using T = std::true_type;
    using F = std::false_type;
    if (pow2) perc ? run(T{}, T{}) : run(T{}, F{});
    else perc ? run(F{}, T{}) : run(F{}, F{});
}

// the DCT-III with known-zero trailing inputs (decode zero skipping) and the
// full one, for tests/test_block_math.py
extern "C" void hb_dct3(int K, const double *in, double *out)
{
    double c[8];
    for (int i = 0; i < 8; ++i) c[i] = in[i];
    switch (K) {
    case 1: vcf::dct3_8r_k<1>(c); break;
    case 2: vcf::dct3_8r_k<2>(c); break;
    case 3: vcf::dct3_8r_k<3>(c); break;
    case 4: vcf::dct3_8r_k<4>(c); break;
    case 5: vcf::dct3_8r_k<5>(c); break;
    case 6: vcf::dct3_8r_k<6>(c); break;
    case 7: vcf::dct3_8r_k<7>(c); break;
    default: vcf::dct3_8r(c); break;
    }
    for (int i = 0; i < 8; ++i) out[i] = c[i];
}
