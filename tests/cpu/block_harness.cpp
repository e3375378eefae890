// Host build of the kernels' per-block arithmetic (vcf_amd/csrc/vcf_dct_block.h)
// for CPU-only parity tests against the oracle (tests/test_block_math.py).
#include <string.h>

#include "vcf_dct_block.h"

using namespace vcf;

template <bool POW2, bool PERC>
static void enc(const uint32_t (&raw)[8][6], const float (&qd)[4], uint8_t *k)
{
    uint8_t kb[3][64];
    encode_block_channel<0, POW2, PERC>(raw, qd, kb[0]);
    encode_block_channel<1, POW2, PERC>(raw, qd, kb[1]);
    encode_block_channel<2, POW2, PERC>(raw, qd, kb[2]);
    for (int n = 0; n < 64; ++n)
        for (int c = 0; c < 3; ++c) k[n * 3 + c] = kb[c][n];
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
