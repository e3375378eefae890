// vcf_dct8.h -- 8-point DCT-II (fp32) and DCT-III (fp64) in pocketfft's exact
// operation order, in the "reduced" form the HIP kernels use.
//
// The reference's block DCT (DCT2D.block_DCT.analyze_image / synthesize_image,
// called at src/2D-DCT.py:303 and :440) runs scipy.fftpack -> pocketfft
// T_dcst23 on every column, then every row, of each 8x8 block.  Bit-exact
// quantization indices need pocketfft's rounding sequence, so these functions
// perform the same floating-point operations, in the same order, on the same
// twiddles (pocketfft sincos_2pibyn, see oracle/vcf_oracle.c), with every
// multiplication by an exact power of two removed:
//
//   * DCT-II: c[0]*=2, c[7]*=2, the 2* factors of radb2/radb4, fct = 1/4 and
//     the 0.5 of the post-twiddle are dropped.  Every signal path carries
//     exactly one of the factors 2, so the result is  out[k] = true[k]/s[k],
//     s = {1/2, 1/4, 1/4, 1/4, 1/2, 1/4, 1/4, 1/4}.
//   * DCT-III: fct = 1/4 is dropped, so out[k] = 4 * true[k].
//
// Scaling by a power of two commutes with IEEE rounding (no overflow or
// subnormals occur for 8-bit video data), so the kernels re-apply the missing
// factors exactly at the end (in the quantizer's divisor, or *1/16 after the
// 2D inverse) and reproduce the oracle bit for bit.  Compile with
// -ffp-contract=off: an FMA would change the rounding.
#pragma once

#if defined(__HIPCC__)
#define VCF_HD __host__ __device__ __forceinline__
#else
#define VCF_HD static inline
#endif

namespace vcf {

// pocketfft twiddles for N = 8 (sincos_2pibyn(32)[i+1].r), fp32 and fp64.
#define VCF_TWF0 0x1.f6297cp-1f
#define VCF_TWF1 0x1.d906bcp-1f
#define VCF_TWF2 0x1.a9b662p-1f
#define VCF_TWF3 0x1.6a09e6p-1f
#define VCF_TWF4 0x1.1c73b4p-1f
#define VCF_TWF5 0x1.87de2ap-2f
#define VCF_TWF6 0x1.8f8b84p-3f
// rfftp N=8 twiddle (sincos_2pibyn(8)[1]); in fp32 re == im == sqrt2*0.5 == tw[3]
#define VCF_HF 0x1.6a09e6p-1f

#define VCF_TWD0 0x1.f6297cff75cb0p-1
#define VCF_TWD1 0x1.d906bcf328d46p-1
#define VCF_TWD2 0x1.a9b66290ea1a3p-1
#define VCF_TWD3 0x1.6a09e667f3bccp-1
#define VCF_TWD4 0x1.1c73b39ae68c8p-1
#define VCF_TWD5 0x1.87de2a6aea963p-2
#define VCF_TWD6 0x1.8f8b83c69a60ap-3
#define VCF_WRD 0x1.6a09e667f3bccp-1   // sin(pi/4) as pocketfft computes it
#define VCF_WID 0x1.6a09e667f3bcdp-1   // cos(pi/4)
#define VCF_SQRT2D 0x1.6a09e667f3bcdp+0
#define VCF_2TW3D 0x1.6a09e667f3bccp+0 // 2*tw[3], exact

// Reduced DCT-II: x -> X/s (see header).
VCF_HD void dct2_8r(float (&c)[8])
{
    // MPINPLACE(c[k+1], c[k]) for k = 1, 3, 5
    const float x1 = c[1] + c[2], x2 = c[2] - c[1];
    const float x3 = c[3] + c[4], x7 = c[3] - c[4];   // x7 = -(c4 - c3): radb2's -2*CC
    const float x5 = c[5] + c[6], x6 = c[6] - c[5];
    // radb2 (ido = 4, l1 = 1)
    const float a0 = c[0] + c[7], a4 = c[0] - c[7];
    const float a1 = x1 + x5, tr2 = x1 - x5;
    const float ti2 = x2 + x6, a2 = x2 - x6;
    const float a6 = VCF_HF * ti2 + VCF_HF * tr2;
    const float a5 = VCF_HF * tr2 - VCF_HF * ti2;
    // radb4 (ido = 1, l1 = 2)
    const float T2 = a0 + x3, T1 = a0 - x3;
    const float r0 = T2 + a1, r4 = T2 - a1, r6 = T1 + a2, r2 = T1 - a2;
    const float U2 = a4 + x7, U1 = a4 - x7;
    const float r1 = U2 + a5, r5 = U2 - a5, r7 = U1 + a6, r3 = U1 - a6;
    // post-twiddle
    float t1, t2;
    t1 = VCF_TWF0 * r7 + VCF_TWF6 * r1; t2 = VCF_TWF0 * r1 - VCF_TWF6 * r7;
    c[1] = t1 + t2; c[7] = t1 - t2;
    t1 = VCF_TWF1 * r6 + VCF_TWF5 * r2; t2 = VCF_TWF1 * r2 - VCF_TWF5 * r6;
    c[2] = t1 + t2; c[6] = t1 - t2;
    t1 = VCF_TWF2 * r5 + VCF_TWF4 * r3; t2 = VCF_TWF2 * r3 - VCF_TWF4 * r5;
    c[3] = t1 + t2; c[5] = t1 - t2;
    c[4] = r4 * VCF_TWF3;
    c[0] = r0 * VCF_HF;
}

// Reduced DCT-III: X -> 4x.
VCF_HD void dct3_8r(double (&c)[8])
{
    const double c0 = c[0] * VCF_SQRT2D;
    double t1, t2;
    t1 = c[1] + c[7]; t2 = c[1] - c[7];
    const double u1 = VCF_TWD0 * t2 + VCF_TWD6 * t1, u7 = VCF_TWD0 * t1 - VCF_TWD6 * t2;
    t1 = c[2] + c[6]; t2 = c[2] - c[6];
    const double u2 = VCF_TWD1 * t2 + VCF_TWD5 * t1, u6 = VCF_TWD1 * t1 - VCF_TWD5 * t2;
    t1 = c[3] + c[5]; t2 = c[3] - c[5];
    const double u3 = VCF_TWD2 * t2 + VCF_TWD4 * t1, u5 = VCF_TWD2 * t1 - VCF_TWD4 * t2;
    const double c4 = c[4] * VCF_2TW3D;
    // radf4 (ido = 1, l1 = 2) on {c0, u1, u2, u3, c4, u5, u6, u7}
    const double tr1 = u6 + u2, h2 = u6 - u2, tr2 = c0 + c4, h1 = c0 - c4;
    const double h0 = tr2 + tr1, h3 = tr2 - tr1;
    const double sr1 = u7 + u3, h6 = u7 - u3, sr2 = u1 + u5, h5 = u1 - u5;
    const double h4 = sr2 + sr1, h7 = sr2 - sr1;
    // radf2 (ido = 4, l1 = 1); o4 = -h7 is folded into the MPINPLACE below
    const double o0 = h0 + h4, o7 = h0 - h4;
    const double tr = VCF_WRD * h5 + VCF_WID * h6, ti = VCF_WRD * h6 - VCF_WID * h5;
    const double o1 = h1 + tr, o5 = h1 - tr;
    const double o2 = ti + h2, o6 = ti - h2;
    // MPINPLACE(c[k], c[k+1]) for k = 1, 3, 5
    c[0] = o0;
    c[1] = o1 - o2; c[2] = o2 + o1;
    c[3] = h3 + h7; c[4] = h3 - h7;      // (h3 - o4), (o4 + h3) with o4 = -h7
    c[5] = o5 - o6; c[6] = o6 + o5;
    c[7] = o7;
}

// dct3_8r with inputs K..7 known to be exactly zero (K = 1..8; K = 8 is
// dct3_8r).  Every operation with a nonzero result is dct3_8r's, on the same
// operands in the same order; an operation with a known-zero operand is
// skipped (x + 0 = x, x - 0 = x, 0 - x = -x and 0 * c = 0 exactly).  Only the
// sign of a zero can differ from pocketfft's (-0 for +0): a signed zero never
// changes a nonzero sum or product, and the decode truncates to int16, where
// both are 0 -- so the decoded bytes are identical (tests/test_dct_gpu.py).
// The zero flags are compile-time constants after inlining: the skipped
// branches vanish (the IDCT of a DC-only block is 2 multiplies per pass).
struct XZ {
    double v;
    bool z;   // known to be exactly zero
};
VCF_HD XZ xz_add(XZ a, XZ b) { return b.z ? a : a.z ? b : XZ{a.v + b.v, false}; }
VCF_HD XZ xz_sub(XZ a, XZ b) { return b.z ? a : a.z ? XZ{-b.v, false} : XZ{a.v - b.v, false}; }
VCF_HD XZ xz_mul(double k, XZ a) { return a.z ? XZ{0.0, true} : XZ{k * a.v, false}; }

template <int K>
VCF_HD void dct3_8r_k(double (&c)[8])
{
    XZ x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = XZ{i < K ? c[i] : 0.0, i >= K};
    const XZ c0 = xz_mul(VCF_SQRT2D, x[0]);   // c[0] * sqrt2 (commutes)
    XZ t1, t2;
    t1 = xz_add(x[1], x[7]); t2 = xz_sub(x[1], x[7]);
    const XZ u1 = xz_add(xz_mul(VCF_TWD0, t2), xz_mul(VCF_TWD6, t1));
    const XZ u7 = xz_sub(xz_mul(VCF_TWD0, t1), xz_mul(VCF_TWD6, t2));
    t1 = xz_add(x[2], x[6]); t2 = xz_sub(x[2], x[6]);
    const XZ u2 = xz_add(xz_mul(VCF_TWD1, t2), xz_mul(VCF_TWD5, t1));
    const XZ u6 = xz_sub(xz_mul(VCF_TWD1, t1), xz_mul(VCF_TWD5, t2));
    t1 = xz_add(x[3], x[5]); t2 = xz_sub(x[3], x[5]);
    const XZ u3 = xz_add(xz_mul(VCF_TWD2, t2), xz_mul(VCF_TWD4, t1));
    const XZ u5 = xz_sub(xz_mul(VCF_TWD2, t1), xz_mul(VCF_TWD4, t2));
    const XZ c4 = xz_mul(VCF_2TW3D, x[4]);
    const XZ tr1 = xz_add(u6, u2), h2 = xz_sub(u6, u2), tr2 = xz_add(c0, c4), h1 = xz_sub(c0, c4);
    const XZ h0 = xz_add(tr2, tr1), h3 = xz_sub(tr2, tr1);
    const XZ sr1 = xz_add(u7, u3), h6 = xz_sub(u7, u3), sr2 = xz_add(u1, u5), h5 = xz_sub(u1, u5);
    const XZ h4 = xz_add(sr2, sr1), h7 = xz_sub(sr2, sr1);
    const XZ o0 = xz_add(h0, h4), o7 = xz_sub(h0, h4);
    const XZ tr = xz_add(xz_mul(VCF_WRD, h5), xz_mul(VCF_WID, h6));
    const XZ ti = xz_sub(xz_mul(VCF_WRD, h6), xz_mul(VCF_WID, h5));
    const XZ o1 = xz_add(h1, tr), o5 = xz_sub(h1, tr);
    const XZ o2 = xz_add(ti, h2), o6 = xz_sub(ti, h2);
    const XZ r[8] = {o0, xz_sub(o1, o2), xz_add(o2, o1), xz_add(h3, h7),
                     xz_sub(h3, h7), xz_sub(o5, o6), xz_add(o6, o5), o7};
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = r[i].z ? 0.0 : r[i].v;
}

// log2(1/s[k]) for the DCT-II reduced outputs.
VCF_HD constexpr int dct2_inv_scale_log2(int k) { return (k & 3) == 0 ? 1 : 2; }

}  // namespace vcf
