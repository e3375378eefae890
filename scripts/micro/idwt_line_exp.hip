// A/B harness for the level-1 line inverse (scripts/micro/idwt_line_exp.py):
// the product kernels compiled alone plus experimental copies, one C entry.
#define VCF_DWT_KERNELS_ONLY
#include "../../vcf_amd/csrc/vcf_dwt.hip"
namespace vcf {
namespace {
#include "idwt_line_exp.h"
}
}
using namespace vcf;
typedef void (*LineK)(const uint8_t *, long long, long long, long long, long long, long long, const double *,
                      long long, int, double *, uint8_t *, int, int, int, int, int, int, int, int);
template <bool RE, bool HB, int NL, int WPE>
static LineK ek() { return idwt_line_exp_kernel<false, true, 0x301u, 1u, 1, true, RE, HB, NL, WPE>; }

extern "C" int exp_line_l1(int variant, const uint8_t *packed, long long packed_stride, long long off_lh,
                           long long off_hl, long long off_hh, const double *prev, long long plane_stride, int lda,
                           uint8_t *rgb, int h, int w, int oh, int ow, int Q, int n_frames, int n_bands, void *stream)
{
    LineK k = nullptr;
    int nl = 128;
    switch (variant) {
    case 0: k = idwt_line_kernel<false, true, 0x301u, 1u, 1, true>; nl = kILC; break;
    case 1: k = ek<false, true, 128, 1>(); break;
    case 2: k = ek<false, false, 128, 1>(); break;
    case 5: k = ek<false, false, 128, 5>(); break;
    case 6: k = ek<false, false, 64, 1>(); nl = 64; break;
    case 7: k = ek<false, false, 64, 5>(); nl = 64; break;
    case 8: k = ek<false, false, 64, 6>(); nl = 64; break;
    default: return -1;
    }
    const int n_tiles = (w + nl - 1) / nl, ohp = (oh + 1) / 2;
    const int brows = (ohp + n_bands - 1) / n_bands;
    n_bands = (ohp + brows - 1) / brows;
    const unsigned grid = (unsigned)(n_tiles * n_bands * n_frames);
    hipLaunchKernelGGL(k, dim3(grid), dim3(3 * nl), 0, (hipStream_t)stream, packed, packed_stride, 0LL, off_lh,
                       off_hl, off_hh, prev, plane_stride, lda, nullptr, rgb, h, w, oh, ow, Q, n_tiles, n_bands,
                       brows);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
