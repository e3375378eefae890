// Host build of the run-time-length block transforms (vcf_pocketfft_rt.h, with
// the Bluestein plans of vcf_pocketfft_blue.h): the plan building and the
// transform code the GPU kernels run, compiled for the CPU (hipcc
// --cuda-host-only -ffp-contract=off) for the oracle parity tests in
// tests/test_rt_math.py.
#include <vector>

#include "vcf_pocketfft_rt.h"

using namespace vcf::pfft;

template <typename T>
static int run(int kind, T *x, int N, int count)
{
    if (N < 1 || (kind != 2 && kind != 3)) return -1;
    RtPlan P;
    std::vector<T> mem;
    rt_fill<T>(N, P, mem);
    std::vector<T> ch((size_t)N), bw((size_t)(rt_line_reals(P) - 2LL * N) + 1);
    const RtFft<T> F{mem.data(), bw.data(), 1};
    for (int r = 0; r < count; ++r) {
        const Line<T> c{x + (size_t)r * N, 1}, h{ch.data(), 1};
        if (kind == 2) F.dct2(c, h, P);
        else F.dct3(c, h, P);
    }
    return 0;
}

extern "C" {
int hb_rt_dct_f32(int kind, float *x, int N, int count) { return run<float>(kind, x, N, count); }
int hb_rt_dct_f64(int kind, double *x, int N, int count) { return run<double>(kind, x, N, count); }
int hb_rt_uses_bluestein(int N) { return rt_uses_bluestein((size_t)N) ? 1 : 0; }
int hb_rt_n2(int N) { return (int)rt_good_size_cmplx(2 * (size_t)N - 1); }
}
