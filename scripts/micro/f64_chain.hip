// Microbenchmark: dependent v_add_f64 / v_mul_f64 chains (C independent chains
// per lane) at W waves per SIMD: cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int C>
__global__ __launch_bounds__(64) void chain(double *out, double a, double b, int iters)
{
    double x[C];
#pragma unroll
    for (int k = 0; k < C; ++k) x[k] = threadIdx.x * 1e-3 + k;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < C; ++k) x[k] = x[k] * b + a;   // mul then add: 2 dependent ops (no fma: -ffp-contract=off)
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < C; ++k) s += x[k];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int C>
void run(double *out, int waves_per_simd)
{
    const int blocks = 256 * 4 * waves_per_simd, iters = 4096;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(chain<C>, dim3(blocks), dim3(64), 0, 0, out, 1.0000001, 0.9999999, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
    }
    // wave-instructions per SIMD: waves_per_simd * iters * C * 2 ops
    const double inst = (double)waves_per_simd * iters * C * 2;
    printf("chains %d waves/SIMD %d: %.2f cycles/wave-instr (at 2.4 GHz)\n", C, waves_per_simd, ms * 1e-3 * 2.4e9 / inst);
}

int main()
{
    double *out;
    (void)hipMalloc(&out, sizeof(double) * 256 * 4 * 16 * 64);
    for (int w : {1, 2, 4, 8}) { run<1>(out, w); run<2>(out, w); run<4>(out, w); }
    return 0;
}
