// Microbenchmark: issue rate of v_add_f64 / v_mul_f64 (8 independent chains per lane).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ __launch_bounds__(256) void chain(double *out, double a, double b, int iters)
{
    double x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 1e-3 + k;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (OP == 0) x[k] = x[k] + a;
            else if (OP == 1) x[k] = x[k] * b;
            else x[k] = __fma_rn(x[k], b, a);
        }
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main()
{
    const int blocks = 256 * 8 * 4, iters = 4096;   // 8 waves/SIMD
    double *out;
    hipMalloc(&out, sizeof(double) * blocks * 256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[3] = {"v_add_f64", "v_mul_f64", "v_fma_f64"};
    for (int op = 0; op < 3; ++op) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            if (op == 0) hipLaunchKernelGGL(chain<0>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001, 0.9999999, iters);
            if (op == 1) hipLaunchKernelGGL(chain<1>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001, 0.9999999, iters);
            if (op == 2) hipLaunchKernelGGL(chain<2>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001, 0.9999999, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double ops = (double)blocks * 256 * iters * 8;
            if (rep) printf("%s: %.2f T lane-ops/s  (%.3f ms)\n", names[op], ops / ms / 1e9, ms);
        }
    }
    return 0;
}
