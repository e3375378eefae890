// Microbenchmark: issue rate of v_add_f32 vs packed v_pk_add_f32 (8 independent
// chains per lane) at 1..8 waves per SIMD (grid = 256 CUs x W workgroups of 4 waves).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ __launch_bounds__(256) void chain(float *out, float a, int iters)
{
    if (OP == 0) {
        float x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 1e-3f + k;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = x[k] + a;
        }
        float s = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) s += x[k];
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    } else {
        f2 x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = f2{threadIdx.x * 1e-3f + k, k * 0.5f};
        const f2 av = {a, a};
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = x[k] + av;
        }
        float s = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) s += x[k].x + x[k].y;
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    }
}

int main()
{
    const int iters = 8192;
    float *out;
    hipMalloc(&out, sizeof(float) * 256 * 8 * 256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w : {1, 2, 3, 4, 6, 8}) {
        const int blocks = 256 * w;
        for (int op = 0; op < 2; ++op) {
            float ms = 0;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                if (op == 0) hipLaunchKernelGGL(chain<0>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001f, iters);
                else hipLaunchKernelGGL(chain<1>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001f, iters);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                hipEventElapsedTime(&ms, e0, e1);
            }
            const double instr = (double)blocks * 4 * iters * 8;   // wave-instructions
            const double per_simd = instr / 1024;
            printf("waves/SIMD %d %s: %.3f ms, %.2f cycles per wave-instruction per SIMD at 2.4 GHz, "
                   "%.1f T elem-ops/s\n", w, op ? "v_pk_add_f32" : "v_add_f32   ", ms,
                   ms * 1e-3 * 2.4e9 / per_simd, instr * 64 * (op ? 2 : 1) / ms / 1e9);
        }
    }
    return 0;
}
