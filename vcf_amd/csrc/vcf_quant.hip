// vcf_quant.hip -- the deadzone quantizer as a stand-alone plug-in:
// deadzone.py CoDec.quantize_fn (:95-102) / dequantize_fn (:107-117) over
// scalar_quantization.Deadzone_Quantizer (assumption A5: encode
// (x / Q).astype(int32), truncation toward zero; decode Q * k in k's dtype).
//
// The fused DCT kernels never call these (they quantize in registers); they
// serve callers of the quantizer surface on arbitrary arrays, e.g. the DWT
// subbands (2D-DWT.py:113-160).  Elementwise, HBM-bound: grid-stride loops,
// 4 elements per lane per iteration.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "vcf_amd.h"
#include "vcf_internal.h"

namespace vcf {
namespace {

// numpy true division: float32 / int -> float32; every other input -> float64
template <typename T>
struct QuantMath {
    using F = double;
};
template <>
struct QuantMath<float> {
    using F = float;
};

template <typename T>
__global__ __launch_bounds__(256) void deadzone_quantize_kernel(const T *__restrict__ x, int64_t n, int32_t Q,
                                                                int32_t *__restrict__ k)
{
    using F = typename QuantMath<T>::F;
    const F q = (F)Q;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const F v = (F)x[i] / q;          // IEEE division (no fast-math)
        k[i] = (int32_t)v;                // astype(int32): truncation toward zero
    }
}

template <typename T>
__global__ __launch_bounds__(256) void deadzone_dequantize_kernel(const T *__restrict__ k, int64_t n, int32_t Q,
                                                                  T *__restrict__ y)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        y[i] = (T)((uint32_t)Q * (uint32_t)(int32_t)k[i]);   // Q * k, wrapping in T
}

unsigned grid_for(int64_t n)
{
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 256 * 64));
}

}  // namespace
}  // namespace vcf

using namespace vcf;

extern "C" {

int vcf_deadzone_quantize(const void *x_dev, int32_t x_dtype, int64_t n, int32_t Q, int32_t *k_dev,
                          void *stream)
{
    if (n < 0) return set_error(VCF_ERR_INVALID, "n < 0");
    if (Q < 1) return set_error(VCF_ERR_INVALID, "quantization step %d out of range", Q);
    if (n == 0) return VCF_OK;
    if (!x_dev || !k_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    const dim3 grid(grid_for(n)), block(256);
    hipStream_t s = (hipStream_t)stream;
    switch (x_dtype) {
    case VCF_DTYPE_F32:
        hipLaunchKernelGGL(deadzone_quantize_kernel<float>, grid, block, 0, s, (const float *)x_dev, n, Q, k_dev);
        break;
    case VCF_DTYPE_F64:
        hipLaunchKernelGGL(deadzone_quantize_kernel<double>, grid, block, 0, s, (const double *)x_dev, n, Q, k_dev);
        break;
    case VCF_DTYPE_I16:
        hipLaunchKernelGGL(deadzone_quantize_kernel<int16_t>, grid, block, 0, s, (const int16_t *)x_dev, n, Q, k_dev);
        break;
    case VCF_DTYPE_I32:
        hipLaunchKernelGGL(deadzone_quantize_kernel<int32_t>, grid, block, 0, s, (const int32_t *)x_dev, n, Q, k_dev);
        break;
    case VCF_DTYPE_U8:
        hipLaunchKernelGGL(deadzone_quantize_kernel<uint8_t>, grid, block, 0, s, (const uint8_t *)x_dev, n, Q, k_dev);
        break;
    default:
        return set_error(VCF_ERR_INVALID, "unsupported input dtype %d", x_dtype);
    }
    return hip_check(hipGetLastError(), "deadzone_quantize launch");
}

int vcf_deadzone_dequantize(const void *k_dev, int32_t k_dtype, int64_t n, int32_t Q, void *y_dev,
                            void *stream)
{
    if (n < 0) return set_error(VCF_ERR_INVALID, "n < 0");
    if (Q < 1) return set_error(VCF_ERR_INVALID, "quantization step %d out of range", Q);
    if (n == 0) return VCF_OK;
    if (!k_dev || !y_dev) return set_error(VCF_ERR_INVALID, "null buffer");
    const dim3 grid(grid_for(n)), block(256);
    hipStream_t s = (hipStream_t)stream;
    switch (k_dtype) {
    case VCF_DTYPE_I16:
        if (Q > 32767) return set_error(VCF_ERR_UNSUPPORTED, "Q > 32767 promotes int16 in numpy");
        hipLaunchKernelGGL(deadzone_dequantize_kernel<int16_t>, grid, block, 0, s, (const int16_t *)k_dev, n, Q,
                           (int16_t *)y_dev);
        break;
    case VCF_DTYPE_I32:
        hipLaunchKernelGGL(deadzone_dequantize_kernel<int32_t>, grid, block, 0, s, (const int32_t *)k_dev, n, Q,
                           (int32_t *)y_dev);
        break;
    default:
        return set_error(VCF_ERR_INVALID, "unsupported index dtype %d", k_dtype);
    }
    return hip_check(hipGetLastError(), "deadzone_dequantize launch");
}

}  // extern "C"
