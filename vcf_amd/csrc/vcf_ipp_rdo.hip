// vcf_ipp_rdo.hip -- IPP block-level rate-distortion mode decision (-R, the
// rdo_lambda > 0 branch of IPP.temporal_filter, src/IPP_DCT.py:441-536) for
// gfx950, and the vcf_ipp_rdo_* entry points of the C ABI.
//
// Per bs x bs block of the full-block area (i, j over range(0, h-bs+1, bs)):
//   * both blocks to luma with cv2.cvtColor(RGB2GRAY) (:449-456; A10);
//   * IPP.rdo_block_decision (:269-342) on the luma blocks:
//       INTER: residual = cur - comp (float64), dct_2d (pocketfft float64,
//       axis 0 then 1), q = round(x / qss) (half to even) as int16,
//       dequantized float32(q) * qss, idct_2d in float32, recon = comp +
//       that (float64), D = mean((cur - recon)^2), R = get_rate(q, inter)
//       (:265-288: 2 nz + 0.2 sum|q| + 4);
//       INTRA: the same on cur itself (R = 3 nz + 0.3 sum|q| + 8);
//       cost = D + lambda R each; P (inter) iff cost_inter <= cost_intra;
//   * numpy's mean is add.reduce, i.e. numpy's pairwise summation over the
//     block in row-major order (8 partial sums per <= 128-element leaf,
//     halves split at multiples of 8), then one division by bs*bs; the
//     restatement below follows it sum by sum.
// Then the frame handed to the spatial codec (:489-505): P blocks
// clip(cur - comp + 128), I blocks cur, everything outside full blocks 128;
// and the reconstruction (:512-526, decode :770-790): P blocks
// clip(comp + rec - 128), I blocks rec, outside full blocks 0.
//
// Mapping: one 64-lane wave per block; lanes < bs run the column / row
// transforms in registers (vcf_pocketfft.h), LDS tiles hold the transposes;
// lane 0 does the pairwise sums and the decision.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "vcf_amd.h"
#include "vcf_internal.h"
#include "vcf_pocketfft.h"
#include "vcf_pocketfft_tables.h"

namespace vcf {
namespace {

__device__ __forceinline__ uint8_t luma(const uint8_t *p)
{
    // cv2 RGB2GRAY for 8-bit images (A10): (4899 R + 9617 G + 1868 B + 8192) >> 14
    return (uint8_t)((4899u * p[0] + 9617u * p[1] + 1868u * p[2] + 8192u) >> 14);
}

// numpy pairwise_sum (umath loops.c.src, PW_BLOCKSIZE 128, unroll 8) of a[0:N]
template <int N>
__device__ __forceinline__ double np_pairwise_sum(const double *a)
{
    if constexpr (N < 8) {
        double res = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) res += a[i];
        return res;
    } else if constexpr (N <= 128) {
        double r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int i = 8;
        for (; i < N - (N % 8); i += 8)
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < N; ++i) res += a[i];
        return res;
    } else {
        constexpr int n2 = N / 2 - (N / 2) % 8;
        return np_pairwise_sum<n2>(a) + np_pairwise_sum<N - n2>(a + n2);
    }
}

template <int BS> struct RdoShared {
    double t[BS * (BS + 1)];   // float64 transpose tile
    float f[BS * (BS + 1)];    // float32 transpose tile
    double sq[BS * BS];        // squared errors, row-major (numpy's flattening)
    uint8_t cg[BS * BS], pg[BS * BS];
    int nz[BS], ms[BS];
};

// One mode's D and R: INTER (residual against pg) or INTRA (cg itself).
template <int BS, bool INTER>
__device__ void rdo_mode(RdoShared<BS> &sh, int lane, int qss, const double *tw64, const float *tw32, double &D,
                         double &R)
{
    constexpr int LD = BS + 1;
    if (lane < BS) {   // column pass (axis 0) of dct_2d, float64
        double v[BS];
#pragma unroll
        for (int y = 0; y < BS; ++y) {
            const double c = (double)sh.cg[y * BS + lane];
            v[y] = INTER ? c - (double)sh.pg[y * BS + lane] : c;
        }
        pfft::dct2<double, BS>(v, tw64);
#pragma unroll
        for (int y = 0; y < BS; ++y) sh.t[y * LD + lane] = v[y];
    }
    __syncthreads();
    if (lane < BS) {   // row pass, quantize (np.round -> int16), dequantize (float32)
        double v[BS];
#pragma unroll
        for (int j = 0; j < BS; ++j) v[j] = sh.t[lane * LD + j];
        pfft::dct2<double, BS>(v, tw64);
        int nz = 0, ms = 0;
        const double dq = (double)qss;
        const float fq = (float)qss;
#pragma unroll
        for (int j = 0; j < BS; ++j) {
            const int16_t q = (int16_t)(int)__builtin_rint(v[j] / dq);
            nz += q != 0;
            ms += q < 0 ? -q : q;
            sh.f[lane * LD + j] = (float)q * fq;
        }
        sh.nz[lane] = nz;
        sh.ms[lane] = ms;
    }
    __syncthreads();
    if (lane < BS) {   // idct_2d column pass, float32
        float v[BS];
#pragma unroll
        for (int y = 0; y < BS; ++y) v[y] = sh.f[y * LD + lane];
        pfft::dct3<float, BS>(v, tw32);
#pragma unroll
        for (int y = 0; y < BS; ++y) sh.f[y * LD + lane] = v[y];
    }
    __syncthreads();
    if (lane < BS) {   // row pass, reconstruction, squared error (float64)
        float v[BS];
#pragma unroll
        for (int j = 0; j < BS; ++j) v[j] = sh.f[lane * LD + j];
        pfft::dct3<float, BS>(v, tw32);
#pragma unroll
        for (int j = 0; j < BS; ++j) {
            const int idx = lane * BS + j;
            const double rec = INTER ? (double)sh.pg[idx] + (double)v[j] : (double)v[j];
            const double e = (double)sh.cg[idx] - rec;
            sh.sq[idx] = e * e;
        }
    }
    __syncthreads();
    if (lane == 0) {
        long long nz = 0, ms = 0;
        for (int y = 0; y < BS; ++y) { nz += sh.nz[y]; ms += sh.ms[y]; }
        D = np_pairwise_sum<BS * BS>(sh.sq) / (double)(BS * BS);
        // get_rate (:265-288): base_rate + magnitude_cost + header_cost
        R = INTER ? ((double)nz * 2.0 + (double)ms * 0.2) + 4.0 : ((double)nz * 3.0 + (double)ms * 0.3) + 8.0;
    }
    __syncthreads();
}

template <int BS>
__global__ __launch_bounds__(64) void ipp_rdo_modes_kernel(const uint8_t *__restrict__ cur,
                                                           const uint8_t *__restrict__ comp, int W, int qss,
                                                           double lambda, uint8_t *__restrict__ modes,
                                                           double *__restrict__ costs)
{
    __shared__ RdoShared<BS> sh;
    const int lane = threadIdx.x;
    const int bx = blockIdx.x, by = blockIdx.y, nbx = gridDim.x;
    const double *tw64 = c_tw_f64 + slot_off(BS);
    const float *tw32 = c_tw_f32 + slot_off(BS);
    for (int e = lane; e < BS * BS; e += 64) {
        const int y = e / BS, x = e % BS;
        const long long o = ((long long)(by * BS + y) * W + bx * BS + x) * 3;
        sh.cg[e] = luma(cur + o);
        sh.pg[e] = luma(comp + o);
    }
    __syncthreads();
    double Di = 0, Ri = 0, Da = 0, Ra = 0;
    rdo_mode<BS, true>(sh, lane, qss, tw64, tw32, Di, Ri);
    rdo_mode<BS, false>(sh, lane, qss, tw64, tw32, Da, Ra);
    if (lane == 0) {
        const double cost_inter = Di + lambda * Ri;
        const double cost_intra = Da + lambda * Ra;
        const int b = by * nbx + bx;
        modes[b] = cost_inter <= cost_intra ? 0 : 1;   // 0 = P (inter), 1 = I (intra)
        if (costs) {
            costs[4 * b + 0] = Di; costs[4 * b + 1] = Ri;
            costs[4 * b + 2] = Da; costs[4 * b + 3] = Ra;
        }
    }
}

// frame_to_encode_shifted (:489-505): P clip(cur - comp + 128), I cur, else 128
__global__ __launch_bounds__(256) void ipp_rdo_residual_kernel(const uint8_t *__restrict__ cur,
                                                               const uint8_t *__restrict__ comp,
                                                               const uint8_t *__restrict__ modes, int H, int W,
                                                               int bs, uint8_t *__restrict__ out)
{
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long long)H * W * 3) return;
    const long long px = e / 3;
    const int y = (int)(px / W), x = (int)(px % W);
    const int nbx = W / bs, nby = H / bs;
    const int by = y / bs, bx = x / bs;
    uint8_t v = 128;
    if (by < nby && bx < nbx) {
        if (modes[by * nbx + bx]) v = cur[e];
        else v = (uint8_t)std::min(255, std::max(0, (int)cur[e] - (int)comp[e] + 128));
    }
    out[e] = v;
}

// recon_P (:512-526, decode :770-790): P clip(comp + rec - 128), I rec, else 0
__global__ __launch_bounds__(256) void ipp_rdo_reconstruct_kernel(const uint8_t *__restrict__ comp,
                                                                  const uint8_t *__restrict__ rec,
                                                                  const uint8_t *__restrict__ modes, int H, int W,
                                                                  int bs, uint8_t *__restrict__ out)
{
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long long)H * W * 3) return;
    const long long px = e / 3;
    const int y = (int)(px / W), x = (int)(px % W);
    const int nbx = W / bs, nby = H / bs;
    const int by = y / bs, bx = x / bs;
    uint8_t v = 0;
    if (by < nby && bx < nbx) {
        if (modes[by * nbx + bx]) v = rec[e];
        else v = (uint8_t)std::min(255, std::max(0, (int)comp[e] + (int)rec[e] - 128));
    }
    out[e] = v;
}

template <int BS>
int launch_modes(const uint8_t *cur, const uint8_t *comp, int H, int W, int qss, double lambda, uint8_t *modes,
                 double *costs, hipStream_t s)
{
    const dim3 grid(W / BS, H / BS);
    hipLaunchKernelGGL((ipp_rdo_modes_kernel<BS>), grid, dim3(64), 0, s, cur, comp, W, qss, lambda, modes, costs);
    return hip_check(hipGetLastError(), "ipp_rdo_modes_kernel launch");
}

int check_frame(const void *a, const void *b, const void *c, int H, int W, int bs)
{
    if (!a || !b || !c) return set_error(VCF_ERR_INVALID, "null buffer");
    if (H <= 0 || W <= 0) return set_error(VCF_ERR_INVALID, "bad frame %d x %d", H, W);
    if (bs < 1) return set_error(VCF_ERR_INVALID, "block size %d", bs);
    if ((long long)H * W * 3 >= (1LL << 31)) return set_error(VCF_ERR_INVALID, "frame too large");
    return VCF_OK;
}

}  // namespace
}  // namespace vcf

using namespace vcf;

extern "C" {

int vcf_ipp_rdo_modes(const uint8_t *cur_dev, const uint8_t *comp_dev, int32_t H, int32_t W, int32_t bs, int32_t Q,
                      double lambda, uint8_t *modes_dev, double *costs_dev, void *stream)
{
    int rc = check_frame(cur_dev, comp_dev, modes_dev, H, W, bs);
    if (rc != VCF_OK) return rc;
    if (Q < 1) return set_error(VCF_ERR_INVALID, "quantization step %d", Q);
    if (H / bs == 0 || W / bs == 0) return VCF_OK;   // no full block: empty mode map
    rc = ensure_tables();
    if (rc != VCF_OK) return rc;
    const hipStream_t s = (hipStream_t)stream;
    switch (bs) {
    case 2: return launch_modes<2>(cur_dev, comp_dev, H, W, Q, lambda, modes_dev, costs_dev, s);
    case 4: return launch_modes<4>(cur_dev, comp_dev, H, W, Q, lambda, modes_dev, costs_dev, s);
    case 8: return launch_modes<8>(cur_dev, comp_dev, H, W, Q, lambda, modes_dev, costs_dev, s);
    case 12: return launch_modes<12>(cur_dev, comp_dev, H, W, Q, lambda, modes_dev, costs_dev, s);
    case 16: return launch_modes<16>(cur_dev, comp_dev, H, W, Q, lambda, modes_dev, costs_dev, s);
    case 24: return launch_modes<24>(cur_dev, comp_dev, H, W, Q, lambda, modes_dev, costs_dev, s);
    case 32: return launch_modes<32>(cur_dev, comp_dev, H, W, Q, lambda, modes_dev, costs_dev, s);
    default:
        return set_error(VCF_ERR_UNSUPPORTED, "RDO block size %d: supported 2, 4, 8, 12, 16, 24, 32", bs);
    }
}

int vcf_ipp_rdo_residual(const uint8_t *cur_dev, const uint8_t *comp_dev, const uint8_t *modes_dev, int32_t H,
                         int32_t W, int32_t bs, uint8_t *out_dev, void *stream)
{
    int rc = check_frame(cur_dev, comp_dev, out_dev, H, W, bs);
    if (rc != VCF_OK) return rc;
    if (!modes_dev && H / bs > 0 && W / bs > 0) return set_error(VCF_ERR_INVALID, "null mode map");
    const long long n = (long long)H * W * 3;
    hipLaunchKernelGGL(ipp_rdo_residual_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, cur_dev, comp_dev, modes_dev, H, W, bs, out_dev);
    return hip_check(hipGetLastError(), "ipp_rdo_residual_kernel launch");
}

int vcf_ipp_rdo_reconstruct(const uint8_t *comp_dev, const uint8_t *rec_dev, const uint8_t *modes_dev, int32_t H,
                            int32_t W, int32_t bs, uint8_t *out_dev, void *stream)
{
    int rc = check_frame(comp_dev, rec_dev, out_dev, H, W, bs);
    if (rc != VCF_OK) return rc;
    if (!modes_dev && H / bs > 0 && W / bs > 0) return set_error(VCF_ERR_INVALID, "null mode map");
    const long long n = (long long)H * W * 3;
    hipLaunchKernelGGL(ipp_rdo_reconstruct_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, comp_dev, rec_dev, modes_dev, H, W, bs, out_dev);
    return hip_check(hipGetLastError(), "ipp_rdo_reconstruct_kernel launch");
}

}  // extern "C"
