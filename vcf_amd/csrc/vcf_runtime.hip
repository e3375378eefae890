// vcf_runtime.hip -- device, memory, stream and event entry points of the
// C ABI (include/vcf_amd.h) plus the thread-local error channel.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

#include "vcf_amd.h"
#include "vcf_internal.h"

namespace vcf {

static thread_local char g_err[512] = "";

int set_error(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int hip_check(hipError_t e, const char *what)
{
    if (e == hipSuccess) return VCF_OK;
    return set_error(VCF_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

}  // namespace vcf

using vcf::hip_check;

extern "C" {

const char *vcf_last_error(void) { return vcf::g_err; }

int vcf_version(int *major, int *minor)
{
    if (!major || !minor) return vcf::set_error(VCF_ERR_INVALID, "null pointer");
    *major = 0;
    *minor = 1;
    return VCF_OK;
}

int vcf_device_count(int *n)
{
    if (!n) return vcf::set_error(VCF_ERR_INVALID, "null pointer");
    return hip_check(hipGetDeviceCount(n), "hipGetDeviceCount");
}

int vcf_set_device(int device) { return hip_check(hipSetDevice(device), "hipSetDevice"); }

int vcf_get_device(int *device)
{
    if (!device) return vcf::set_error(VCF_ERR_INVALID, "null pointer");
    return hip_check(hipGetDevice(device), "hipGetDevice");
}

int vcf_device_sync(void) { return hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize"); }

int vcf_malloc(void **ptr, size_t bytes)
{
    if (!ptr) return vcf::set_error(VCF_ERR_INVALID, "null pointer");
    return hip_check(hipMalloc(ptr, bytes), "hipMalloc");
}

int vcf_free(void *ptr) { return hip_check(hipFree(ptr), "hipFree"); }

int vcf_host_alloc(void **ptr, size_t bytes)
{
    if (!ptr) return vcf::set_error(VCF_ERR_INVALID, "null pointer");
    return hip_check(hipHostMalloc(ptr, bytes, hipHostMallocDefault), "hipHostMalloc");
}

int vcf_host_free(void *ptr) { return hip_check(hipHostFree(ptr), "hipHostFree"); }

int vcf_memcpy_htod(void *dst, const void *src, size_t bytes, void *stream)
{
    return hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream),
                     "hipMemcpyAsync(H2D)");
}

int vcf_memcpy_dtoh(void *dst, const void *src, size_t bytes, void *stream)
{
    return hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream),
                     "hipMemcpyAsync(D2H)");
}

int vcf_memcpy_dtod(void *dst, const void *src, size_t bytes, void *stream)
{
    return hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream),
                     "hipMemcpyAsync(D2D)");
}

int vcf_memset(void *dst, int value, size_t bytes, void *stream)
{
    return hip_check(hipMemsetAsync(dst, value, bytes, (hipStream_t)stream), "hipMemsetAsync");
}

int vcf_stream_create(void **stream)
{
    if (!stream) return vcf::set_error(VCF_ERR_INVALID, "null pointer");
    hipStream_t s;
    int rc = hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    if (rc == VCF_OK) *stream = (void *)s;
    return rc;
}

int vcf_stream_destroy(void *stream)
{
    return hip_check(hipStreamDestroy((hipStream_t)stream), "hipStreamDestroy");
}

int vcf_stream_sync(void *stream)
{
    return hip_check(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize");
}

int vcf_event_create(void **event)
{
    if (!event) return vcf::set_error(VCF_ERR_INVALID, "null pointer");
    hipEvent_t e;
    int rc = hip_check(hipEventCreate(&e), "hipEventCreate");
    if (rc == VCF_OK) *event = (void *)e;
    return rc;
}

int vcf_event_destroy(void *event)
{
    return hip_check(hipEventDestroy((hipEvent_t)event), "hipEventDestroy");
}

int vcf_event_record(void *event, void *stream)
{
    return hip_check(hipEventRecord((hipEvent_t)event, (hipStream_t)stream), "hipEventRecord");
}

int vcf_event_sync(void *event)
{
    return hip_check(hipEventSynchronize((hipEvent_t)event), "hipEventSynchronize");
}

// piece p: table[3p] = source offset, table[3p + 1] = destination offset,
// table[3p + 2] = bytes; one workgroup per piece, dword copies when aligned
__global__ __launch_bounds__(256) void copy_pieces_kernel(const uint8_t *__restrict__ src,
                                                          const int64_t *__restrict__ table,
                                                          uint8_t *__restrict__ dst)
{
    const int64_t so = table[3 * blockIdx.x], d = table[3 * blockIdx.x + 1], nb = table[3 * blockIdx.x + 2];
    const uint8_t *s = src + so;
    uint8_t *o = dst + d;
    if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(o)) & 3) == 0) {
        const int64_t nw = nb >> 2;
        for (int64_t i = threadIdx.x; i < nw; i += 256)
            reinterpret_cast<uint32_t *>(o)[i] = reinterpret_cast<const uint32_t *>(s)[i];
        for (int64_t i = 4 * nw + threadIdx.x; i < nb; i += 256) o[i] = s[i];
    } else {
        for (int64_t i = threadIdx.x; i < nb; i += 256) o[i] = s[i];
    }
}

int vcf_copy_pieces(const uint8_t *src_dev, const int64_t *table_dev, int64_t n_pieces, uint8_t *dst_dev, void *stream)
{
    if (n_pieces < 0 || n_pieces > 0x7FFFFFFF) return vcf::set_error(VCF_ERR_INVALID, "piece count");
    if (n_pieces == 0) return VCF_OK;
    if (!src_dev || !table_dev || !dst_dev) return vcf::set_error(VCF_ERR_INVALID, "null buffer");
    copy_pieces_kernel<<<(unsigned)n_pieces, 256, 0, (hipStream_t)stream>>>(src_dev, table_dev, dst_dev);
    return hip_check(hipGetLastError(), "copy_pieces_kernel");
}

int vcf_stream_wait_event(void *stream, void *event)
{
    return hip_check(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0), "hipStreamWaitEvent");
}

int vcf_event_elapsed_ms(void *start, void *stop, float *ms)
{
    if (!ms) return vcf::set_error(VCF_ERR_INVALID, "null pointer");
    return hip_check(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop),
                     "hipEventElapsedTime");
}

}  // extern "C"
