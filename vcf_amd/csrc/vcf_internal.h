// vcf_internal.h -- helpers shared by the translation units of libvcf_amd.so.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace vcf {
int set_error(int code, const char *fmt, ...);
int hip_check(hipError_t e, const char *what);
// block sizes other than 8 (vcf_dct_any.hip)
int dct_any_encode_u8(const uint8_t *rgb_dev, int64_t n_frames, int32_t H, int32_t W, int32_t B, int32_t Q,
                      uint32_t flags, uint8_t *k_dev, void *stream);
int dct_any_decode_u8(const uint8_t *k_dev, int64_t n_frames, int32_t H, int32_t W, int32_t B, int32_t Q,
                      uint32_t flags, uint8_t *rgb_dev, void *stream);
}  // namespace vcf
