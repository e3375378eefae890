// vcf_internal.h -- helpers shared by the translation units of libvcf_amd.so.
#pragma once
#include <hip/hip_runtime.h>

namespace vcf {
int set_error(int code, const char *fmt, ...);
int hip_check(hipError_t e, const char *what);
}  // namespace vcf
