// vcf_pocketfft_tables.h -- the twiddle tables vcf_pocketfft.h's transforms
// read: pocketfft's sincos_2pibyn values (computed on the host in double,
// exactly as pocketfft computes them) for every covered length, uploaded once
// per device into __constant__ memory.  Each translation unit that includes
// this gets its own copy of the tables (no relocatable device code).
// Restates pocketfft (BSD-3-Clause, Copyright (C) 2010-2019 Max-Planck-Society);
// license text in THIRD_PARTY_NOTICES.md.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <mutex>

#include "vcf_amd.h"
#include "vcf_internal.h"
#include "vcf_pocketfft.h"
#include "vcf_sincos.h"

namespace vcf {
namespace {

// supported lengths: the 5-smooth B <= 128 (pocketfft's radix-2/3/4/5 passes)
constexpr int kNumSlots = 38;
constexpr int kLens[kNumSlots] = {1,  2,  3,  4,  5,  6,  8,  9,  10, 12,  15,  16,  18,  20,  24,  25,  27,  30,  32,
                                  36, 40, 45, 48, 50, 54, 60, 64, 72, 75, 80, 81, 90, 96, 100, 108, 120, 125, 128};
constexpr int slot_of(int n)
{
    for (int i = 0; i < kNumSlots; ++i)
        if (kLens[i] == n) return i;
    return -1;
}
// a length's table: its rfftp twiddles, then N DCT twiddles, then fct (<= 2N + 1 values)
constexpr int slot_size(int n) { return 2 * n + 1; }
constexpr int slot_off(int n)
{
    int off = 0;
    for (int i = 0; i < kNumSlots && kLens[i] != n; ++i) off += slot_size(kLens[i]);
    return off;
}
constexpr int kTableSize = slot_off(1 << 30);   // all slots

__constant__ float c_tw_f32[kTableSize];
__constant__ double c_tw_f64[kTableSize];

// One slot: rfftp<T>::comp_twiddle values, T_dcst23's twiddle, fct.
template <typename T> void fill_slot(int n, T *slot)
{
    const pfft::Factors F = pfft::factorize(n);
    size_t l1 = 1;
    for (int k = 0; k < F.n; ++k) {
        const int ip = F.f[k], ido = n / ((int)l1 * ip);
        if (k < F.n - 1)
            for (int j = 1; j < ip; ++j)
                for (int i = 1; i <= (ido - 1) / 2; ++i) {
                    T re, im;
                    sincos_2pibyn<T>((size_t)n, (size_t)j * l1 * i, re, im);
                    slot[F.tw_off[k] + (j - 1) * (ido - 1) + 2 * i - 2] = re;
                    slot[F.tw_off[k] + (j - 1) * (ido - 1) + 2 * i - 1] = im;
                }
        l1 *= ip;
    }
    for (int i = 0; i < n; ++i) {
        T re, im;
        sincos_2pibyn<T>(4 * (size_t)n, (size_t)i + 1, re, im);
        slot[F.tw_len + i] = re;
    }
    slot[F.tw_len + n] = T(1 / std::sqrt((long double)(2 * n)));   // pypocketfft norm_fct
}

int ensure_tables()
{
    static std::mutex mu;
    static bool done[64] = {};
    int dev = 0;
    int rc = hip_check(hipGetDevice(&dev), "hipGetDevice");
    if (rc != VCF_OK) return rc;
    if (dev < 0 || dev >= 64) return set_error(VCF_ERR_INVALID, "device %d", dev);
    std::lock_guard<std::mutex> lock(mu);
    if (done[dev]) return VCF_OK;
    static float tf[kTableSize];
    static double td[kTableSize];
    for (int s = 0; s < kNumSlots; ++s) {
        fill_slot<float>(kLens[s], tf + slot_off(kLens[s]));
        fill_slot<double>(kLens[s], td + slot_off(kLens[s]));
    }
    rc = hip_check(hipMemcpyToSymbol(HIP_SYMBOL(c_tw_f32), tf, sizeof(tf)), "twiddle upload");
    if (rc != VCF_OK) return rc;
    rc = hip_check(hipMemcpyToSymbol(HIP_SYMBOL(c_tw_f64), td, sizeof(td)), "twiddle upload");
    if (rc != VCF_OK) return rc;
    done[dev] = true;
    return VCF_OK;
}


}  // namespace
}  // namespace vcf
