// vcf_pipeline.h -- frame pipelines over library streams (shared by the
// 2D-DWT and DCT launchers).  A batch of independent frames is cut into
// chunks whose launches run on the library's own streams, forked from the
// caller's stream by an event and joined back to it, so a call keeps its
// stream semantics; each chunk touches only its own frames' buffers.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>

#include "vcf_amd.h"
#include "vcf_internal.h"

namespace vcf {
namespace {

constexpr int kAuxStreams = 4, kMaxChunks = 16;

// stagger: the level that fills the chip (level 1 of either direction) of
// chunk k waits for chunk k-1's to finish, so those kernels run one after
// another at full width while the small levels fill in beside them
struct PipeHook {
    hipEvent_t wait = nullptr;   // before the big level (null: none)
    hipEvent_t rec = nullptr;    // recorded after it
};

struct AuxStreams {
    std::mutex mu;
    bool ready = false;
    hipStream_t s[kAuxStreams] = {};
    hipEvent_t fork = nullptr, join[kAuxStreams] = {}, big[kMaxChunks] = {};

    int init()
    {
        if (ready) return VCF_OK;
        int rc = hip_check(hipEventCreateWithFlags(&fork, hipEventDisableTiming), "hipEventCreate");
        for (int j = 0; rc == VCF_OK && j < kAuxStreams; ++j) {
            rc = hip_check(hipStreamCreateWithFlags(&s[j], hipStreamNonBlocking), "hipStreamCreate");
            if (rc == VCF_OK) rc = hip_check(hipEventCreateWithFlags(&join[j], hipEventDisableTiming), "hipEventCreate");
        }
        for (int j = 0; rc == VCF_OK && j < kMaxChunks; ++j)
            rc = hip_check(hipEventCreateWithFlags(&big[j], hipEventDisableTiming), "hipEventCreate");
        ready = rc == VCF_OK;
        return rc;
    }
};

AuxStreams &aux_for_current_device()
{
    static AuxStreams per_dev[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    return per_dev[dev];
}

// how a batch is pipelined: `chunks` chunks of consecutive frames round-robin
// over `streams` library streams, staggered or not; streams == 0: no pipeline
struct PipeShape {
    int streams = 0, chunks = 0;
    bool stagger = false;
    bool caller = false;   // the caller's stream is stream 0 (no fork wait or join on it)
};

// run chain(first_frame, n, stream, hook) per chunk, ordered after and before
// the caller's stream s
template <typename Chain>
int run_pipelined(long long n_frames, PipeShape ps, hipStream_t s, Chain &&chain)
{
    AuxStreams &ax = aux_for_current_device();
    std::lock_guard<std::mutex> lock(ax.mu);
    int rc = ax.init();
    if (rc != VCF_OK) return rc;
    const int ns = std::max(1, std::min(ps.streams, kAuxStreams));
    const long long nc = std::max(1LL, std::min<long long>({(long long)ps.chunks, (long long)kMaxChunks, n_frames}));
    const long long chunk = (n_frames + nc - 1) / nc;
    // stream j of the pipeline: the caller's own for j = 0 when ps.caller, else a library stream
    const int j0 = ps.caller ? 1 : 0;
    auto stream_of = [&](int j) { return ps.caller && j == 0 ? s : ax.s[j - j0]; };
    if ((rc = hip_check(hipEventRecord(ax.fork, s), "hipEventRecord")) != VCF_OK) return rc;
    for (int j = j0; j < ns; ++j)
        if ((rc = hip_check(hipStreamWaitEvent(stream_of(j), ax.fork, 0), "hipStreamWaitEvent")) != VCF_OK)
            return rc;
    int k = 0;
    for (long long f0 = 0; f0 < n_frames; f0 += chunk, ++k) {
        PipeHook hook;
        if (ps.stagger) {
            hook.wait = k > 0 ? ax.big[k - 1] : nullptr;
            hook.rec = ax.big[k];
        }
        if ((rc = chain(f0, std::min(chunk, n_frames - f0), stream_of(k % ns), ps.stagger ? &hook : nullptr)) !=
            VCF_OK)
            break;
    }
    // join every library stream even after an error, so the caller's stream never runs ahead
    for (int j = 0; j < ns - j0; ++j) {
        int r2 = hip_check(hipEventRecord(ax.join[j], ax.s[j]), "hipEventRecord");
        if (r2 == VCF_OK) r2 = hip_check(hipStreamWaitEvent(s, ax.join[j], 0), "hipStreamWaitEvent");
        if (rc == VCF_OK) rc = r2;
    }
    return rc;
}

[[maybe_unused]] int hook_wait(const PipeHook *h, hipStream_t s)
{
    return h && h->wait ? hip_check(hipStreamWaitEvent(s, h->wait, 0), "hipStreamWaitEvent") : VCF_OK;
}
[[maybe_unused]] int hook_rec(const PipeHook *h, hipStream_t s)
{
    return h && h->rec ? hip_check(hipEventRecord(h->rec, s), "hipEventRecord") : VCF_OK;
}


}  // namespace
}  // namespace vcf
