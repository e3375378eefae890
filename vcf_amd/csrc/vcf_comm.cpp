// vcf_comm.cpp -- the cross-rank exchange of the frame-sharded drivers on
// RCCL over xGMI.
//
// Replaces the reference's sequential frame loop as the place where coded
// frames come together (src/III.py:77-115 encode, :132-144 decode: one
// process writes /tmp/encoded_%04d.* for every frame).  With frames sharded
// across one process per GPU the only exchange is after coding:
//   1. an all-gather of the per-frame code-stream sizes (int64), and
//   2. a gather of the variable-length payloads to rank 0.
// RCCL has no gatherv, so (2) is one grouped ncclSend per peer and P-1
// ncclRecv on the root: on xGMI every peer has its own link to rank 0, the
// P-1 transfers run concurrently and the step is link-bound, not ring-bound.
//
// librccl (~570 MB) is opened with dlopen on first use, so processes that
// never exchange anything do not pay for loading it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

#include "vcf_amd.h"
#include "vcf_internal.h"

namespace vcf {
namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
    decltype(&ncclCommInitRankConfig) commInitRankConfig = nullptr;
    decltype(&ncclCommGetAsyncError) commGetAsyncError = nullptr;
    decltype(&ncclCommAbort) commAbort = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclGetErrorString) getErrorString = nullptr;
    decltype(&ncclAllGather) allGather = nullptr;
    decltype(&ncclAllReduce) allReduce = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    bool ok = false;
    char why[256] = "";
};

Rccl &rccl()
{
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char *names[] = {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"};
        void *h = nullptr;
        for (const char *n : names)
            if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) {
            snprintf(r.why, sizeof(r.why), "dlopen(librccl.so.1): %s", dlerror());
            return;
        }
#define VCF_SYM(field, name)                                                  \
    r.field = reinterpret_cast<decltype(r.field)>(dlsym(h, name));            \
    if (!r.field) {                                                           \
        snprintf(r.why, sizeof(r.why), "librccl: symbol %s missing", name);   \
        return;                                                               \
    }
        VCF_SYM(getUniqueId, "ncclGetUniqueId");
        VCF_SYM(commInitRank, "ncclCommInitRank");
        VCF_SYM(commInitRankConfig, "ncclCommInitRankConfig");
        VCF_SYM(commGetAsyncError, "ncclCommGetAsyncError");
        VCF_SYM(commAbort, "ncclCommAbort");
        VCF_SYM(commDestroy, "ncclCommDestroy");
        VCF_SYM(getErrorString, "ncclGetErrorString");
        VCF_SYM(allGather, "ncclAllGather");
        VCF_SYM(allReduce, "ncclAllReduce");
        VCF_SYM(send, "ncclSend");
        VCF_SYM(recv, "ncclRecv");
        VCF_SYM(groupStart, "ncclGroupStart");
        VCF_SYM(groupEnd, "ncclGroupEnd");
#undef VCF_SYM
        r.ok = true;
    });
    return r;
}

int need_rccl()
{
    Rccl &r = rccl();
    return r.ok ? VCF_OK : set_error(VCF_ERR_UNSUPPORTED, "%s", r.why);
}

int nccl_check(ncclResult_t e, const char *what)
{
    if (e == ncclSuccess) return VCF_OK;
    return set_error(VCF_ERR_HIP, "%s: %s", what, rccl().getErrorString(e));
}

using Clock = std::chrono::steady_clock;

int64_t default_timeout_ms()
{
    const char *e = getenv("VCF_COMM_TIMEOUT_MS");
    const long long v = e ? atoll(e) : 0;
    return v > 0 ? (int64_t)v : 120000;
}

// Poll a non-blocking communicator until its pending operation (init, an
// enqueue, a group end) has left ncclInProgress.  Past the deadline the
// communicator is aborted: a peer that never arrives ends the job with an
// error instead of a hang (the launcher then sees a non-zero exit).
int settle(ncclComm_t c, ncclResult_t first, int64_t timeout_ms, const char *what, bool *aborted)
{
    Rccl &R = rccl();
    if (first != ncclSuccess && first != ncclInProgress) {
        R.commAbort(c);
        *aborted = true;
        return nccl_check(first, what);
    }
    const auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms);
    for (;;) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t q = R.commGetAsyncError(c, &st);
        if (q != ncclSuccess) st = q;
        if (st == ncclSuccess) return VCF_OK;
        if (st != ncclInProgress) {
            R.commAbort(c);
            *aborted = true;
            return nccl_check(st, what);
        }
        if (Clock::now() > deadline) {
            R.commAbort(c);
            *aborted = true;
            return set_error(VCF_ERR_TIMEOUT, "%s: no progress within %lld ms (RCCL communicator aborted)", what,
                             (long long)timeout_ms);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

}  // namespace
}  // namespace vcf

struct vcf_comm {
    ncclComm_t comm;
    int rank;
    int world;
    int device;
    int64_t timeout_ms;
    bool aborted;
};

static int comm_usable(vcf_comm_t c)
{
    if (!c) return vcf::set_error(VCF_ERR_INVALID, "null communicator");
    if (c->aborted) return vcf::set_error(VCF_ERR_TIMEOUT, "the communicator was aborted after an earlier failure");
    return VCF_OK;
}

using vcf::nccl_check;
using vcf::set_error;

extern "C" {

int vcf_comm_unique_id(uint8_t *id, size_t cap)
{
    if (!id || cap < VCF_COMM_ID_BYTES) return set_error(VCF_ERR_INVALID, "id buffer smaller than %d bytes",
                                                         VCF_COMM_ID_BYTES);
    if (int s = vcf::need_rccl()) return s;
    ncclUniqueId u;
    if (int s = nccl_check(vcf::rccl().getUniqueId(&u), "ncclGetUniqueId")) return s;
    static_assert(sizeof(u) == VCF_COMM_ID_BYTES, "ncclUniqueId size");
    memcpy(id, &u, sizeof(u));
    return VCF_OK;
}

int vcf_comm_init_timeout(vcf_comm_t *out, const uint8_t *id, int rank, int world, int64_t timeout_ms)
{
    if (!out || !id) return set_error(VCF_ERR_INVALID, "null pointer");
    *out = nullptr;
    if (world < 1 || rank < 0 || rank >= world) return set_error(VCF_ERR_INVALID, "rank %d of %d", rank, world);
    if (int s = vcf::need_rccl()) return s;
    if (timeout_ms <= 0) timeout_ms = vcf::default_timeout_ms();
    int dev = 0;
    if (int s = vcf::hip_check(hipGetDevice(&dev), "hipGetDevice")) return s;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    const ncclResult_t r = vcf::rccl().commInitRankConfig(&c, world, u, rank, &cfg);
    if (!c) return nccl_check(r == ncclSuccess ? ncclInternalError : r, "ncclCommInitRankConfig");
    bool aborted = false;
    if (int s = vcf::settle(c, r, timeout_ms, "ncclCommInitRankConfig", &aborted)) return s;
    *out = new vcf_comm{c, rank, world, dev, timeout_ms, false};
    return VCF_OK;
}

int vcf_comm_init(vcf_comm_t *out, const uint8_t *id, int rank, int world)
{
    return vcf_comm_init_timeout(out, id, rank, world, 0);
}

int vcf_comm_destroy(vcf_comm_t comm)
{
    if (!comm) return VCF_OK;
    int s = VCF_OK;
    if (!comm->aborted) s = nccl_check(vcf::rccl().commDestroy(comm->comm), "ncclCommDestroy");
    delete comm;
    return s;
}

int vcf_comm_wait(vcf_comm_t comm, void *stream)
{
    if (int s = comm_usable(comm)) return s;
    vcf::Rccl &R = vcf::rccl();
    const auto deadline = vcf::Clock::now() + std::chrono::milliseconds(comm->timeout_ms);
    int status = VCF_OK;
    for (;;) {
        const hipError_t e = hipStreamQuery((hipStream_t)stream);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) {
            status = vcf::hip_check(e, "hipStreamQuery");
            break;
        }
        ncclResult_t st = ncclSuccess;
        R.commGetAsyncError(comm->comm, &st);
        if (st != ncclSuccess && st != ncclInProgress) {
            R.commAbort(comm->comm);
            comm->aborted = true;
            status = nccl_check(st, "RCCL (asynchronous error)");
            break;
        }
        if (vcf::Clock::now() > deadline) {
            R.commAbort(comm->comm);
            comm->aborted = true;
            status = set_error(VCF_ERR_TIMEOUT, "stream did not finish within %lld ms (RCCL communicator aborted)",
                               (long long)comm->timeout_ms);
            break;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    (void)hipGetLastError();   // hipStreamQuery's hipErrorNotReady must not reach a later launch check
    return status;
}

int vcf_comm_rank(vcf_comm_t comm, int *rank, int *world)
{
    if (!comm || !rank || !world) return set_error(VCF_ERR_INVALID, "null pointer");
    *rank = comm->rank;
    *world = comm->world;
    return VCF_OK;
}

int vcf_comm_allgather_i64(vcf_comm_t comm, const int64_t *send_dev, int64_t count, int64_t *recv_dev,
                           void *stream)
{
    if (int s = comm_usable(comm)) return s;
    if (count < 0 || (count > 0 && (!send_dev || !recv_dev)))
        return set_error(VCF_ERR_INVALID, "bad all-gather arguments");
    if (count == 0) return VCF_OK;
    return vcf::settle(comm->comm,
                       vcf::rccl().allGather(send_dev, recv_dev, (size_t)count, ncclInt64, comm->comm,
                                             (hipStream_t)stream),
                       comm->timeout_ms, "ncclAllGather", &comm->aborted);
}

int vcf_comm_allreduce_f64(vcf_comm_t comm, const double *send_dev, double *recv_dev, int64_t count, int op,
                           void *stream)
{
    if (int s = comm_usable(comm)) return s;
    if (count < 0 || (count > 0 && (!send_dev || !recv_dev)))
        return set_error(VCF_ERR_INVALID, "bad all-reduce arguments");
    ncclRedOp_t o;
    switch (op) {
    case VCF_COMM_SUM: o = ncclSum; break;
    case VCF_COMM_MAX: o = ncclMax; break;
    case VCF_COMM_MIN: o = ncclMin; break;
    default: return set_error(VCF_ERR_INVALID, "unknown reduction %d", op);
    }
    if (count == 0) return VCF_OK;
    return vcf::settle(comm->comm,
                       vcf::rccl().allReduce(send_dev, recv_dev, (size_t)count, ncclFloat64, o, comm->comm,
                                             (hipStream_t)stream),
                       comm->timeout_ms, "ncclAllReduce", &comm->aborted);
}

int vcf_comm_gatherv(vcf_comm_t comm, const void *send_dev, int64_t send_bytes, void *recv_dev,
                     const int64_t *counts, int root, void *stream)
{
    if (int s = comm_usable(comm)) return s;
    if (!counts || root < 0 || root >= comm->world || send_bytes < 0)
        return set_error(VCF_ERR_INVALID, "bad gather arguments");
    if (counts[comm->rank] != send_bytes)
        return set_error(VCF_ERR_INVALID, "counts[%d]=%lld but this rank sends %lld bytes", comm->rank,
                         (long long)counts[comm->rank], (long long)send_bytes);
    if (send_bytes > 0 && !send_dev) return set_error(VCF_ERR_INVALID, "null send buffer");
    int64_t total = 0;
    for (int r = 0; r < comm->world; ++r) {
        if (counts[r] < 0) return set_error(VCF_ERR_INVALID, "negative count for rank %d", r);
        total += counts[r];
    }
    if (comm->rank == root && total > 0 && !recv_dev) return set_error(VCF_ERR_INVALID, "null receive buffer");
    hipStream_t s = (hipStream_t)stream;
    vcf::Rccl &R = vcf::rccl();
    if (comm->world == 1) {   // the root alone: a device copy, no RCCL call
        if (send_bytes == 0) return VCF_OK;
        return vcf::hip_check(hipMemcpyAsync(recv_dev, send_dev, (size_t)send_bytes, hipMemcpyDeviceToDevice, s),
                              "hipMemcpyAsync");
    }
    int64_t root_off = 0;   // the root's own bytes: a device copy on the same stream
    for (int r = 0; r < root; ++r) root_off += counts[r];
    if (comm->rank == root && send_bytes > 0)
        if (int st = vcf::hip_check(hipMemcpyAsync((uint8_t *)recv_dev + root_off, send_dev, (size_t)send_bytes,
                                                   hipMemcpyDeviceToDevice, s),
                                    "hipMemcpyAsync"))
            return st;
    if (int st = nccl_check(R.groupStart(), "ncclGroupStart")) return st;
    int status = VCF_OK;
    if (comm->rank == root) {
        int64_t off = 0;
        for (int r = 0; r < comm->world && status == VCF_OK; ++r) {
            if (counts[r] > 0 && r != root) {
                const ncclResult_t e = R.recv((uint8_t *)recv_dev + off, (size_t)counts[r], ncclUint8, r,
                                              comm->comm, s);
                if (e != ncclSuccess && e != ncclInProgress) status = nccl_check(e, "ncclRecv");
            }
            off += counts[r];
        }
    } else if (send_bytes > 0) {
        const ncclResult_t e = R.send(send_dev, (size_t)send_bytes, ncclUint8, root, comm->comm, s);
        if (e != ncclSuccess && e != ncclInProgress) status = nccl_check(e, "ncclSend");
    }
    const int end = vcf::settle(comm->comm, R.groupEnd(), comm->timeout_ms, "ncclGroupEnd", &comm->aborted);
    return status != VCF_OK ? status : end;
}

}  // extern "C"
