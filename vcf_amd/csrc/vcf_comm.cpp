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

#include <cstring>
#include <mutex>

#include "vcf_amd.h"
#include "vcf_internal.h"

namespace vcf {
namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
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

}  // namespace
}  // namespace vcf

struct vcf_comm {
    ncclComm_t comm;
    int rank;
    int world;
    int device;
};

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

int vcf_comm_init(vcf_comm_t *out, const uint8_t *id, int rank, int world)
{
    if (!out || !id) return set_error(VCF_ERR_INVALID, "null pointer");
    if (world < 1 || rank < 0 || rank >= world) return set_error(VCF_ERR_INVALID, "rank %d of %d", rank, world);
    if (int s = vcf::need_rccl()) return s;
    int dev = 0;
    if (int s = vcf::hip_check(hipGetDevice(&dev), "hipGetDevice")) return s;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    if (int s = nccl_check(vcf::rccl().commInitRank(&c, world, u, rank), "ncclCommInitRank")) return s;
    *out = new vcf_comm{c, rank, world, dev};
    return VCF_OK;
}

int vcf_comm_destroy(vcf_comm_t comm)
{
    if (!comm) return VCF_OK;
    int s = nccl_check(vcf::rccl().commDestroy(comm->comm), "ncclCommDestroy");
    delete comm;
    return s;
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
    if (!comm || count < 0 || (count > 0 && (!send_dev || !recv_dev)))
        return set_error(VCF_ERR_INVALID, "bad all-gather arguments");
    if (count == 0) return VCF_OK;
    return nccl_check(vcf::rccl().allGather(send_dev, recv_dev, (size_t)count, ncclInt64, comm->comm,
                                            (hipStream_t)stream),
                      "ncclAllGather");
}

int vcf_comm_allreduce_f64(vcf_comm_t comm, const double *send_dev, double *recv_dev, int64_t count, int op,
                           void *stream)
{
    if (!comm || count < 0 || (count > 0 && (!send_dev || !recv_dev)))
        return set_error(VCF_ERR_INVALID, "bad all-reduce arguments");
    ncclRedOp_t o;
    switch (op) {
    case VCF_COMM_SUM: o = ncclSum; break;
    case VCF_COMM_MAX: o = ncclMax; break;
    case VCF_COMM_MIN: o = ncclMin; break;
    default: return set_error(VCF_ERR_INVALID, "unknown reduction %d", op);
    }
    if (count == 0) return VCF_OK;
    return nccl_check(vcf::rccl().allReduce(send_dev, recv_dev, (size_t)count, ncclFloat64, o, comm->comm,
                                            (hipStream_t)stream),
                      "ncclAllReduce");
}

int vcf_comm_gatherv(vcf_comm_t comm, const void *send_dev, int64_t send_bytes, void *recv_dev,
                     const int64_t *counts, int root, void *stream)
{
    if (!comm || !counts || root < 0 || root >= comm->world || send_bytes < 0)
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
    if (int st = nccl_check(R.groupStart(), "ncclGroupStart")) return st;
    int status = VCF_OK;
    if (comm->rank == root) {
        int64_t off = 0;
        for (int r = 0; r < comm->world && status == VCF_OK; ++r) {
            uint8_t *dst = (uint8_t *)recv_dev + off;
            if (counts[r] > 0) {
                if (r == root)
                    status = vcf::hip_check(hipMemcpyAsync(dst, send_dev, (size_t)counts[r],
                                                           hipMemcpyDeviceToDevice, s),
                                            "hipMemcpyAsync");
                else
                    status = nccl_check(R.recv(dst, (size_t)counts[r], ncclUint8, r, comm->comm, s), "ncclRecv");
            }
            off += counts[r];
        }
    } else if (send_bytes > 0) {
        status = nccl_check(R.send(send_dev, (size_t)send_bytes, ncclUint8, root, comm->comm, s), "ncclSend");
    }
    int end = nccl_check(R.groupEnd(), "ncclGroupEnd");
    return status != VCF_OK ? status : end;
}

}  // extern "C"
