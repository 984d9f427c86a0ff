// RCCL communicators owned by the caller and used by the library itself (ABI 10): the SEGNN SyncBN
// all-reduces (the multi-GPU form of the reference's train-mode BatchNorm, models/segnn/segnn.py:233-235,
// 257-261, 282-283) are enqueued by libnbx on the launch stream, so a sharded forward or rollout has
// no host round trip per BatchNorm and can be captured into a HIP graph.
//
// RCCL is the one in the process: under PyTorch that is torch's librccl.so.1 (same soname), so the
// communicator here and torch.distributed's share one implementation.
#include <rccl/rccl.h>

#include "nbx_internal.h"

namespace nbx {

int comm_allreduce_f64(double* buf, int64_t count, void* comm, hipStream_t st) {
    const ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, ncclFloat64, ncclSum, (ncclComm_t)comm, st);
    if (r != ncclSuccess) {
        set_error("ncclAllReduce (BatchNorm sums) failed: %s", ncclGetErrorString(r));
        return NBX_E_HIP;
    }
    return NBX_OK;
}

}  // namespace nbx

extern "C" int nbx_comm_unique_id(void* id_out) {
    NBX_CHECK_ARG(id_out != nullptr, "nbx_comm_unique_id: null output");
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        nbx::set_error("ncclGetUniqueId failed: %s", ncclGetErrorString(r));
        return NBX_E_HIP;
    }
    static_assert(sizeof(ncclUniqueId) == NBX_COMM_ID_BYTES, "RCCL unique id size");
    memcpy(id_out, &id, sizeof(id));
    return NBX_OK;
}

extern "C" int nbx_comm_init(const void* id, int32_t nranks, int32_t rank, int32_t device, void** comm_out) {
    NBX_CHECK_ARG(id != nullptr && comm_out != nullptr, "nbx_comm_init: null argument");
    NBX_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "nbx_comm_init: bad rank %d of %d", rank, nranks);
    NBX_HIP(hipSetDevice(device));
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = ncclCommInitRank(&comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        nbx::set_error("ncclCommInitRank failed: %s", ncclGetErrorString(r));
        return NBX_E_HIP;
    }
    *comm_out = comm;
    return NBX_OK;
}

extern "C" int nbx_comm_destroy(void* comm) {
    if (!comm) return NBX_OK;
    const ncclResult_t r = ncclCommDestroy((ncclComm_t)comm);
    if (r != ncclSuccess) {
        nbx::set_error("ncclCommDestroy failed: %s", ncclGetErrorString(r));
        return NBX_E_HIP;
    }
    return NBX_OK;
}

extern "C" int nbx_comm_allreduce_f64(double* buf, int64_t count, void* comm, void* stream) {
    NBX_CHECK_ARG(buf != nullptr && comm != nullptr && count >= 0, "nbx_comm_allreduce_f64: bad arguments");
    return nbx::comm_allreduce_f64(buf, count, comm, (hipStream_t)stream);
}
