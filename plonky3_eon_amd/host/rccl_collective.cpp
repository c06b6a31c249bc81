// eon_collective over RCCL: the lane-sharded prove's two all-gathers (partial quotients,
// per-column records) as ncclAllGather and the four-step DFT's transposes as ncclAllToAll, on
// device buffers, enqueued on the context's stream -- xGMI peer-to-peer on an MI355X node, no host
// staging.
#include <rccl/rccl.h>

#include <cstring>

#include "eon_prove.h"

namespace {

int rccl_all_gather(void* user, const void* send, void* recv, uint64_t bytes, void* stream) {
    ncclComm_t comm = static_cast<ncclComm_t>(user);
    const ncclResult_t r =
        ncclAllGather(send, recv, (size_t)bytes, ncclUint8, comm, static_cast<hipStream_t>(stream));
    return r == ncclSuccess ? 0 : -(int)r;
}

int rccl_all_to_all(void* user, const void* send, void* recv, uint64_t bytes, void* stream) {
    ncclComm_t comm = static_cast<ncclComm_t>(user);
    const ncclResult_t r =
        ncclAllToAll(send, recv, (size_t)bytes, ncclUint8, comm, static_cast<hipStream_t>(stream));
    return r == ncclSuccess ? 0 : -(int)r;
}

}  // namespace

extern "C" {

int eon_rccl_unique_id(uint8_t id[128]) {
    if (!id) return EON_E_ARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return EON_E_DEVICE;
    static_assert(sizeof(u.internal) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(id, u.internal, 128);
    return EON_OK;
}

int eon_rccl_collective_init(uint32_t rank, uint32_t world, const uint8_t id[128], eon_collective* out) {
    if (!id || !out || world == 0 || rank >= world) return EON_E_ARG;
    ncclUniqueId u;
    std::memcpy(u.internal, id, 128);
    ncclComm_t comm = nullptr;
    if (ncclCommInitRank(&comm, (int)world, u, (int)rank) != ncclSuccess) return EON_E_DEVICE;
    out->rank = rank;
    out->world = world;
    out->all_gather = rccl_all_gather;
    out->all_to_all = rccl_all_to_all;
    out->user = comm;
    return EON_OK;
}

void eon_rccl_collective_finalize(eon_collective* coll) {
    if (!coll || !coll->user) return;
    ncclCommDestroy(static_cast<ncclComm_t>(coll->user));
    coll->user = nullptr;
    coll->all_gather = nullptr;
    coll->all_to_all = nullptr;
}

}  // extern "C"
