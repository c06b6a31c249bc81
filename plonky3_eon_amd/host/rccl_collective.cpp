// eon_collective over RCCL: the lane-sharded prove's two all-gathers (partial quotients,
// per-column records) as ncclAllGather and the four-step DFT's transposes as ncclAllToAll, on
// device buffers, enqueued on the context's stream -- xGMI peer-to-peer on an MI355X node, no host
// staging.
#include <hip/hip_runtime_api.h>
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

// Emulated exchanges for the one-GPU proxy of an N-rank prove: every slot of the all-gather's
// output receives this rank's own block, and the all-to-all sends every block to itself, as
// device-to-device copies on the same stream.  The bytes and the stream ordering are the real
// collective's; the other ranks' data are not (the results are meaningless by design).
int emulated_all_gather(void* user, const void* send, void* recv, uint64_t bytes, void* stream) {
    const uint32_t world = (uint32_t)(uintptr_t)user;
    for (uint32_t g = 0; g < world; g++)
        if (hipMemcpyAsync(static_cast<char*>(recv) + (uint64_t)g * bytes, send, bytes, hipMemcpyDeviceToDevice,
                           static_cast<hipStream_t>(stream)) != hipSuccess)
            return 1;
    return 0;
}

int emulated_all_to_all(void* user, const void* send, void* recv, uint64_t bytes, void* stream) {
    const uint32_t world = (uint32_t)(uintptr_t)user;
    return hipMemcpyAsync(recv, send, bytes * world, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)) ==
                   hipSuccess
               ? 0
               : 1;
}

}  // namespace

extern "C" {

int eon_emulated_collective_init(uint32_t rank, uint32_t world, eon_collective* out) {
    if (!out || world == 0 || rank >= world) return EON_E_ARG;
    out->rank = rank;
    out->world = world;
    out->all_gather = emulated_all_gather;
    out->all_to_all = emulated_all_to_all;
    out->user = (void*)(uintptr_t)world;
    return EON_OK;
}

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

int eon_rccl_collective_info(const eon_collective* coll, int32_t* count, int32_t* user_rank, int32_t* device,
                             char* pci_bus_id, uint32_t pci_len) {
    if (!coll || !coll->user || coll->all_gather != rccl_all_gather) return EON_E_ARG;
    ncclComm_t comm = static_cast<ncclComm_t>(coll->user);
    int n = -1, r = -1, d = -1;
    if (ncclCommCount(comm, &n) != ncclSuccess || ncclCommUserRank(comm, &r) != ncclSuccess ||
        ncclCommCuDevice(comm, &d) != ncclSuccess)
        return EON_E_DEVICE;
    if (count) *count = n;
    if (user_rank) *user_rank = r;
    if (device) *device = d;
    if (pci_bus_id && pci_len > 0) {
        pci_bus_id[0] = 0;
        if (hipDeviceGetPCIBusId(pci_bus_id, (int)pci_len, d) != hipSuccess) return EON_E_DEVICE;
    }
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
