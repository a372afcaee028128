// comm.cpp -- RCCL exchange (see comm.h).
#include "comm.h"

#include <rccl/rccl.h>

#include <cstring>
#include <string>

namespace sbmf {

[[noreturn]] void comm_fail(const char* what, ncclResult_t r);

Comm::~Comm() {
    if (comm_) (void)ncclCommDestroy((ncclComm_t)comm_);
}

void Comm::unique_id(uint8_t id[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId u;
    ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) comm_fail("ncclGetUniqueId", r);
    std::memcpy(id, &u, 128);
}

void Comm::init(int nranks, int rank, const uint8_t id[128]) {
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    ncclComm_t c;
    ncclResult_t r = ncclCommInitRank(&c, nranks, u, rank);
    if (r != ncclSuccess) comm_fail("ncclCommInitRank", r);
    comm_ = c;
    nranks_ = nranks;
    rank_ = rank;
}

void Comm::bcast_ranges(void* base, size_t unit_bytes, const std::vector<uint64_t>& bounds, hipStream_t st) {
    if (!comm_ || nranks_ <= 1) return;
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) comm_fail("ncclGroupStart", r);
    for (int k = 0; k < nranks_; ++k) {
        const size_t bytes = (size_t)(bounds[k + 1] - bounds[k]) * unit_bytes;
        if (bytes == 0) continue;
        char* p = static_cast<char*>(base) + (size_t)bounds[k] * unit_bytes;
        r = ncclBroadcast(p, p, bytes, ncclUint8, k, (ncclComm_t)comm_, st);
        if (r != ncclSuccess) comm_fail("ncclBroadcast", r);
    }
    r = ncclGroupEnd();
    if (r != ncclSuccess) comm_fail("ncclGroupEnd", r);
}

}  // namespace sbmf
