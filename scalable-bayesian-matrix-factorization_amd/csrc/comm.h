// comm.h -- RCCL (over xGMI) exchange between the ranks of one node.
// One process per GPU.  Users and items are block-partitioned by row; after
// each half-sweep every rank holds fresh rows only for its own block, and the
// blocks are exchanged with one grouped set of in-place ncclBroadcast calls
// (an all-gather with per-rank row counts: no padding, no repack).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace sbmf {

// RCCL's message for an ncclResult_t (RCCL is dlopen'ed on first multi-GPU use).
const char* rccl_error_string(int r);

// Test-only alternative (SBMF_COMM=host when the id is made): the same
// exchange through a POSIX shared-memory segment and a process-shared
// barrier, so the multi-rank sampler can run as several processes on ONE GPU
// (RCCL rejects two ranks on one device).  Synchronous; not a product path.
class Comm {
  public:
    Comm() = default;
    ~Comm();
    Comm(const Comm&) = delete;
    Comm& operator=(const Comm&) = delete;
    static void unique_id(uint8_t id[128]);
    void init(int nranks, int rank, const uint8_t id[128]);
    // Test only (sbmf_test_rccl_selftest): a one-rank RCCL communicator whose calls
    // are issued as with several ranks -- the block broadcasts with rank 0 as every
    // owner, the point-to-point exchange including the rank itself -- so one GPU runs
    // the exact RCCL calls of the exchange through the same dlsym table.
    void init_loopback();
    bool active() const { return comm_ != nullptr || shm_ != nullptr; }
    // ncclCommAbort: tear the communicator down without waiting for its queued
    // work (a stuck self-test); the object is inactive afterwards.
    void abort();
    // Rank k owns units [bounds[k], bounds[k+1]) of unit_bytes each, starting
    // at base; after the call every rank holds every rank's units.
    void bcast_ranges(void* base, size_t unit_bytes, const std::vector<uint64_t>& bounds, hipStream_t st);
    // The same for blocks that need not tile a range: rank k owns units
    // [starts[k], ends[k]) (a pipelined stage of every rank's block).
    void bcast_blocks(void* base, size_t unit_bytes, const std::vector<uint64_t>& starts,
                      const std::vector<uint64_t>& ends, hipStream_t st);
    // Point-to-point exchange (grouped ncclSend / ncclRecv): to every other
    // rank k, send [soff[k], soff[k] + scnt[k]) of sendbuf, and receive
    // rcnt[k] bytes from it at recvbuf + roff[k] (byte offsets and counts).
    void alltoallv(const void* sendbuf, const std::vector<size_t>& soff, const std::vector<size_t>& scnt,
                   void* recvbuf, const std::vector<size_t>& roff, const std::vector<size_t>& rcnt, hipStream_t st);

    // Bracket several of the calls below into one RCCL group (nests; no-op for
    // the host backend): their transfers run concurrently, started at group_end.
    void group_begin();
    void group_end();
    // All-gather of equal blocks (ncclAllGather): rank k's `bytes` at sendbuf
    // land at recvbuf + k * bytes on every rank.
    void allgather(const void* sendbuf, size_t bytes, void* recvbuf, hipStream_t st);
    int nranks() const { return nranks_; }
    int rank() const { return rank_; }

  private:
    void host_barrier();
    bool live() const { return nranks_ > 1 || loopback_; }
    void* comm_ = nullptr;  // ncclComm_t
    bool loopback_ = false;
    unsigned char* shm_ = nullptr;  // host backend: [barrier header | window]
    size_t shm_bytes_ = 0;
    int sense_ = 0;
    int nranks_ = 1, rank_ = 0;
};

}  // namespace sbmf
