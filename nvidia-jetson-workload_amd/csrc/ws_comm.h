// y-slab halo exchange over RCCL between the processes of a slab decomposition: the plan
// of ws_halo.h (one packed message per neighbour), moved with ncclSend / ncclRecv.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <vector>

#include "ws_halo.h"
#include "ws_internal.h"

namespace ws {

struct CommError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// Balanced row partition: rank r owns [H*r/n, H*(r+1)/n).
inline void slab_rows(int H, int rank, int nranks, int* row0, int* rows) {
    const int r0 = (int)((int64_t)H * rank / nranks), r1 = (int)((int64_t)H * (rank + 1) / nranks);
    *row0 = r0;
    *rows = r1 - r0;
}

class SlabComm {
public:
    static void unique_id(uint8_t* id128);
    SlabComm(int rank, int nranks, const uint8_t* id128);
    ~SlabComm();
    SlabComm(const SlabComm&) = delete;
    SlabComm& operator=(const SlabComm&) = delete;

    int rank() const { return rank_; }
    int nranks() const { return nranks_; }

    // Exchange `depth` halo rows of `nfields` level-stacked fields (row 0 of level 0 at
    // fields[i]) with both neighbours, enqueued on `stream`: pack each neighbour's segments
    // into one message (halo_pack), one grouped RCCL send / recv per neighbour, unpack.
    // periodic: the ring closes (rank 0 <-> rank n-1; make_halo_plan), always packed.
    void exchange(void* const* fields, int nfields, int elem_size, const Geom& g, int depth, hipStream_t stream,
                  bool periodic = false);
    // Block all-to-all (the vorticity model's spectrum transposes): send[i] goes to rank
    // send[i].peer, recv[i] arrives from rank recv[i].peer -- one block per peer and direction,
    // so the pairs match whatever the posting order; this rank's own block is a device copy.
    struct Block {
        void* ptr;
        size_t bytes;
        int peer;
    };
    void alltoall(const std::vector<Block>& send, const std::vector<Block>& recv, hipStream_t stream);
    // rank `root`'s n int32 values to every rank (host in, host out; synchronises `stream`)
    void broadcast_i32(int32_t* v, int n, int root, hipStream_t stream);
    // In-place max over ranks of one double (device scratch owned by the comm).
    double allreduce_max(double v, hipStream_t stream);
    // In-place max over ranks of n uint64 values in DEVICE memory, enqueued on `stream` (the
    // CFL reduction's per-level bit patterns, ws_reduce.hip)
    void allreduce_max_u64_device(uint64_t* d, int n, hipStream_t stream);
    void barrier(hipStream_t stream);

private:
    int rank_ = 0, nranks_ = 1;
    void* comm_ = nullptr;  // ncclComm_t
    double* scratch_ = nullptr;
    HaloStaging staging_;
};

}  // namespace ws
