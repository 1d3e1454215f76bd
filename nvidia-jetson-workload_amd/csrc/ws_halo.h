// Halo exchange plan of the y-slab decomposition, and its pack / unpack kernels.
//
// The reference has no distributed path; this is new. Rank r owns rows
// [row0, row0 + H) of the global grid. For an exchange of `depth` rows of `nfields`
// level-stacked fields, its top `depth` rows of every (field, level) go to rank r-1 (which
// stores them as rows [H', H' + depth) of the same field and level) and its bottom `depth`
// rows go to rank r+1 (stored as rows [-depth, 0)). The plan lists every such segment as a
// byte range relative to the field's row 0 of level 0, in the order the segments are
// concatenated into the ONE message per neighbour: field-major, then level. The transports
// (RCCL send/recv between processes, ws_comm.cpp; device copies between the slabs of one
// process, ws_runtime.cpp group_exchange) both pack the plan's send segments into a staging
// buffer with halo_pack, move the message, and scatter it with halo_unpack -- so one plan
// and one pair of kernels serve both, and the slab-group tests exercise them on the GPU.
// The global top / bottom edges keep the reference's clamp-to-self stencil
// (Geom::top_clamp / bot_clamp): no segment there. A periodic plan (the doubly periodic
// layered model, ws_layered_pe.hip) closes the ring instead: rank 0's upper neighbour is rank
// n-1 and rank n-1's lower one rank 0 -- with two ranks both neighbours are the same peer,
// so the transports post the sends side 0 then side 1 and the receives side 1 then side 0:
// a pair's k-th send meets the peer's k-th receive (my top rows -> its bottom halo first).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "ws_internal.h"

namespace ws {

// one segment of an exchange (mirrors ws_xfer_t of the C ABI)
struct HaloXfer {
    int32_t peer;         // neighbour rank
    int32_t kind;         // 0 = send, 1 = receive
    int32_t field;        // index into the exchanged field list
    int32_t level;
    int64_t offset;       // bytes from the field's row 0 of level 0
    int64_t bytes;
    int64_t msg_offset;   // bytes into the message exchanged with `peer`
};

constexpr int kMaxHaloFields = 8;

// side 0 = the upper neighbour (rank - 1), side 1 = the lower one (rank + 1)
struct HaloPlan {
    int32_t nfields = 0, L = 0, depth = 0;
    int64_t seg_bytes = 0;   // depth rows
    int64_t lbytes = 0;      // level stride
    bool has[2] = {false, false};
    int32_t peer[2] = {-1, -1};
    int64_t send_off[2] = {0, 0}, recv_off[2] = {0, 0};  // within one level, from row 0
    int64_t msg_bytes() const { return seg_bytes * nfields * L; }
    std::vector<HaloXfer> xfers() const;
};

HaloPlan make_halo_plan(const Geom& g, int elem_size, int rank, int nranks, int nfields, int depth,
                        bool periodic = false);

// Transport choice: with few segments per neighbour (SWE: 3 fields x 1 level) each segment
// moves by its own send / receive straight between the field rows (no pack / unpack
// kernels on the exchange's critical path); with many (PE: 3 x L levels) they are packed
// into one message per neighbour.
constexpr int kDirectSegs = 4;
inline bool halo_direct(const HaloPlan& p) { return p.nfields * p.L <= kDirectSegs; }

struct HaloFields {
    char* f[kMaxHaloFields];
};

// gather side `side`'s send segments of `fields` into dst (msg_bytes), in plan order
hipError_t halo_pack(const HaloPlan& p, const HaloFields& fields, int side, void* dst, hipStream_t s);
// scatter a received message into side `side`'s halo rows of `fields`
hipError_t halo_unpack(const HaloPlan& p, const HaloFields& fields, int side, const void* src, hipStream_t s);

// Measurement aid (a slab without a communicator, ws_sim_create_slab_emulated): one workgroup that
// holds the stream for `us` microseconds of wall clock -- the place of the transfer in the
// schedule, without the transfer.
hipError_t emulated_transfer(double us, hipStream_t s);

// Per-slab staging buffers for the two neighbour messages (send and receive), grown on
// demand (device memory, freed with the slab).
class HaloStaging {
public:
    HaloStaging() = default;
    ~HaloStaging();
    HaloStaging(const HaloStaging&) = delete;
    HaloStaging& operator=(const HaloStaging&) = delete;
    void ensure(int64_t bytes);  // throws std::runtime_error on allocation failure
    void* send[2] = {nullptr, nullptr};
    void* recv[2] = {nullptr, nullptr};

private:
    int64_t cap_ = 0;
};

}  // namespace ws
