// RCCL halo exchange for y-slab decomposition (see ws_comm.h).
#include "ws_comm.h"

#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>

namespace ws {
namespace {

void check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw CommError(std::string(what) + ": " + ncclGetErrorString(r));
}

void hcheck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw CommError(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

static_assert(sizeof(ncclUniqueId) <= 128, "unique id larger than WS_COMM_ID_BYTES");

void SlabComm::unique_id(uint8_t* id128) {
    ncclUniqueId id;
    check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    std::memset(id128, 0, 128);
    std::memcpy(id128, &id, sizeof(id));
}

SlabComm::SlabComm(int rank, int nranks, const uint8_t* id128) : rank_(rank), nranks_(nranks) {
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof(id));
    ncclComm_t c = nullptr;
    check(ncclCommInitRank(&c, nranks, id, rank), "ncclCommInitRank");
    comm_ = c;
    hcheck(hipMalloc(&scratch_, 16 * sizeof(double)), "hipMalloc");
}

SlabComm::~SlabComm() {
    if (comm_) ncclCommDestroy((ncclComm_t)comm_);
    if (scratch_) (void)hipFree(scratch_);
}

void SlabComm::exchange(void* const* fields, int nfields, int elem_size, const Geom& g, int depth, hipStream_t stream,
                        bool periodic) {
    if (nranks_ == 1) return;
    if (nfields > kMaxHaloFields) throw CommError("too many fields for one exchange");
    const HaloPlan plan = make_halo_plan(g, elem_size, rank_, nranks_, nfields, depth, periodic);
    const ncclComm_t c = (ncclComm_t)comm_;
    if (halo_direct(plan) && !periodic) {
        // the plan executed literally: one send / receive per (field, level) segment, posted
        // in plan order (per neighbour: sends, then receives, field-major) on every rank, so
        // the k-th send to a peer meets that peer's k-th receive from us
        check(ncclGroupStart(), "ncclGroupStart");
        for (const HaloXfer& x : plan.xfers()) {
            char* p = (char*)fields[x.field] + x.offset;
            if (x.kind == 0) check(ncclSend(p, (size_t)x.bytes, ncclChar, x.peer, c, stream), "ncclSend");
            else check(ncclRecv(p, (size_t)x.bytes, ncclChar, x.peer, c, stream), "ncclRecv");
        }
        check(ncclGroupEnd(), "ncclGroupEnd");
        return;
    }
    staging_.ensure(plan.msg_bytes());
    HaloFields hf{};
    for (int f = 0; f < nfields; ++f) hf.f[f] = (char*)fields[f];
    for (int side = 0; side < 2; ++side)
        if (plan.has[side]) hcheck(halo_pack(plan, hf, side, staging_.send[side], stream), "halo_pack");
    const size_t bytes = (size_t)plan.msg_bytes();
    // sends side 0, side 1, then receives side 1, side 0 (ws_halo.h: with a periodic ring of
    // two ranks both sides are the same peer, and a pair's k-th send meets its k-th receive)
    check(ncclGroupStart(), "ncclGroupStart");
    for (int side = 0; side < 2; ++side)
        if (plan.has[side]) check(ncclSend(staging_.send[side], bytes, ncclChar, plan.peer[side], c, stream), "ncclSend");
    for (int side = 1; side >= 0; --side)
        if (plan.has[side]) check(ncclRecv(staging_.recv[side], bytes, ncclChar, plan.peer[side], c, stream), "ncclRecv");
    check(ncclGroupEnd(), "ncclGroupEnd");
    for (int side = 0; side < 2; ++side)
        if (plan.has[side]) hcheck(halo_unpack(plan, hf, side, staging_.recv[side], stream), "halo_unpack");
}

void SlabComm::alltoall(const std::vector<Block>& send, const std::vector<Block>& recv, hipStream_t stream) {
    const ncclComm_t c = (ncclComm_t)comm_;
    for (const Block& s : send)
        if (s.peer == rank_)
            for (const Block& r : recv)
                if (r.peer == rank_) {
                    if (r.bytes != s.bytes) throw CommError("alltoall: own block sizes differ");
                    hcheck(hipMemcpyAsync(r.ptr, s.ptr, s.bytes, hipMemcpyDeviceToDevice, stream), "hipMemcpyAsync");
                }
    if (nranks_ == 1) return;
    check(ncclGroupStart(), "ncclGroupStart");
    for (const Block& s : send)
        if (s.peer != rank_) check(ncclSend(s.ptr, s.bytes, ncclChar, s.peer, c, stream), "ncclSend");
    for (const Block& r : recv)
        if (r.peer != rank_) check(ncclRecv(r.ptr, r.bytes, ncclChar, r.peer, c, stream), "ncclRecv");
    check(ncclGroupEnd(), "ncclGroupEnd");
}

void SlabComm::broadcast_i32(int32_t* v, int n, int root, hipStream_t stream) {
    if (nranks_ == 1 || n <= 0) return;
    if (n > 16) throw CommError("broadcast_i32: at most 16 values");
    int32_t* d = (int32_t*)scratch_;  // scratch_ holds 16 doubles = 32 int32
    hcheck(hipMemcpyAsync(d, v, n * sizeof(int32_t), hipMemcpyHostToDevice, stream), "hipMemcpyAsync");
    check(ncclBroadcast(d, d, n, ncclInt32, root, (ncclComm_t)comm_, stream), "ncclBroadcast");
    hcheck(hipMemcpyAsync(v, d, n * sizeof(int32_t), hipMemcpyDeviceToHost, stream), "hipMemcpyAsync");
    hcheck(hipStreamSynchronize(stream), "hipStreamSynchronize");
}

double SlabComm::allreduce_max(double v, hipStream_t stream) {
    hcheck(hipMemcpyAsync(scratch_, &v, sizeof(double), hipMemcpyHostToDevice, stream), "hipMemcpyAsync");
    if (nranks_ > 1)
        check(ncclAllReduce(scratch_, scratch_, 1, ncclFloat64, ncclMax, (ncclComm_t)comm_, stream), "ncclAllReduce");
    double out = v;
    hcheck(hipMemcpyAsync(&out, scratch_, sizeof(double), hipMemcpyDeviceToHost, stream), "hipMemcpyAsync");
    hcheck(hipStreamSynchronize(stream), "hipStreamSynchronize");
    return out;
}

void SlabComm::allreduce_max_u64_device(uint64_t* d, int n, hipStream_t stream) {
    if (nranks_ == 1 || n <= 0) return;
    check(ncclAllReduce(d, d, (size_t)n, ncclUint64, ncclMax, (ncclComm_t)comm_, stream), "ncclAllReduce");
}

void SlabComm::barrier(hipStream_t stream) { (void)allreduce_max(0.0, stream); }

}  // namespace ws
