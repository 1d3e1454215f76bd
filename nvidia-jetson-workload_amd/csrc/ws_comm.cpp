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
    hcheck(hipMalloc(&scratch_, sizeof(double)), "hipMalloc");
}

SlabComm::~SlabComm() {
    if (comm_) ncclCommDestroy((ncclComm_t)comm_);
    if (scratch_) (void)hipFree(scratch_);
}

void SlabComm::exchange(void* const* fields, int nfields, int elem_size, const Geom& g, int depth, hipStream_t stream) {
    if (nranks_ == 1) return;
    const ncclComm_t c = (ncclComm_t)comm_;
    const size_t row_bytes = (size_t)g.pitch * elem_size;
    const size_t bytes = row_bytes * depth;
    const size_t lbytes = (size_t)g.lstride * elem_size;
    check(ncclGroupStart(), "ncclGroupStart");
    for (int f = 0; f < nfields; ++f) {
        char* base = (char*)fields[f];
        for (int l = 0; l < g.L; ++l) {
            char* lv = base + (size_t)l * lbytes;
            if (rank_ > 0) {  // my top rows <-> upper neighbour's bottom rows
                check(ncclSend(lv, bytes, ncclChar, rank_ - 1, c, stream), "ncclSend");
                check(ncclRecv(lv - bytes, bytes, ncclChar, rank_ - 1, c, stream), "ncclRecv");
            }
            if (rank_ < nranks_ - 1) {
                check(ncclSend(lv + (size_t)(g.H - depth) * row_bytes, bytes, ncclChar, rank_ + 1, c, stream),
                      "ncclSend");
                check(ncclRecv(lv + (size_t)g.H * row_bytes, bytes, ncclChar, rank_ + 1, c, stream), "ncclRecv");
            }
        }
    }
    check(ncclGroupEnd(), "ncclGroupEnd");
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

void SlabComm::barrier(hipStream_t stream) { (void)allreduce_max(0.0, stream); }

}  // namespace ws
