// Halo exchange plan and pack / unpack kernels (see ws_halo.h).
#include "ws_halo.h"

#include <algorithm>
#include <stdexcept>
#include <string>

namespace ws {

HaloPlan make_halo_plan(const Geom& g, int elem_size, int rank, int nranks, int nfields, int depth, bool periodic) {
    HaloPlan p;
    p.nfields = nfields;
    p.L = g.L;
    p.depth = depth;
    const int64_t row = g.pitch * (int64_t)elem_size;
    p.seg_bytes = row * depth;
    p.lbytes = g.lstride * (int64_t)elem_size;
    const bool ring = periodic && nranks > 1;
    // upper neighbour: my top rows [0, depth) <-> its bottom rows, received into [-depth, 0)
    p.has[0] = rank > 0 || ring;
    p.peer[0] = rank > 0 ? rank - 1 : (ring ? nranks - 1 : -1);
    p.send_off[0] = 0;
    p.recv_off[0] = -p.seg_bytes;
    // lower neighbour: my bottom rows [H - depth, H) <-> its top rows, received into [H, H + depth)
    p.has[1] = rank < nranks - 1 || ring;
    p.peer[1] = rank < nranks - 1 ? rank + 1 : (ring ? 0 : -1);
    p.send_off[1] = (int64_t)(g.H - depth) * row;
    p.recv_off[1] = (int64_t)g.H * row;
    return p;
}

namespace {
__global__ void delay_kernel(uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
}
}  // namespace

hipError_t emulated_transfer(double us, hipStream_t s) {
    int dev = 0, khz = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, s, (uint64_t)(us * khz / 1000.0));
    return hipGetLastError();
}

std::vector<HaloXfer> HaloPlan::xfers() const {
    std::vector<HaloXfer> out;
    for (int side = 0; side < 2; ++side) {
        if (!has[side]) continue;
        for (int kind = 0; kind < 2; ++kind)
            for (int f = 0; f < nfields; ++f)
                for (int l = 0; l < L; ++l) {
                    HaloXfer x;
                    x.peer = peer[side];
                    x.kind = kind;
                    x.field = f;
                    x.level = l;
                    x.offset = (int64_t)l * lbytes + (kind == 0 ? send_off[side] : recv_off[side]);
                    x.bytes = seg_bytes;
                    x.msg_offset = (int64_t)(f * L + l) * seg_bytes;
                    out.push_back(x);
                }
    }
    return out;
}

namespace {

using V4 = unsigned int __attribute__((ext_vector_type(4)));

// segment i = (f, l) of the message: seg units of U each (16-byte vectors; 4-byte words when
// a row is not a multiple of 16 bytes -- the layered model's unpadded rows); one thread per unit
template <bool PACK, typename U>
__global__ __launch_bounds__(256) void halo_copy_kernel(HaloFields fields, int L, int64_t lbytes, int64_t off,
                                                        int64_t seg_vec, char* msg, int64_t total_vec) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total_vec; i += (int64_t)gridDim.x * 256) {
        const int64_t seg = i / seg_vec, j = i - seg * seg_vec;
        const int f = (int)(seg / L), l = (int)(seg - (int64_t)f * L);
        U* field = (U*)(fields.f[f] + (int64_t)l * lbytes + off) + j;
        U* m = (U*)msg + i;
        if constexpr (PACK) *m = *field;
        else *field = *m;
    }
}

template <typename U>
void launch_halo_copy(bool pack, const HaloPlan& p, const HaloFields& fields, int64_t off, char* msg, hipStream_t s) {
    const int64_t seg_vec = p.seg_bytes / (int64_t)sizeof(U), total = seg_vec * p.nfields * p.L;
    const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 4096);
    if (pack)
        hipLaunchKernelGGL((halo_copy_kernel<true, U>), dim3(blocks), dim3(256), 0, s, fields, p.L, p.lbytes, off,
                           seg_vec, msg, total);
    else
        hipLaunchKernelGGL((halo_copy_kernel<false, U>), dim3(blocks), dim3(256), 0, s, fields, p.L, p.lbytes, off,
                           seg_vec, msg, total);
}

hipError_t halo_copy(bool pack, const HaloPlan& p, const HaloFields& fields, int side, void* msg, hipStream_t s) {
    if (!p.has[side] || p.msg_bytes() == 0) return hipSuccess;
    if (p.seg_bytes % 4 != 0 || p.lbytes % 4 != 0 || p.nfields > kMaxHaloFields) return hipErrorInvalidValue;
    const int64_t off = pack ? p.send_off[side] : p.recv_off[side];
    // (field rows start 16-byte aligned when rows and level strides are multiples of 16 bytes)
    if (p.seg_bytes % 16 == 0 && p.lbytes % 16 == 0 && off % 16 == 0)
        launch_halo_copy<V4>(pack, p, fields, off, (char*)msg, s);
    else
        launch_halo_copy<unsigned int>(pack, p, fields, off, (char*)msg, s);
    return hipGetLastError();
}

}  // namespace

hipError_t halo_pack(const HaloPlan& p, const HaloFields& fields, int side, void* dst, hipStream_t s) {
    return halo_copy(true, p, fields, side, dst, s);
}

hipError_t halo_unpack(const HaloPlan& p, const HaloFields& fields, int side, const void* src, hipStream_t s) {
    return halo_copy(false, p, fields, side, const_cast<void*>(src), s);
}

HaloStaging::~HaloStaging() {
    for (void* b : {send[0], send[1], recv[0], recv[1]})
        if (b) (void)hipFree(b);
}

void HaloStaging::ensure(int64_t bytes) {
    if (bytes <= cap_) return;
    for (void** b : {&send[0], &send[1], &recv[0], &recv[1]}) {
        if (*b) (void)hipFree(*b);
        *b = nullptr;
    }
    cap_ = 0;
    for (void** b : {&send[0], &send[1], &recv[0], &recv[1]}) {
        const hipError_t e = hipMalloc(b, (size_t)bytes);
        if (e != hipSuccess) throw std::runtime_error(std::string("halo staging hipMalloc: ") + hipGetErrorString(e));
    }
    cap_ = bytes;
}

}  // namespace ws
