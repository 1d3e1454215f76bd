// CFL number of the current state: a device max-reduction (north_star: "wavefront-level
// reductions for the CFL / diagnostic passes"; the reference has no CFL, its dt is fixed).
//
// Per cell c = max((|u| + sqrt(g h)) dt / dx, (|v| + sqrt(g h)) dt / dy) (the explicit
// gravity-wave CFL of the shallow-water system; h < 0 gives NaN, which the max propagates),
// per level the maximum over the H x W cells. HBM-bound: 3 words read per cell, one pass.
//
// Reduction: values are non-negative doubles (or NaN), whose IEEE bit patterns order like
// unsigned 64-bit integers (NaN above +inf), so the max runs on the bits: per thread over
// its cells, then across the wave by DPP (quad_perm x2, row_half_mirror, row_mirror,
// row_bcast:15, row_bcast:31 -- the total lands in lane 63, no LDS traffic), across the
// workgroup's waves through LDS, and across workgroups by a second one-workgroup-per-level
// pass over the partials (deterministic, no atomics). The per-level results stay on the
// device for the slab decomposition's RCCL max-allreduce (ws_comm.cpp).
#include "ws_reduce.h"

namespace ws {
namespace {

constexpr int kThreads = 256;


template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
    // lanes the control does not write keep their own value (old = src, bound_ctrl off)
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    const uint32_t nlo = (uint32_t)__builtin_amdgcn_update_dpp((int)lo, (int)lo, CTRL, ROW_MASK, 0xF, false);
    const uint32_t nhi = (uint32_t)__builtin_amdgcn_update_dpp((int)hi, (int)hi, CTRL, ROW_MASK, 0xF, false);
    return ((uint64_t)nhi << 32) | nlo;
}

__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

// max over the wave's 64 lanes, valid in lane 63
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
    v = umax64(v, dpp_u64<0xB1, 0xF>(v));   // quad_perm [1,0,3,2]
    v = umax64(v, dpp_u64<0x4E, 0xF>(v));   // quad_perm [2,3,0,1]
    v = umax64(v, dpp_u64<0x141, 0xF>(v));  // row_half_mirror
    v = umax64(v, dpp_u64<0x140, 0xF>(v));  // row_mirror: every lane holds its row's max
    v = umax64(v, dpp_u64<0x142, 0xA>(v));  // row_bcast:15 -> rows 1, 3
    v = umax64(v, dpp_u64<0x143, 0xC>(v));  // row_bcast:31 -> rows 2, 3
    return v;
}

// workgroup max -> thread 0
__device__ __forceinline__ uint64_t block_max_u64(uint64_t v) {
    __shared__ uint64_t part[kThreads / 64];
    v = wave_max_u64(v);
    const int lane = threadIdx.x % 64, wave = threadIdx.x / 64;
    if (lane == 63) part[wave] = v;
    __syncthreads();
    uint64_t m = 0;
    if (threadIdx.x == 0)
        for (int i = 0; i < kThreads / 64; ++i) m = umax64(m, part[i]);
    return m;
}

// per-cell CFL value as the bits of a double (T arithmetic, NaN-propagating max of the two)
template <typename T>
__device__ __forceinline__ uint64_t cfl_bits(T u, T v, T h, T gravity, T cx, T cy) {
    const T c = sqrt(gravity * h);
    const T a = (fabs(u) + c) * cx;
    const T b = (fabs(v) + c) * cy;
    return (uint64_t)__double_as_longlong((double)(a >= b || a != a ? a : b));
}

// Workgroup (b, level) reduces rows b, b + gridDim.x, ... of one level. A row is read in
// 16-byte vectors (rows are padded to 64 elements, so they are whole vectors; lanes past W
// are masked), kUnroll independent vector triples in flight per thread.
template <typename T>
__global__ __launch_bounds__(kThreads) void cfl_partial_kernel(const T* __restrict__ u, const T* __restrict__ v,
                                                              const T* __restrict__ h, Geom g, T gravity, T cx, T cy,
                                                              uint64_t* __restrict__ partial) {
    constexpr int VW = 16 / (int)sizeof(T);
    constexpr int kUnroll = 4;
    using V = T __attribute__((ext_vector_type(VW)));
    const int level = blockIdx.y;
    const int64_t lofs = (int64_t)level * g.lstride;
    const int nvec = (int)(g.pitch / VW);
    uint64_t m = 0;
    for (int y = blockIdx.x; y < g.H; y += gridDim.x) {
        const int64_t row = lofs + (int64_t)y * g.pitch;
        const V* U = (const V*)(u + row);
        const V* Vv = (const V*)(v + row);
        const V* Hh = (const V*)(h + row);
        for (int x0 = threadIdx.x; x0 < nvec; x0 += kThreads * kUnroll) {
            V uu[kUnroll], vv[kUnroll], hh[kUnroll];
#pragma unroll
            for (int k = 0; k < kUnroll; ++k) {
                const int xv = x0 + k * kThreads;
                if (xv < nvec) {
                    uu[k] = U[xv];
                    vv[k] = Vv[xv];
                    hh[k] = Hh[xv];
                }
            }
#pragma unroll
            for (int k = 0; k < kUnroll; ++k) {
                const int xv = x0 + k * kThreads;
#pragma unroll
                for (int j = 0; j < VW; ++j)
                    if (xv < nvec && xv * VW + j < g.W) m = umax64(m, cfl_bits<T>(uu[k][j], vv[k][j], hh[k][j], gravity, cx, cy));
            }
        }
    }
    m = block_max_u64(m);
    if (threadIdx.x == 0) partial[(int64_t)level * gridDim.x + blockIdx.x] = m;
}

__global__ __launch_bounds__(kThreads) void cfl_final_kernel(const uint64_t* __restrict__ partial, int nparts,
                                                            uint64_t* __restrict__ out) {
    const int level = blockIdx.x;
    uint64_t m = 0;
    for (int i = threadIdx.x; i < nparts; i += kThreads) m = umax64(m, partial[(int64_t)level * nparts + i]);
    m = block_max_u64(m);
    if (threadIdx.x == 0) out[level] = m;
}

}  // namespace

int cfl_partials(const Geom& g) { return g.H < 1024 ? g.H : 1024; }

template <typename T>
hipError_t launch_cfl(const T* u, const T* v, const T* h, const Geom& g, T gravity, T dt_dx, T dt_dy,
                      uint64_t* partial, uint64_t* out, hipStream_t s) {
    if (g.W <= 0 || g.H <= 0 || g.L <= 0 || g.L > 65535) return hipErrorInvalidValue;
    const int nb = cfl_partials(g);
    hipLaunchKernelGGL((cfl_partial_kernel<T>), dim3(nb, g.L), dim3(kThreads), 0, s, u, v, h, g, gravity, dt_dx,
                       dt_dy, partial);
    hipLaunchKernelGGL(cfl_final_kernel, dim3(g.L), dim3(kThreads), 0, s, partial, nb, out);
    return hipGetLastError();
}

template hipError_t launch_cfl<float>(const float*, const float*, const float*, const Geom&, float, float, float,
                                      uint64_t*, uint64_t*, hipStream_t);
template hipError_t launch_cfl<double>(const double*, const double*, const double*, const Geom&, double, double,
                                       double, uint64_t*, uint64_t*, hipStream_t);

}  // namespace ws
