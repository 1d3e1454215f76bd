// HIP kernels for the weather-sim time step on MI355X (gfx950, CDNA4).
//
// Bandwidth-bound 5-point stencils; no MFMA. Compiled with -ffp-contract=off and IEEE
// division so every cell reproduces the reference CPU arithmetic bit-for-bit
// (reference: src/weather-sim/cpp/src/weather_simulation.cpp:473-540 for the tendency,
// :160-455 for the stage updates, src/weather_grid.cpp:82-121 for the diagnostics).
#include "ws_internal.h"
#include "ws_repeat_add.h"

namespace ws {
namespace {

// Centred difference (a_r - a_l) / (2 d). When 2d is a power of two the reciprocal is
// exact and x * (1/2d) == x / 2d bit-for-bit (both are the correctly rounded quotient),
// so the IEEE divide is replaced by a multiply.
template <typename T>
__device__ __forceinline__ T cdiff(T ar, T al, T two_d, T inv, int pow2) {
    return pow2 ? (ar - al) * inv : (ar - al) / two_d;
}

// SWE tendency at one cell (weather_simulation.cpp:521-537), evaluation order preserved:
//   du = (((-u)*u_x - v*u_y) - g*h_x) + f*v
//   dv = (((-u)*v_x - v*v_y) - g*h_y) - f*u
//   dh = ((-h)*(u_x + v_y) - u*h_x) - v*h_y
template <typename T>
struct Tend {
    T du, dv, dh;
};

template <typename T>
__device__ __forceinline__ Tend<T> swe_tendency(T u, T v, T h, T ul, T ur, T ut, T ub, T vl, T vr, T vt, T vb, T hl,
                                                T hr, T ht, T hb, const Spacing<T>& sp, T g, T f) {
    const T u_x = cdiff(ur, ul, sp.two_dx, sp.inv2dx, sp.pow2x);
    const T u_y = cdiff(ub, ut, sp.two_dy, sp.inv2dy, sp.pow2y);
    const T v_x = cdiff(vr, vl, sp.two_dx, sp.inv2dx, sp.pow2x);
    const T v_y = cdiff(vb, vt, sp.two_dy, sp.inv2dy, sp.pow2y);
    const T h_x = cdiff(hr, hl, sp.two_dx, sp.inv2dx, sp.pow2x);
    const T h_y = cdiff(hb, ht, sp.two_dy, sp.inv2dy, sp.pow2y);
    Tend<T> t;
    t.du = -u * u_x - v * u_y - g * h_x + f * v;
    t.dv = -u * v_x - v * v_y - g * h_y - f * u;
    t.dh = -h * (u_x + v_y) - u * h_x - v * h_y;
    return t;
}

constexpr int kBX = 64;
constexpr int kBY = 4;

// v1: one cell per lane, 64x4 blocks, neighbours through the vector L1 / L2.
template <typename T, int MODE>
__global__ __launch_bounds__(kBX* kBY) void stage_kernel(StageArgs<T> a, Geom g) {
    const int x = blockIdx.x * kBX + threadIdx.x;
    const int y = blockIdx.y * kBY + threadIdx.y;
    if (x >= g.W || y >= g.H) return;
    const int64_t idx = (int64_t)blockIdx.z * g.lstride + (int64_t)y * g.pitch + x;
    const int64_t il = x > 0 ? idx - 1 : idx;
    const int64_t ir = x < g.W - 1 ? idx + 1 : idx;
    const int64_t it = (y > 0 || !g.top_clamp) ? idx - g.pitch : idx;
    const int64_t ib = (y < g.H - 1 || !g.bot_clamp) ? idx + g.pitch : idx;

    const T u = a.in_u[idx], v = a.in_v[idx], h = a.in_h[idx];
    const Tend<T> k = swe_tendency<T>(u, v, h, a.in_u[il], a.in_u[ir], a.in_u[it], a.in_u[ib], a.in_v[il], a.in_v[ir],
                                      a.in_v[it], a.in_v[ib], a.in_h[il], a.in_h[ir], a.in_h[it], a.in_h[ib], a.sp,
                                      a.gravity, a.coriolis_f);
    if constexpr (MODE == kAxpy) {
        a.out_u[idx] = a.base_u[idx] + a.c * k.du;
        a.out_v[idx] = a.base_v[idx] + a.c * k.dv;
        a.out_h[idx] = a.base_h[idx] + a.c * k.dh;
    } else if constexpr (MODE == kAxpyStore) {
        a.k2_u[idx] = k.du;
        a.k2_v[idx] = k.dv;
        a.k2_h[idx] = k.dh;
        a.out_u[idx] = a.base_u[idx] + a.c * k.du;
        a.out_v[idx] = a.base_v[idx] + a.c * k.dv;
        a.out_h[idx] = a.base_h[idx] + a.c * k.dh;
    } else {
        const T two = T(2);
        a.out_u[idx] = a.base_u[idx] + a.c * (((k.du + two * a.k2_u[idx]) + two * a.k3_u[idx]) + k.du);
        a.out_v[idx] = a.base_v[idx] + a.c * (((k.dv + two * a.k2_v[idx]) + two * a.k3_v[idx]) + k.dv);
        a.out_h[idx] = a.base_h[idx] + a.c * (((k.dh + two * a.k2_h[idx]) + two * a.k3_h[idx]) + k.dh);
    }
}

// weather_grid.cpp:82-121 -- left/right = max(0,x-1)/min(W-1,x+1), same for y
template <typename T>
__global__ __launch_bounds__(kBX* kBY) void diag_kernel(const T* __restrict__ u, const T* __restrict__ v,
                                                        T* __restrict__ vort, T* __restrict__ div, Spacing<T> sp,
                                                        Geom g) {
    const int x = blockIdx.x * kBX + threadIdx.x;
    const int y = blockIdx.y * kBY + threadIdx.y;
    if (x >= g.W || y >= g.H) return;
    const int64_t idx = (int64_t)blockIdx.z * g.lstride + (int64_t)y * g.pitch + x;
    const int64_t il = x > 0 ? idx - 1 : idx;
    const int64_t ir = x < g.W - 1 ? idx + 1 : idx;
    const int64_t it = (y > 0 || !g.top_clamp) ? idx - g.pitch : idx;
    const int64_t ib = (y < g.H - 1 || !g.bot_clamp) ? idx + g.pitch : idx;
    const T dv_dx = cdiff(v[ir], v[il], sp.two_dx, sp.inv2dx, sp.pow2x);
    const T du_dy = cdiff(u[ib], u[it], sp.two_dy, sp.inv2dy, sp.pow2y);
    const T du_dx = cdiff(u[ir], u[il], sp.two_dx, sp.inv2dx, sp.pow2x);
    const T dv_dy = cdiff(v[ib], v[it], sp.two_dy, sp.inv2dy, sp.pow2y);
    vort[idx] = dv_dx - du_dy;
    div[idx] = du_dx + dv_dy;
}

template <typename T>
__global__ __launch_bounds__(kBX* kBY) void affine_kernel(T* __restrict__ out, const T* __restrict__ in, T c, T tend,
                                                          Geom g) {
    const int x = blockIdx.x * kBX + threadIdx.x;
    const int y = blockIdx.y * kBY + threadIdx.y;
    if (x >= g.W || y >= g.H) return;
    const int64_t idx = (int64_t)blockIdx.z * g.lstride + (int64_t)y * g.pitch + x;
    out[idx] = in[idx] + c * tend;
}

// PE T and P in one pass: out = in + ct with ct = dt * tend rounded once on the host (the
// reference's per-cell `dt_ * tendency` has the same operands everywhere, so the same
// rounding). Each level's rows [0, H) are one contiguous run of H * pitch elements (pitch
// columns padded to 64 elements): 16-byte vectors over it, padding columns included (never
// read as cells).
// (The outputs may alias the inputs: every element is loaded before it is stored.)
template <typename T>
__global__ __launch_bounds__(256) void affine2_kernel(T* oT, const T* iT, T cT, T* oP, const T* iP, T cP,
                                                      int64_t vec_per_level, int64_t lstride, int nrep, T* oT2,
                                                      T* oP2, int jrep) {
    using V = T __attribute__((ext_vector_type(16 / sizeof(T))));
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= vec_per_level) return;
    const int64_t off = (int64_t)blockIdx.y * lstride + i * (int64_t)(16 / sizeof(T));
    V t = *(const V*)(iT + off);
    V p = *(const V*)(iP + off);
    // nrep steps' updates, each rounded as a separate addition: (x + c) + c ...; the values
    // after jrep of them go to the second outputs. repeat_add (ws_repeat_add.h) takes the steps
    // that stay in one binade at once -- bit-identical to the loop, O(binades) instead of O(nrep)
    // (a 200-step C4 run's flush: 200 dependent additions per value before)
    V tj, pj;
#pragma unroll
    for (int i = 0; i < (int)(16 / sizeof(T)); ++i) {
        tj[i] = repeat_add(t[i], cT, jrep);
        pj[i] = repeat_add(p[i], cP, jrep);
        t[i] = repeat_add(tj[i], cT, nrep - jrep);
        p[i] = repeat_add(pj[i], cP, nrep - jrep);
    }
    if (oT2) {
        __builtin_nontemporal_store(tj, (V*)(oT2 + off));
        __builtin_nontemporal_store(pj, (V*)(oP2 + off));
    }
    __builtin_nontemporal_store(t, (V*)(oT + off));
    __builtin_nontemporal_store(p, (V*)(oP + off));
}

template <typename T>
__global__ __launch_bounds__(kBX* kBY) void fill_kernel(T* __restrict__ out, T value, Geom g) {
    const int x = blockIdx.x * kBX + threadIdx.x;
    const int y = blockIdx.y * kBY + threadIdx.y;
    if (x >= g.W || y >= g.H) return;
    out[(int64_t)blockIdx.z * g.lstride + (int64_t)y * g.pitch + x] = value;
}

inline dim3 grid2d(const Geom& g) {
    return dim3((g.W + kBX - 1) / kBX, (g.H + kBY - 1) / kBY, g.L);
}

}  // namespace

template <typename T>
hipError_t launch_stage(int mode, const StageArgs<T>& a, const Geom& g, hipStream_t s) {
    const dim3 block(kBX, kBY);
    switch (mode) {
        case kAxpy: hipLaunchKernelGGL((stage_kernel<T, kAxpy>), grid2d(g), block, 0, s, a, g); break;
        case kAxpyStore: hipLaunchKernelGGL((stage_kernel<T, kAxpyStore>), grid2d(g), block, 0, s, a, g); break;
        case kRk4Final: hipLaunchKernelGGL((stage_kernel<T, kRk4Final>), grid2d(g), block, 0, s, a, g); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <typename T>
hipError_t launch_diagnostics(const T* u, const T* v, T* vort, T* div, const Spacing<T>& sp, const Geom& g,
                              hipStream_t s) {
    hipLaunchKernelGGL((diag_kernel<T>), grid2d(g), dim3(kBX, kBY), 0, s, u, v, vort, div, sp, g);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_affine(T* out, const T* in, T c, T tend, const Geom& g, hipStream_t s) {
    hipLaunchKernelGGL((affine_kernel<T>), grid2d(g), dim3(kBX, kBY), 0, s, out, in, c, tend, g);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_affine2(T* oT, const T* iT, T cT, T* oP, const T* iP, T cP, const Geom& g, hipStream_t s,
                          int nrep, T* oT2, T* oP2, int jrep) {
    const int64_t n = (int64_t)g.H * g.pitch;
    if (n % (16 / (int64_t)sizeof(T)) != 0 || g.L > 65535 || nrep < 1) return hipErrorInvalidValue;
    if ((oT2 == nullptr) != (oP2 == nullptr) || jrep < 0 || jrep >= nrep) return hipErrorInvalidValue;
    const int64_t nv = n / (16 / (int64_t)sizeof(T));
    if (nv <= 0) return hipSuccess;
    const dim3 grid((unsigned)((nv + 255) / 256), (unsigned)g.L);
    hipLaunchKernelGGL((affine2_kernel<T>), grid, dim3(256), 0, s, oT, iT, cT, oP, iP, cP, nv, g.lstride, nrep, oT2,
                       oP2, jrep);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_fill(T* out, T value, const Geom& g, hipStream_t s) {
    hipLaunchKernelGGL((fill_kernel<T>), grid2d(g), dim3(kBX, kBY), 0, s, out, value, g);
    return hipGetLastError();
}

#define WS_INSTANTIATE(T)                                                                                      \
    template hipError_t launch_stage<T>(int, const StageArgs<T>&, const Geom&, hipStream_t);                    \
    template hipError_t launch_diagnostics<T>(const T*, const T*, T*, T*, const Spacing<T>&, const Geom&,       \
                                              hipStream_t);                                                     \
    template hipError_t launch_affine<T>(T*, const T*, T, T, const Geom&, hipStream_t);                         \
    template hipError_t launch_affine2<T>(T*, const T*, T, T*, const T*, T, const Geom&, hipStream_t, int, T*, \
                                          T*, int);                                                             \
    template hipError_t launch_fill<T>(T*, T, const Geom&, hipStream_t);
WS_INSTANTIATE(float)
WS_INSTANTIATE(double)
#undef WS_INSTANTIATE

}  // namespace ws
