// Internal interfaces between the HIP kernels (ws_kernels.hip) and the host runtime
// (ws_runtime.cpp). Not part of the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace ws {

// Halo rows allocated above and below every field: a slab exchanges up to 6 time steps'
// worth of RK4 dependency cone (6 x 4 rows) at once (see ws_runtime.cpp, slab blocks).
constexpr int kHalo = 24;

enum StageMode : int {
    kAxpy = 0,       // out = base + c * k(in)                         (Euler, RK2, RK4 stage 1)
    kAxpyStore = 1,  // K = k(in); out = base + c * K                  (RK4 stages 2, 3)
    kRk4Final = 2,   // out = base + c * (((k(in) + 2 K2) + 2 K3) + k(in))  (RK4 stage 4, k1 alias)
};

// Geometry of one level-stacked field: element (l, y, x) at base[l*lstride + y*pitch + x],
// y in [-kHalo, H + kHalo).
struct Geom {
    int32_t W, H, L;
    int64_t pitch;    // elements
    int64_t lstride;  // elements
    int32_t top_clamp, bot_clamp;  // 1: y-1 / y+1 clamp to self at row 0 / H-1 (global edge)
    int32_t halo;                  // rows addressable above row 0 / below row H-1 (non-clamped sides)
};

template <typename T>
struct Spacing {
    T two_dx, two_dy;  // divisors as the reference computes them: (2.0f * dx)
    T inv2dx, inv2dy;  // exact reciprocals, valid when pow2x / pow2y
    int32_t pow2x, pow2y;
};

template <typename T>
struct StageArgs {
    const T *in_u, *in_v, *in_h;
    const T *base_u, *base_v, *base_h;
    T *out_u, *out_v, *out_h;
    T *k2_u, *k2_v, *k2_h;               // kAxpyStore: written; kRk4Final: read (K2)
    const T *k3_u, *k3_v, *k3_h;         // kRk4Final: read (K3)
    T c;
    T gravity, coriolis_f;
    Spacing<T> sp;
};

template <typename T>
hipError_t launch_stage(int mode, const StageArgs<T>& a, const Geom& g, hipStream_t s);

// vorticity / divergence (weather_grid.cpp:82-121)
template <typename T>
hipError_t launch_diagnostics(const T* u, const T* v, T* vort, T* div, const Spacing<T>& sp, const Geom& g,
                              hipStream_t s);

// out = in + c * tend_const   (PE T/P stale-tendency update, weather_simulation.cpp:201-214)
template <typename T>
hipError_t launch_affine(T* out, const T* in, T c, T tend, const Geom& g, hipStream_t s);
// both PE updates in one pass: oT = iT + cT, oP = iP + cP (cX = dt * tendency, rounded in T);
// nrep > 1 applies nrep steps' updates in one pass, each rounded: oT = ((iT + cT) + cT) ...;
// oT2 / oP2 (optional) receive the values after jrep (< nrep) of them in the same pass. The
// outputs may alias the inputs (element-wise: each element is read before it is written).
template <typename T>
hipError_t launch_affine2(T* oT, const T* iT, T cT, T* oP, const T* iP, T cP, const Geom& g, hipStream_t s,
                          int nrep = 1, T* oT2 = nullptr, T* oP2 = nullptr, int jrep = 0);

// fill all rows [0,H) of all levels with value
template <typename T>
hipError_t launch_fill(T* out, T value, const Geom& g, hipStream_t s);

}  // namespace ws
