// Fused multi-stage time-step kernel (ws_fused.hip).
#pragma once

#include "ws_internal.h"

namespace ws {

constexpr int kFusedCols = 256;  // lanes (= columns) per workgroup strip

template <typename T>
struct FusedArgs {
    const T *in_u, *in_v, *in_h;  // y_n (rows [-kHalo, H + kHalo) addressable)
    T *out_u, *out_v, *out_h;     // y_{n+1}
    T c_half;                     // 0.5f * dt
    T c_dt;                       // dt
    T c_dt6;                      // dt / 6.0f
    T gravity, coriolis_f;
    Spacing<T> sp1;               // stage 1: spacing of the current grid
    Spacing<T> sp2;               // later stages: spacing of the temp grid (= config)
    int32_t seg_rows;             // output rows per workgroup segment
};

// nstages: 1 (Euler), 2 (RK2 midpoint), 4 (RK4-as-implemented)
// LDS variant: 256-lane workgroups, horizontal neighbours through LDS, one barrier per row.
template <typename T>
hipError_t launch_fused_step(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s);
// DPP variant: independent 64-lane waves, horizontal neighbours by DPP lane shifts.
constexpr int kDppCols = 64;
template <typename T>
hipError_t launch_fused_step_dpp(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s);

}  // namespace ws
