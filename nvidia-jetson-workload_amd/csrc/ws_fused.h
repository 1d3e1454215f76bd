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
    // segments processed by this launch: local index i < seg_na -> seg_a + i,
    // else seg_b + (i - seg_na); seg_n in total (slab interior / edge split)
    int32_t seg_a, seg_na, seg_b, seg_n;
};

__host__ __device__ inline int fused_segment(int i, int seg_a, int seg_na, int seg_b) {
    return i < seg_na ? seg_a + i : seg_b + (i - seg_na);
}

// nstages: 1 (Euler), 2 (RK2 midpoint), 4 (RK4-as-implemented)
// LDS variant: 256-lane workgroups, horizontal neighbours through LDS, one barrier per row.
template <typename T>
hipError_t launch_fused_step(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s);
// DPP variant: independent 64-lane waves, horizontal neighbours by DPP lane shifts.
constexpr int kDppCols = 64;
template <typename T>
hipError_t launch_fused_step_dpp(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s);

// x2 variant: independent 64-lane waves, two adjacent columns per lane (128-column strips).
int fused_x2_out_cols(int nstages);
template <typename T>
hipError_t launch_fused_step_x2(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s);

}  // namespace ws
