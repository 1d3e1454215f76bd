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
    int32_t out_w;                // output columns per strip (<= strip columns - 2 margins)
    int32_t seg_rows;             // output rows per workgroup segment
    // Output rows of this launch: two row groups, each cut into segments of seg_rows rows
    // (the last one clipped): group A = [ga_y0, ga_y1) (ga_n segments), then group B =
    // [gb_y0, gb_y1); seg_n segments in total. One group = the whole grid; a slab's
    // interior launch uses A = the rows whose cone avoids the halo, its edge launch uses
    // A, B = the few rows at the two slab boundaries.
    int32_t ga_y0, ga_y1, ga_n;
    int32_t gb_y0, gb_y1;
    int32_t seg_n;
    // 1 = "scaled tendencies" (set by scale_tendencies, below): the kernels leave the
    // central differences unscaled and every constant that multiplies them carries the
    // 1/(2 dx) factor instead; 0 = the kernels divide by (2 dx) as the reference writes it
    int32_t scaled;
};

// Scaled tendencies. When 2dx = 2dy = 2^-k for both spacings (s = 1/(2dx) = 2^k), every
// tendency the reference computes is s times the same expression evaluated on the raw
// differences D = (ar - al): multiplying by a power of two commutes with IEEE rounding, so
//   (-u)*(s*D) = s*round((-u)*D),   g*(s*D) = s*round(g*D),   s*A - s*B = s*round(A - B),
//   f*v = s*round((f/s)*v),   y + c*(s*K) = y + round((c*s)*K),   s*a + 2*(s*b) = s*round(a + 2*b),
// with f/s and c*s exact. The kernels evaluate K = k/s (g unchanged, f -> f/s) and the
// update constants carry s, skipping the 6 multiplications by s per stage (RK4: 24 of ~170
// fp64 ops per cell). Results are bit-identical to the reference's
// evaluation order whenever no intermediate is subnormal (|x| < 2^-1022 fp64, 2^-126 fp32)
// or within a factor 2^|k| of overflow. Subnormal intermediates do occur (the reference
// fixture "mountain" fp32 after 50 steps: values ~1e-42 ahead of the wave front differ in
// their last subnormal bits), so this is OPT-IN (WS_SCALED=1): the default is bit-exact.
// Spacing modes of the fused kernels (template parameter): divide as the reference writes
// it; multiply by the exact reciprocal (2dx, 2dy powers of two: bit-identical); scaled.
enum SpacingMode : int { kSpDiv = 0, kSpMul = 1, kSpScaled = 2 };
template <typename T>
inline int fused_sp_mode(const FusedArgs<T>& a) {
    if (a.scaled) return kSpScaled;
    return a.sp1.pow2x && a.sp1.pow2y && a.sp2.pow2x && a.sp2.pow2y ? kSpMul : kSpDiv;
}

template <typename T>
inline void scale_tendencies(FusedArgs<T>& a) {
    const Spacing<T>& p = a.sp1;
    const Spacing<T>& q = a.sp2;
    a.scaled = p.pow2x && p.pow2y && q.pow2x && q.pow2y && p.inv2dx == p.inv2dy && q.inv2dx == q.inv2dy &&
               p.inv2dx == q.inv2dx;
    if (!a.scaled) return;
    const T s = p.inv2dx;
    a.c_half *= s;
    a.c_dt *= s;
    a.c_dt6 *= s;
    a.coriolis_f /= s;
}

template <typename T>
__host__ __device__ inline void fused_rows(const FusedArgs<T>& a, int i, int& y0, int& y1) {
    if (i < a.ga_n) {
        y0 = a.ga_y0 + i * a.seg_rows;
        y1 = y0 + a.seg_rows < a.ga_y1 ? y0 + a.seg_rows : a.ga_y1;
    } else {
        y0 = a.gb_y0 + (i - a.ga_n) * a.seg_rows;
        y1 = y0 + a.seg_rows < a.gb_y1 ? y0 + a.seg_rows : a.gb_y1;
    }
}

// nstages: 1 (Euler), 2 (RK2 midpoint), 4 (RK4-as-implemented)
// LDS variant: 256-lane workgroups, horizontal neighbours through LDS, one barrier per row.
template <typename T>
hipError_t launch_fused_step(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s);
// DPP variant: independent 64-lane waves, horizontal neighbours by DPP lane shifts.
constexpr int kDppCols = 64;
// y rows: loaded into a VGPR ring (kDppVgpr), staged through LDS by LDS-DMA (16 B per lane)
// and copied to the VGPR ring (kDppDma), or LDS-DMA staged and read from LDS in place
// (kDppLdsY: fewer VGPRs, three waves per SIMD)
enum DppMode : int { kDppVgpr = 0, kDppDma = 1, kDppLdsY = 2 };
template <typename T>
hipError_t launch_fused_step_dpp(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s, int mode);
// the three modes' launchers (one translation unit each)
template <typename T>
hipError_t launch_dpp_vgpr(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s);
template <typename T>
hipError_t launch_dpp_dma(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s);
template <typename T>
hipError_t launch_dpp_ldsy(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s);

// Strip geometry, per variant: columns per strip and the left margin (the dependency cone;
// the x2 variant rounds it up to whole column pairs). The output window of strip s is
// [s * out_w, (s + 1) * out_w); out_w is at most columns - 2 * margin, and when `aligned`
// it is rounded down to whole 128-byte lines so no two strips write parts of one line.
enum FusedVariant : int { kFusedLds = 0, kFusedDpp = 1, kFusedX2 = 2, kFusedDppDma = 3, kFusedDppLdsY = 4,
                          kFusedX2Y = 5 };
inline int fused_strip_cols(int variant) {
    return variant == kFusedX2 || variant == kFusedX2Y ? 128
           : (variant == kFusedDpp || variant == kFusedDppDma || variant == kFusedDppLdsY) ? 64
                                                                                             : 256;
}
// (the DMA variant rounds it up to whole 16-byte chunks: a strip's LDS-DMA chunks then
// never straddle column 0, where a partly negative chunk would be dropped whole by the
// buffer range check)
inline int fused_margin(int variant, int nstages, int elem_bytes) {
    if (variant == kFusedX2) return (nstages + 1) / 2 * 2;
    if (variant == kFusedDppDma || variant == kFusedDppLdsY || variant == kFusedX2Y) {
        const int g = 16 / elem_bytes;
        return (nstages + g - 1) / g * g;
    }
    return nstages;
}
inline int fused_out_w(int variant, int nstages, int elem_bytes, bool aligned) {
    const int w = fused_strip_cols(variant) - 2 * fused_margin(variant, nstages, elem_bytes);
    const int line = 128 / elem_bytes;
    return aligned && w >= line ? w / line * line : w;
}

// x2 variant: independent 64-lane waves, two adjacent columns per lane (128-column strips).
template <typename T>
hipError_t launch_fused_step_x2(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s);
// x2y variant: column pairs with y rows staged by LDS-DMA and read from LDS in place
template <typename T>
hipError_t launch_fused_step_x2y(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s);

}  // namespace ws
