// Fused multi-stage time-step kernel (ws_fused.hip).
#pragma once

#include "ws_internal.h"

namespace ws {

constexpr int kFusedCols = 256;  // lanes (= columns) per workgroup strip

// One march of a chain-scheduled launch: output rows [y0, y1) of march column `unit`
// (= level * strips + strip). See FusedArgs::chains.
struct ChainSeg {
    int32_t unit, y0, y1, pad;
};

template <typename T>
struct FusedArgs {
    const T *in_u, *in_v, *in_h;  // y_n (rows [-kHalo, H + kHalo) addressable)
    T *out_u, *out_v, *out_h;     // y_{n+1}
    T c_half;                     // 0.5f * dt
    T c_dt;                       // dt
    T c_dt6;                      // dt / 6.0f (fast numerics: dt / 3 * s, see prepare_fast)
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
    // spacing / numerics mode of the launch (SpacingMode below), set by the host
    int32_t sp_mode;
    // Chain schedule (dppy / x2y / pc / pc2; nullptr = the segments above): workgroup w marches
    // chains[w] -- one long segment per workgroup, sized by the host (ws_schedule.cpp
    // chain_table) so that every chain of a launch costs the same (edge strips / segments run
    // the dearer clamped code), with r chains per SIMD (r x 4 x CUs waves in all, whatever the
    // kernel's occupancy): no round of short-lived waves to quantise, one warm-up per chain.
    // seg_rows then holds the longest chain's rows.
    const ChainSeg* chains;
    int32_t nchains;
    // wave issue priority of the launch (s_setprio; 0 = normal): an overlapped slab block's
    // edge bands run beside its interior on the same SIMDs and are the block's critical path
    int32_t prio;
    // output stores cached (1) or nontemporal (0): a launch whose output fits the Infinity Cache
    // (the next launch reads it back from there) stores cached (ws_schedule.cpp fused_launch)
    int32_t cached;
};

// Spacing / numerics modes of the fused kernels (a template parameter, chosen per launch).
//  * kSpDiv: the central difference (ar - al) / (2 dx) divides, as the reference writes it;
//  * kSpMul: multiplies by the exact reciprocal (2dx, 2dy powers of two) -- bit-identical;
//  * kSpFast / kSpFast0 ("fast numerics", fp64 tolerance mode): the reference's tendencies
//    re-associated for the hardware. With s = 1 / (2 dx) = 1 / (2 dy) (isotropic spacing,
//    any value) every tendency is s times the same expression on the raw differences
//    D = ar - al, so the kernel evaluates K = k / s with fused multiply-adds (f -> f / s)
//    and the update constants carry s; RK4-as-implemented's final combination
//    y + dt/6 (((k4 + 2 k2) + 2 k3) + k4) is evaluated as y + (dt/3)((k2 + k3) + k4).
//    kSpFast0 drops the Coriolis terms (f == 0). Not bit-identical: every result differs
//    from the reference by rounding only (fp64: <= 1e-10 relative L2 is the north_star
//    tolerance; tests/test_gpu_numerics.py measures it), and about half the fp64 VALU work
//    of the exact evaluation order.
enum SpacingMode : int { kSpDiv = 0, kSpMul = 1, kSpFast = 2, kSpFast0 = 3 };

template <typename T>
inline int exact_sp_mode(const FusedArgs<T>& a) {
    return a.sp1.pow2x && a.sp1.pow2y && a.sp2.pow2x && a.sp2.pow2y ? kSpMul : kSpDiv;
}

// Set up a launch's constants for fast numerics when the spacing allows it (isotropic, and
// the same on both grids); otherwise leave the exact mode. Returns the mode chosen.
template <typename T>
inline int prepare_fast(FusedArgs<T>& a) {
    const Spacing<T>& p = a.sp1;
    const Spacing<T>& q = a.sp2;
    if (!(p.two_dx == p.two_dy && q.two_dx == q.two_dy && p.two_dx == q.two_dx)) return a.sp_mode = exact_sp_mode(a);
    const T s = T(1) / p.two_dx;
    const T dt = a.c_dt;
    a.c_half *= s;
    a.c_dt = dt * s;
    a.c_dt6 = dt / T(3) * s;  // fast mode: the final combination's dt/3
    a.coriolis_f /= s;
    return a.sp_mode = a.coriolis_f == T(0) ? kSpFast0 : kSpFast;
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

// nstages: 1 (Euler), 2 (RK2 midpoint), 4 (RK4-as-implemented). Three variants, all giving
// identical results (the autotuner picks one per grid, ws_runtime.cpp):
// "lds": 256-lane workgroups, horizontal neighbours through LDS, one barrier per row.
template <typename T>
hipError_t launch_fused_step(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s);
// "dppy": independent 64-lane waves, one column per lane, horizontal neighbours by DPP lane
// shifts, y rows staged by LDS-DMA and read from LDS in place. "x2y": the same kernel with an
// adjacent column pair per lane (128-column strips). variant = kFusedDppLdsY or kFusedX2Y;
// nsteps = time steps per launch (1, 2 or 4: temporal blocking, see ws_fused_dppy_kernel.h;
// fused_tb_ok says which)
template <typename T>
hipError_t launch_fused_step_dppy(int variant, int nstages, int nsteps, const FusedArgs<T>& a, const Geom& g,
                                  hipStream_t s);
// one translation unit per (T, steps per launch, columns per lane): the kernel instantiations
template <typename T, int NSTEP, int CPL>
hipError_t launch_dppy_tu(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s, int nstrips, int nsegs);
// "pc" / "pc2": the dppy / x2y kernel's two-step march split over a producer and a consumer
// wave (ws_fused_dppy_kernel.h, SPLIT), one translation unit per (T, CPL):
// ws_fused_dppypc{,2}_<t>.hip
template <typename T, int CPL>
hipError_t launch_dppy_pc_tu(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s, int nstrips, int nsegs);
// workgroups of one instantiation one CU holds at once (occupancy; the chain schedule's rounds)
template <typename T, int NSTEP, int CPL>
int dppy_blocks_per_cu_tu(int nstages, int sp_mode);
template <typename T, int CPL>
int dppy_pc_blocks_per_cu_tu(int nstages, int sp_mode);
template <typename T>
int fused_dppy_blocks_per_cu(int variant, int nstages, int nsteps, int sp_mode);

// Strip geometry, per variant: columns per strip and the left margin (the dependency cone,
// rounded up to whole 16-byte DMA chunks for the LDS-DMA variants: a strip's chunks then
// never straddle column 0, where a partly negative chunk would be dropped whole by the
// buffer range check). Middle strips output out_w columns, at most columns - 2 * margin, and
// when `aligned` rounded down to whole 128-byte lines so no two strips write parts of one line;
// the first and last strips lean on the global edges (strip_geom below). The lds variant keeps
// the plain layout: strip s outputs [s * out_w, (s + 1) * out_w). (Variant ids are ABI values,
// ws_sim_fused_variant; 1-3 belonged to variants removed after never winning a config.)
enum FusedVariant : int { kFusedLds = 0, kFusedDppLdsY = 4, kFusedX2Y = 5, kFusedPc = 6, kFusedPc2 = 7 };
// the variants of the wave-independent kernel (ws_fused_dppy_kernel.h), and their lane width
inline bool fused_is_dppy(int variant) {
    return variant == kFusedDppLdsY || variant == kFusedX2Y || variant == kFusedPc || variant == kFusedPc2;
}
inline bool fused_pairs(int variant) { return variant == kFusedX2Y || variant == kFusedPc2; }
inline bool fused_split(int variant) { return variant == kFusedPc || variant == kFusedPc2; }
// steps per launch a variant can take: 1 and 2 (the split variants: 2 only); 4 for the
// one-wave march at Euler / RK2 and 8 at Euler (an 8-deep cone, the RK4 two-step kernel's) in
// fp32, and fp64 one column per lane (fp64 pairs would need > 256 VGPRs)
inline bool fused_tb_ok(int variant, int tb, int nstages, int elem_bytes) {
    if (tb == 1) return !fused_split(variant);
    if (tb == 2) return fused_is_dppy(variant);
    if (tb == 4)
        return (variant == kFusedDppLdsY || (variant == kFusedX2Y && elem_bytes == 4)) && nstages <= 2;
    if (tb == 8)  // Euler: the same cone of 8
        return (variant == kFusedDppLdsY || (variant == kFusedX2Y && elem_bytes == 4)) && nstages == 1;
    return false;
}
inline int fused_strip_cols(int variant) {
    return fused_pairs(variant) ? 128 : fused_is_dppy(variant) ? 64 : 256;
}
inline int fused_margin(int variant, int nstages, int elem_bytes) {
    if (fused_is_dppy(variant)) {
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

// Strip layout of the dppy family (round 5: edge-aware). A strip is a window of SW
// (fused_strip_cols) columns whose outputs keep kM (fused_margin: the cone in whole 16-byte
// chunks of kC columns) columns from the window's edges -- except at a global edge, where the
// clamp takes the margin's place: the first strip's window starts at column 0 and the last
// strip's is right-aligned to the row's end (rounded up to a chunk), so each outputs kM more
// columns and a row may need one strip fewer (C4's 1024 columns: 9 pair strips instead of 10).
// Middle strips output out_w columns. (With whole-line windows, out_w < SW - 2 kM, the first
// strip outputs out_w columns too, keeping every middle window on 128-byte lines.)
struct StripGeom {
    int xs, o0, o1;  // window start column; output columns [o0, o1)
};
__host__ __device__ inline int strip_first_out(int SW, int kM, int out_w) {
    return out_w == SW - 2 * kM ? SW - kM : out_w;
}
__host__ __device__ inline int strip_last_xs(int W, int SW, int kC) { return (W - SW + kC - 1) / kC * kC; }
__host__ __device__ inline int strip_count(int W, int SW, int kM, int kC, int out_w) {
    if (W <= SW) return 1;
    const int need = strip_last_xs(W, SW, kC) + kM - strip_first_out(SW, kM, out_w);
    return 2 + (need > 0 ? (need + out_w - 1) / out_w : 0);
}
__host__ __device__ inline StripGeom strip_geom(int s, int n, int W, int SW, int kM, int kC, int out_w) {
    if (n == 1) return {0, 0, W};
    const int first = strip_first_out(SW, kM, out_w);
    if (s == 0) return {0, 0, first < W ? first : W};
    const int o0 = first + (s - 1) * out_w;
    if (s == n - 1) return {strip_last_xs(W, SW, kC), o0, W};
    return {o0 - kM, o0, o0 + out_w < W ? o0 + out_w : W};
}
// the same for a launch: strips of a W-column row for variant / cone / element size / out_w
inline int fused_strips(int variant, int W, int cone, int elem_bytes, int out_w) {
    return strip_count(W, fused_strip_cols(variant), fused_margin(variant, cone, elem_bytes), 16 / elem_bytes, out_w);
}
inline StripGeom fused_strip_geom(int variant, int s, int n, int W, int cone, int elem_bytes, int out_w) {
    return strip_geom(s, n, W, fused_strip_cols(variant), fused_margin(variant, cone, elem_bytes), 16 / elem_bytes, out_w);
}

}  // namespace ws
