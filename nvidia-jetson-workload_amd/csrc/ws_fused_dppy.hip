// Host launcher of the dppy / x2y fused step kernel (kernel: ws_fused_dppy_kernel.h; its
// instantiations: ws_fused_dppy{,2}_{f32,f64}_{1,2}.hip, and the four-step launches
// ws_fused_dppy_{f32,f64}_4.hip, ws_fused_dppy2_f32_4.hip; eight-step (Euler) launches
// ws_fused_dppy_{f32,f64}_8.hip, ws_fused_dppy2_f32_8.hip).
#include "ws_fused.h"

namespace ws {

template <typename T>
hipError_t launch_fused_step_dppy(int variant, int nstages, int nsteps, const FusedArgs<T>& a, const Geom& g,
                                  hipStream_t s) {
    const int out_w = a.out_w;
    if (!fused_is_dppy(variant)) return hipErrorInvalidValue;
    if (!fused_tb_ok(variant, nsteps, nstages, (int)sizeof(T)) && !(fused_split(variant) && nsteps == 1))
        return hipErrorInvalidValue;
    const int ns = nstages * nsteps;  // the launch's cone depth
    if (out_w < 1 || out_w > fused_strip_cols(variant) - 2 * fused_margin(variant, ns, (int)sizeof(T)))
        return hipErrorInvalidValue;
    if (out_w % (16 / (int)sizeof(T)) != 0) return hipErrorInvalidValue;  // chunk-aligned strips
    // column pairs are stored whole: an odd width's last pair ends in the row padding
    if (fused_pairs(variant) && (g.pitch % 2 != 0 || g.pitch < g.W + (g.W % 2))) return hipErrorInvalidValue;
    const int nstrips = fused_strips(variant, g.W, ns, (int)sizeof(T), out_w);
    const int nsegs = a.seg_n;
    if (a.chains ? a.nchains <= 0 : nsegs <= 0) return hipSuccess;
    const int64_t nblocks = a.chains ? (int64_t)a.nchains : (int64_t)nstrips * nsegs * g.L;
    if (nblocks > 0x7fffffff) return hipErrorInvalidValue;
    // buffer descriptors span one segment's rows (+ margins); offsets are 32-bit and the
    // dropped-store voffset is 2^31
    const int64_t span = (int64_t)(a.seg_rows + 2 * ns + 48) * g.pitch * (int64_t)sizeof(T);
    if (span >= 0x7fffffff) return hipErrorInvalidValue;
    // pc / pc2 split a two-step launch; their one-step launches (a run's odd step, a slab
    // block's last) are the dppy / x2y kernel's, on the same strips
    if (fused_split(variant) && nsteps == 2)
        return fused_pairs(variant) ? launch_dppy_pc_tu<T, 2>(nstages, a, g, s, nstrips, nsegs)
                                    : launch_dppy_pc_tu<T, 1>(nstages, a, g, s, nstrips, nsegs);
    if (fused_pairs(variant)) {
        if (nsteps == 4 || nsteps == 8) {
            if constexpr (sizeof(T) == 4)
                return nsteps == 4 ? launch_dppy_tu<T, 4, 2>(nstages, a, g, s, nstrips, nsegs)
                                   : launch_dppy_tu<T, 8, 2>(nstages, a, g, s, nstrips, nsegs);
            return hipErrorInvalidValue;
        }
        return nsteps == 1 ? launch_dppy_tu<T, 1, 2>(nstages, a, g, s, nstrips, nsegs)
                           : launch_dppy_tu<T, 2, 2>(nstages, a, g, s, nstrips, nsegs);
    }
    if (nsteps == 4) return launch_dppy_tu<T, 4, 1>(nstages, a, g, s, nstrips, nsegs);
    if (nsteps == 8) return launch_dppy_tu<T, 8, 1>(nstages, a, g, s, nstrips, nsegs);
    return nsteps == 1 ? launch_dppy_tu<T, 1, 1>(nstages, a, g, s, nstrips, nsegs)
                       : launch_dppy_tu<T, 2, 1>(nstages, a, g, s, nstrips, nsegs);
}

template <typename T>
int fused_dppy_blocks_per_cu(int variant, int nstages, int nsteps, int sp_mode) {
    if (fused_split(variant) && nsteps == 2)
        return fused_pairs(variant) ? dppy_pc_blocks_per_cu_tu<T, 2>(nstages, sp_mode)
                                    : dppy_pc_blocks_per_cu_tu<T, 1>(nstages, sp_mode);
    if (fused_pairs(variant)) {
        if (nsteps == 4 || nsteps == 8) {
            if constexpr (sizeof(T) == 4)
                return nsteps == 4 ? dppy_blocks_per_cu_tu<T, 4, 2>(nstages, sp_mode)
                                   : dppy_blocks_per_cu_tu<T, 8, 2>(nstages, sp_mode);
            return 0;
        }
        return nsteps == 1 ? dppy_blocks_per_cu_tu<T, 1, 2>(nstages, sp_mode) : dppy_blocks_per_cu_tu<T, 2, 2>(nstages, sp_mode);
    }
    if (nsteps == 4) return dppy_blocks_per_cu_tu<T, 4, 1>(nstages, sp_mode);
    if (nsteps == 8) return dppy_blocks_per_cu_tu<T, 8, 1>(nstages, sp_mode);
    return nsteps == 1 ? dppy_blocks_per_cu_tu<T, 1, 1>(nstages, sp_mode) : dppy_blocks_per_cu_tu<T, 2, 1>(nstages, sp_mode);
}
template int fused_dppy_blocks_per_cu<float>(int, int, int, int);
template int fused_dppy_blocks_per_cu<double>(int, int, int, int);

template hipError_t launch_fused_step_dppy<float>(int, int, int, const FusedArgs<float>&, const Geom&, hipStream_t);
template hipError_t launch_fused_step_dppy<double>(int, int, int, const FusedArgs<double>&, const Geom&, hipStream_t);

}  // namespace ws
