// fused_dppy_kernel instantiations for float, two time steps per launch split over a producer and a
// consumer wave, a column pair per lane (variant pc2; see ws_fused_dppy_kernel.h, SPLIT)
#include "ws_fused_dppy_kernel.h"

namespace ws {
template <typename T, int CPL>
hipError_t launch_dppy_pc_tu(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s, int nstrips, int nsegs) {
    return launch_dppy_impl<T, 2, CPL, true>(nstages, a, g, s, nstrips, nsegs);
}
template hipError_t launch_dppy_pc_tu<float, 2>(int, const FusedArgs<float>&, const Geom&, hipStream_t, int, int);
template <typename T, int CPL>
int dppy_pc_blocks_per_cu_tu(int nstages, int sp_mode) {
    return dppy_blocks_per_cu_impl<T, 2, CPL, true>(nstages, sp_mode);
}
template int dppy_pc_blocks_per_cu_tu<float, 2>(int, int);
}  // namespace ws
