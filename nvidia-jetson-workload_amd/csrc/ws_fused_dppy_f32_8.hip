// fused_dppy_kernel instantiations for float, 8 time steps per launch (Euler), one column per lane (variant dppy)
// (see ws_fused_dppy_kernel.h)
#include "ws_fused_dppy_kernel.h"

namespace ws {
template <typename T, int NSTEP, int CPL>
hipError_t launch_dppy_tu(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s, int nstrips, int nsegs) {
    return launch_dppy_impl<T, NSTEP, CPL>(nstages, a, g, s, nstrips, nsegs);
}
template hipError_t launch_dppy_tu<float, 8, 1>(int, const FusedArgs<float>&, const Geom&, hipStream_t, int, int);
template <typename T, int NSTEP, int CPL>
int dppy_blocks_per_cu_tu(int nstages, int sp_mode) {
    return dppy_blocks_per_cu_impl<T, NSTEP, CPL>(nstages, sp_mode);
}
template int dppy_blocks_per_cu_tu<float, 8, 1>(int, int);
}  // namespace ws
