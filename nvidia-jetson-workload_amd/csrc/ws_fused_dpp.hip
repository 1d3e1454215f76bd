// DPP fused step kernel, VGPR-prefetch mode, and the mode dispatcher (the kernel itself:
// ws_fused_dpp_kernel.h).
#include "ws_fused_dpp_kernel.h"

namespace ws {

template <typename T>
hipError_t launch_dpp_vgpr(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s) {
    return launch_dpp_impl<T, WS_DPP_PF>(nstages, a, g, s);
}

template <typename T>
hipError_t launch_fused_step_dpp(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s, int mode) {
    switch (mode) {
        case kDppVgpr: return launch_dpp_vgpr<T>(nstages, a, g, s);
        case kDppDma: return launch_dpp_dma<T>(nstages, a, g, s);
        case kDppLdsY: return launch_dpp_ldsy<T>(nstages, a, g, s);
        default: return hipErrorInvalidValue;
    }
}

template hipError_t launch_fused_step_dpp<float>(int, const FusedArgs<float>&, const Geom&, hipStream_t, int);
template hipError_t launch_fused_step_dpp<double>(int, const FusedArgs<double>&, const Geom&, hipStream_t, int);

}  // namespace ws
