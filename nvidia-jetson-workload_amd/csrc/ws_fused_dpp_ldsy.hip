// DPP fused step kernel, LDS-resident-y mode (y rows read from the LDS-DMA ring in place); the kernel: ws_fused_dpp_kernel.h.
#include "ws_fused_dpp_kernel.h"

namespace ws {

template <typename T>
hipError_t launch_dpp_ldsy(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s) {
    return launch_dpp_impl<T, -1>(nstages, a, g, s);
}

template hipError_t launch_dpp_ldsy<float>(int, const FusedArgs<float>&, const Geom&, hipStream_t);
template hipError_t launch_dpp_ldsy<double>(int, const FusedArgs<double>&, const Geom&, hipStream_t);

}  // namespace ws
