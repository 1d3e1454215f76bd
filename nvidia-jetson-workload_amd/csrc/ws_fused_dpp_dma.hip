// DPP fused step kernel, LDS-DMA mode (y rows staged through LDS, copied to the VGPR ring); the kernel: ws_fused_dpp_kernel.h.
#include "ws_fused_dpp_kernel.h"

namespace ws {

template <typename T>
hipError_t launch_dpp_dma(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s) {
    return launch_dpp_impl<T, 0>(nstages, a, g, s);
}

template hipError_t launch_dpp_dma<float>(int, const FusedArgs<float>&, const Geom&, hipStream_t);
template hipError_t launch_dpp_dma<double>(int, const FusedArgs<double>&, const Geom&, hipStream_t);

}  // namespace ws
