// CFL max-reduction (ws_reduce.hip).
#pragma once

#include "ws_internal.h"

namespace ws {

// partial results per level of launch_cfl (scratch: L x cfl_partials(g) uint64)
int cfl_partials(const Geom& g);
// per level l: out[l] = bits of max over cells of max((|u| + sqrt(g h)) dt_dx, (|v| + sqrt(g h)) dt_dy),
// as a double's IEEE bit pattern (non-negative doubles order as unsigned integers)
template <typename T>
hipError_t launch_cfl(const T* u, const T* v, const T* h, const Geom& g, T gravity, T dt_dx, T dt_dy,
                      uint64_t* partial, uint64_t* out, hipStream_t s);

}  // namespace ws
