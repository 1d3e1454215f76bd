/* CPU oracle for the weather-sim time step -- TEST INFRASTRUCTURE ONLY (see
 * ws_oracle_impl.h for the reference file:line map). Builds liboracle.so exporting
 * ws_oracle_f32_* and ws_oracle_f64_*; loaded only by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg. */
#include <stdlib.h>
#include <string.h>

#define WS_T float
#define WS_SFX f32
#include "ws_oracle_impl.h"
#undef WS_T
#undef WS_SFX

#define WS_T double
#define WS_SFX f64
#include "ws_oracle_impl.h"
#undef WS_T
#undef WS_SFX
