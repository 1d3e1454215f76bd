/* Host-code sanitizer check (ASan + UBSan) of libws_hip.so's host paths that run without a
 * GPU: configuration defaults, the slab partition, the halo exchange plan, argument
 * validation and the no-device error paths of the C ABI. Built and run by
 * tools/sanitize/host_sanitize.sh (tests/test_host_sanitizers.py); any sanitizer report
 * aborts with a non-zero status. */
#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ws_hip.h"

static int check_partition(void) {
    for (int H = 1; H <= 300; ++H)
        for (int n = 1; n <= 9 && n <= H; ++n) {
            int32_t next = 0;
            for (int r = 0; r < n; ++r) {
                int32_t row0 = -1, rows = -1;
                if (ws_slab_partition(H, r, n, &row0, &rows) != WS_OK) return 1;
                if (row0 != next || rows < H / n || rows > H / n + 1) return 2;
                next = row0 + rows;
            }
            if (next != H) return 3;
        }
    int32_t a, b;
    if (ws_slab_partition(10, 3, 3, &a, &b) == WS_OK) return 4; /* rank out of range */
    return 0;
}

static int check_plan(void) {
    for (int dtype = WS_F32; dtype <= WS_F64; ++dtype)
        for (int nr = 1; nr <= 4; ++nr)
            for (int rank = 0; rank < nr; ++rank)
                for (int L = 1; L <= 33; L += 16)
                    for (int depth = 1; depth <= 24; depth += 7) {
                        int32_t count = -1;
                        int64_t pitch = 0, lstride = 0;
                        if (ws_slab_exchange_plan(97, 40, L, dtype, rank, nr, 3, depth, NULL, 0, &count, &pitch,
                                                  &lstride) != WS_OK)
                            return 10;
                        const int nb = (rank > 0) + (rank < nr - 1);
                        if (count != 2 * 3 * L * nb) return 11;
                        ws_xfer_t* x = (ws_xfer_t*)malloc(sizeof(ws_xfer_t) * (size_t)(count > 0 ? count : 1));
                        int32_t c2 = 0;
                        if (count > 0 && ws_slab_exchange_plan(97, 40, L, dtype, rank, nr, 3, depth, x, count - 1, &c2,
                                                               NULL, NULL) == WS_OK)
                            return 12; /* capacity too small must fail */
                        if (ws_slab_exchange_plan(97, 40, L, dtype, rank, nr, 3, depth, x, count, &c2, NULL, NULL) !=
                            WS_OK)
                            return 13;
                        for (int i = 0; i < count; ++i)
                            if (x[i].bytes != (int64_t)depth * pitch * (dtype == WS_F64 ? 8 : 4)) return 14;
                        free(x);
                    }
    int32_t c;
    if (ws_slab_exchange_plan(97, 40, 1, WS_F64, 0, 2, 3, 25, NULL, 0, &c, NULL, NULL) == WS_OK) return 15;
    if (ws_slab_exchange_plan(0, 40, 1, WS_F64, 0, 2, 3, 2, NULL, 0, &c, NULL, NULL) == WS_OK) return 16;
    return 0;
}

static int check_no_device_paths(void) {
    ws_config_t cfg;
    ws_config_default(&cfg);
    if (cfg.grid_width != 256 || cfg.grid_height != 256 || cfg.integration_method != WS_RK4) return 20;
    int32_t ok = 1;
    if (ws_is_available(&ok) != WS_OK) return 21;
    ws_sim_t* sim = NULL;
    if (!ok) { /* a GPU-less host: every creating call fails loudly (no CPU fallback) */
        if (ws_sim_create(&cfg, &sim) != WS_ERR_DEVICE || sim != NULL) return 22;
        const char* msg = ws_last_error();
        if (!msg || strlen(msg) == 0) return 23;
        ws_grid_t* g = NULL;
        if (ws_grid_create(16, 16, 1, WS_F32, 0, &g) == WS_OK) return 26;
    }
    cfg.grid_width = 0;
    if (ws_sim_create(&cfg, &sim) == WS_OK) return 24;
    if (ws_sim_create(NULL, &sim) == WS_OK) return 25;
    if (ws_launch_shallow_water_kernel(NULL, NULL, NULL, NULL, NULL, NULL, 8, 8, 8, 0.01, 9.81, 1, 1, 0, WS_F32,
                                       NULL) != WS_ERR_INVALID)
        return 27;
    double d = 0;
    if (ws_sim_cfl(NULL, &d, NULL, 0, NULL) != WS_ERR_INVALID) return 28;
    ws_config_default(&cfg);
    int32_t r0 = 0, nr = 0;
    /* a NULL communicator id is an error (the measurement slab has its own entry point) */
    if (ws_sim_create_slab(&cfg, 0, 2, NULL, &sim, &r0, &nr) != WS_ERR_INVALID) return 29;
    if (ws_sim_create_slab_emulated(&cfg, 0, 1, 5.0, &sim, &r0, &nr) != WS_ERR_INVALID) return 30;
    if (ws_sim_create_slab_emulated(&cfg, 0, 2, -1.0, &sim, &r0, &nr) != WS_ERR_INVALID) return 31;
    if (ws_sim_pin_variant(NULL, -1, -1, -1, -1) != WS_ERR_INVALID) return 32;
    if (ws_sim_set_slab_schedule(NULL, 6, WS_OVERLAP_AUTO) != WS_ERR_INVALID) return 33;
    if (ws_bvort_create_poisson(&cfg, 7, NULL) != WS_ERR_INVALID) return 34;
    return 0;
}

int main(void) {
    int rc;
    if ((rc = check_partition())) return rc;
    if ((rc = check_plan())) return rc;
    if ((rc = check_no_device_paths())) return rc;
    printf("host sanitizer check ok\n");
    return 0;
}
