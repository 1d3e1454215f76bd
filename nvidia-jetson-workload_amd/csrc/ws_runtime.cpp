// Host runtime of libws_hip.so: device-resident grids and simulations, and the C ABI of
// both (include/ws_hip.h; internal interfaces in ws_sim.h).
//
// Owns device-resident grids (SoA, one allocation per field, rows padded to a 64-element
// pitch, kHalo spare rows above/below each level for slab halos) and the simulation objects
// whose step / run (ws_schedule.cpp) replace WeatherSimulation::step/run (reference
// src/weather-sim/cpp/src/weather_simulation.cpp:68-158). Fields leave the device only
// through ws_grid_get_field.
#include <algorithm>
#include <cstdio>

#include "ws_ic.h"
#include "ws_reduce.h"
#include "ws_sim.h"

namespace wsr {

thread_local std::string g_last_error;

int device_count() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void set_device(int dev) {
    const int n = device_count();
    if (n <= 0) throw WsError(WS_ERR_DEVICE, "no HIP device available (MI355X build has no CPU path)");
    if (dev < 0 || dev >= n) throw WsError(WS_ERR_DEVICE, "device_id out of range");
    WS_HIP_CHECK(hipSetDevice(dev));
}

static void grid_alloc(ws_grid* g, unsigned nfields) {
    g->pitch = layout_pitch(g->W);
    g->lstride = layout_lstride(g->H, g->pitch);
    g->nfields = nfields;
    const size_t es = elem_size(g->dtype);
    for (unsigned i = 0; i < nfields; ++i) {
        WS_HIP_CHECK(hipMalloc(&g->alloc[i], g->bytes_per_field()));
        // on the grid's own stream: a legacy-stream hipMemset is not ordered with the
        // non-blocking streams the kernels run on, and returns before it completes -- it raced
        // with the first launches writing a freshly allocated overlap grid (slab groups)
        WS_HIP_CHECK(hipMemsetAsync(g->alloc[i], 0, g->bytes_per_field(), g->stream));
        g->f[i] = (char*)g->alloc[i] + (size_t)ws::kHalo * g->pitch * es;
    }
}

void grid_free(ws_grid* g) {
    for (auto& a : g->alloc)
        if (a) { (void)hipFree(a); a = nullptr; }
    for (auto& e : g->tev)
        if (e) { (void)hipEventDestroy(e); e = nullptr; }
}

template <typename T>
static void grid_reset_t(ws_grid* g) {
    const ws::Geom ge = g->geom();
    // weather_grid.cpp:57-71 (float literals, widened for the fp64 build)
    const T vals[8] = {T(0.0f), T(0.0f), T(10.0f), T(1013.25f), T(288.15f), T(0.0f), T(0.0f), T(0.0f)};
    for (unsigned i = 0; i < g->nfields; ++i) WS_HIP_CHECK(ws::launch_fill<T>((T*)g->f[i], vals[i], ge, g->stream));
    g->diag_pending = false;
}

void grid_reset(ws_grid* g) {
    if (g->dtype == WS_F64) grid_reset_t<double>(g);
    else grid_reset_t<float>(g);
}

template <typename T>
static void grid_diag_t(ws_grid* g) {
    WS_HIP_CHECK(ws::launch_diagnostics<T>((const T*)g->f[WS_FIELD_U], (const T*)g->f[WS_FIELD_V],
                                           (T*)g->f[WS_FIELD_VORTICITY], (T*)g->f[WS_FIELD_DIVERGENCE],
                                           make_spacing<T>(g->dx, g->dy), g->geom(), g->stream));
}

void materialize_diag(ws_grid* g) {
    if (!g->diag_pending) return;
    if (g->dtype == WS_F64) grid_diag_t<double>(g);
    else grid_diag_t<float>(g);
    g->diag_pending = false;
}

ws_grid* new_grid(int32_t W, int32_t H, int32_t L, int32_t dtype, int32_t device, unsigned nfields, hipStream_t s) {
    require(W > 0 && H > 0 && L > 0, WS_ERR_INVALID, "Grid dimensions must be positive");
    require(dtype == WS_F32 || dtype == WS_F64, WS_ERR_INVALID, "dtype must be WS_F32 or WS_F64");
    set_device(device);
    ws_grid* g = new ws_grid;
    g->W = W; g->H = H; g->L = L; g->dtype = dtype; g->device = device; g->stream = s;
    g->row0 = 0; g->gH = H;
    try {
        grid_alloc(g, nfields);
        if (nfields == 8) grid_reset(g);
    } catch (...) {
        grid_free(g);
        delete g;
        throw;
    }
    return g;
}

template <typename Dst, typename Src>
static void convert(Dst* d, const Src* s, size_t n) {
    for (size_t i = 0; i < n; ++i) d[i] = static_cast<Dst>(s[i]);
}

}  // namespace wsr

int ws_sim::launch_tb() const {
    if (kernel == wsr::kKernLds) return 1;
    int t = tb;
    while (t > 1 && !ws::fused_tb_ok(kernel, t, wsr::fused_stages(this), (int)wsr::elem_size(dtype))) t /= 2;
    return std::max(t, 1);
}

int32_t ws_sim::seg_for_blocks(int nst, int64_t want_blocks, int64_t min_rows) const {
    const ws_grid* g = slot[0];
    const int64_t per_seg = strips(nst * launch_tb()) * g->L;
    const int64_t want_segs = std::max<int64_t>(1, (want_blocks + per_seg - 1) / per_seg);
    int64_t rows = (g->H + want_segs - 1) / want_segs;
    rows = std::max<int64_t>(rows, min_rows);
    const int cone = nst * launch_tb();
    rows = (rows + 2 * cone + 7) / 8 * 8 - 2 * cone;
    return (int32_t)std::max<int64_t>(1, std::min<int64_t>(rows, g->H));
}

int32_t ws_sim::seg_rows(int nst) const {
    if (seg_override > 0 || (wsr::chain_rounds(seg_override) > 0 && kernel != wsr::kKernLds)) return seg_override;
    const int64_t want_blocks = ws::fused_pairs(kernel) ? 2048 : ws::fused_is_dppy(kernel) ? 4096 : 512;
    return seg_for_blocks(nst, want_blocks, 24 * nst);
}

namespace wsr {

void sim_free(ws_sim* s) {
    for (ws_grid* g : {s->slot[0], s->slot[1], s->tmpA, s->tmpB, s->K2, s->K3, s->ov[0], s->ov[1], s->ov[2], s->ov[3]})
        if (g) { grid_free(g); delete g; }
    for (hipEvent_t e : {s->ev0, s->ev1, s->aux_in, s->aux_out, s->ev_edge, s->ev_join, s->ev_trial[0], s->ev_trial[1]})
        if (e) (void)hipEventDestroy(e);
    if (s->aux) (void)hipStreamDestroy(s->aux);
    if (s->edge) (void)hipStreamDestroy(s->edge);
    if (s->stream && s->own_stream) (void)hipStreamDestroy(s->stream);
    if (s->cfl_scratch) (void)hipFree(s->cfl_scratch);
    for (auto& t : s->chain_tables)
        if (t.dev) (void)hipFree(t.dev);
    delete s->comm;
    delete s->staging;
    delete s;
}

ws_sim* sim_build(const ws_config_t* cfg, SlabInfo slab, ws::SlabComm* comm, hipStream_t stream) {
    const int32_t local_rows = slab.nranks == 1 ? (cfg ? cfg->grid_height : 0) : slab.rows;
    const int32_t row0 = slab.row0;
    require(cfg != nullptr, WS_ERR_INVALID, "null config");
    require(cfg->grid_width > 0 && cfg->grid_height > 0 && cfg->num_levels > 0, WS_ERR_INVALID,
            "Grid dimensions must be positive");
    require(cfg->dx > 0 && cfg->dy > 0, WS_ERR_INVALID, "Grid spacing must be positive");
    // The reference runs every backend through its CPU solver (selectOptimalBackend,
    // weather_simulation.cpp:562-591; the CUDA branch is a placeholder). This library has only
    // the HIP path, which every backend runs -- CPU included (the reference's own tests request
    // it "for consistent tests", weather_simulation_test.cpp:68, and the HIP results are the
    // CPU solver's bits); the Python layer warns once that CPU work ran on the GPU (D8).
    require(cfg->compute_backend >= WS_BACKEND_CUDA && cfg->compute_backend <= WS_BACKEND_ADAPTIVE_HYBRID,
            WS_ERR_INVALID, "unknown compute_backend");
    set_device(cfg->device_id);
    ws_sim* s = new ws_sim;
    s->cfg = *cfg;
    s->dtype = cfg->double_precision ? WS_F64 : WS_F32;
    s->device = cfg->device_id;
    s->dt = to_prec(cfg->dt, s->dtype);
    s->comm = comm;
    s->row0 = row0;
    s->rank = slab.rank;
    s->nranks = slab.nranks;
    try {
        if (stream) {
            s->stream = stream;
            s->own_stream = false;
        } else {
            WS_HIP_CHECK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        }
        WS_HIP_CHECK(hipEventCreate(&s->ev0));
        WS_HIP_CHECK(hipEventCreate(&s->ev1));
        const int W = cfg->grid_width, H = local_rows, L = cfg->num_levels;
        for (int i = 0; i < 2; ++i) s->slot[i] = new_grid(W, H, L, s->dtype, s->device, 8, s->stream);
        // environment switches (include/ws_hip.h lists every one the library reads)
        if (const char* e = env_str("WS_FUSED")) s->fused = std::atoi(e) != 0;
        // numerics: fast for fp64 (north_star tolerance), exact for fp32; WS_NUMERICS overrides
        s->numerics = s->dtype == WS_F64 ? WS_NUMERICS_FAST : WS_NUMERICS_EXACT;
        if (const char* e = env_str("WS_NUMERICS")) {
            require(std::strcmp(e, "exact") == 0 || std::strcmp(e, "fast") == 0, WS_ERR_INVALID,
                    "WS_NUMERICS must be exact or fast");
            s->numerics = std::strcmp(e, "fast") == 0 ? WS_NUMERICS_FAST : WS_NUMERICS_EXACT;
        }
        if (const char* e = env_str("WS_KERNEL")) {
            static const std::pair<const char*, int> names[] = {
                {"lds", kKernLds}, {"dppy", kKernDppLdsY}, {"x2y", kKernX2Y}, {"pc", kKernPc}, {"pc2", kKernPc2}};
            int k = -1;
            for (const auto& n : names)
                if (std::strcmp(e, n.first) == 0) k = n.second;
            require(k >= 0, WS_ERR_INVALID, "WS_KERNEL must be x2y, dppy, pc, pc2 or lds");
            s->kernel = k;
            s->kernel_fixed = true;
            s->kernel_env = true;
            if (ws::fused_split(k)) s->tb = 2;  // the split variants advance two steps per launch
        }
        if (const char* e = env_str("WS_TB")) {
            s->tb = std::atoi(e);
            // (4 / 8: where the kernel takes them -- Euler / RK2 (8: Euler) on dppy, x2y in
            // fp32 -- else the largest it takes: ws_sim::launch_tb)
            require(s->tb == 1 || s->tb == 2 || s->tb == 4 || s->tb == 8, WS_ERR_INVALID, "WS_TB must be 1, 2, 4 or 8");
            require(!(s->kernel_env && ws::fused_split(s->kernel) && s->tb == 1), WS_ERR_INVALID,
                    "WS_KERNEL=pc / pc2 advance two steps per launch: WS_TB must be 2 (or unset)");
            s->tb_fixed = true;
        }
        if (const char* e = env_str("WS_SEG_ROWS")) {  // n > 0 rows, or -2, -3, ...: chain schedule
            s->seg_override = std::atoi(e);
            s->seg_fixed = s->seg_override > 0 || (chain_rounds(s->seg_override) > 0 &&
                                                   chain_rounds(s->seg_override) <= kMaxChainRounds);
            if (!s->seg_fixed) s->seg_override = 0;
        }
        s->tuned = env_int("WS_AUTOTUNE", 1) == 0;

        const int method = effective_method(*cfg);
        if (slab.nranks > 1 && s->fused) {
            // steps per exchange: as many as the halo (kHalo rows) and the thinnest slab
            // (floor(H / nranks) rows, the same on every rank: neighbours must agree) allow,
            // at most 6: an exchange is a fixed RCCL latency (~10 us) plus the transfer, the
            // extended rows cost (block - 2) NST rows per side and launch (C2 at 8 slabs,
            // block 6: 3 % more rows computed, one exchange per 6 steps instead of 3)
            const int nst = method == WS_EULER ? 1 : method == WS_RK2 ? 2 : 4;
            const int thin = cfg->grid_height / slab.nranks;
            s->block = std::max(1, std::min(6, std::min(ws::kHalo, thin) / nst));
            // overlap schedule (overlap_block): WS_SLAB_OVERLAP=0|1 fixes it; by default it is
            // decided at the first run from a measured halo exchange (choose_slab_schedule)
            s->overlap_mode = kOverlapAuto;
            if (const char* e = env_str("WS_SLAB_OVERLAP")) s->overlap_mode = std::atoi(e) != 0 ? kOverlapOn : kOverlapOff;
            s->overlap = s->overlap_mode == kOverlapOn;
        } else if (comm && s->fused) {
            // a one-rank communicator slab runs overlap_block itself only when asked
            s->overlap = env_int("WS_SLAB_OVERLAP", 0) != 0;
            s->overlap_mode = s->overlap ? kOverlapOn : kOverlapOff;
        }
        if (!s->fused && method != WS_EULER) s->tmpA = new_grid(W, H, L, s->dtype, s->device, 3, s->stream);
        if (!s->fused && method == WS_RK4) {
            s->tmpB = new_grid(W, H, L, s->dtype, s->device, 3, s->stream);
            s->K2 = new_grid(W, H, L, s->dtype, s->device, 3, s->stream);
            s->K3 = new_grid(W, H, L, s->dtype, s->device, 3, s->stream);
        }
        for (ws_grid* g : {s->slot[0], s->slot[1], s->tmpA, s->tmpB, s->K2, s->K3}) {
            if (!g) continue;
            g->owned = true;
            g->dx = to_prec(cfg->dx, s->dtype);
            g->dy = to_prec(cfg->dy, s->dtype);
            if (slab.nranks > 1) {
                g->top_clamp = slab.rank == 0;
                g->bot_clamp = slab.rank == slab.nranks - 1;
                g->row0 = row0;
                g->gH = cfg->grid_height;
            }
        }
        WS_HIP_CHECK(hipStreamSynchronize(s->stream));
    } catch (...) {
        s->comm = nullptr;  // caller keeps ownership on failure
        sim_free(s);
        throw;
    }
    return s;
}


}  // namespace wsr

using namespace wsr;

extern "C" {

const char* ws_last_error(void) { return g_last_error.c_str(); }

int ws_abi_version(void) { return WS_ABI_VERSION; }

int ws_is_available(int32_t* available) {
    return guarded([&] {
        require(available != nullptr, WS_ERR_INVALID, "null pointer");
        *available = device_count() > 0;
    });
}

int ws_device_count(int32_t* count) {
    return guarded([&] {
        require(count != nullptr, WS_ERR_INVALID, "null pointer");
        *count = device_count();
    });
}

int ws_device_info(int32_t device, ws_device_info_t* out) {
    return guarded([&] {
        require(out != nullptr, WS_ERR_INVALID, "null pointer");
        set_device(device);
        hipDeviceProp_t p;
        WS_HIP_CHECK(hipGetDeviceProperties(&p, device));
        std::memset(out, 0, sizeof(*out));
        std::snprintf(out->device_name, sizeof(out->device_name), "%s", p.name);
        std::snprintf(out->arch, sizeof(out->arch), "%s", p.gcnArchName);
        out->compute_capability_major = p.major;
        out->compute_capability_minor = p.minor;
        out->multiprocessors = p.multiProcessorCount;
        out->cuda_cores = p.multiProcessorCount * 64;
        out->global_memory = (int64_t)p.totalGlobalMem;
        out->shared_memory_per_block = (int32_t)p.sharedMemPerBlock;
        out->max_threads_per_block = p.maxThreadsPerBlock;
        out->max_threads_per_multiprocessor = p.maxThreadsPerMultiProcessor;
        out->clock_rate_khz = p.clockRate;
        out->memory_clock_rate_khz = p.memoryClockRate;
        out->memory_bus_width = p.memoryBusWidth;
        out->wavefront_size = p.warpSize;
    });
}

int ws_device_memory(int32_t device, int64_t* free_bytes, int64_t* total_bytes) {
    return guarded([&] {
        set_device(device);
        size_t fr = 0, tot = 0;
        WS_HIP_CHECK(hipMemGetInfo(&fr, &tot));
        if (free_bytes) *free_bytes = (int64_t)fr;
        if (total_bytes) *total_bytes = (int64_t)tot;
    });
}

void ws_config_default(ws_config_t* c) {
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    // SimulationConfig defaults (weather_sim.hpp:155-191)
    c->model = WS_MODEL_SHALLOW_WATER;
    c->grid_type = 1;  // Staggered
    c->integration_method = WS_RK4;
    c->boundary_condition = 0;  // Periodic (accepted, not read: clamp-to-self)
    c->grid_width = 256;
    c->grid_height = 256;
    c->num_levels = 1;
    c->dx = 1.0; c->dy = 1.0; c->dt = 0.01;
    c->gravity = 9.81; c->coriolis_f = 0.0;
    c->compute_backend = WS_BACKEND_CUDA;
    c->double_precision = 0;
    c->device_id = 0;
    c->num_threads = 0;
    c->max_time = 10.0;
    c->max_steps = 1000;
    c->output_interval = 10;
    c->random_seed = 0;
}

// ---- grid ----
int ws_grid_create(int32_t width, int32_t height, int32_t num_levels, int32_t dtype, int32_t device,
                   ws_grid_t** out) {
    return guarded([&] {
        require(out != nullptr, WS_ERR_INVALID, "null pointer");
        ws_grid* g = new_grid(width, height, num_levels, dtype, device, 8, nullptr);
        WS_HIP_CHECK(hipStreamSynchronize(nullptr));
        *out = g;
    });
}

int ws_grid_destroy(ws_grid_t* g) {
    return guarded([&] {
        if (!g) return;
        require(!g->owned, WS_ERR_INVALID, "grid is owned by a simulation");
        set_device(g->device);
        grid_free(g);
        delete g;
    });
}

int ws_grid_reset(ws_grid_t* g) {
    return guarded([&] {
        require(g != nullptr, WS_ERR_INVALID, "null grid");
        set_device(g->device);
        grid_reset(g);
        WS_HIP_CHECK(hipStreamSynchronize(g->stream));
    });
}

int ws_grid_get_dims(const ws_grid_t* g, int32_t* w, int32_t* h, int32_t* l, int32_t* dt) {
    return guarded([&] {
        require(g != nullptr, WS_ERR_INVALID, "null grid");
        if (w) *w = g->W;
        if (h) *h = g->H;
        if (l) *l = g->L;
        if (dt) *dt = g->dtype;
    });
}

int ws_grid_set_spacing(ws_grid_t* g, double dx, double dy) {
    return guarded([&] {
        require(g != nullptr, WS_ERR_INVALID, "null grid");
        require(dx > 0.0 && dy > 0.0, WS_ERR_INVALID, "Grid spacing must be positive");
        g->dx = to_prec(dx, g->dtype);
        g->dy = to_prec(dy, g->dtype);
    });
}

int ws_grid_get_spacing(const ws_grid_t* g, double* dx, double* dy) {
    return guarded([&] {
        require(g != nullptr, WS_ERR_INVALID, "null grid");
        if (dx) *dx = g->dx;
        if (dy) *dy = g->dy;
    });
}

static void check_field_args(const ws_grid* g, int32_t field, int32_t level, int32_t height, int32_t width,
                             int32_t dtype, bool writing) {
    require(g != nullptr, WS_ERR_INVALID, "null grid");
    require(field >= 0 && field < (int)g->nfields, WS_ERR_INVALID, "bad field id");
    require(!writing || field < WS_FIELD_VORTICITY, WS_ERR_INVALID, "diagnostic fields are read-only");
    require(level >= -1 && level < g->L, WS_ERR_INVALID, "level out of range");
    require(dtype == WS_F32 || dtype == WS_F64, WS_ERR_INVALID, "dtype must be WS_F32 or WS_F64");
    require(height == g->H && width == g->W, WS_ERR_SHAPE, "Array dimensions must match field dimensions");
}

static void copy_field(ws_grid* g, int32_t field, int32_t level, void* host, int32_t dtype, bool to_device) {
    const size_t es = elem_size(g->dtype), n = (size_t)g->W * g->H;
    const int l0 = level < 0 ? 0 : level, l1 = level < 0 ? g->L : level + 1;
    std::vector<char> tmp;
    for (int l = l0; l < l1; ++l) {
        char* hp = (char*)host + (size_t)(l - l0) * n * elem_size(dtype);
        void* src_or_dst = hp;
        if (dtype != g->dtype) {
            tmp.resize(n * es);
            src_or_dst = tmp.data();
            if (to_device) {
                if (g->dtype == WS_F32) convert((float*)tmp.data(), (const double*)hp, n);
                else convert((double*)tmp.data(), (const float*)hp, n);
            }
        }
        char* dev = (char*)g->f[field] + (size_t)l * g->lstride * es;
        if (to_device)
            WS_HIP_CHECK(hipMemcpy2DAsync(dev, g->pitch * es, src_or_dst, g->W * es, g->W * es, g->H,
                                          hipMemcpyHostToDevice, g->stream));
        else
            WS_HIP_CHECK(hipMemcpy2DAsync(src_or_dst, g->W * es, dev, g->pitch * es, g->W * es, g->H,
                                          hipMemcpyDeviceToHost, g->stream));
        WS_HIP_CHECK(hipStreamSynchronize(g->stream));
        if (!to_device && dtype != g->dtype) {
            if (g->dtype == WS_F32) convert((double*)hp, (const float*)tmp.data(), n);
            else convert((float*)hp, (const double*)tmp.data(), n);
        }
    }
}

int ws_grid_set_field(ws_grid_t* g, int32_t field, int32_t level, const void* host, int32_t height, int32_t width,
                      int32_t dtype) {
    return guarded([&] {
        check_field_args(g, field, level, height, width, dtype, true);
        require(host != nullptr, WS_ERR_INVALID, "null host pointer");
        set_device(g->device);
        // keep vorticity what calculateDiagnostics made of the OLD u, v (reference setters
        // do not recompute diagnostics)
        if (field == WS_FIELD_U || field == WS_FIELD_V) materialize_diag(g);
        copy_field(g, field, level, const_cast<void*>(host), dtype, true);
    });
}

int ws_grid_get_field(ws_grid_t* g, int32_t field, int32_t level, void* host, int32_t height, int32_t width,
                      int32_t dtype) {
    return guarded([&] {
        check_field_args(g, field, level, height, width, dtype, false);
        require(host != nullptr, WS_ERR_INVALID, "null host pointer");
        set_device(g->device);
        if (field >= WS_FIELD_VORTICITY) materialize_diag(g);
        copy_field(g, field, level, host, dtype, false);
    });
}

int ws_grid_device_field(ws_grid_t* g, int32_t field, void** dptr, int64_t* pitch, int64_t* level_stride) {
    return guarded([&] {
        require(g != nullptr && field >= 0 && field < (int)g->nfields, WS_ERR_INVALID, "bad grid/field");
        set_device(g->device);
        if (field >= WS_FIELD_VORTICITY) {
            materialize_diag(g);
            WS_HIP_CHECK(hipStreamSynchronize(g->stream));
        }
        if (dptr) *dptr = g->f[field];
        if (pitch) *pitch = g->pitch;
        if (level_stride) *level_stride = g->lstride;
    });
}

int ws_grid_calculate_diagnostics(ws_grid_t* g) {
    return guarded([&] {
        require(g != nullptr, WS_ERR_INVALID, "null grid");
        g->diag_pending = true;
    });
}

int ws_grid_apply_initial_condition(ws_grid_t* g, const char* name, const double* params, int32_t nparams,
                                    const char* sparam, int32_t level) {
    return guarded([&] {
        require(g != nullptr && name != nullptr, WS_ERR_INVALID, "null argument");
        require(level >= -1 && level < g->L, WS_ERR_INVALID, "level out of range");
        set_device(g->device);
        const std::string nm(name), sp(sparam ? sparam : "");
        auto apply = [&](auto tag) {
            using T = decltype(tag);
            ws::IcFields<T> f(g->W, g->gH, g->row0, g->H);
            require(ws::compute_initial_condition<T>(nm, params, nparams, sp, f), WS_ERR_INVALID,
                    "unknown initial condition");
            materialize_diag(g);
            const std::pair<unsigned, std::vector<T>*> m[6] = {{ws::kU, &f.u}, {ws::kV, &f.v}, {ws::kH, &f.h},
                                                               {ws::kP, &f.p}, {ws::kT, &f.t}, {ws::kQ, &f.q}};
            const int l0 = level < 0 ? 0 : level, l1 = level < 0 ? g->L : level + 1;
            for (int i = 0; i < 6; ++i)
                if (f.wrote & m[i].first)
                    for (int l = l0; l < l1; ++l) copy_field(g, i, l, m[i].second->data(), g->dtype, true);
        };
        if (g->dtype == WS_F64) apply(double{});
        else apply(float{});
        g->diag_pending = true;  // every IC ends with grid.calculateDiagnostics()
    });
}

// ---- simulation ----
int ws_sim_create(const ws_config_t* cfg, ws_sim_t** out) {
    return guarded([&] {
        require(out != nullptr, WS_ERR_INVALID, "null pointer");
        *out = sim_build(cfg, SlabInfo{}, nullptr);
    });
}

int ws_sim_destroy(ws_sim_t* s) {
    return guarded([&] {
        if (!s) return;
        require(!s->in_group, WS_ERR_INVALID, "simulation is owned by a slab group");
        set_device(s->device);
        (void)hipStreamSynchronize(s->stream);
        sim_free(s);
    });
}

int ws_sim_grid(ws_sim_t* s, int32_t which, ws_grid_t** out) {
    return guarded([&] {
        require(s != nullptr && out != nullptr && (which == 0 || which == 1), WS_ERR_INVALID, "bad argument");
        *out = s->slot[which == 0 ? s->cur : 1 - s->cur];
    });
}

int ws_sim_initialize(ws_sim_t* s) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        set_device(s->device);
        s->time = 0.0;
        s->step = 0;
        s->tp_lazy = false;  // no drift of an earlier run may land on the reset fields
        s->tp_steps = 0;
        std::memset(&s->metrics, 0, sizeof(s->metrics));
        grid_reset(s->slot[s->cur]);
        WS_HIP_CHECK(hipStreamSynchronize(s->stream));
    });
}

int ws_sim_inject_failure(ws_sim_t* s, int32_t after_launches) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        s->fail_after = after_launches;
    });
}

int ws_sim_step(ws_sim_t* s) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        run_steps(s, 1);
    });
}

int ws_sim_run(ws_sim_t* s, int32_t n, int32_t* taken) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        const int k = plan_steps(s, n);
        if (k > 0) run_steps(s, k);
        if (taken) *taken = k;
    });
}

int ws_sim_run_until(ws_sim_t* s, double max_time, int32_t* taken) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        int k = 0;
        // weather_simulation.cpp:105-115, evaluated in scalar_t
        if (s->dtype == WS_F64) {
            const double mt = max_time, t = s->time;
            if (!(mt <= t)) k = plan_steps(s, (int)((mt - t) / s->dt) + 1);
        } else {
            const float mt = (float)max_time, t = (float)s->time;
            if (!(mt <= t)) k = plan_steps(s, (int)((mt - t) / (float)s->dt) + 1);
        }
        if (k > 0) run_steps(s, k);
        if (taken) *taken = k;
    });
}

int ws_sim_get_time(const ws_sim_t* s, double* t) {
    return guarded([&] {
        require(s && t, WS_ERR_INVALID, "null pointer");
        *t = s->time;
    });
}

int ws_sim_get_step(const ws_sim_t* s, int32_t* st) {
    return guarded([&] {
        require(s && st, WS_ERR_INVALID, "null pointer");
        *st = s->step;
    });
}

int ws_sim_get_dt(const ws_sim_t* s, double* dt) {
    return guarded([&] {
        require(s && dt, WS_ERR_INVALID, "null pointer");
        *dt = s->dt;
    });
}

int ws_sim_set_dt(ws_sim_t* s, double dt) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        s->dt = to_prec(dt, s->dtype);
    });
}

int ws_sim_get_config(const ws_sim_t* s, ws_config_t* cfg) {
    return guarded([&] {
        require(s && cfg, WS_ERR_INVALID, "null pointer");
        *cfg = s->cfg;
    });
}

int ws_sim_get_metrics(const ws_sim_t* s, ws_metrics_t* m) {
    return guarded([&] {
        require(s && m, WS_ERR_INVALID, "null pointer");
        *m = s->metrics;
    });
}

int ws_sim_reset_metrics(ws_sim_t* s) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        std::memset(&s->metrics, 0, sizeof(s->metrics));
    });
}

int ws_sim_synchronize(ws_sim_t* s) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        set_device(s->device);
        WS_HIP_CHECK(hipStreamSynchronize(s->stream));
    });
}

int ws_sim_last_run_stats(const ws_sim_t* s, double* ms, int64_t* launches) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        if (ms) *ms = s->last_ms;
        if (launches) *launches = s->last_launches;
    });
}

// ---- KernelAdapter ----
// The adapter's timing events live on the grid that is timed (created at its first adapter
// call, destroyed with it): a step costs no event creation.
static void adapter_events(ws_grid* g) {
    for (auto& e : g->tev)
        if (!e) WS_HIP_CHECK(hipEventCreate(&e));
}

// One explicit-Euler step in -> out (the reference adapter's executeShallowWaterStep: the fused
// CUDA Euler kernel, shallow_water_kernels.cu:704-719), with the PE T / P update for the
// primitive-equations entry point. The step runs the fused one-step kernel (fused_dppy, NST = 1,
// exact numerics: bit-identical to the reference) over the whole grid; widths below two columns
// take the per-stage kernel.
static int adapter_step(ws_grid* in, ws_grid* out, double dt, double g, double f, double* ms, bool pe) {
    return guarded([&] {
        require(in && out && in != out, WS_ERR_INVALID, "in and out must be distinct grids");
        require(in->W == out->W && in->H == out->H && in->L == out->L && in->dtype == out->dtype &&
                    in->device == out->device && out->nfields == 8,
                WS_ERR_SHAPE, "grids must have identical dimensions and precision");
        set_device(in->device);
        adapter_events(in);
        auto body = [&](auto tag) {
            using T = decltype(tag);
            const ws::Geom ge = in->geom();
            if (in->W >= 2) {
                ws::FusedArgs<T> a{};
                a.in_u = (const T*)in->f[0]; a.in_v = (const T*)in->f[1]; a.in_h = (const T*)in->f[2];
                a.out_u = (T*)out->f[0]; a.out_v = (T*)out->f[1]; a.out_h = (T*)out->f[2];
                a.c_dt = (T)dt;
                a.c_half = T(0.5f) * a.c_dt;
                a.c_dt6 = a.c_dt / T(6.0f);
                a.gravity = (T)g;
                a.coriolis_f = (T)f;
                a.sp1 = a.sp2 = make_spacing<T>(in->dx, in->dy);
                a.sp_mode = ws::exact_sp_mode(a);
                a.out_w = ws::fused_out_w(kKernDppLdsY, 1, (int)sizeof(T), false);
                // segments for ~4 waves per SIMD of the chip (1024 SIMDs), at least 16 rows
                const int64_t strips = (in->W + a.out_w - 1) / a.out_w;
                a.seg_rows = (int)std::max<int64_t>(16, (strips * in->H * in->L + 4095) / 4096);
                a.seg_rows = std::min(a.seg_rows, in->H);
                a.ga_y0 = 0; a.ga_y1 = in->H; a.ga_n = (in->H + a.seg_rows - 1) / a.seg_rows;
                a.gb_y0 = a.gb_y1 = 0;
                a.seg_n = a.ga_n;
                WS_HIP_CHECK(ws::launch_fused_step_dppy<T>(kKernDppLdsY, 1, 1, a, ge, in->stream));
            } else {
                ws::StageArgs<T> a{};
                a.in_u = (const T*)in->f[0]; a.in_v = (const T*)in->f[1]; a.in_h = (const T*)in->f[2];
                a.base_u = a.in_u; a.base_v = a.in_v; a.base_h = a.in_h;
                a.out_u = (T*)out->f[0]; a.out_v = (T*)out->f[1]; a.out_h = (T*)out->f[2];
                a.c = (T)dt; a.gravity = (T)g; a.coriolis_f = (T)f;
                a.sp = make_spacing<T>(in->dx, in->dy);
                WS_HIP_CHECK(ws::launch_stage<T>(ws::kAxpy, a, ge, in->stream));
            }
            if (pe) {
                WS_HIP_CHECK(ws::launch_affine<T>((T*)out->f[WS_FIELD_T], (const T*)in->f[WS_FIELD_T], (T)dt,
                                                  T(288.15f), ge, in->stream));
                WS_HIP_CHECK(ws::launch_affine<T>((T*)out->f[WS_FIELD_P], (const T*)in->f[WS_FIELD_P], (T)dt,
                                                  T(1013.25f), ge, in->stream));
            }
        };
        WS_HIP_CHECK(hipEventRecord(in->tev[0], in->stream));
        if (in->dtype == WS_F64) body(double{});
        else body(float{});
        WS_HIP_CHECK(hipEventRecord(in->tev[1], in->stream));
        WS_HIP_CHECK(hipEventSynchronize(in->tev[1]));
        float t = 0.f;
        WS_HIP_CHECK(hipEventElapsedTime(&t, in->tev[0], in->tev[1]));
        out->diag_pending = true;
        if (ms) *ms = t;
    });
}

int ws_adapter_execute_shallow_water_step(ws_grid_t* in, ws_grid_t* out, double dt, double g, double f, double* ms) {
    return adapter_step(in, out, dt, g, f, ms, false);
}
int ws_adapter_execute_barotropic_step(ws_grid_t* in, ws_grid_t* out, double dt, double g, double f, double* ms) {
    return adapter_step(in, out, dt, g, f, ms, false);
}
int ws_adapter_execute_primitive_equations_step(ws_grid_t* in, ws_grid_t* out, double dt, double g, double f,
                                                double* ms) {
    return adapter_step(in, out, dt, g, f, ms, true);
}
int ws_adapter_execute_gcm_step(ws_grid_t* in, ws_grid_t* out, double dt, double g, double f, double* ms) {
    return adapter_step(in, out, dt, g, f, ms, false);
}

int ws_adapter_calculate_diagnostics(ws_grid_t* g, double* ms) {
    return guarded([&] {
        require(g != nullptr, WS_ERR_INVALID, "null grid");
        set_device(g->device);
        adapter_events(g);
        WS_HIP_CHECK(hipEventRecord(g->tev[0], g->stream));
        g->diag_pending = true;
        materialize_diag(g);
        WS_HIP_CHECK(hipEventRecord(g->tev[1], g->stream));
        WS_HIP_CHECK(hipEventSynchronize(g->tev[1]));
        float t = 0.f;
        WS_HIP_CHECK(hipEventElapsedTime(&t, g->tev[0], g->tev[1]));
        if (ms) *ms = t;
    });
}

// ---- raw kernel ABI ----
int ws_launch_shallow_water_kernel(const void* d_u, const void* d_v, const void* d_h, void* d_u_out, void* d_v_out,
                                   void* d_h_out, int32_t width, int32_t height, int64_t pitch, double dt,
                                   double gravity, double dx, double dy, double coriolis_f, int32_t dtype,
                                   void* stream) {
    return guarded([&] {
        require(d_u && d_v && d_h && d_u_out && d_v_out && d_h_out, WS_ERR_INVALID, "null device pointer");
        require(width > 0 && height > 0 && pitch >= width, WS_ERR_INVALID, "bad dimensions");
        require(dx > 0 && dy > 0, WS_ERR_INVALID, "Grid spacing must be positive");
        ws::Geom g{};
        g.W = width; g.H = height; g.L = 1; g.pitch = pitch; g.lstride = pitch * height;
        g.top_clamp = 1; g.bot_clamp = 1; g.halo = 0;
        auto body = [&](auto tag) {
            using T = decltype(tag);
            ws::StageArgs<T> a{};
            a.in_u = (const T*)d_u; a.in_v = (const T*)d_v; a.in_h = (const T*)d_h;
            a.base_u = a.in_u; a.base_v = a.in_v; a.base_h = a.in_h;
            a.out_u = (T*)d_u_out; a.out_v = (T*)d_v_out; a.out_h = (T*)d_h_out;
            a.c = (T)dt; a.gravity = (T)gravity; a.coriolis_f = (T)coriolis_f;
            a.sp = make_spacing<T>(to_prec(dx, dtype), to_prec(dy, dtype));
            WS_HIP_CHECK(ws::launch_stage<T>(ws::kAxpy, a, g, (hipStream_t)stream));
        };
        require(dtype == WS_F32 || dtype == WS_F64, WS_ERR_INVALID, "bad dtype");
        if (dtype == WS_F64) body(double{});
        else body(float{});
    });
}

int ws_launch_diagnostics_kernels(const void* d_u, const void* d_v, void* d_vort, void* d_div, int32_t width,
                                  int32_t height, int64_t pitch, double dx, double dy, int32_t dtype, void* stream) {
    return guarded([&] {
        require(d_u && d_v && d_vort && d_div, WS_ERR_INVALID, "null device pointer");
        require(width > 0 && height > 0 && pitch >= width, WS_ERR_INVALID, "bad dimensions");
        require(dx > 0 && dy > 0, WS_ERR_INVALID, "Grid spacing must be positive");
        require(dtype == WS_F32 || dtype == WS_F64, WS_ERR_INVALID, "bad dtype");
        ws::Geom g{};
        g.W = width; g.H = height; g.L = 1; g.pitch = pitch; g.lstride = pitch * height;
        g.top_clamp = 1; g.bot_clamp = 1; g.halo = 0;
        if (dtype == WS_F64)
            WS_HIP_CHECK(ws::launch_diagnostics<double>((const double*)d_u, (const double*)d_v, (double*)d_vort,
                                                        (double*)d_div, make_spacing<double>(dx, dy), g,
                                                        (hipStream_t)stream));
        else
            WS_HIP_CHECK(ws::launch_diagnostics<float>((const float*)d_u, (const float*)d_v, (float*)d_vort,
                                                       (float*)d_div, make_spacing<float>((float)dx, (float)dy), g,
                                                       (hipStream_t)stream));
    });
}





int ws_sim_set_kernel_timing(ws_sim_t* s, int32_t enable) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        set_device(s->device);
        s->timer.enable(enable != 0);
        s->timer.reset();
        if (enable > 1) s->timer.reserve((size_t)enable);
    });
}

int ws_sim_kernel_timing(const ws_sim_t* s, int32_t kind, int64_t* launches, double* total_ms,
                         double* bytes_per_launch) {
    return guarded([&] {
        require(s != nullptr && kind >= 0 && kind < ws::KernelTimer::kKinds, WS_ERR_INVALID, "bad argument");
        const auto& st = s->timer.stat(kind);
        if (launches) *launches = st.launches;
        if (total_ms) *total_ms = st.total_ms;
        if (bytes_per_launch) *bytes_per_launch = st.bytes_per_launch;
    });
}

int ws_sim_fused_variant(const ws_sim_t* s, int32_t* kernel, int32_t* seg_rows, int32_t* out_cols) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        const bool fused = use_fused(s);
        if (kernel) *kernel = fused ? s->kernel : -1;
        if (seg_rows) *seg_rows = fused ? s->seg_rows(fused_stages(s)) : 0;
        if (out_cols) *out_cols = fused ? s->out_w(fused_stages(s) * s->launch_tb()) : 0;
    });
}

int ws_sim_kernel_occupancy(const ws_sim_t* s, int32_t* waves_per_simd) {
    return guarded([&] {
        require(s != nullptr && waves_per_simd != nullptr, WS_ERR_INVALID, "null pointer");
        set_device(s->device);
        *waves_per_simd = s->dtype == WS_F64 ? fused_waves_per_simd<double>(s) : fused_waves_per_simd<float>(s);
    });
}

int ws_sim_cfl(ws_sim_t* s, double* cfl, double* per_level, int32_t nlevels, double* ms) {
    return guarded([&] {
        require(s != nullptr && cfl != nullptr, WS_ERR_INVALID, "null pointer");
        set_device(s->device);
        const ws_grid* c = s->slot[s->cur];
        const ws::Geom g = c->geom();
        require(per_level == nullptr || nlevels >= g.L, WS_ERR_INVALID, "per_level needs num_levels entries");
        const int64_t need = (int64_t)g.L * (ws::cfl_partials(g) + 1);
        if (s->cfl_scratch_n < need) {
            if (s->cfl_scratch) WS_HIP_CHECK(hipFree(s->cfl_scratch));
            s->cfl_scratch = nullptr;
            s->cfl_scratch_n = 0;
            WS_HIP_CHECK(hipMalloc(&s->cfl_scratch, need * sizeof(uint64_t)));
            s->cfl_scratch_n = need;
        }
        uint64_t* out = s->cfl_scratch;
        uint64_t* partial = s->cfl_scratch + g.L;
        WS_HIP_CHECK(hipEventRecord(s->ev0, s->stream));
        auto go = [&](auto tag) {
            using T = decltype(tag);
            const T dt = (T)s->dt;
            WS_HIP_CHECK(ws::launch_cfl<T>((const T*)c->f[WS_FIELD_U], (const T*)c->f[WS_FIELD_V],
                                           (const T*)c->f[WS_FIELD_H], g, (T)s->cfg.gravity, dt / (T)c->dx,
                                           dt / (T)c->dy, partial, out, s->stream));
        };
        if (s->dtype == WS_F64) go(double{});
        else go(float{});
        WS_HIP_CHECK(hipEventRecord(s->ev1, s->stream));
        // slab decomposition: the per-level maxima over every rank, on the device (RCCL)
        if (s->comm) s->comm->allreduce_max_u64_device(out, g.L, s->stream);
        std::vector<uint64_t> bits(g.L);
        WS_HIP_CHECK(hipMemcpyAsync(bits.data(), out, g.L * sizeof(uint64_t), hipMemcpyDeviceToHost, s->stream));
        WS_HIP_CHECK(hipStreamSynchronize(s->stream));
        uint64_t m = 0;
        for (int l = 0; l < g.L; ++l) {
            m = std::max(m, bits[l]);
            if (per_level) std::memcpy(&per_level[l], &bits[l], sizeof(double));
        }
        std::memcpy(cfl, &m, sizeof(double));
        if (ms) {
            float t = 0.f;
            WS_HIP_CHECK(hipEventElapsedTime(&t, s->ev0, s->ev1));
            *ms = t;
        }
    });
}

int ws_sim_steps_per_launch(const ws_sim_t* s, int32_t* steps) {
    return guarded([&] {
        require(s != nullptr && steps != nullptr, WS_ERR_INVALID, "null pointer");
        *steps = use_fused(s) ? s->launch_tb() : 1;
    });
}


int ws_sim_set_numerics(ws_sim_t* s, int32_t mode) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        require(mode == WS_NUMERICS_EXACT || mode == WS_NUMERICS_FAST, WS_ERR_INVALID,
                "numerics must be WS_NUMERICS_EXACT or WS_NUMERICS_FAST");
        if (mode != s->numerics && s->tune_free()) s->tuned = env_int("WS_AUTOTUNE", 1) == 0;  // re-rank
        s->numerics = mode;
    });
}

int ws_sim_get_numerics(const ws_sim_t* s, int32_t* mode) {
    return guarded([&] {
        require(s && mode, WS_ERR_INVALID, "null pointer");
        *mode = s->numerics;
    });
}




int ws_sim_pin_variant(ws_sim_t* s, int32_t kernel, int32_t steps_per_launch, int32_t seg_rows, int32_t align) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        require(kernel == -1 || kernel == kKernLds || ws::fused_is_dppy(kernel), WS_ERR_INVALID,
                "kernel must be -1, WS_KERNEL_LDS, WS_KERNEL_DPPY, WS_KERNEL_X2Y, WS_KERNEL_PC or WS_KERNEL_PC2");
        require(steps_per_launch == -1 || steps_per_launch == 1 || steps_per_launch == 2 || steps_per_launch == 4 ||
                    steps_per_launch == 8,
                WS_ERR_INVALID, "steps_per_launch must be -1, 1, 2, 4 or 8");
        require(seg_rows == -1 || seg_rows > 0 || (chain_rounds(seg_rows) > 0 && chain_rounds(seg_rows) <= kMaxChainRounds),
                WS_ERR_INVALID, "seg_rows must be -1, positive, or -2 .. -9 (chain schedule of 1 .. 8 rounds)");
        require(align == -1 || align == 0 || align == 1, WS_ERR_INVALID, "align must be -1, 0 or 1");
        const int k = kernel != -1 ? kernel : s->kernel_fixed ? s->kernel : -1;
        const int tb = steps_per_launch != -1 ? steps_per_launch : s->tb_fixed ? s->tb : -1;
        require(!(k != -1 && ws::fused_split(k) && tb == 1), WS_ERR_INVALID,
                "the split variants (WS_KERNEL_PC, WS_KERNEL_PC2) advance two steps per launch: "
                "steps_per_launch must be 2 or -1");
        require(!(k == kKernLds && tb > 1), WS_ERR_INVALID, "WS_KERNEL_LDS advances one step per launch");
        if (kernel != -1) { s->kernel = kernel; s->kernel_fixed = true; }
        if (steps_per_launch != -1) { s->tb = steps_per_launch; s->tb_fixed = true; }
        else if (k != -1 && ws::fused_split(k)) s->tb = 2;  // the only choice left for a split kernel
        if (seg_rows != -1) { s->seg_override = seg_rows; s->seg_fixed = true; }
        if (align != -1) { s->align = align != 0; s->align_fixed = true; }
        // re-rank what is left free, restricted to the pinned parts
        s->tuned = !s->tune_free() || env_int("WS_AUTOTUNE", 1) == 0;
    });
}

}  // extern "C"

namespace ws {
int abi_guarded(const std::function<void()>& f) { return wsr::guarded(f); }
void abi_set_device(int device) { wsr::set_device(device); }
}  // namespace ws
