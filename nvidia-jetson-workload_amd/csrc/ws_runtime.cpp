// Host runtime of libws_hip.so: the C ABI declared in include/ws_hip.h.
//
// Owns device-resident grids (SoA, one allocation per field, rows padded to a 64-element
// pitch, kHalo spare rows above/below each level for slab halos) and the time stepper that
// replaces WeatherSimulation::step/run (reference src/weather-sim/cpp/src/
// weather_simulation.cpp:68-158). Fields leave the device only through ws_grid_get_field.
#include "ws_hip.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "ws_abi.h"
#include "ws_comm.h"
#include "ws_fused.h"
#include "ws_halo.h"
#include "ws_reduce.h"
#include "ws_ic.h"
#include "ws_internal.h"
#include "ws_timer.h"

namespace {

thread_local std::string g_last_error;

struct WsError : std::runtime_error {
    int code;
    WsError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define WS_HIP_CHECK(expr)                                                                                \
    do {                                                                                                  \
        hipError_t e_ = (expr);                                                                           \
        if (e_ != hipSuccess)                                                                             \
            throw WsError(WS_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));              \
    } while (0)

template <typename F>
int guarded(F&& f) {
    try {
        f();
        return WS_OK;
    } catch (const WsError& e) {
        g_last_error = e.what();
        return e.code;
    } catch (const ws::AbiError& e) {
        g_last_error = e.what();
        return e.code;
    } catch (const ws::CommError& e) {
        g_last_error = e.what();
        return WS_ERR_COMM;
    } catch (const std::bad_alloc&) {
        g_last_error = "out of host memory";
        return WS_ERR_DEVICE;
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return WS_ERR_INVALID;
    }
}

void require(bool cond, int code, const char* msg) {
    if (!cond) throw WsError(code, msg);
}

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

size_t elem_size(int dtype) { return dtype == WS_F64 ? 8 : 4; }

bool is_pow2(double v) {
    if (!(v > 0) || !std::isfinite(v)) return false;
    int e;
    return std::frexp(v, &e) == 0.5;
}

// value rounded to the simulation precision (the reference stores scalar_t)
double to_prec(double v, int dtype) { return dtype == WS_F64 ? v : (double)(float)v; }

}  // namespace

struct ws_grid {
    int32_t W = 0, H = 0, L = 1, dtype = WS_F32, device = 0;
    int64_t pitch = 0, lstride = 0;
    double dx = 1.0, dy = 1.0;  // already rounded to the grid precision
    void* alloc[8] = {};
    void* f[8] = {};            // row 0 of level 0
    unsigned nfields = 8;
    bool diag_pending = false;
    bool owned = false;         // owned by a ws_sim
    int32_t top_clamp = 1, bot_clamp = 1;
    int32_t row0 = 0, gH = 0;   // slab: first global row, global height (ICs use global coordinates)
    hipStream_t stream = nullptr;

    ws::Geom geom() const {
        ws::Geom g;
        g.W = W; g.H = H; g.L = L; g.pitch = pitch; g.lstride = lstride;
        g.top_clamp = top_clamp; g.bot_clamp = bot_clamp;
        g.halo = ws::kHalo;
        return g;
    }
    size_t bytes_per_field() const { return (size_t)L * lstride * elem_size(dtype); }
};

namespace {

int64_t env_int(const char* name, int64_t dflt) {
    const char* e = std::getenv(name);
    return e ? std::atoll(e) : dflt;
}

// row pitch (elements) and level stride of a W x H grid: rows padded to 64 elements, kHalo
// halo rows above and below every level (the layout ws_slab_exchange_plan reports)
int64_t layout_pitch(int64_t W) { return (W + 63) / 64 * 64 + env_int("WS_PITCH_PAD", 0) / 64 * 64; }
int64_t layout_lstride(int64_t H, int64_t pitch) { return (H + 2 * ws::kHalo) * pitch; }

void grid_alloc(ws_grid* g, unsigned nfields) {
    g->pitch = layout_pitch(g->W);
    g->lstride = layout_lstride(g->H, g->pitch);
    g->nfields = nfields;
    const size_t es = elem_size(g->dtype);
    const size_t stagger = (size_t)env_int("WS_FIELD_STAGGER", 0) / 256 * 256;  // bytes, field i offset by i*stagger
    for (unsigned i = 0; i < nfields; ++i) {
        WS_HIP_CHECK(hipMalloc(&g->alloc[i], g->bytes_per_field() + i * stagger));
        // on the grid's own stream: a legacy-stream hipMemset is not ordered with the
        // non-blocking streams the kernels run on, and returns before it completes -- it raced
        // with the first launches writing a freshly allocated overlap grid (slab groups)
        WS_HIP_CHECK(hipMemsetAsync(g->alloc[i], 0, g->bytes_per_field() + i * stagger, g->stream));
        g->f[i] = (char*)g->alloc[i] + i * stagger + (size_t)ws::kHalo * g->pitch * es;
    }
}

void grid_free(ws_grid* g) {
    for (auto& a : g->alloc)
        if (a) { (void)hipFree(a); a = nullptr; }
}

template <typename T>
ws::Spacing<T> make_spacing(double dx, double dy) {
    ws::Spacing<T> s;
    s.two_dx = T(2.0f) * (T)dx;
    s.two_dy = T(2.0f) * (T)dy;
    s.pow2x = is_pow2((double)s.two_dx);
    s.pow2y = is_pow2((double)s.two_dy);
    s.inv2dx = s.pow2x ? T(1) / s.two_dx : T(0);
    s.inv2dy = s.pow2y ? T(1) / s.two_dy : T(0);
    return s;
}

template <typename T>
void grid_reset_t(ws_grid* g) {
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
void grid_diag_t(ws_grid* g) {
    WS_HIP_CHECK(ws::launch_diagnostics<T>((const T*)g->f[WS_FIELD_U], (const T*)g->f[WS_FIELD_V],
                                           (T*)g->f[WS_FIELD_VORTICITY], (T*)g->f[WS_FIELD_DIVERGENCE],
                                           make_spacing<T>(g->dx, g->dy), g->geom(), g->stream));
}

// Run pending diagnostics now (lazy vorticity / divergence).
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
void convert(Dst* d, const Src* s, size_t n) {
    for (size_t i = 0; i < n; ++i) d[i] = static_cast<Dst>(s[i]);
}

}  // namespace

// ------------------------------------------------------------------------------------
// simulation
// ------------------------------------------------------------------------------------
enum FusedKernel : int { kKernLds = ws::kFusedLds, kKernDppLdsY = ws::kFusedDppLdsY, kKernX2Y = ws::kFusedX2Y };

struct ws_sim {
    ws_config_t cfg{};
    int32_t dtype = WS_F32;
    int32_t device = 0;
    ws_grid* slot[2] = {nullptr, nullptr};
    int cur = 0;
    ws_grid* tmpA = nullptr;  // RK stage state ping-pong (u, v, h only)
    ws_grid* tmpB = nullptr;
    ws_grid* K2 = nullptr;    // RK4 stage-2 / stage-3 tendencies
    ws_grid* K3 = nullptr;
    double time = 0.0;        // rounded to the precision after every add
    double dt = 0.01;
    int32_t step = 0;
    ws_metrics_t metrics{};
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // PE: the T / P update runs on a second stream beside the stencil kernels (independent
    // fields, see run_steps); joined with the main stream at the start and end of every run
    hipStream_t aux = nullptr;
    hipEvent_t aux_in = nullptr, aux_out = nullptr;
    bool aux_active = false;
    double last_ms = 0.0;
    int64_t last_launches = 0;
    ws::KernelTimer timer;
    int32_t rank = 0, nranks = 1;                       // y-slab position (1 = whole domain)
    bool own_stream = true;
    bool in_group = false;                              // a slab of a ws_group (local halo transport)
    bool fused = true;       // one fused kernel per step (WS_FUSED=0: one kernel per RK stage)
    int kernel = kKernX2Y;    // fused kernel variant (WS_KERNEL=x2y|dppy|lds fixes it)
    int32_t seg_override = 0; // WS_SEG_ROWS (fixes it)
    bool align = false;       // strip output windows on whole 128-byte lines (WS_ALIGN fixes it)
    bool kernel_fixed = false, seg_fixed = false, align_fixed = false;
    // time steps per fused launch (temporal blocking; the dppy kernel only): 1, or 2 = two
    // steps per launch inside run(k) (WS_TB=1|2 fixes it, else the autotuner picks)
    int32_t tb = 1;
    bool tb_fixed = false;
    int numerics = WS_NUMERICS_EXACT;  // fused kernels: exact or fast numerics (ws_fused.h)
    bool tuned = false;       // autotune done (first run; WS_AUTOTUNE=0 disables)
    int32_t block = 1;        // slab: steps per halo exchange (deep halo), see step_rows
    int32_t block_pos = 0;    // position in the current block (0 = exchange first)
    int32_t want_blocks_override = 0;  // WS_WANT_BLOCKS
    // slab overlap schedule (overlap_block): a block's edge bands run on `edge`, the halo
    // exchange follows them there, the interior runs meanwhile on `stream`
    bool overlap = false;
    hipStream_t edge = nullptr;
    hipEvent_t ev_edge = nullptr, ev_join = nullptr;
    ws_grid* ov[4] = {};      // interior ping-pong (0, 1), edge-band ping-pong (2, 3); u, v, h
    double emu_xfer_us = -1.0;  // no communicator (measurement aid): WS_EMU_XFER_US, see slab_exchange
    // slab decomposition
    ws::SlabComm* comm = nullptr;
    ws::HaloStaging* staging = nullptr;  // slab of a group: its halo messages (group_exchange)
    uint64_t* cfl_scratch = nullptr;     // ws_sim_cfl: per-level partial maxima + results (device)
    int64_t cfl_scratch_n = 0;
    int32_t row0 = 0;

    // cone = stages per launch (NST x steps per launch): the strip margins
    int out_w(int cone) const { return ws::fused_out_w(kernel, cone, (int)elem_size(dtype), align); }
    int64_t strips(int cone) const { return (slot[0]->W + out_w(cone) - 1) / out_w(cone); }
    // steps per launch the tuned configuration asks for (1 unless dppy with tb = 2)
    int launch_tb() const { return kernel == kKernLds ? 1 : tb; }
    // segment rows giving about want_blocks workgroups (at least min_rows rows; the march
    // length rows + 2 NST a multiple of the unroll)
    int32_t seg_for_blocks(int nst, int64_t want_blocks, int64_t min_rows) const {
        const ws_grid* g = slot[0];
        const int64_t per_seg = strips(nst * launch_tb()) * g->L;
        const int64_t want_segs = std::max<int64_t>(1, (want_blocks + per_seg - 1) / per_seg);
        int64_t rows = (g->H + want_segs - 1) / want_segs;
        rows = std::max<int64_t>(rows, min_rows);
        const int cone = nst * launch_tb();
        rows = (rows + 2 * cone + 7) / 8 * 8 - 2 * cone;
        return (int32_t)std::max<int64_t>(1, std::min<int64_t>(rows, g->H));
    }
    // Rows per fused-kernel segment: enough workgroups to fill the chip (64-lane waves of
    // 64 / 128 columns vs 256-lane workgroups), segments long enough that the 2*NST
    // warm-up rows stay a small overhead. The autotuner also tries other counts.
    int32_t seg_rows(int nst) const {
        if (seg_override > 0) return seg_override;
        int64_t want_blocks = kernel == kKernX2Y ? 2048 : kernel == kKernDppLdsY ? 4096 : 512;
        if (want_blocks_override > 0) want_blocks = want_blocks_override;
        return seg_for_blocks(nst, want_blocks, 24 * nst);
    }
};

namespace {

// Integrator actually executed (weather_simulation.cpp:122-142, :334-338, :457-471).
int effective_method(const ws_config_t& c) {
    switch (c.integration_method) {
        case WS_RK2: return WS_RK2;
        case WS_RK4: return c.model == WS_MODEL_SHALLOW_WATER ? WS_RK4 : WS_RK2;
        default: return WS_EULER;
    }
}

template <typename T>
ws::StageArgs<T> stage_args(const ws_grid* in, const ws_grid* base, ws_grid* out, T c, const ws_sim* s) {
    ws::StageArgs<T> a{};
    a.in_u = (const T*)in->f[0]; a.in_v = (const T*)in->f[1]; a.in_h = (const T*)in->f[2];
    a.base_u = (const T*)base->f[0]; a.base_v = (const T*)base->f[1]; a.base_h = (const T*)base->f[2];
    a.out_u = (T*)out->f[0]; a.out_v = (T*)out->f[1]; a.out_h = (T*)out->f[2];
    a.c = c;
    a.gravity = (T)s->cfg.gravity;
    a.coriolis_f = (T)s->cfg.coriolis_f;
    a.sp = make_spacing<T>(in->dx, in->dy);
    return a;
}

template <typename T>
void launch(ws_sim* s, int mode, const ws::StageArgs<T>& a, const ws_grid* in, int kind, int words) {
    if (s->comm) s->comm->exchange(in->f, 3, (int)sizeof(T), in->geom(), 1, s->stream);
    const ws::Geom g = s->slot[0]->geom();
    s->timer.begin(kind, (double)words * sizeof(T) * g.W * g.H * g.L, s->stream);
    WS_HIP_CHECK(ws::launch_stage<T>(mode, a, g, s->stream));
    s->timer.end(s->stream);
    ++s->last_launches;
}

int fused_stages(const ws_sim* s) {
    const int m = effective_method(s->cfg);
    return m == WS_EULER ? 1 : m == WS_RK2 ? 2 : 4;
}

bool use_fused(const ws_sim* s) { return s->fused && s->slot[0]->W >= 2; }

void slab_exchange(ws_sim* s, ws_grid* g, int nfields, int depth, hipStream_t st);

// Output rows of a fused launch: [y0, y1) (empty if y1 <= y0).
struct RowRange {
    int y0, y1;
    int rows() const { return y1 > y0 ? y1 - y0 : 0; }
};

// Slab blocks. A slab advances `block` steps per halo exchange: the exchange moves
// block * NST rows of u, v, h from each neighbour, and step j = 0 .. block-1 of the block
// computes its rows extended by (block - 1 - j) * NST into the halo on each non-global
// side, so every step's dependency cone is covered by rows already on the device and the
// last step of the block ends on exactly the owned rows. The extra work is
// (block - 1) * NST * (block) rows per side per block; the saving is block - 1 exchanges and
// every cross-stream synchronisation: the exchange is stream-ordered on the compute
// stream (measured on MI355X: two cross-stream event waits per step cost more than an
// overlapped edge launch saves).
RowRange step_rows(const ws_sim* s, int nst, int nsteps = 1) {
    const ws_grid* g = s->slot[0];
    // a launch of nsteps steps ends on the rows of its last step, block position + nsteps - 1
    const int e = (s->block - nsteps - s->block_pos) * nst;
    return {g->top_clamp ? 0 : -e, g->bot_clamp ? g->H : g->H + e};
}

// Launch the fused step kernel over the output rows A U B (segments of seg_rows rows).
template <typename T>
void fused_launch(ws_sim* s, int nst, int nsteps, RowRange A, RowRange B, int seg_rows, hipStream_t st = nullptr,
                  ws_grid* in = nullptr, ws_grid* out = nullptr) {
    if (!st) st = s->stream;
    const int nA = (A.rows() + seg_rows - 1) / seg_rows, nB = (B.rows() + seg_rows - 1) / seg_rows;
    if (nA + nB <= 0) return;
    ws_grid* c = in ? in : s->slot[s->cur];    // (the autotuner times launches on other grids)
    ws_grid* n = out ? out : s->slot[1 - s->cur];
    const T dt = (T)s->dt;
    ws::FusedArgs<T> a{};
    a.in_u = (const T*)c->f[0]; a.in_v = (const T*)c->f[1]; a.in_h = (const T*)c->f[2];
    a.out_u = (T*)n->f[0]; a.out_v = (T*)n->f[1]; a.out_h = (T*)n->f[2];
    a.c_half = T(0.5f) * dt;  // `0.5f * dt_` (weather_simulation.cpp:249)
    a.c_dt = dt;
    a.c_dt6 = dt / T(6.0f);   // `dt_ / 6.0f` (:438)
    a.gravity = (T)s->cfg.gravity;
    a.coriolis_f = (T)s->cfg.coriolis_f;
    a.sp1 = make_spacing<T>(c->dx, c->dy);
    a.sp2 = make_spacing<T>(to_prec(s->cfg.dx, s->dtype), to_prec(s->cfg.dy, s->dtype));
    a.out_w = s->out_w(nst * nsteps);
    a.seg_rows = seg_rows;
    a.ga_y0 = A.y0; a.ga_y1 = A.y1; a.ga_n = nA;
    a.gb_y0 = B.y0; a.gb_y1 = B.y1;
    a.seg_n = nA + nB;
    // numerics (ws_fused.h): exact = the reference's evaluation order, bit-identical;
    // fast = re-associated with FMAs (isotropic spacing; otherwise exact)
    if (s->numerics == WS_NUMERICS_FAST) ws::prepare_fast(a);
    else a.sp_mode = ws::exact_sp_mode(a);
    const ws::Geom g = c->geom();
    if (nsteps > 1 && s->kernel == kKernLds) throw WsError(WS_ERR_INVALID, "multi-step launch needs dppy or x2y");
    if (s->kernel == kKernLds) WS_HIP_CHECK(ws::launch_fused_step<T>(nst, a, g, st));
    else WS_HIP_CHECK(ws::launch_fused_step_dppy<T>(s->kernel, nst, nsteps, a, g, st));
    ++s->last_launches;
}

// Phase 1 of a step: everything that does not need this step's halo rows.
//  * single domain: the whole step (fused or stage kernels);
//  * slab, fused: start the RCCL halo exchange on the comm stream (after the previous
//    step's output is complete) and run the interior segments meanwhile.
template <typename T>
void step_begin(ws_sim* s, int nsteps = 1) {
    ws_grid* c = s->slot[s->cur];
    ws_grid* n = s->slot[1 - s->cur];
    const T dt = (T)s->dt;
    const T half = T(0.5f) * dt;
    const int method = effective_method(s->cfg);
    const ws::Geom g = c->geom();
    if (use_fused(s)) {
        const int nst = fused_stages(s);
        // algorithmic bytes of the launch: 6 words per cell-update (read u, v, h + write u, v,
        // h: the compulsory traffic of one step) x the cell-updates it performs
        s->timer.begin(0, 6.0 * sizeof(T) * g.W * g.H * g.L * nsteps, s->stream);
        // slab: at a block start, the block's halo (group slabs: copied by group_step)
        if (s->block_pos == 0) slab_exchange(s, c, 3, s->block * nst, s->stream);
        fused_launch<T>(s, nst, nsteps, step_rows(s, nst, nsteps), {0, 0}, s->seg_rows(nst));
        return;
    }
    require(nsteps == 1, WS_ERR_INVALID, "multi-step launches need the fused kernels");
    if (method == WS_EULER) {
        launch<T>(s, ws::kAxpy, stage_args<T>(c, c, n, dt, s), c, 0, 6);
    } else if (method == WS_RK2) {
        launch<T>(s, ws::kAxpy, stage_args<T>(c, c, s->tmpA, half, s), c, 0, 6);
        launch<T>(s, ws::kAxpy, stage_args<T>(s->tmpA, c, n, dt, s), s->tmpA, 1, 9);
    } else {
        launch<T>(s, ws::kAxpy, stage_args<T>(c, c, s->tmpA, half, s), c, 0, 6);
        auto a2 = stage_args<T>(s->tmpA, c, s->tmpB, half, s);
        a2.k2_u = (T*)s->K2->f[0]; a2.k2_v = (T*)s->K2->f[1]; a2.k2_h = (T*)s->K2->f[2];
        launch<T>(s, ws::kAxpyStore, a2, s->tmpA, 1, 12);
        auto a3 = stage_args<T>(s->tmpB, c, s->tmpA, dt, s);
        a3.k2_u = (T*)s->K3->f[0]; a3.k2_v = (T*)s->K3->f[1]; a3.k2_h = (T*)s->K3->f[2];
        launch<T>(s, ws::kAxpyStore, a3, s->tmpB, 2, 12);
        auto a4 = stage_args<T>(s->tmpA, c, n, dt / T(6.0f), s);  // `dt_ / 6.0f`
        a4.k2_u = (T*)s->K2->f[0]; a4.k2_v = (T*)s->K2->f[1]; a4.k2_h = (T*)s->K2->f[2];
        a4.k3_u = (const T*)s->K3->f[0]; a4.k3_v = (const T*)s->K3->f[1]; a4.k3_h = (const T*)s->K3->f[2];
        launch<T>(s, ws::kRk4Final, a4, s->tmpA, 3, 15);
    }
}

// Phase 2: the segments that need the halo (after it arrived), the PE T/P update, and the
// grid rotation of the reference (current <-> next shared_ptr swap).
//
// A two-step launch (temporal blocking) reads the current grid and writes u, v, h two steps
// on into the next grid (PE: one T / P pass applies both steps' updates, also into the next
// grid); the reference's rotation after two steps puts the current grid back in place, so
// the storage of those fields is exchanged between the two grids instead of the slots: the
// current grid holds the new state and the other fields are where two rotations leave them.
// (The intermediate state is never materialised: the non-current grid then holds the state
// of two steps back instead of one -- visible only through a grid handle held across run(),
// DESIGN.md deviation D6.)
template <typename T>
void rotate(ws_sim* s, int nsteps);

template <typename T>
void step_end(ws_sim* s, int nsteps = 1) {
    if (use_fused(s)) {
        s->timer.end(s->stream);
        s->block_pos = (s->block_pos + nsteps) % s->block;
    }
    rotate<T>(s, nsteps);
}

// After nsteps steps written into the next grid: the PE T / P update (nsteps updates in one
// pass) and the reference's grid rotation.
template <typename T>
void rotate(ws_sim* s, int nsteps) {
    const T dt = (T)s->dt;
    ws_grid* c = s->slot[s->cur];
    ws_grid* n = s->slot[1 - s->cur];
    const bool pe = s->cfg.model == WS_MODEL_PRIMITIVE_EQUATIONS;
    if (pe) {
        // stale tendency: the tendency grid's T/P keep their reset values 288.15f / 1013.25f
        // (`dt_ * tendency` has the same operands in every cell: one rounding, done here);
        // all nsteps updates in one pass, each rounded as the reference rounds it
        const ws::Geom g = c->geom();
        const T cT = dt * T(288.15f), cP = dt * T(1013.25f);
        WS_HIP_CHECK(ws::launch_affine2<T>((T*)n->f[WS_FIELD_T], (const T*)c->f[WS_FIELD_T], cT,
                                           (T*)n->f[WS_FIELD_P], (const T*)c->f[WS_FIELD_P], cP, g,
                                           s->aux_active ? s->aux : s->stream, nsteps));
        s->last_launches += 1;
    }
    if (nsteps % 2 == 1) {
        s->cur = 1 - s->cur;
    } else {
        // two steps: exchange the storage of the fields written into the next grid (u, v, h
        // and, for PE, T and P), so the current grid holds the new state
        for (int f : {WS_FIELD_U, WS_FIELD_V, WS_FIELD_H, WS_FIELD_T, WS_FIELD_P}) {
            if (!pe && (f == WS_FIELD_T || f == WS_FIELD_P)) continue;
            std::swap(c->alloc[f], n->alloc[f]);
            std::swap(c->f[f], n->f[f]);
        }
        n->diag_pending = true;
    }
    s->slot[s->cur]->diag_pending = true;  // step() ends with calculateDiagnostics (:149)
}

// Steps the next launch advances, of `remaining`: 2 when the tuned configuration launches
// two steps at once, the slab block has room for both, and both steps see the config's
// spacing (the kernel's later stages use it); else 1.
// The halo exchange of a slab: RCCL (ws_comm.cpp), or -- a slab created without a
// communicator, the measurement aid of ws_sim_create_slab -- the pack / unpack kernels
// around a WS_EMU_XFER_US wall-clock wait in place of the transfer (the halo rows then hold
// the slab's own edge rows: timing only).
void slab_exchange(ws_sim* s, ws_grid* g, int nfields, int depth, hipStream_t st) {
    if (s->comm) {
        s->comm->exchange(g->f, nfields, (int)elem_size(s->dtype), g->geom(), depth, st);
        return;
    }
    if (s->nranks < 2 || s->emu_xfer_us < 0 || s->in_group) return;
    const ws::HaloPlan plan = ws::make_halo_plan(g->geom(), (int)elem_size(s->dtype), s->rank, s->nranks, nfields, depth);
    if (ws::halo_direct(plan)) {  // direct sends (ws_comm.cpp): the transfer only
        WS_HIP_CHECK(ws::emulated_transfer(s->emu_xfer_us, st));
        return;
    }
    if (!s->staging) s->staging = new ws::HaloStaging;
    s->staging->ensure(plan.msg_bytes());
    ws::HaloFields hf{};
    for (int f = 0; f < nfields; ++f) hf.f[f] = (char*)g->f[f];
    for (int side = 0; side < 2; ++side)
        if (plan.has[side]) WS_HIP_CHECK(ws::halo_pack(plan, hf, side, s->staging->send[side], st));
    WS_HIP_CHECK(ws::emulated_transfer(s->emu_xfer_us, st));
    for (int side = 0; side < 2; ++side)
        if (plan.has[side]) WS_HIP_CHECK(ws::halo_unpack(plan, hf, side, s->staging->send[side], st));
}

bool config_spacing(const ws_sim* s) {
    const double dx = to_prec(s->cfg.dx, s->dtype), dy = to_prec(s->cfg.dy, s->dtype);
    for (const ws_grid* g : {s->slot[0], s->slot[1]})
        if (g->dx != dx || g->dy != dy) return false;
    return true;
}

int launch_steps(const ws_sim* s, int remaining) {
    if (remaining < 2 || !use_fused(s) || s->launch_tb() < 2) return 1;
    if (s->nranks > 1 && s->block_pos + 2 > s->block) return 1;  // a slab's block (one domain: no blocks)
    return config_spacing(s) ? 2 : 1;
}

// One time step on the stream (no host synchronisation).
template <typename T>
void enqueue_steps(ws_sim* s, int nsteps) {
    step_begin<T>(s, nsteps);
    step_end<T>(s, nsteps);
}

// ------------------------------------------------------------------------------------
// Slab overlap schedule (north_star: the halo exchange overlapped with interior compute on a
// second HIP stream). A block of `steps` steps (one halo exchange, depth D = steps x NST
// rows, as in the stream-ordered schedule above) is split by rows:
//   * edge bands, on the slab's `edge` stream: the rows within 2D of a non-global side,
//     advanced the whole block through their own ping-pong grids (ov[2], ov[3]); launch j
//     (cumulative cone C_j) computes rows [C_j - D, 2D - C_j) at the top and
//     [H - 2D + C_j, H + D - C_j) at the bottom, so the last launch writes exactly rows
//     [0, D) and [H - D, H) of the next grid -- the rows the neighbours need. The exchange of
//     the next block's halo follows on the same stream;
//   * interior, on the compute stream meanwhile: launch j computes rows [C_j, H - C_j)
//     through ov[0], ov[1]; it reads only owned rows (never the halo), and its last launch
//     writes rows [D, H - D) of the next grid.
// Every launch reads exactly the rows its predecessor in the same band wrote (the
// dependency cone shrinks by the launch's NST x steps per side), so both parts are
// bit-identical to the stream-ordered schedule. Two cross-stream waits per block: the edge
// launches of block k read rows [D, 2D) that the interior of block k-1 wrote (ev_join), and
// the interior of block k reads rows [0, D) that the edges of block k-1 wrote (ev_edge). The
// exchange itself is waited on only by the next block's edges (stream order on `edge`).
// ------------------------------------------------------------------------------------

// steps per launch within a block (2 while the tuned configuration launches two at once)
std::vector<int> block_launches(const ws_sim* s, int steps) {
    const bool two = use_fused(s) && s->launch_tb() >= 2 && config_spacing(s);
    std::vector<int> n;
    for (int left = steps; left > 0;) {
        const int k = two && left >= 2 ? 2 : 1;
        n.push_back(k);
        left -= k;
    }
    return n;
}

// launch j's interior rows and edge-band rows (two ranges; merged into A when they touch)
struct BandRows {
    RowRange interior, A, B;
};

BandRows band_rows(const ws_grid* g, int C, int D) {
    const int H = g->H;
    const int lo = g->top_clamp ? 0 : C - D, hi = g->bot_clamp ? H : H + D - C;
    BandRows r{{g->top_clamp ? 0 : C, g->bot_clamp ? H : H - C}, {0, 0}, {0, 0}};
    RowRange top{0, 0}, bot{0, 0};
    if (!g->top_clamp) top = {lo, std::min(hi, 2 * D - C)};
    if (!g->bot_clamp) bot = {std::max(lo, H - 2 * D + C), hi};
    if (top.rows() > 0 && bot.rows() > 0 && top.y1 >= bot.y0) {
        r.A = {top.y0, bot.y1};
    } else {
        r.A = top.rows() > 0 ? top : bot;
        r.B = top.rows() > 0 ? bot : RowRange{0, 0};
    }
    return r;
}

// the overlap grids (allocated on first use; same layout and slab flags as the slots)
void ensure_overlap_grids(ws_sim* s) {
    if (!s->edge) {
        // (a high-priority edge stream measured no different: tools/rank_timing.py)
        WS_HIP_CHECK(hipStreamCreateWithFlags(&s->edge, hipStreamNonBlocking));
        WS_HIP_CHECK(hipEventCreateWithFlags(&s->ev_edge, hipEventDisableTiming));
        WS_HIP_CHECK(hipEventCreateWithFlags(&s->ev_join, hipEventDisableTiming));
    }
    const ws_grid* c = s->slot[0];
    for (auto& g : s->ov) {
        if (g) continue;
        g = new_grid(c->W, c->H, c->L, s->dtype, s->device, 3, s->stream);
        g->owned = true;
        g->dx = c->dx; g->dy = c->dy;
        g->top_clamp = c->top_clamp; g->bot_clamp = c->bot_clamp;
        g->row0 = c->row0; g->gH = c->gH;
    }
}

// Phase 1 (compute stream): join the previous block and hand the edge stream its start.
void overlap_begin(ws_sim* s, bool first) {
    if (!first) WS_HIP_CHECK(hipStreamWaitEvent(s->stream, s->ev_edge, 0));  // rows [0, D) of block k-1
    WS_HIP_CHECK(hipEventRecord(s->ev_join, s->stream));
    WS_HIP_CHECK(hipStreamWaitEvent(s->edge, s->ev_join, 0));
}

// Phase 2 (edge stream): the edge bands of the block; ev_edge marks them done.
template <typename T>
void overlap_edges(ws_sim* s, int steps) {
    const int nst = fused_stages(s), D = steps * nst;
    const std::vector<int> n = block_launches(s, steps);
    ws_grid* in = s->slot[s->cur];
    int C = 0;
    for (size_t j = 0; j < n.size(); ++j) {
        C += n[j] * nst;
        ws_grid* out = j + 1 == n.size() ? s->slot[1 - s->cur] : s->ov[2 + j % 2];
        const BandRows r = band_rows(in, C, D);
        // the tuned segment rows (one segment per band -- fewer warm-up rows, longer marches
        // -- measured no faster: the edges are on the critical path at 8 slabs)
        fused_launch<T>(s, nst, n[j], r.A, r.B, s->seg_rows(nst), s->edge, in, out);
        in = out;
    }
    WS_HIP_CHECK(hipEventRecord(s->ev_edge, s->edge));
}

// Phase 3 (compute stream): the interior of the block, then the PE T / P update and rotation.
template <typename T>
void overlap_interior(ws_sim* s, int steps) {
    const int nst = fused_stages(s), D = steps * nst;
    const std::vector<int> n = block_launches(s, steps);
    ws_grid* in = s->slot[s->cur];
    const ws::Geom g = in->geom();
    int C = 0;
    for (size_t j = 0; j < n.size(); ++j) {
        C += n[j] * nst;
        ws_grid* out = j + 1 == n.size() ? s->slot[1 - s->cur] : s->ov[j % 2];
        const BandRows r = band_rows(in, C, D);
        s->timer.begin(0, 6.0 * sizeof(T) * g.W * r.interior.rows() * g.L * n[j], s->stream);
        fused_launch<T>(s, nst, n[j], r.interior, {0, 0}, s->seg_rows(nst), s->stream, in, out);
        s->timer.end(s->stream);
        in = out;
    }
    rotate<T>(s, steps);
}

// Whether run() uses the overlap schedule: a slab of the fused path whose grids all have the
// configured spacing (the two-step launches' later stages assume it).
// (A one-rank RCCL slab runs it only when WS_SLAB_OVERLAP=1: no edge bands, no-op exchanges.)
bool overlap_active(const ws_sim* s) {
    return s->overlap && (s->nranks > 1 || s->comm) && use_fused(s) && config_spacing(s);
}

// One overlapped block of a slab with an RCCL communicator.
template <typename T>
void overlap_block(ws_sim* s, int steps, bool first, bool last) {
    const int depth = s->block * fused_stages(s);
    if (first) slab_exchange(s, s->slot[s->cur], 3, depth, s->stream);
    overlap_begin(s, first);
    overlap_edges<T>(s, steps);
    if (!last) slab_exchange(s, s->slot[1 - s->cur], 3, depth, s->edge);  // the next block's halo, behind the edge bands
    overlap_interior<T>(s, steps);
}

template <typename T>
double advance_time(double t, double dt) {
    T tt = (T)t;
    tt += (T)dt;
    return (double)tt;
}

// Decide on the host how many of n steps run(n) takes (weather_simulation.cpp:77-90).
int plan_steps(const ws_sim* s, int n) {
    if (n <= 0) return 0;
    const bool f64 = s->dtype == WS_F64;
    const double max_time = to_prec(s->cfg.max_time, s->dtype);
    double t = s->time;
    int k = 0;
    while (k < n) {
        t = f64 ? advance_time<double>(t, s->dt) : advance_time<float>(t, s->dt);
        ++k;
        if (t >= max_time) break;
    }
    return k;
}

// Pick the fused-kernel variant (and segment length) for this grid by timing each
// candidate on the real fields once, at the first run: all variants produce bit-identical
// results (each is the reference's arithmetic), they differ only in speed, and which is
// fastest depends on precision, integrator, width and level count. A candidate launch
// reads the current state and writes the next-state buffer, which the real step then
// overwrites, so tuning leaves no trace in the results.
template <typename T>
void autotune_time(ws_sim* s) {
    const int nst = fused_stages(s);
    struct Cand {
        int kernel, seg;
        bool align;
        int tb;
        float ms;  // per time step
    };
    std::vector<Cand> cands;
    const int fixed_seg = s->seg_override;
    const int fixed_tb = s->tb;
    // two steps per launch only where a run can use them (slab blocks of >= 2 steps)
    const bool tb2_ok = s->block >= 2 || s->nranks == 1;
    for (int k : {kKernDppLdsY, kKernX2Y, kKernLds})
      for (int tb : {1, 2}) {
        if (tb == 2 && (k == kKernLds || !tb2_ok)) continue;
        if (s->tb_fixed && k != kKernLds && tb != fixed_tb) continue;
        s->tb = tb;
        const int cone = nst * tb;
        for (bool al : {false, true}) {
            if (s->align_fixed && al != s->align) continue;
            s->kernel = k;
            const bool same = ws::fused_out_w(k, cone, (int)elem_size(s->dtype), true) ==
                              ws::fused_out_w(k, cone, (int)elem_size(s->dtype), false);
            if (al && same) continue;  // already aligned
            // aligned windows below 3/4 of the strip waste too much recomputation
            if (al && 4 * ws::fused_out_w(k, cone, (int)elem_size(s->dtype), true) < 3 * ws::fused_strip_cols(k))
                continue;
            const bool save_al = s->align;
            s->align = al;
            if (s->seg_fixed) {
                cands.push_back({k, fixed_seg, al, tb, 0.f});
            } else {
                // the default, and segment lengths giving whole multiples of the chip's wave
                // slots (1024 SIMDs; an LDS workgroup is 4 waves) so no SIMD runs a lone
                // extra wave
                s->seg_override = 0;
                std::vector<int> segs{s->seg_rows(nst)};
                const int wave_per_block = k == kKernLds ? 4 : 1;
                for (int64_t waves : {1024, 2048, 3072, 4096, 6144})
                    segs.push_back(s->seg_for_blocks(nst, waves / wave_per_block, 5 * nst));
                if (k == kKernDppLdsY || k == kKernX2Y)  // more waves per SIMD fit: shorter segments pay
                    for (int64_t waves : {8192, 12288}) segs.push_back(s->seg_for_blocks(nst, waves, 5 * nst));
                std::sort(segs.begin(), segs.end());
                segs.erase(std::unique(segs.begin(), segs.end()), segs.end());
                for (int seg : segs) cands.push_back({k, seg, al, tb, 0.f});
            }
            s->align = save_al;
        }
      }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    WS_HIP_CHECK(hipEventCreate(&e0));
    WS_HIP_CHECK(hipEventCreate(&e1));
    // Launches alternate current -> next and next -> scratch (a u, v, h grid allocated for
    // the tuning only), so every launch but the first reads what the one before it wrote,
    // as in a run: on grids that fit the 256 MB Infinity Cache, re-reading one unchanged
    // input would favour the candidates that read most. Nothing the real step reads changes.
    ws_grid* cur = s->slot[s->cur];
    ws_grid* scratch = new_grid(cur->W, cur->H, cur->L, s->dtype, s->device, 3, s->stream);
    scratch->dx = cur->dx;
    scratch->dy = cur->dy;
    scratch->top_clamp = cur->top_clamp;
    scratch->bot_clamp = cur->bot_clamp;
    // round-robin rounds, best-of per candidate: robust to clock ramp-up and noise
    auto time_cand = [&](Cand& c, int reps) {
        s->kernel = c.kernel;
        s->seg_override = c.seg;
        s->align = c.align;
        s->tb = c.tb;
        const int H = s->slot[0]->H, seg = s->seg_rows(nst);
        WS_HIP_CHECK(hipEventRecord(e0, s->stream));
        for (int i = 0; i < reps; ++i)
            if (i % 2 == 0) fused_launch<T>(s, nst, c.tb, {0, H}, {0, 0}, seg);
            else fused_launch<T>(s, nst, c.tb, {0, H}, {0, 0}, seg, nullptr, s->slot[1 - s->cur], scratch);
        WS_HIP_CHECK(hipEventRecord(e1, s->stream));
        WS_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        WS_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        return ms / reps / c.tb;
    };
    float first = 0.f;
    for (Cand& c : cands) first += time_cand(c, 1);  // warm-up (code load, clocks)
    const int reps = (int)std::clamp(10.0f * (float)cands.size() / std::max(first, 1e-3f), 2.0f, 8.0f);
    for (Cand& c : cands) c.ms = 1e30f;
    // at least 3 rounds, and until ~150 ms of device time: the chip's clocks ramp up over
    // tens of milliseconds of load, and only warm timings rank the candidates right
    float spent = first;
    for (int round = 0; round < 12 && (round < 3 || spent < 150.f); ++round)
        for (Cand& c : cands) {
            const float t = time_cand(c, reps);
            c.ms = std::min(c.ms, t);
            spent += t * reps * c.tb;
        }
    // final: the three fastest by best-of, timed again over longer windows (>= 16 launches,
    // 4 round-robin rounds, mean): best-of over short windows let one lucky window pick a
    // segment length a few % slower in a run (C2: seg 48 over 88, -4 %)
    // plus the segment lengths next to the best one (+-8, +-16 rows: the march constraint
    // seg + 2 cone = 0 mod 8 keeps them valid) when the heuristic list skipped them
    {
        const Cand b = *std::min_element(cands.begin(), cands.end(),
                                         [](const Cand& x, const Cand& y) { return x.ms < y.ms; });
        if (!s->seg_fixed)
            for (int d : {-16, -8, 8, 16}) {
                const int seg = b.seg + d;
                if (seg < 8 || seg > s->slot[0]->H) continue;
                const bool have = std::any_of(cands.begin(), cands.end(), [&](const Cand& c) {
                    return c.kernel == b.kernel && c.tb == b.tb && c.align == b.align && c.seg == seg;
                });
                if (!have) cands.push_back({b.kernel, seg, b.align, b.tb, 0.f});
            }
    }
    std::vector<Cand*> top;
    for (Cand& c : cands) top.push_back(&c);
    std::sort(top.begin(), top.end(), [](const Cand* a, const Cand* b) { return a->ms < b->ms; });
    // the new neighbours (ms = 0) sort first; keep them and the three fastest timed ones
    size_t keep = 0;
    while (keep < top.size() && top[keep]->ms == 0.f) ++keep;
    if (top.size() > keep + 3) top.resize(keep + 3);
    if (top.size() > 1) {
        std::vector<float> sum(top.size(), 0.f);
        const int long_reps = std::max(reps, 16);
        for (int round = 0; round < 4; ++round)
            for (size_t i = 0; i < top.size(); ++i) sum[i] += time_cand(*top[i], long_reps);
        for (size_t i = 0; i < top.size(); ++i) top[i]->ms = sum[i] / 4;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    WS_HIP_CHECK(hipStreamSynchronize(s->stream));
    grid_free(scratch);
    delete scratch;
    const Cand* best = top[0];
    for (const Cand* c : top)
        if (c->ms < best->ms) best = c;
    if (env_int("WS_TUNE_LOG", 0))
        for (const Cand& c : cands)
            std::fprintf(stderr, "ws autotune: kernel %d tb %d seg %d align %d  %.4f ms/step%s\n", c.kernel, c.tb, c.seg,
                         (int)c.align, c.ms, &c == best ? "  <- chosen" : "");
    s->kernel = best->kernel;
    s->seg_override = best->seg;
    s->align = best->align;
    s->tb = best->tb;
    s->last_launches = 0;
}

// Autotune results, per process (and optionally a file, WS_TUNE_CACHE=path): a drop-in user
// creating many simulations of one shape pays the tuning once. The key is everything the
// ranking depends on.
struct TuneKey {
    int32_t W, H, L, dtype, nst, numerics, top, bot, block, device;
    bool operator<(const TuneKey& o) const {
        return std::memcmp(this, &o, sizeof(TuneKey)) < 0;
    }
};
struct TuneChoice {
    int32_t kernel, seg, align, tb;
};
std::mutex g_tune_mu;
std::map<TuneKey, TuneChoice> g_tune_cache;
bool g_tune_file_loaded = false;

TuneKey tune_key(const ws_sim* s) {
    const ws_grid* g = s->slot[0];
    TuneKey k;
    std::memset(&k, 0, sizeof(k));
    k.W = g->W; k.H = g->H; k.L = g->L; k.dtype = s->dtype; k.nst = fused_stages(s);
    k.numerics = s->numerics; k.top = g->top_clamp; k.bot = g->bot_clamp; k.block = s->block;
    k.device = s->device;
    return k;
}

void tune_file_load_locked() {
    if (g_tune_file_loaded) return;
    g_tune_file_loaded = true;
    const char* path = std::getenv("WS_TUNE_CACHE");
    if (!path) return;
    FILE* f = std::fopen(path, "r");
    if (!f) return;
    TuneKey k;
    TuneChoice c;
    std::memset(&k, 0, sizeof(k));
    while (std::fscanf(f, "%d %d %d %d %d %d %d %d %d %d %d %d %d %d", &k.W, &k.H, &k.L, &k.dtype, &k.nst,
                       &k.numerics, &k.top, &k.bot, &k.block, &k.device, &c.kernel, &c.seg, &c.align, &c.tb) == 14)
        if ((c.kernel == kKernLds || c.kernel == kKernDppLdsY || c.kernel == kKernX2Y) && (c.tb == 1 || c.tb == 2))
            g_tune_cache[k] = c;
    std::fclose(f);
}

void tune_file_append_locked(const TuneKey& k, const TuneChoice& c) {
    const char* path = std::getenv("WS_TUNE_CACHE");
    if (!path) return;
    if (FILE* f = std::fopen(path, "a")) {
        std::fprintf(f, "%d %d %d %d %d %d %d %d %d %d %d %d %d %d\n", k.W, k.H, k.L, k.dtype, k.nst, k.numerics,
                     k.top, k.bot, k.block, k.device, c.kernel, c.seg, c.align, c.tb);
        std::fclose(f);
    }
}

// Pick the variant for this simulation: from the cache, or by timing (autotune_time). A slab
// of a multi-rank decomposition takes rank 0's choice (one broadcast), so every rank runs the
// same kernel and segment length and no rank runs behind on a different pick.
template <typename T>
void autotune(ws_sim* s) {
    s->tuned = true;
    if (!use_fused(s)) return;
    const bool lead = !s->comm || s->comm->rank() == 0;
    if (lead && !s->kernel_fixed) {
        const TuneKey key = tune_key(s);
        bool hit = false;
        {
            std::lock_guard<std::mutex> lk(g_tune_mu);
            tune_file_load_locked();
            auto it = g_tune_cache.find(key);
            if (it != g_tune_cache.end() && !s->seg_fixed && !s->align_fixed && !s->tb_fixed) {
                s->kernel = it->second.kernel;
                s->seg_override = it->second.seg;
                s->align = it->second.align != 0;
                s->tb = it->second.tb;
                hit = true;
            }
        }
        if (!hit) {
            autotune_time<T>(s);
            if (!s->seg_fixed && !s->align_fixed && !s->tb_fixed) {
                std::lock_guard<std::mutex> lk(g_tune_mu);
                const TuneChoice c{s->kernel, s->seg_override, s->align ? 1 : 0, s->tb};
                g_tune_cache[key] = c;
                tune_file_append_locked(key, c);
            }
        }
    }
    if (s->comm && s->comm->nranks() > 1) {
        int32_t v[4] = {s->kernel, s->seg_override, s->align ? 1 : 0, s->tb};
        s->comm->broadcast_i32(v, 4, 0, s->stream);
        s->kernel = v[0];
        s->seg_override = v[1];
        s->align = v[2] != 0;
        s->tb = v[3];
    }
}

void run_steps(ws_sim* s, int k) {
    require(!s->in_group, WS_ERR_INVALID, "a slab of a group steps only with ws_group_run");
    set_device(s->device);
    if (!s->tuned && k > 0) {
        if (s->dtype == WS_F64) autotune<double>(s);
        else autotune<float>(s);
    }
    s->last_launches = 0;
    s->block_pos = 0;  // every run starts a block: the halo is refreshed first
    // one fused launch per step and nothing else on the stream: the kernel's mean duration
    // is the run's span / k (no timestamp packets between the launches being measured)
    const bool span = s->timer.enabled() && use_fused(s) && !s->comm &&
                      s->cfg.model != WS_MODEL_PRIMITIVE_EQUATIONS;
    s->timer.suspend(span);
    // otherwise (halo exchanges or PE T/P updates share the stream) time every 8th launch
    s->timer.sample_period(span || !use_fused(s) ? 1 : 8);
    WS_HIP_CHECK(hipEventRecord(s->ev0, s->stream));
    // PE: T / P updates on the aux stream, in step order there, concurrent with the stencil
    // kernels (they touch neither u, v, h nor each other's inputs across streams); the aux
    // stream starts after everything queued so far and the main stream waits for it at the end
    s->aux_active = k > 0 && s->cfg.model == WS_MODEL_PRIMITIVE_EQUATIONS && env_int("WS_PE_AUX", 1) != 0;
    if (s->aux_active) {
        if (!s->aux) {
            WS_HIP_CHECK(hipStreamCreateWithFlags(&s->aux, hipStreamNonBlocking));
            WS_HIP_CHECK(hipEventCreateWithFlags(&s->aux_in, hipEventDisableTiming));
            WS_HIP_CHECK(hipEventCreateWithFlags(&s->aux_out, hipEventDisableTiming));
        }
        WS_HIP_CHECK(hipEventRecord(s->aux_in, s->stream));
        WS_HIP_CHECK(hipStreamWaitEvent(s->aux, s->aux_in, 0));
    }
    const bool ovl = k > 0 && overlap_active(s);
    if (ovl) ensure_overlap_grids(s);
    for (int i = 0; i < k;) {
        // overlap schedule: one block per iteration; else one launch
        const int n = ovl ? std::min(s->block, k - i) : launch_steps(s, k - i);
        if (ovl) {
            if (s->dtype == WS_F64) overlap_block<double>(s, n, i == 0, i + n == k);
            else overlap_block<float>(s, n, i == 0, i + n == k);
        } else if (s->dtype == WS_F64) {
            enqueue_steps<double>(s, n);
        } else {
            enqueue_steps<float>(s, n);
        }
        for (int j = 0; j < n; ++j) {
            s->time = s->dtype == WS_F64 ? advance_time<double>(s->time, s->dt) : advance_time<float>(s->time, s->dt);
            s->step++;
        }
        i += n;
    }
    if (ovl) WS_HIP_CHECK(hipStreamWaitEvent(s->stream, s->ev_edge, 0));  // the last block's edge bands
    if (s->aux_active) {
        WS_HIP_CHECK(hipEventRecord(s->aux_out, s->aux));
        WS_HIP_CHECK(hipStreamWaitEvent(s->stream, s->aux_out, 0));
        s->aux_active = false;
    }
    WS_HIP_CHECK(hipEventRecord(s->ev1, s->stream));
    if (k > 0 && s->comm) {
        // Diagnostics at slab seams read the neighbours' CURRENT rows: every rank refreshes a
        // one-row u, v halo and computes them here, collectively (a lazy per-rank exchange
        // would deadlock when only one rank reads vorticity).
        ws_grid* c = s->slot[s->cur];
        s->comm->exchange(c->f, 2, (int)elem_size(s->dtype), c->geom(), 1, s->stream);
        materialize_diag(c);
    }
    WS_HIP_CHECK(hipEventSynchronize(s->ev1));
    s->timer.collect();
    float ms = 0.f;
    WS_HIP_CHECK(hipEventElapsedTime(&ms, s->ev0, s->ev1));
    if (span) {
        const ws::Geom g = s->slot[0]->geom();
        // per launch: 6 words per cell-update x the cell-updates of the run / its launches
        s->timer.add_span(0, 6.0 * elem_size(s->dtype) * g.W * g.H * g.L * k / std::max<int64_t>(1, s->last_launches),
                          s->last_launches, ms);
        s->timer.suspend(false);
    }
    s->last_ms = ms;
    s->metrics.compute_time_ms += ms;
    s->metrics.total_time_ms += ms;
    s->metrics.num_steps += k;
}

void sim_free(ws_sim* s) {
    for (ws_grid* g : {s->slot[0], s->slot[1], s->tmpA, s->tmpB, s->K2, s->K3, s->ov[0], s->ov[1], s->ov[2], s->ov[3]})
        if (g) { grid_free(g); delete g; }
    for (hipEvent_t e : {s->ev0, s->ev1, s->aux_in, s->aux_out, s->ev_edge, s->ev_join})
        if (e) (void)hipEventDestroy(e);
    if (s->aux) (void)hipStreamDestroy(s->aux);
    if (s->edge) (void)hipStreamDestroy(s->edge);
    if (s->stream && s->own_stream) (void)hipStreamDestroy(s->stream);
    if (s->cfl_scratch) (void)hipFree(s->cfl_scratch);
    delete s->comm;
    delete s->staging;
    delete s;
}

// Where a simulation sits in a y-slab decomposition (rank 0 of 1: the whole domain).
struct SlabInfo {
    int32_t rank = 0, nranks = 1, row0 = 0, rows = 0;
};

// cfg describes the GLOBAL grid; the simulation owns rows [row0, row0 + rows). `stream`:
// use this (caller-owned) stream instead of creating one (slabs of a group share one).
ws_sim* sim_build(const ws_config_t* cfg, SlabInfo slab, ws::SlabComm* comm, hipStream_t stream = nullptr) {
    const int32_t local_rows = slab.nranks == 1 ? (cfg ? cfg->grid_height : 0) : slab.rows;
    const int32_t row0 = slab.row0;
    require(cfg != nullptr, WS_ERR_INVALID, "null config");
    require(cfg->grid_width > 0 && cfg->grid_height > 0 && cfg->num_levels > 0, WS_ERR_INVALID,
            "Grid dimensions must be positive");
    require(cfg->dx > 0 && cfg->dy > 0, WS_ERR_INVALID, "Grid spacing must be positive");
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
        if (const char* e = std::getenv("WS_FUSED")) s->fused = std::atoi(e) != 0;
        // numerics: fast for fp64 (north_star tolerance), exact for fp32; WS_NUMERICS overrides
        s->numerics = s->dtype == WS_F64 ? WS_NUMERICS_FAST : WS_NUMERICS_EXACT;
        if (const char* e = std::getenv("WS_NUMERICS")) {
            require(std::strcmp(e, "exact") == 0 || std::strcmp(e, "fast") == 0, WS_ERR_INVALID,
                    "WS_NUMERICS must be exact or fast");
            s->numerics = std::strcmp(e, "fast") == 0 ? WS_NUMERICS_FAST : WS_NUMERICS_EXACT;
        }
        if (const char* e = std::getenv("WS_KERNEL")) {
            require(std::strcmp(e, "lds") == 0 || std::strcmp(e, "dppy") == 0 || std::strcmp(e, "x2y") == 0,
                    WS_ERR_INVALID, "WS_KERNEL must be x2y, dppy or lds");
            s->kernel = std::strcmp(e, "lds") == 0 ? kKernLds : std::strcmp(e, "dppy") == 0 ? kKernDppLdsY : kKernX2Y;
            s->kernel_fixed = true;
        }
        if (const char* e = std::getenv("WS_WANT_BLOCKS")) s->want_blocks_override = std::atoi(e);
        if (const char* e = std::getenv("WS_TB")) {
            s->tb = std::atoi(e);
            require(s->tb == 1 || s->tb == 2, WS_ERR_INVALID, "WS_TB must be 1 or 2");
            s->tb_fixed = true;
        }
        if (const char* e = std::getenv("WS_SEG_ROWS")) {
            s->seg_override = std::atoi(e);
            s->seg_fixed = s->seg_override > 0;
        }
        if (const char* e = std::getenv("WS_AUTOTUNE")) s->tuned = std::atoi(e) == 0;
        if (const char* e = std::getenv("WS_ALIGN")) {
            s->align = std::atoi(e) != 0;
            s->align_fixed = true;
        }

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
            if (const char* e = std::getenv("WS_SLAB_BLOCK")) s->block = std::max(1, std::min(s->block, std::atoi(e)));
            // overlap schedule (overlap_block) when the slabs have an interior beside the two
            // edge bands: its edge bands cost ~11 % more stencil work plus two cross-stream
            // waits per block, which the hidden exchange repays from ~2 / 20 / 35 us per
            // exchange at C2's 2 / 4 / 8 slabs (tools/rank_timing.py; a 2.4 MB
            // message per neighbour over one xGMI link is ~40-55 us). Every rank decides
            // alike (global quantities only).
            s->overlap = thin >= 3 * s->block * nst;
            if (const char* e = std::getenv("WS_SLAB_OVERLAP")) s->overlap = std::atoi(e) != 0;
        } else if (comm && s->fused) {
            s->overlap = env_int("WS_SLAB_OVERLAP", 0) != 0;
        }
        if (!comm && slab.nranks > 1 && std::getenv("WS_EMU_XFER_US")) s->emu_xfer_us = std::atof(std::getenv("WS_EMU_XFER_US"));
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

}  // namespace

// ------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------
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
        std::memset(&s->metrics, 0, sizeof(s->metrics));
        grid_reset(s->slot[s->cur]);
        WS_HIP_CHECK(hipStreamSynchronize(s->stream));
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
static int adapter_step(ws_grid* in, ws_grid* out, double dt, double g, double f, double* ms, bool pe) {
    return guarded([&] {
        require(in && out && in != out, WS_ERR_INVALID, "in and out must be distinct grids");
        require(in->W == out->W && in->H == out->H && in->L == out->L && in->dtype == out->dtype &&
                    in->device == out->device && out->nfields == 8,
                WS_ERR_SHAPE, "grids must have identical dimensions and precision");
        set_device(in->device);
        hipEvent_t e0, e1;
        WS_HIP_CHECK(hipEventCreate(&e0));
        WS_HIP_CHECK(hipEventCreate(&e1));
        auto body = [&](auto tag) {
            using T = decltype(tag);
            ws::StageArgs<T> a{};
            a.in_u = (const T*)in->f[0]; a.in_v = (const T*)in->f[1]; a.in_h = (const T*)in->f[2];
            a.base_u = a.in_u; a.base_v = a.in_v; a.base_h = a.in_h;
            a.out_u = (T*)out->f[0]; a.out_v = (T*)out->f[1]; a.out_h = (T*)out->f[2];
            a.c = (T)dt; a.gravity = (T)g; a.coriolis_f = (T)f;
            a.sp = make_spacing<T>(in->dx, in->dy);
            WS_HIP_CHECK(ws::launch_stage<T>(ws::kAxpy, a, in->geom(), in->stream));
            if (pe) {
                WS_HIP_CHECK(ws::launch_affine<T>((T*)out->f[WS_FIELD_T], (const T*)in->f[WS_FIELD_T], (T)dt,
                                                  T(288.15f), in->geom(), in->stream));
                WS_HIP_CHECK(ws::launch_affine<T>((T*)out->f[WS_FIELD_P], (const T*)in->f[WS_FIELD_P], (T)dt,
                                                  T(1013.25f), in->geom(), in->stream));
            }
        };
        WS_HIP_CHECK(hipEventRecord(e0, in->stream));
        if (in->dtype == WS_F64) body(double{});
        else body(float{});
        WS_HIP_CHECK(hipEventRecord(e1, in->stream));
        WS_HIP_CHECK(hipEventSynchronize(e1));
        float t = 0.f;
        WS_HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
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
        hipEvent_t e0, e1;
        WS_HIP_CHECK(hipEventCreate(&e0));
        WS_HIP_CHECK(hipEventCreate(&e1));
        WS_HIP_CHECK(hipEventRecord(e0, g->stream));
        g->diag_pending = true;
        materialize_diag(g);
        WS_HIP_CHECK(hipEventRecord(e1, g->stream));
        WS_HIP_CHECK(hipEventSynchronize(e1));
        float t = 0.f;
        WS_HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
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

// ---- slab decomposition ----
int ws_comm_get_unique_id(uint8_t id[WS_COMM_ID_BYTES]) {
    return guarded([&] {
        require(id != nullptr, WS_ERR_INVALID, "null pointer");
        ws::SlabComm::unique_id(id);
    });
}

int ws_sim_create_slab(const ws_config_t* cfg, int32_t rank, int32_t nranks, const uint8_t id[WS_COMM_ID_BYTES],
                       ws_sim_t** out, int32_t* row0, int32_t* rows) {
    return guarded([&] {
        require(cfg && out, WS_ERR_INVALID, "null pointer");
        require(nranks >= 1 && rank >= 0 && rank < nranks, WS_ERR_INVALID, "bad rank / nranks");
        require(cfg->grid_height >= nranks, WS_ERR_INVALID, "fewer rows than ranks");
        int r0 = 0, nrows = 0;
        ws::slab_rows(cfg->grid_height, rank, nranks, &r0, &nrows);
        require(nranks == 1 || nrows >= 4, WS_ERR_INVALID, "a slab needs at least 4 rows per rank");
        const int r1 = r0 + nrows;
        set_device(cfg->device_id);
        // a 1-rank slab still gets its communicator: same code path as N>1 (the exchanges
        // are no-ops), so a 1-GPU run exercises the RCCL bootstrap
        // (id == NULL: no communicator, exchanges skipped -- the measurement aid of ws_hip.h)
        ws::SlabComm* comm = id ? new ws::SlabComm(rank, nranks, id) : nullptr;
        ws_sim* s = nullptr;
        try {
            SlabInfo si;
            si.rank = rank; si.nranks = nranks; si.row0 = r0; si.rows = nrows;
            s = sim_build(cfg, si, comm, nullptr);
        } catch (...) {
            delete comm;
            throw;
        }
        *out = s;
        if (row0) *row0 = r0;
        if (rows) *rows = r1 - r0;
    });
}

int ws_slab_partition(int32_t height, int32_t rank, int32_t nranks, int32_t* row0, int32_t* rows) {
    return guarded([&] {
        require(row0 && rows, WS_ERR_INVALID, "null pointer");
        require(nranks >= 1 && rank >= 0 && rank < nranks && height >= nranks, WS_ERR_INVALID, "bad partition");
        int r0 = 0, n = 0;
        ws::slab_rows(height, rank, nranks, &r0, &n);
        *row0 = r0;
        *rows = n;
    });
}

int ws_sim_comm_allreduce_max(ws_sim_t* s, double value, double* out) {
    return guarded([&] {
        require(s && out, WS_ERR_INVALID, "null pointer");
        set_device(s->device);
        *out = s->comm ? s->comm->allreduce_max(value, s->stream) : value;
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

int ws_sim_slab_schedule(const ws_sim_t* s, int32_t* block, int32_t* overlap) {
    return guarded([&] {
        require(s != nullptr && block != nullptr && overlap != nullptr, WS_ERR_INVALID, "null pointer");
        *block = s->block;
        *overlap = overlap_active(s) ? 1 : 0;
    });
}

int ws_sim_set_numerics(ws_sim_t* s, int32_t mode) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        require(mode == WS_NUMERICS_EXACT || mode == WS_NUMERICS_FAST, WS_ERR_INVALID,
                "numerics must be WS_NUMERICS_EXACT or WS_NUMERICS_FAST");
        if (mode != s->numerics && !s->kernel_fixed) s->tuned = env_int("WS_AUTOTUNE", 1) == 0;  // re-rank
        s->numerics = mode;
    });
}

int ws_sim_get_numerics(const ws_sim_t* s, int32_t* mode) {
    return guarded([&] {
        require(s && mode, WS_ERR_INVALID, "null pointer");
        *mode = s->numerics;
    });
}

int ws_slab_exchange_plan(int32_t width, int32_t rows, int32_t levels, int32_t dtype, int32_t rank, int32_t nranks,
                          int32_t nfields, int32_t depth, ws_xfer_t* out, int32_t capacity, int32_t* count,
                          int64_t* pitch, int64_t* level_stride) {
    return guarded([&] {
        require(width > 0 && rows > 0 && levels > 0, WS_ERR_INVALID, "Grid dimensions must be positive");
        require(dtype == WS_F32 || dtype == WS_F64, WS_ERR_INVALID, "bad dtype");
        require(nranks >= 1 && rank >= 0 && rank < nranks, WS_ERR_INVALID, "bad rank / nranks");
        require(nfields >= 1 && nfields <= ws::kMaxHaloFields, WS_ERR_INVALID, "bad field count");
        require(depth >= 1 && depth <= ws::kHalo && depth <= rows, WS_ERR_INVALID, "bad halo depth");
        // the slab grids' layout (grid_alloc)
        ws::Geom g{};
        g.W = width; g.H = rows; g.L = levels;
        g.pitch = layout_pitch(width);
        g.lstride = layout_lstride(rows, g.pitch);
        g.top_clamp = rank == 0; g.bot_clamp = rank == nranks - 1; g.halo = ws::kHalo;
        const auto x = ws::make_halo_plan(g, (int)elem_size(dtype), rank, nranks, nfields, depth).xfers();
        if (count) *count = (int32_t)x.size();
        if (pitch) *pitch = g.pitch;
        if (level_stride) *level_stride = g.lstride;
        if (out) {
            require(capacity >= (int32_t)x.size(), WS_ERR_INVALID, "plan capacity too small");
            for (size_t i = 0; i < x.size(); ++i) {
                out[i].peer = x[i].peer; out[i].kind = x[i].kind; out[i].field = x[i].field;
                out[i].level = x[i].level; out[i].offset = x[i].offset; out[i].bytes = x[i].bytes;
                out[i].msg_offset = x[i].msg_offset;
            }
        }
    });
}

int ws_sim_comm_barrier(ws_sim_t* s) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        set_device(s->device);
        if (s->comm) s->comm->barrier(s->stream);
        WS_HIP_CHECK(hipStreamSynchronize(s->stream));
    });
}

}  // extern "C"

// ------------------------------------------------------------------------------------
// slab group: the y-slab decomposition inside one process on one device, halo rows moved
// by device copies instead of RCCL. It runs exactly the multi-rank step schedule
// (interior segments -> halo exchange -> edge segments) and is how the decomposition is
// verified bitwise against the single-domain run on a one-GPU box.
// ------------------------------------------------------------------------------------
struct ws_group {
    std::vector<ws_sim*> slabs;
    hipStream_t stream = nullptr;
    // overlap schedule: the transport between the slabs' edge streams (what RCCL does on each
    // rank's edge stream), created on first use
    hipStream_t xstream = nullptr;
    hipEvent_t ev_x = nullptr;
    int device = 0;
};

namespace {

// The halo exchange of every slab of the group, by the plan of ws_halo.h: each slab packs
// its neighbour messages (halo_pack), the messages move by device copies into the
// neighbours' receive staging (what RCCL does between processes, ws_comm.cpp), and each slab
// unpacks them -- the same plan and kernels as the multi-process path.
void group_exchange(ws_group* gr, int nfields, int depth, bool next = false, hipStream_t st = nullptr) {
    if (!st) st = gr->stream;
    const int n = (int)gr->slabs.size();
    std::vector<ws::HaloPlan> plans(n);
    std::vector<ws::HaloFields> hf(n);
    auto grid = [&](int r) { ws_sim* s = gr->slabs[r]; return s->slot[next ? 1 - s->cur : s->cur]; };
    for (int r = 0; r < n; ++r) {
        const ws_grid* me = grid(r);
        plans[r] = ws::make_halo_plan(me->geom(), (int)elem_size(me->dtype), r, n, nfields, depth);
    }
    if (ws::halo_direct(plans[0])) {
        // the direct transport (ws_comm.cpp): every send segment of the plan lands on the
        // receive segment the peer's plan lists for it (same field / level, the k-th of each)
        for (int r = 0; r < n; ++r)
            for (const ws::HaloXfer& x : plans[r].xfers()) {
                if (x.kind != 0) continue;
                for (const ws::HaloXfer& y : plans[x.peer].xfers())
                    if (y.kind == 1 && y.peer == r && y.field == x.field && y.level == x.level) {
                        require(y.bytes == x.bytes, WS_ERR_COMM, "halo segment size mismatch");
                        WS_HIP_CHECK(hipMemcpyAsync((char*)grid(x.peer)->f[y.field] + y.offset,
                                                    (const char*)grid(r)->f[x.field] + x.offset, (size_t)x.bytes,
                                                    hipMemcpyDeviceToDevice, st));
                    }
            }
        return;
    }
    for (int r = 0; r < n; ++r) {
        ws_sim* s = gr->slabs[r];
        const ws_grid* me = grid(r);
        if (!s->staging) s->staging = new ws::HaloStaging;
        s->staging->ensure(plans[r].msg_bytes());
        for (int f = 0; f < nfields; ++f) hf[r].f[f] = (char*)me->f[f];
        for (int side = 0; side < 2; ++side)
            if (plans[r].has[side])
                WS_HIP_CHECK(ws::halo_pack(plans[r], hf[r], side, s->staging->send[side], st));
    }
    for (int r = 0; r < n; ++r)
        for (int side = 0; side < 2; ++side) {
            if (!plans[r].has[side]) continue;
            ws_sim* peer = gr->slabs[plans[r].peer[side]];
            WS_HIP_CHECK(hipMemcpyAsync(peer->staging->recv[1 - side], gr->slabs[r]->staging->send[side],
                                        (size_t)plans[r].msg_bytes(), hipMemcpyDeviceToDevice, st));
        }
    for (int r = 0; r < n; ++r)
        for (int side = 0; side < 2; ++side)
            if (plans[r].has[side])
                WS_HIP_CHECK(ws::halo_unpack(plans[r], hf[r], side, gr->slabs[r]->staging->recv[side], st));
}

// One overlapped block of every slab (overlap_block with the group's device-copy transport
// on xstream between the slabs' edge streams).
template <typename T>
void group_overlap_block(ws_group* gr, int steps, bool first, bool last) {
    ws_sim* s0 = gr->slabs[0];
    const int depth = s0->block * fused_stages(s0);
    if (first) group_exchange(gr, 3, depth);
    for (ws_sim* s : gr->slabs) overlap_begin(s, first);
    for (ws_sim* s : gr->slabs) overlap_edges<T>(s, steps);
    if (!last) {
        if (!gr->xstream) {
            WS_HIP_CHECK(hipStreamCreateWithFlags(&gr->xstream, hipStreamNonBlocking));
            WS_HIP_CHECK(hipEventCreateWithFlags(&gr->ev_x, hipEventDisableTiming));
        }
        for (ws_sim* s : gr->slabs) WS_HIP_CHECK(hipStreamWaitEvent(gr->xstream, s->ev_edge, 0));
        group_exchange(gr, 3, depth, true, gr->xstream);
        WS_HIP_CHECK(hipEventRecord(gr->ev_x, gr->xstream));
        for (ws_sim* s : gr->slabs) WS_HIP_CHECK(hipStreamWaitEvent(s->edge, gr->ev_x, 0));
    }
    for (ws_sim* s : gr->slabs) overlap_interior<T>(s, steps);
}

template <typename T>
void group_step(ws_group* gr, int nsteps) {
    ws_sim* s0 = gr->slabs[0];
    if (s0->block_pos == 0) {  // a block starts: the block's halo, by device copies
        group_exchange(gr, 3, s0->block * fused_stages(s0));
    }
    for (ws_sim* s : gr->slabs) step_begin<T>(s, nsteps);
    for (ws_sim* s : gr->slabs) step_end<T>(s, nsteps);
}

}  // namespace

extern "C" {

int ws_group_create(const ws_config_t* cfg, int32_t nslabs, ws_group_t** out) {
    return guarded([&] {
        require(cfg && out, WS_ERR_INVALID, "null pointer");
        require(nslabs >= 1 && cfg->grid_height >= nslabs * 4, WS_ERR_INVALID, "a slab needs >= 4 rows");
        set_device(cfg->device_id);
        ws_group* gr = new ws_group;
        gr->device = cfg->device_id;
        try {
            WS_HIP_CHECK(hipStreamCreateWithFlags(&gr->stream, hipStreamNonBlocking));
            for (int r = 0; r < nslabs; ++r) {
                SlabInfo si;
                si.rank = r;
                si.nranks = nslabs;
                ws::slab_rows(cfg->grid_height, r, nslabs, &si.row0, &si.rows);
                ws_sim* s = sim_build(cfg, si, nullptr, gr->stream);
                s->in_group = true;
                gr->slabs.push_back(s);
                require(use_fused(s), WS_ERR_UNSUPPORTED, "slab groups need the fused step kernel (WS_FUSED=1)");
            }
        } catch (...) {
            for (ws_sim* s : gr->slabs) sim_free(s);
            if (gr->stream) (void)hipStreamDestroy(gr->stream);
            delete gr;
            throw;
        }
        *out = gr;
    });
}

int ws_group_destroy(ws_group_t* gr) {
    return guarded([&] {
        if (!gr) return;
        set_device(gr->device);
        (void)hipStreamSynchronize(gr->stream);
        for (ws_sim* s : gr->slabs) sim_free(s);
        (void)hipStreamDestroy(gr->stream);
        if (gr->xstream) (void)hipStreamDestroy(gr->xstream);
        if (gr->ev_x) (void)hipEventDestroy(gr->ev_x);
        delete gr;
    });
}

int ws_group_slab(ws_group_t* gr, int32_t rank, ws_sim_t** sim, int32_t* row0, int32_t* rows) {
    return guarded([&] {
        require(gr && sim && rank >= 0 && rank < (int)gr->slabs.size(), WS_ERR_INVALID, "bad argument");
        ws_sim* s = gr->slabs[rank];
        *sim = s;
        if (row0) *row0 = s->row0;
        if (rows) *rows = s->slot[0]->H;
    });
}

int ws_group_run(ws_group_t* gr, int32_t n, int32_t* taken) {
    return guarded([&] {
        require(gr != nullptr, WS_ERR_INVALID, "null group");
        set_device(gr->device);
        const int k = plan_steps(gr->slabs[0], n);
        ws_sim* s0 = gr->slabs[0];
        if (!s0->tuned && k > 0) {  // tune on slab 0, apply everywhere
            if (s0->dtype == WS_F64) autotune<double>(s0);
            else autotune<float>(s0);
            for (ws_sim* s : gr->slabs) {
                s->kernel = s0->kernel;
                s->seg_override = s0->seg_override;
                s->align = s0->align;
                s->tb = s0->tb;
                s->tuned = true;
            }
        }
        for (ws_sim* s : gr->slabs) s->block_pos = 0;
        WS_HIP_CHECK(hipEventRecord(s0->ev0, gr->stream));
        bool ovl = k > 0;  // every slab must agree
        for (ws_sim* s : gr->slabs) ovl = ovl && overlap_active(s);
        if (ovl)
            for (ws_sim* s : gr->slabs) ensure_overlap_grids(s);
        for (int i = 0; i < k;) {
            int n = 2;  // every slab must agree (they share the block position and the choice)
            for (ws_sim* s : gr->slabs) n = std::min(n, launch_steps(s, k - i));
            if (ovl) n = std::min(s0->block, k - i);
            if (ovl && s0->dtype == WS_F64) group_overlap_block<double>(gr, n, i == 0, i + n == k);
            else if (ovl) group_overlap_block<float>(gr, n, i == 0, i + n == k);
            else if (s0->dtype == WS_F64) group_step<double>(gr, n);
            else group_step<float>(gr, n);
            for (ws_sim* s : gr->slabs)
                for (int j = 0; j < n; ++j) {
                    s->time = s->dtype == WS_F64 ? advance_time<double>(s->time, s->dt) : advance_time<float>(s->time, s->dt);
                    s->step++;
                }
            i += n;
        }
        if (ovl)
            for (ws_sim* s : gr->slabs) WS_HIP_CHECK(hipStreamWaitEvent(gr->stream, s->ev_edge, 0));
        WS_HIP_CHECK(hipEventRecord(s0->ev1, gr->stream));
        if (k > 0) {  // seam diagnostics need the neighbours' current rows (see run_steps)
            group_exchange(gr, 2, 1);
            for (ws_sim* s : gr->slabs) materialize_diag(s->slot[s->cur]);
        }
        WS_HIP_CHECK(hipStreamSynchronize(gr->stream));
        WS_HIP_CHECK(hipEventSynchronize(s0->ev1));
        float ms = 0.f;
        WS_HIP_CHECK(hipEventElapsedTime(&ms, s0->ev0, s0->ev1));
        for (ws_sim* s : gr->slabs) {
            s->timer.collect();
            s->last_ms = ms;
            s->metrics.compute_time_ms += ms;
            s->metrics.total_time_ms += ms;
            s->metrics.num_steps += k;
        }
        if (taken) *taken = k;
    });
}

}  // extern "C"

namespace ws {
int abi_guarded(const std::function<void()>& f) { return guarded(f); }
void abi_set_device(int device) { set_device(device); }
}  // namespace ws
