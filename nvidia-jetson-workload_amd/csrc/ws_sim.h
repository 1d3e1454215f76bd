// Internal types and interfaces of the host runtime, shared by its translation units:
//   ws_runtime.cpp   device-resident grids and simulations, and the C ABI of both (grid,
//                    simulation, KernelAdapter, raw launchers, CFL);
//   ws_schedule.cpp  the time-step schedules: one domain, slab blocks (stream-ordered and
//                    overlapped with the halo exchange on a second stream), run();
//   ws_autotune.cpp  the fused-kernel variant choice (timed candidates, per-process / file
//                    cache, rank 0's choice broadcast) and the slab schedule choice;
//   ws_slab.cpp      the multi-GPU slab ABI (RCCL communicator, partition, exchange plan) and
//                    the one-process slab group.
// Not part of the C ABI (include/ws_hip.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "ws_abi.h"
#include "ws_comm.h"
#include "ws_fused.h"
#include "ws_halo.h"
#include "ws_hip.h"
#include "ws_internal.h"
#include "ws_timer.h"

namespace wsr {

extern thread_local std::string g_last_error;

struct WsError : std::runtime_error {
    int code;
    WsError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define WS_HIP_CHECK(expr)                                                                                \
    do {                                                                                                  \
        hipError_t e_ = (expr);                                                                           \
        if (e_ != hipSuccess)                                                                             \
            throw ::wsr::WsError(WS_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));       \
    } while (0)

// Runs f; maps what it throws to a status code + ws_last_error() (no exception crosses the ABI).
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

inline void require(bool cond, int code, const char* msg) {
    if (!cond) throw WsError(code, msg);
}

int device_count();
void set_device(int dev);  // WS_ERR_DEVICE without a HIP device: there is no CPU path

inline size_t elem_size(int dtype) { return dtype == WS_F64 ? 8 : 4; }

inline bool is_pow2(double v) {
    if (!(v > 0) || !std::isfinite(v)) return false;
    int e;
    return std::frexp(v, &e) == 0.5;
}

// value rounded to the simulation precision (the reference stores scalar_t)
inline double to_prec(double v, int dtype) { return dtype == WS_F64 ? v : (double)(float)v; }

// The library's environment switches (every one is listed in include/ws_hip.h).
inline const char* env_str(const char* name) { return std::getenv(name); }
inline int64_t env_int(const char* name, int64_t dflt) {
    const char* e = std::getenv(name);
    return e ? std::atoll(e) : dflt;
}

}  // namespace wsr

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
    hipEvent_t tev[2] = {};     // timing events of the KernelAdapter entry points (created once)

    ws::Geom geom() const {
        ws::Geom g;
        g.W = W; g.H = H; g.L = L; g.pitch = pitch; g.lstride = lstride;
        g.top_clamp = top_clamp; g.bot_clamp = bot_clamp;
        g.halo = ws::kHalo;
        return g;
    }
    size_t bytes_per_field() const { return (size_t)L * lstride * wsr::elem_size(dtype); }
};

namespace wsr {

// row pitch (elements) and level stride of a W x H grid: rows padded to 64 elements, kHalo
// halo rows above and below every level (the layout ws_slab_exchange_plan reports)
// (row pitch padding by 8 / 64 / 128 elements measured +-1 %)
inline int64_t layout_pitch(int64_t W) { return (W + 63) / 64 * 64; }
inline int64_t layout_lstride(int64_t H, int64_t pitch) { return (H + 2 * ws::kHalo) * pitch; }

void grid_free(ws_grid* g);
void grid_reset(ws_grid* g);
void materialize_diag(ws_grid* g);  // run pending diagnostics now (lazy vorticity / divergence)
ws_grid* new_grid(int32_t W, int32_t H, int32_t L, int32_t dtype, int32_t device, unsigned nfields, hipStream_t s);

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

enum FusedKernel : int { kKernLds = ws::kFusedLds, kKernDppLdsY = ws::kFusedDppLdsY, kKernX2Y = ws::kFusedX2Y, kKernPc = ws::kFusedPc,
                         kKernPc2 = ws::kFusedPc2 };

// slab schedule choice (ws_sim::overlap_mode)
enum OverlapMode : int { kOverlapOff = 0, kOverlapOn = 1, kOverlapAuto = 2 };

}  // namespace wsr

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
    // PE T / P drift deferred inside run() (ws_schedule.cpp rotate / run_steps): the steps not
    // yet applied, the last launch's steps, and the buffers holding the run's starting T / P
    bool tp_lazy = false;
    int64_t tp_steps = 0;
    int tp_last = 0;
    void* tp_src[2] = {nullptr, nullptr};
    int64_t fail_after = -1;  // test hook (ws_sim_inject_failure): throw once this many launches ran
    double last_ms = 0.0;
    int64_t last_launches = 0;
    ws::KernelTimer timer;
    int32_t rank = 0, nranks = 1;                       // y-slab position (1 = whole domain)
    bool own_stream = true;
    bool in_group = false;                              // a slab of a ws_group (local halo transport)
    bool fused = true;       // one fused kernel per step (WS_FUSED=0: one kernel per RK stage)
    int kernel = wsr::kKernX2Y;  // fused kernel variant (WS_KERNEL / ws_sim_pin_variant fix it)
    int32_t seg_override = 0;    // rows per segment (WS_SEG_ROWS / pin fix it)
    bool align = false;          // strip output windows on whole 128-byte lines (pin fixes it)
    bool kernel_fixed = false, seg_fixed = false, align_fixed = false;
    bool kernel_env = false;  // WS_KERNEL pins process-wide: no autotuning of what it leaves free
    // time steps per fused launch (temporal blocking; the dppy / x2y kernels): 1, or 2 = two
    // steps per launch inside run(k) (WS_TB / pin fix it, else the autotuner picks)
    int32_t tb = 1;
    bool tb_fixed = false;
    int numerics = WS_NUMERICS_EXACT;  // fused kernels: exact or fast numerics (ws_fused.h)
    bool tuned = false;       // autotune done (first run; WS_AUTOTUNE=0 disables)
    // whether the autotuner has anything left to choose: parts ws_sim_pin_variant leaves at -1
    // are tuned (restricted to the pinned parts); a WS_KERNEL environment pin disables tuning
    bool tune_free() const { return !kernel_env && !(kernel_fixed && seg_fixed && align_fixed && tb_fixed); }
    int32_t block = 1;        // slab: steps per halo exchange (deep halo), see step_rows
    int32_t block_pos = 0;    // position in the current block (0 = exchange first)
    // slab overlap schedule (overlap_block): a block's edge bands run on `edge`, the halo
    // exchange follows them there, the interior runs meanwhile on `stream`
    int overlap_mode = wsr::kOverlapOff;  // off / on / auto (decided from a measured exchange)
    bool overlap = false;                 // the schedule in use
    double xfer_us = -1.0;                // measured halo exchange (auto mode), microseconds
    bool overlap_trial = false;           // auto mode: time one block of each schedule at the next run
    double trial_ms[2] = {-1.0, -1.0};    // that trial: ms per block stream-ordered, overlapped
    hipEvent_t ev_trial[2] = {};
    hipStream_t edge = nullptr;
    hipEvent_t ev_edge = nullptr, ev_join = nullptr;
    ws_grid* ov[4] = {};      // interior ping-pong (0, 1), edge-band ping-pong (2, 3); u, v, h
    int ov_edge_wgs[8] = {};  // workgroups of the current block's edge launches (launch j)
    bool ov_thin = false;     // the block's edge bands are a large share of its rows (overlap_edges)
    double emu_xfer_us = -1.0;  // measurement slab (ws_sim_create_slab_emulated): transfer stand-in
    // slab decomposition
    ws::SlabComm* comm = nullptr;
    ws::HaloStaging* staging = nullptr;  // measurement slab: its pack / unpack staging
    uint64_t* cfl_scratch = nullptr;     // ws_sim_cfl: per-level partial maxima + results (device)
    int64_t cfl_scratch_n = 0;
    int32_t row0 = 0;
    // chain-schedule tables (ws_schedule.cpp chain_table), one per launch shape, on the device
    struct ChainTable {
        int64_t key[12];
        ws::ChainSeg* dev = nullptr;
        int32_t n = 0, max_rows = 0;
    };
    std::vector<ChainTable> chain_tables;
    int32_t num_cus = 0;  // the device's compute units (chain-schedule round size), queried once

    // cone = stages per launch (NST x steps per launch): the strip margins
    int out_w(int cone) const { return ws::fused_out_w(kernel, cone, (int)wsr::elem_size(dtype), align); }
    int64_t strips(int cone) const {
        return kernel == wsr::kKernLds ? (slot[0]->W + out_w(cone) - 1) / out_w(cone)
                                       : ws::fused_strips(kernel, slot[0]->W, cone, (int)wsr::elem_size(dtype), out_w(cone));
    }
    // steps per launch the tuned configuration launches where a run has room: tb, capped to
    // what the kernel takes at this integrator and precision (ws::fused_tb_ok: 4 -> 2 -> 1)
    int launch_tb() const;
    // segment rows giving about want_blocks workgroups (at least min_rows rows; the march
    // length rows + 2 NST a multiple of the unroll)
    int32_t seg_for_blocks(int nst, int64_t want_blocks, int64_t min_rows) const;
    // Rows per fused-kernel segment: enough workgroups to fill the chip (64-lane waves of
    // 64 / 128 columns vs 256-lane workgroups), segments long enough that the 2*NST
    // warm-up rows stay a small overhead. The autotuner also tries other counts.
    int32_t seg_rows(int nst) const;
};

namespace wsr {
// A segment choice (seg_override, ws_sim_pin_variant's seg_rows) of -2, -3, ... selects the chain
// schedule (ws_fused.h FusedArgs::chains) with 1, 2, ... chains (waves) per SIMD.
inline int chain_rounds(int seg) { return seg <= -2 ? -seg - 1 : 0; }
constexpr int seg_chains(int rounds) { return -(rounds + 1); }
constexpr int kMaxChainRounds = 8;
}  // namespace wsr

namespace wsr {

// ---- ws_schedule.cpp ----
int effective_method(const ws_config_t& c);  // the integrator the reference actually runs
int fused_stages(const ws_sim* s);           // stages per step of the fused kernels (1, 2, 4)
inline bool use_fused(const ws_sim* s) { return s->fused && s->slot[0]->W >= 2; }
bool config_spacing(const ws_sim* s);        // both grids carry the configured dx, dy

// Output rows of a fused launch: [y0, y1) (empty if y1 <= y0).
struct RowRange {
    int y0, y1;
    int rows() const { return y1 > y0 ? y1 - y0 : 0; }
};

// the fused step kernel over the output rows A U B (segments of seg_rows rows); in / out
// default to the current / next grid
template <typename T>
// want > 0: a chain schedule's chain count (default: its rounds x the chip's wave slots); returns
// the workgroups launched
int fused_launch(ws_sim* s, int nst, int nsteps, RowRange A, RowRange B, int seg_rows, hipStream_t st = nullptr,
                 ws_grid* in = nullptr, ws_grid* out = nullptr, int want = 0, int prio = 0, int min2 = 4);
template <typename T>
void step_begin(ws_sim* s, int nsteps = 1);
template <typename T>
void step_end(ws_sim* s, int nsteps = 1);
int launch_steps(const ws_sim* s, int remaining);
template <typename T>
int fused_waves_per_simd(const ws_sim* s);  // occupancy of the chosen fused variant (0: none)
// overlap schedule pieces (the slab group runs them per slab, ws_slab.cpp)
bool overlap_active(const ws_sim* s);
void ensure_overlap_grids(ws_sim* s);
void overlap_begin(ws_sim* s, bool first);
template <typename T>
void overlap_edges(ws_sim* s, int steps);
template <typename T>
void overlap_interior(ws_sim* s, int steps);
// the halo exchange of a slab (RCCL, or the measurement slab's stand-in)
void slab_exchange(ws_sim* s, ws_grid* g, int nfields, int depth, hipStream_t st);
double advance_time(const ws_sim* s, double t);  // t + dt in the simulation's precision
int plan_steps(const ws_sim* s, int n);          // steps run(n) takes (max_time cap)
void run_steps(ws_sim* s, int k);

// ---- ws_slab.cpp ----
void group_diag_halo(ws_group* gr);  // one-row u, v halos of every slab (diagnostics at seams)

// ---- ws_autotune.cpp ----
void autotune(ws_sim* s);  // variant choice at the first run (cache, timing, rank-0 broadcast)
void choose_slab_schedule(ws_sim* s);  // auto overlap: from a measured halo exchange

// ---- ws_runtime.cpp ----
void sim_free(ws_sim* s);
// Where a simulation sits in a y-slab decomposition (rank 0 of 1: the whole domain).
struct SlabInfo {
    int32_t rank = 0, nranks = 1, row0 = 0, rows = 0;
};
// cfg describes the GLOBAL grid; the simulation owns rows [row0, row0 + rows). `stream`:
// use this (caller-owned) stream instead of creating one (slabs of a group share one).
ws_sim* sim_build(const ws_config_t* cfg, SlabInfo slab, ws::SlabComm* comm, hipStream_t stream = nullptr);

}  // namespace wsr
