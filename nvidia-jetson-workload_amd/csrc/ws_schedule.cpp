// Time-step schedules of the host runtime (internal interfaces: ws_sim.h).
//
// run_steps replaces WeatherSimulation::run's loop of step() calls (reference
// src/weather-sim/cpp/src/weather_simulation.cpp:68-158): the steps of one run() are
// enqueued on the simulation's stream without host synchronisation --
//   * one domain: one fused launch per one or two time steps (temporal blocking), or the
//     per-stage kernels (WS_FUSED=0);
//   * a y-slab of a multi-GPU decomposition: deep-halo blocks of up to 6 steps per halo
//     exchange, stream-ordered or overlapped (the exchange behind the edge bands on a second
//     stream while the interior runs, overlap_block);
// then the reference's grid rotation, the PE T / P update and the float time accumulation.
#include <algorithm>
#include <cstdio>

#include "ws_knobs.h"
#include "ws_sim.h"

namespace wsr {

// Integrator actually executed (weather_simulation.cpp:122-142, :334-338, :457-471).
int effective_method(const ws_config_t& c) {
    switch (c.integration_method) {
        case WS_RK2: return WS_RK2;
        case WS_RK4: return c.model == WS_MODEL_SHALLOW_WATER ? WS_RK4 : WS_RK2;
        default: return WS_EULER;
    }
}

template <typename T>
static ws::StageArgs<T> stage_args(const ws_grid* in, const ws_grid* base, ws_grid* out, T c, const ws_sim* s) {
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
static void launch_stage(ws_sim* s, int mode, const ws::StageArgs<T>& a, const ws_grid* in, int kind, int words) {
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




// Slab blocks. A slab advances `block` steps per halo exchange: the exchange moves
// block * NST rows of u, v, h from each neighbour, and step j = 0 .. block-1 of the block
// computes its rows extended by (block - 1 - j) * NST into the halo on each non-global
// side, so every step's dependency cone is covered by rows already on the device and the
// last step of the block ends on exactly the owned rows. The extra work is
// (block - 1) * NST * (block) rows per side per block; the saving is block - 1 exchanges and
// every cross-stream synchronisation: the exchange is stream-ordered on the compute
// stream (measured on MI355X: two cross-stream event waits per step cost more than an
// overlapped edge launch saves).
static RowRange step_rows(const ws_sim* s, int nst, int nsteps) {
    const ws_grid* g = s->slot[0];
    // a launch of nsteps steps ends on the rows of its last step, block position + nsteps - 1
    const int e = (s->block - nsteps - s->block_pos) * nst;
    return {g->top_clamp ? 0 : -e, g->bot_clamp ? g->H : g->H + e};
}

// Chain schedule (ws_fused.h FusedArgs::chains): `rounds` waves per SIMD, each marching ONE chain -- a run of rows of one strip (and level) -- sized so that every
// chain of a launch costs about the same. A strip whose window touches a global x edge runs the
// clamped march (kXClampCost x the instructions per row of an interior strip, the fp64 RK4
// two-step kernel's steady loops: tools/isa_mix.py) and a chain reaching into a global y edge's
// cone the y-clamped march (kYClampCost), so those get fewer rows. Chains of neighbouring strips
// at the same rows are adjacent in the table: xcd_work_item() puts them on one XCD (shared halo
// columns in its L2). Built on first use per launch shape and kept on the device.
// Timed, not counted (round 6, profiles/r06_ab_clamp_cost_*.txt): the fp64 one-column march's
// clamped bodies cost 3.0 / 2.0 x (C2 RK4 0.1146-0.1157 -> 0.1085-0.1089 ms/step against the
// instruction-count weights 1.73 / 1.34); the fp32 pair march (C3) keeps 1.73 / 1.34, which it
// runs fastest with (0.0131-0.0132 against 0.0135-0.0137 at 3.0 / 2.0).
#ifndef WS_XCLAMP_COST
#define WS_XCLAMP_COST 3.0
#endif
#ifndef WS_YCLAMP_COST
#define WS_YCLAMP_COST 2.0
#endif
constexpr double kXClampCost64 = WS_XCLAMP_COST, kYClampCost64 = WS_YCLAMP_COST;
#ifndef WS_XCLAMP_COST_DEF
#define WS_XCLAMP_COST_DEF 1.73
#endif
#ifndef WS_YCLAMP_COST_DEF
#define WS_YCLAMP_COST_DEF 1.34
#endif
constexpr double kXClampCostDef = WS_XCLAMP_COST_DEF, kYClampCostDef = WS_YCLAMP_COST_DEF;

template <typename T>
static const ws_sim::ChainTable& chain_table(ws_sim* s, int nst, int nsteps, RowRange A, RowRange B, int rounds,
                                             int out_w, int sp_mode, int want_chains, int min2) {
    const ws_grid* g = s->slot[0];
    const int64_t key[12] = {nst, nsteps, A.y0, A.y1, B.y0, B.y1, rounds, out_w, s->kernel, sp_mode, want_chains, min2};
    for (const auto& t : s->chain_tables)
        if (std::equal(key, key + 12, t.key)) return t;
    if (s->num_cus == 0) {
        int cus = 0;
        WS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device));
        s->num_cus = cus;
    }
    // `rounds` chains per SIMD (4 per CU; a split variant's workgroup is two waves): a whole
    // number of waves on every SIMD whatever the kernel's occupancy (C3's launch with 1.5 waves
    // per SIMD ran half its SIMDs idle for the last 40 %, profiles/r04_timeline_c3.txt)
    const int waves_per_wg = ws::fused_split(s->kernel) ? 2 : 1;
    const int64_t want = want_chains > 0 ? want_chains : (int64_t)rounds * 4 * std::max(1, s->num_cus) / waves_per_wg;
    const int cone = nst * nsteps;
    const int nstrips = (int)ws::fused_strips(s->kernel, g->W, cone, (int)elem_size(s->dtype), out_w);
    const bool col64 = s->dtype == WS_F64 && !ws::fused_pairs(s->kernel);
    const double kXClampCost = col64 ? kXClampCost64 : kXClampCostDef;
    const double kYClampCost = col64 ? kYClampCost64 : kYClampCostDef;
    struct Group {
        int unit;
        RowRange r;
        double wx;  // cost per row of the strip
        int n = 1;
        double frac = 0;
    };
    std::vector<Group> groups;
    double total = 0;
    for (int l = 0; l < g->L; ++l)
        for (int st = 0; st < nstrips; ++st)
            for (const RowRange& r : {A, B}) {
                if (r.rows() <= 0) continue;
                const ws::StripGeom sg = ws::fused_strip_geom(s->kernel, st, nstrips, g->W, cone, (int)elem_size(s->dtype), out_w);
                const bool xc = sg.o0 <= cone || sg.o1 + cone >= g->W;  // the kernel's xclamp test
                Group gr{l * nstrips + st, r, xc ? kXClampCost : 1.0};
                total += gr.wx * r.rows();
                groups.push_back(gr);
            }
    // chains per group in proportion to its cost (largest remainder), at least one, and none
    // shorter than min2 half cones (default 2 cones, the march's warm-up): a band of few rows --
    // an overlapped block's edge bands -- gets few long chains, not a chip's worth of stubs (a
    // thin slab's edge bands, the latency-critical path of its block, take chains of one cone)
    const int min_rows = std::max(1, min2 * cone / 2);
    auto cap = [&](const Group& gr) { return std::max(1, gr.r.rows() / min_rows); };
    // ... and none longer than a 32-bit buffer descriptor spans (the launcher's check: rows +
    // 2 cone + 48 rows of pitch below 2^31 bytes; C5's 16384-row strips at one chain per strip)
    const int64_t row_bytes = (int64_t)g->pitch * (int64_t)elem_size(s->dtype);
    // (nine tenths of it: the y-edge weights below lengthen the other chains of a group a little)
    const int64_t span_rows = 0x7fffffff / row_bytes - 2 * cone - 49;  // longest chain the launcher takes
    const int max_rows = (int)std::max<int64_t>(min_rows, span_rows * 9 / 10);
    auto floor_n = [&](const Group& gr) { return (gr.r.rows() + max_rows - 1) / max_rows; };
    int64_t assigned = 0;
    for (Group& gr : groups) {
        const double ideal = (double)want * gr.wx * gr.r.rows() / total;
        gr.n = (int)std::max(1.0, std::floor(ideal));
        gr.n = std::max(floor_n(gr), std::min(gr.n, cap(gr)));
        gr.frac = ideal - std::floor(ideal);
        assigned += gr.n;
    }
    std::vector<size_t> order(groups.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return groups[x].frac > groups[y].frac; });
    for (size_t i = 0; assigned < want && i < order.size(); ++i) {
        Group& gr = groups[order[i]];
        if (gr.n < cap(gr)) { ++gr.n; ++assigned; }
    }
    // rows of each group's chains: equal cost, the chains in a y edge's cone priced kYClampCost
    auto yclamped = [&](int y0, int y1) { return (g->top_clamp && y0 < cone) || (g->bot_clamp && y1 > g->H - cone); };
    std::vector<std::vector<ws::ChainSeg>> per(groups.size());
    int maxn = 0;
    auto split = [&](const Group& gr, int n) {
        const int rows = gr.r.rows();
        const bool top = yclamped(gr.r.y0, gr.r.y0 + 1), bot = yclamped(gr.r.y1 - 1, gr.r.y1);
        // weights of the first / last chain (y-clamped ones are dearer per row)
        std::vector<double> w(n, 1.0);
        if (top) w[0] = kYClampCost;
        if (bot) w[n - 1] = n == 1 ? std::max(w[n - 1], kYClampCost) : kYClampCost;
        double inv = 0;
        for (double x : w) inv += 1.0 / x;
        std::vector<ws::ChainSeg> out;
        int y = gr.r.y0;
        double acc = 0;
        for (int c = 0; c < n; ++c) {
            acc += (1.0 / w[c]) / inv * rows;
            int y1 = c == n - 1 ? gr.r.y1 : gr.r.y0 + (int)std::lround(acc);
            y1 = std::max(y1, y + 1);
            y1 = std::min(y1, gr.r.y1 - (n - 1 - c));  // leave a row for every later chain
            out.push_back(ws::ChainSeg{gr.unit, y, y1, 0});
            y = y1;
        }
        return out;
    };
    for (size_t gi = 0; gi < groups.size(); ++gi) {
        // the edge weights lengthen a group's other chains: one more chain until every chain
        // fits the descriptor span
        for (int n = groups[gi].n;; ++n) {
            per[gi] = split(groups[gi], n);
            bool fits = true;
            for (const ws::ChainSeg& cs : per[gi]) fits = fits && cs.y1 - cs.y0 <= span_rows;
            if (fits) break;
        }
        maxn = std::max(maxn, (int)per[gi].size());
    }
    // table order: chain position, then unit -- neighbouring strips at the same rows adjacent
    ws_sim::ChainTable t;
    std::copy(key, key + 12, t.key);
    std::vector<ws::ChainSeg> tab;
    for (int c = 0; c < maxn; ++c)
        for (size_t gi = 0; gi < groups.size(); ++gi)
            if (c < (int)per[gi].size()) {
                tab.push_back(per[gi][c]);
                t.max_rows = std::max(t.max_rows, per[gi][c].y1 - per[gi][c].y0);
            }
    t.n = (int32_t)tab.size();
    require(t.max_rows <= span_rows, WS_ERR_INVALID, "chain longer than a buffer descriptor spans");
    WS_HIP_CHECK(hipMalloc(&t.dev, tab.size() * sizeof(ws::ChainSeg)));
    WS_HIP_CHECK(hipMemcpy(t.dev, tab.data(), tab.size() * sizeof(ws::ChainSeg), hipMemcpyHostToDevice));
    s->chain_tables.push_back(t);
    return s->chain_tables.back();
}

// Launch the fused step kernel over the output rows A U B (segments of seg_rows rows, or the
// chain schedule when seg_rows encodes one: chain_rounds).
template <typename T>
int fused_launch(ws_sim* s, int nst, int nsteps, RowRange A, RowRange B, int seg_rows, hipStream_t st, ws_grid* in,
                 ws_grid* out, int want, int prio, int min2) {
    if (!st) st = s->stream;
    const int rounds = s->kernel == kKernLds ? 0 : chain_rounds(seg_rows);
    if (rounds == 0 && seg_rows <= 0) throw WsError(WS_ERR_INVALID, "bad segment rows");
    const int nA = rounds ? (A.rows() > 0) : (A.rows() + seg_rows - 1) / seg_rows;
    const int nB = rounds ? (B.rows() > 0) : (B.rows() + seg_rows - 1) / seg_rows;
    if (nA + nB <= 0) return 0;
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
    a.prio = prio;
    {
        const ws::Geom og = n->geom();
        const double out_mb = 3.0 * sizeof(T) * og.W * ((double)og.H + 2 * og.halo) * og.L / 1e6;
        a.cached = (WS_CACHED_PREC >> (sizeof(T) == 8 ? 1 : 0) & 1) && out_mb <= WS_CACHED_MAX_MB ? 1 : 0;
    }
    a.ga_y0 = A.y0; a.ga_y1 = A.y1; a.ga_n = nA;
    a.gb_y0 = B.y0; a.gb_y1 = B.y1;
    a.seg_n = nA + nB;
    // numerics (ws_fused.h): exact = the reference's evaluation order, bit-identical;
    // fast = re-associated with FMAs (isotropic spacing; otherwise exact)
    if (s->numerics == WS_NUMERICS_FAST) ws::prepare_fast(a);
    else a.sp_mode = ws::exact_sp_mode(a);
    if (rounds) {
        const ws_sim::ChainTable& t = chain_table<T>(s, nst, nsteps, A, B, rounds, a.out_w, a.sp_mode, want, min2);
        a.chains = t.dev;
        a.nchains = t.n;
        a.seg_rows = t.max_rows;  // the launcher's descriptor-span check
    }
    const ws::Geom g = c->geom();
    if (nsteps > 1 && s->kernel == kKernLds) throw WsError(WS_ERR_INVALID, "multi-step launch needs dppy, x2y, pc or pc2");
    if (s->kernel == kKernLds) WS_HIP_CHECK(ws::launch_fused_step<T>(nst, a, g, st));
    else WS_HIP_CHECK(ws::launch_fused_step_dppy<T>(s->kernel, nst, nsteps, a, g, st));
    ++s->last_launches;
    return rounds ? a.nchains : (nA + nB) * (int)s->strips(nst * nsteps) * g.L;
}

// Waves per SIMD the chosen fused variant's launches hold (hipOccupancy of the instantiation a
// tb-step launch runs; 0 for the per-stage kernels / fused_lds): what the VALU issue rate of the
// march depends on (bench.py prices VALU issue cycles by it).
template <typename T>
int fused_waves_per_simd(const ws_sim* s) {
    if (!use_fused(s) || s->kernel == kKernLds) return 0;
    ws::FusedArgs<T> a{};
    a.c_dt = (T)s->dt;
    a.sp1 = make_spacing<T>(s->slot[s->cur]->dx, s->slot[s->cur]->dy);
    a.sp2 = make_spacing<T>(to_prec(s->cfg.dx, s->dtype), to_prec(s->cfg.dy, s->dtype));
    if (s->numerics == WS_NUMERICS_FAST) ws::prepare_fast(a);
    else a.sp_mode = ws::exact_sp_mode(a);
    const int wgs = ws::fused_dppy_blocks_per_cu<T>(s->kernel, fused_stages(s), s->launch_tb(), a.sp_mode);
    return wgs * (ws::fused_split(s->kernel) ? 2 : 1) / 4;
}
template int fused_waves_per_simd<float>(const ws_sim*);
template int fused_waves_per_simd<double>(const ws_sim*);

// Phase 1 of a step: everything that does not need this step's halo rows.
//  * single domain: the whole step (fused or stage kernels);
//  * slab, fused: start the RCCL halo exchange on the comm stream (after the previous
//    step's output is complete) and run the interior segments meanwhile.
template <typename T>
void step_begin(ws_sim* s, int nsteps) {
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
        launch_stage<T>(s, ws::kAxpy, stage_args<T>(c, c, n, dt, s), c, 0, 6);
    } else if (method == WS_RK2) {
        launch_stage<T>(s, ws::kAxpy, stage_args<T>(c, c, s->tmpA, half, s), c, 0, 6);
        launch_stage<T>(s, ws::kAxpy, stage_args<T>(s->tmpA, c, n, dt, s), s->tmpA, 1, 9);
    } else {
        launch_stage<T>(s, ws::kAxpy, stage_args<T>(c, c, s->tmpA, half, s), c, 0, 6);
        auto a2 = stage_args<T>(s->tmpA, c, s->tmpB, half, s);
        a2.k2_u = (T*)s->K2->f[0]; a2.k2_v = (T*)s->K2->f[1]; a2.k2_h = (T*)s->K2->f[2];
        launch_stage<T>(s, ws::kAxpyStore, a2, s->tmpA, 1, 12);
        auto a3 = stage_args<T>(s->tmpB, c, s->tmpA, dt, s);
        a3.k2_u = (T*)s->K3->f[0]; a3.k2_v = (T*)s->K3->f[1]; a3.k2_h = (T*)s->K3->f[2];
        launch_stage<T>(s, ws::kAxpyStore, a3, s->tmpB, 2, 12);
        auto a4 = stage_args<T>(s->tmpA, c, n, dt / T(6.0f), s);  // `dt_ / 6.0f`
        a4.k2_u = (T*)s->K2->f[0]; a4.k2_v = (T*)s->K2->f[1]; a4.k2_h = (T*)s->K2->f[2];
        a4.k3_u = (const T*)s->K3->f[0]; a4.k3_v = (const T*)s->K3->f[1]; a4.k3_h = (const T*)s->K3->f[2];
        launch_stage<T>(s, ws::kRk4Final, a4, s->tmpA, 3, 15);
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
static void rotate(ws_sim* s, int nsteps);

template <typename T>
void step_end(ws_sim* s, int nsteps) {
    if (use_fused(s)) {
        s->timer.end(s->stream);
        s->block_pos = (s->block_pos + nsteps) % s->block;
    }
    rotate<T>(s, nsteps);
}

// After nsteps steps written into the next grid: the PE T / P update (nsteps updates in one
// pass) and the reference's grid rotation.
template <typename T>
static void rotate(ws_sim* s, int nsteps) {
    const T dt = (T)s->dt;
    ws_grid* c = s->slot[s->cur];
    ws_grid* n = s->slot[1 - s->cur];
    const bool pe = s->cfg.model == WS_MODEL_PRIMITIVE_EQUATIONS;
    if (pe && s->tp_lazy) {
        // inside run(): the drift is applied once, at the run's end (tp_flush)
        s->tp_steps += nsteps;
        s->tp_last = nsteps;
    } else if (pe) {
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
            if ((!pe || s->tp_lazy) && (f == WS_FIELD_T || f == WS_FIELD_P)) continue;  // (lazy: not written yet)
            std::swap(c->alloc[f], n->alloc[f]);
            std::swap(c->f[f], n->f[f]);
        }
        n->diag_pending = true;
    }
    s->slot[s->cur]->diag_pending = true;  // step() ends with calculateDiagnostics (:149)
}

// The PE T / P drift of a run, deferred by rotate() while tp_lazy: every launch of the run
// moved T / P from the current grid to the next (each step's `+ dt tendency` rounded in turn)
// and left the new values in the grid that ends current, the previous ones in the other --
// so after launches n_1 .. n_m (k steps) the current grid holds T0 + k updates and the other
// T0 + (k - n_m), T0 = the run's starting T (tp_src, which never moved: lazy launches swap no
// T / P storage). One pass computes both (launch_affine2's second output), on the aux stream.
template <typename T>
static void tp_flush(ws_sim* s) {
    s->tp_lazy = false;
    if (s->tp_steps <= 0) return;
    ws_grid* c = s->slot[s->cur];
    ws_grid* n = s->slot[1 - s->cur];
    const T dt = (T)s->dt;
    const T cT = dt * T(288.15f), cP = dt * T(1013.25f);
    WS_HIP_CHECK(ws::launch_affine2<T>((T*)c->f[WS_FIELD_T], (const T*)s->tp_src[0], cT, (T*)c->f[WS_FIELD_P],
                                       (const T*)s->tp_src[1], cP, c->geom(), s->aux_active ? s->aux : s->stream,
                                       (int)s->tp_steps, (T*)n->f[WS_FIELD_T], (T*)n->f[WS_FIELD_P],
                                       (int)(s->tp_steps - s->tp_last)));
    s->last_launches += 1;
    s->tp_steps = 0;
}

// The halo exchange of a slab: RCCL (ws_comm.cpp), or -- the communicator-less measurement
// slab of ws_sim_create_slab_emulated -- a device-side wait of emu_xfer_us in place of the
// transfer (around the pack / unpack kernels for the packed transport; the halo rows then
// hold the slab's own edge rows: timing only).
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

// The largest launch (8, 4, 2 or 1 steps) of at most `room` steps the tuned configuration
// allows: its steps per launch, and every step of a multi-step launch sees the config's
// spacing (the kernel's later stages use it).
static int launch_of(const ws_sim* s, int room) {
    if (room < 2 || !use_fused(s) || s->launch_tb() < 2 || !config_spacing(s)) return 1;
    for (int k : {8, 4, 2})
        if (k <= s->launch_tb() && k <= room &&
            ws::fused_tb_ok(s->kernel, k, fused_stages(s), (int)elem_size(s->dtype)))
            return k;
    return 1;
}

// Steps the next launch advances, of `remaining` (a slab's block bounds it too: one domain
// has no blocks).
int launch_steps(const ws_sim* s, int remaining) {
    return launch_of(s, s->nranks > 1 ? std::min(remaining, s->block - s->block_pos) : remaining);
}

// One time step on the stream (no host synchronisation).
template <typename T>
static void enqueue_steps(ws_sim* s, int nsteps) {
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
static std::vector<int> block_launches(const ws_sim* s, int steps) {
    std::vector<int> n;
    for (int left = steps; left > 0;) {
        const int k = launch_of(s, left);
        n.push_back(k);
        left -= k;
    }
    return n;
}

// launch j's interior rows and edge-band rows (two ranges; merged into A when they touch)
struct BandRows {
    RowRange interior, A, B;
};

static BandRows band_rows(const ws_grid* g, int C, int D) {
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
        // A thin slab (C2 at 8 GPUs: the edge bands are 18 % of the first launch's rows) runs its
        // edge bands in chains of one cone, at a raised wave priority, and its interior leaves
        // them their wave slots (overlap_interior): the edges and the exchange behind them are
        // the block's critical path. A deep slab (C5 at 8 GPUs: 5 %) keeps few long edge chains
        // and a full-chip interior -- there the short-chain edges took half the chip.
        if (j == 0) {
            const int e = r.A.rows() + r.B.rows(), i = r.interior.rows();
            s->ov_thin = chain_rounds(s->seg_rows(nst)) > 0 && 100 * e >= WS_THIN_PCT * (e + i);
        }
        // the tuned segment rows (one segment per band -- fewer warm-up rows, longer marches
        // -- measured no faster: the edges are on the critical path at 8 slabs)
        const int wgs = fused_launch<T>(s, nst, n[j], r.A, r.B, s->seg_rows(nst), s->edge, in, out, 0,
                                        s->ov_thin ? WS_EDGE_PRIO : 0, s->ov_thin ? WS_CHAIN_MIN2 : 4);
        if (j < 8) s->ov_edge_wgs[j] = wgs;
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
        // a chain schedule's interior leaves the wave slots the concurrent edge launch takes:
        // both launches are then resident together (an interior sized to fill the chip made the
        // edge bands wait for its waves to drain, and the edges are the block's critical path)
        const int seg = s->seg_rows(nst);
        int want = 0;
        if (s->ov_thin && chain_rounds(seg) > 0 && j < 8 && s->ov_edge_wgs[j] > 0) {
            const int slots = chain_rounds(seg) * 4 * std::max(1, s->num_cus) / (ws::fused_split(s->kernel) ? 2 : 1);
            want = std::max(slots / 2, slots - s->ov_edge_wgs[j]);
        }
        fused_launch<T>(s, nst, n[j], r.interior, {0, 0}, seg, s->stream, in, out, want);
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
static void overlap_block(ws_sim* s, int steps, bool first, bool last) {
    const int depth = s->block * fused_stages(s);
    if (first) slab_exchange(s, s->slot[s->cur], 3, depth, s->stream);
    overlap_begin(s, first);
    overlap_edges<T>(s, steps);
    if (!last) slab_exchange(s, s->slot[1 - s->cur], 3, depth, s->edge);  // the next block's halo, behind the edge bands
    overlap_interior<T>(s, steps);
}

template <typename T>
static double add_time(double t, double dt) {
    T tt = (T)t;
    tt += (T)dt;
    return (double)tt;
}

double advance_time(const ws_sim* s, double t) {
    return s->dtype == WS_F64 ? add_time<double>(t, s->dt) : add_time<float>(t, s->dt);
}

// Decide on the host how many of n steps run(n) takes (weather_simulation.cpp:77-90).
int plan_steps(const ws_sim* s, int n) {
    if (n <= 0) return 0;
    const bool f64 = s->dtype == WS_F64;
    const double max_time = to_prec(s->cfg.max_time, s->dtype);
    double t = s->time;
    int k = 0;
    while (k < n) {
        t = f64 ? add_time<double>(t, s->dt) : add_time<float>(t, s->dt);
        ++k;
        if (t >= max_time) break;
    }
    return k;
}

void run_steps(ws_sim* s, int k) {
    require(!s->in_group, WS_ERR_INVALID, "a slab of a group steps only with ws_group_run");
    set_device(s->device);
    if (!s->tuned && k > 0) autotune(s);
    if (k > 0 && s->overlap_mode == kOverlapAuto && s->xfer_us < 0) choose_slab_schedule(s);
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
    const bool pe_run = k > 0 && s->cfg.model == WS_MODEL_PRIMITIVE_EQUATIONS;
    s->aux_active = pe_run;
    if (s->aux_active) {
        if (!s->aux) {
            WS_HIP_CHECK(hipStreamCreateWithFlags(&s->aux, hipStreamNonBlocking));
            WS_HIP_CHECK(hipEventCreateWithFlags(&s->aux_in, hipEventDisableTiming));
            WS_HIP_CHECK(hipEventCreateWithFlags(&s->aux_out, hipEventDisableTiming));
        }
        WS_HIP_CHECK(hipEventRecord(s->aux_in, s->stream));
        WS_HIP_CHECK(hipStreamWaitEvent(s->aux, s->aux_in, 0));
    }
    if (pe_run) {
        // the T / P drift of the whole run in one pass at its end (tp_flush; on a throw, the
        // guard below applies the completed launches' drift before the error leaves run())
        s->tp_lazy = true;
        s->tp_steps = 0;
        s->tp_src[0] = s->slot[s->cur]->f[WS_FIELD_T];
        s->tp_src[1] = s->slot[s->cur]->f[WS_FIELD_P];
    }
    // A run that throws after some launches (a HIP / RCCL error) must not leave the T / P drift
    // pending: T / P would lag u, v, h, and a later flush would overwrite fields reset or set in
    // between. The guard flushes what the completed launches owe (normal exits flushed already)
    // and, like the normal exit, joins the aux stream back into the compute stream: the flush
    // runs on the aux stream, which ws_sim_synchronize, field reads and grid resets never wait on.
    struct TpGuard {
        ws_sim* s;
        ~TpGuard() {
            try {
                if (s->tp_lazy) {
                    if (s->dtype == WS_F64) tp_flush<double>(s);
                    else tp_flush<float>(s);
                }
            } catch (...) {
            }
            s->tp_lazy = false;
            s->tp_steps = 0;
            if (s->aux_active) {
                if (hipEventRecord(s->aux_out, s->aux) != hipSuccess ||
                    hipStreamWaitEvent(s->stream, s->aux_out, 0) != hipSuccess)
                    (void)hipStreamSynchronize(s->aux);  // (the join by events failed: drain it)
                s->aux_active = false;
            }
        }
    } tp_guard{s};
    // n steps from a block boundary on one schedule: stream-ordered launches, or the overlap
    // schedule's blocks (edge bands + exchange on the edge stream, interior on the compute stream)
    // (marks: events recorded on the compute stream after the first block and after the last)
    auto segment = [&](int n_steps, bool ovl, hipEvent_t mark0 = nullptr, hipEvent_t mark1 = nullptr) {
        if (n_steps <= 0) return;
        if (ovl) ensure_overlap_grids(s);
        s->block_pos = 0;
        for (int i = 0; i < n_steps;) {
            const int n = ovl ? std::min(s->block, n_steps - i) : launch_steps(s, n_steps - i);
            if (ovl) {
                if (s->dtype == WS_F64) overlap_block<double>(s, n, i == 0, i + n == n_steps);
                else overlap_block<float>(s, n, i == 0, i + n == n_steps);
            } else if (s->dtype == WS_F64) {
                enqueue_steps<double>(s, n);
            } else {
                enqueue_steps<float>(s, n);
            }
            for (int j = 0; j < n; ++j) {
                s->time = advance_time(s, s->time);
                s->step++;
            }
            if (s->fail_after >= 0 && s->last_launches >= s->fail_after) {  // ws_sim_inject_failure (tests)
                s->fail_after = -1;
                throw WsError(WS_ERR_DEVICE, "injected failure after a launch (ws_sim_inject_failure)");
            }
            const int prev = i;
            i += n;
            if (mark0 && prev < s->block && i >= s->block) WS_HIP_CHECK(hipEventRecord(mark0, s->stream));
        }
        if (mark1) WS_HIP_CHECK(hipEventRecord(mark1, s->stream));
        if (ovl) WS_HIP_CHECK(hipStreamWaitEvent(s->stream, s->ev_edge, 0));  // the last block's edge bands
    };
    // (the trial runs where the overlap schedule could: a fused slab with the configured spacing)
    const bool trial_ok = (s->nranks > 1 || s->comm) && use_fused(s) && config_spacing(s);
    if (k > 0 && s->overlap_trial && trial_ok && k >= 16 * s->block) {
        // the auto schedule's decision (choose_slab_schedule): four-block segments alternating
        // stream-ordered / overlapped / stream-ordered / overlapped, each timed on the compute
        // stream from the end of its first block to the end of its last: three block periods in
        // the steady state (a run's first overlapped block exchanges its halo before any interior
        // work, and first launches of new shapes, the overlap grids and chain tables are set up
        // in it). Over three periods the overlap's whole dependency cycle is inside the window --
        // interior k-1 -> edge bands k -> exchange -> interior k+1 -- so the exchange is charged
        // as far as the interior does not hide it. The better of the two samples per schedule is
        // compared, so a clock still ramping up favours neither. Both give the same bits, so
        // these are real steps of the run; the slower rank's times decide, identically on every
        // rank.
        auto timed = [&](bool ovl) {
            segment(4 * s->block, ovl, s->ev_trial[0], s->ev_trial[1]);
            WS_HIP_CHECK(hipEventSynchronize(s->ev_trial[1]));
            float ms = 0.f;
            WS_HIP_CHECK(hipEventElapsedTime(&ms, s->ev_trial[0], s->ev_trial[1]));
            return ms / 3.0;
        };
        double so = timed(false), ov = timed(true);
        so = std::min(so, timed(false));
        ov = std::min(ov, timed(true));
        if (s->comm && s->comm->nranks() > 1) {
            so = s->comm->allreduce_max(so, s->stream);
            ov = s->comm->allreduce_max(ov, s->stream);
        }
        s->trial_ms[0] = so;
        s->trial_ms[1] = ov;
        // a near-tie keeps the stream-ordered schedule (no cross-stream waits): the samples of
        // two schedules that cost the same differ by sync jitter, box to box
        s->overlap = ov < so * (1.0 - WS_OVERLAP_MARGIN);
        s->overlap_trial = false;
        segment(k - 16 * s->block, s->overlap && overlap_active(s));
    } else {
        segment(k, k > 0 && overlap_active(s));
    }
    if (s->tp_lazy) {
        if (s->dtype == WS_F64) tp_flush<double>(s);
        else tp_flush<float>(s);
    }
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

template int fused_launch<float>(ws_sim*, int, int, RowRange, RowRange, int, hipStream_t, ws_grid*, ws_grid*, int, int, int);
template int fused_launch<double>(ws_sim*, int, int, RowRange, RowRange, int, hipStream_t, ws_grid*, ws_grid*, int, int, int);
template void step_begin<float>(ws_sim*, int);
template void step_begin<double>(ws_sim*, int);
template void step_end<float>(ws_sim*, int);
template void step_end<double>(ws_sim*, int);
template void overlap_edges<float>(ws_sim*, int);
template void overlap_edges<double>(ws_sim*, int);
template void overlap_interior<float>(ws_sim*, int);
template void overlap_interior<double>(ws_sim*, int);

}  // namespace wsr
