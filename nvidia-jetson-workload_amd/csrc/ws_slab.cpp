// Multi-GPU y-slabs (the reference has no distributed path) and the
// one-process slab group (internal interfaces: ws_sim.h).
//
// A slab is a ws_sim owning rows [row0, row0 + rows) of the global grid with an RCCL
// communicator (ws_comm.cpp) for its halo exchanges; ws_schedule.cpp steps it. The slab group
// runs N slabs of one grid in one process on one device with device copies as the transport:
// the same per-slab schedule, plan and kernels, so the decomposition is checked bitwise
// against one domain on a one-GPU box.
#include <algorithm>

#include "ws_sim.h"

using namespace wsr;

extern "C" {

int ws_comm_get_unique_id(uint8_t id[WS_COMM_ID_BYTES]) {
    return guarded([&] {
        require(id != nullptr, WS_ERR_INVALID, "null pointer");
        ws::SlabComm::unique_id(id);
    });
}

// One rank's slab: rows [row0, row0 + rows) of the global grid, `comm` its halo transport
// (RCCL), or none for the measurement slab (emulated transfer of xfer_us microseconds).
static void create_slab(const ws_config_t* cfg, int32_t rank, int32_t nranks, const uint8_t* id, double xfer_us,
                        ws_sim_t** out, int32_t* row0, int32_t* rows) {
    require(cfg && out, WS_ERR_INVALID, "null pointer");
    require(nranks >= 1 && rank >= 0 && rank < nranks, WS_ERR_INVALID, "bad rank / nranks");
    require(cfg->grid_height >= nranks, WS_ERR_INVALID, "fewer rows than ranks");
    int r0 = 0, nrows = 0;
    ws::slab_rows(cfg->grid_height, rank, nranks, &r0, &nrows);
    require(nranks == 1 || nrows >= 4, WS_ERR_INVALID, "a slab needs at least 4 rows per rank");
    set_device(cfg->device_id);
    // a 1-rank slab still gets its communicator: same code path as N>1 (the exchanges are
    // no-ops), so a 1-GPU run exercises the RCCL bootstrap
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
    if (!id) s->emu_xfer_us = xfer_us;
    *out = s;
    if (row0) *row0 = r0;
    if (rows) *rows = nrows;
}

int ws_sim_create_slab(const ws_config_t* cfg, int32_t rank, int32_t nranks, const uint8_t id[WS_COMM_ID_BYTES],
                       ws_sim_t** out, int32_t* row0, int32_t* rows) {
    return guarded([&] {
        require(id != nullptr, WS_ERR_INVALID, "null communicator id (ws_sim_create_slab_emulated is the "
                                               "communicator-less measurement slab)");
        create_slab(cfg, rank, nranks, id, -1.0, out, row0, rows);
    });
}

int ws_sim_create_slab_emulated(const ws_config_t* cfg, int32_t rank, int32_t nranks, double xfer_us,
                                ws_sim_t** out, int32_t* row0, int32_t* rows) {
    return guarded([&] {
        require(nranks >= 2, WS_ERR_INVALID, "an emulated slab needs nranks >= 2");
        require(xfer_us >= 0.0 && std::isfinite(xfer_us), WS_ERR_INVALID, "xfer_us must be finite and >= 0");
        create_slab(cfg, rank, nranks, nullptr, xfer_us, out, row0, rows);
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

int ws_sim_slab_schedule(const ws_sim_t* s, int32_t* block, int32_t* overlap) {
    return guarded([&] {
        require(s != nullptr && block != nullptr && overlap != nullptr, WS_ERR_INVALID, "null pointer");
        *block = s->block;
        *overlap = overlap_active(s) ? 1 : 0;
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

int ws_sim_set_slab_schedule(ws_sim_t* s, int32_t block, int32_t overlap) {
    return guarded([&] {
        require(s != nullptr, WS_ERR_INVALID, "null sim");
        require(overlap >= WS_OVERLAP_OFF && overlap <= WS_OVERLAP_AUTO, WS_ERR_INVALID,
                "overlap must be WS_OVERLAP_OFF, WS_OVERLAP_ON or WS_OVERLAP_AUTO");
        require(s->nranks > 1 || s->comm || block <= 1, WS_ERR_INVALID, "a whole domain has no slab blocks");
        if (block > 0) {
            const int nst = fused_stages(s);
            const int thin = s->cfg.grid_height / std::max(1, s->nranks);
            require(block * nst <= std::min(ws::kHalo, thin), WS_ERR_INVALID,
                    "block x stages exceeds the halo rows or the thinnest slab");
            if (block != s->block && s->tune_free()) s->tuned = env_int("WS_AUTOTUNE", 1) == 0;  // re-rank
            s->block = block;
        }
        s->overlap_mode = overlap;
        s->overlap = overlap == WS_OVERLAP_ON;
        s->xfer_us = -1.0;  // auto: measured again at the next run
        s->overlap_trial = false;
        s->trial_ms[0] = s->trial_ms[1] = -1.0;
    });
}

int ws_sim_slab_exchange_us(const ws_sim_t* s, double* us) {
    return guarded([&] {
        require(s != nullptr && us != nullptr, WS_ERR_INVALID, "null pointer");
        *us = s->xfer_us;
    });
}

int ws_sim_slab_trial_ms(const ws_sim_t* s, double* ms) {
    return guarded([&] {
        require(s != nullptr && ms != nullptr, WS_ERR_INVALID, "null pointer");
        ms[0] = s->trial_ms[0];
        ms[1] = s->trial_ms[1];
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

namespace wsr {

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

// The auto schedule in a group: overlap where every slab has an interior (there is no
// transfer to measure: the device copies stand in for RCCL).
void group_auto_schedule(ws_group* gr) {
    for (ws_sim* s : gr->slabs)
        if (s->overlap_mode == kOverlapAuto)
            s->overlap = gr->slabs.size() > 1 && use_fused(s) &&
                         s->cfg.grid_height / (int)gr->slabs.size() >= 3 * s->block * fused_stages(s);
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

// After field writes outside run() (initial conditions, setters): every slab's one-row u, v
// halo from its neighbours, so diagnostics read next see the neighbours' current rows at the
// seams (run() refreshes it at its end, see run_steps)
void group_diag_halo(ws_group* gr) {
    set_device(gr->device);
    group_exchange(gr, 2, 1);
    for (ws_sim* s : gr->slabs) s->slot[s->cur]->diag_pending = true;
    WS_HIP_CHECK(hipStreamSynchronize(gr->stream));
}

}  // namespace wsr

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
            group_auto_schedule(gr);
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
            autotune(s0);
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
        group_auto_schedule(gr);
        bool ovl = k > 0;  // every slab must agree
        for (ws_sim* s : gr->slabs) ovl = ovl && overlap_active(s);
        if (ovl)
            for (ws_sim* s : gr->slabs) ensure_overlap_grids(s);
        for (int i = 0; i < k;) {
            int n = 8;  // every slab must agree (they share the block position and the choice)
            for (ws_sim* s : gr->slabs) n = std::min(n, launch_steps(s, k - i));
            if (ovl) n = std::min(s0->block, k - i);
            if (ovl && s0->dtype == WS_F64) group_overlap_block<double>(gr, n, i == 0, i + n == k);
            else if (ovl) group_overlap_block<float>(gr, n, i == 0, i + n == k);
            else if (s0->dtype == WS_F64) group_step<double>(gr, n);
            else group_step<float>(gr, n);
            for (ws_sim* s : gr->slabs)
                for (int j = 0; j < n; ++j) {
                    s->time = advance_time(s, s->time);
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
