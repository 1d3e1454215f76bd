// Fused-kernel variant choice and slab schedule choice (internal interfaces: ws_sim.h).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>

#include "ws_sim.h"

namespace wsr {

// Pick the fused-kernel variant (and segment length) for this grid by timing each
// candidate on the real fields once, at the first run: all variants produce bit-identical
// results (each is the reference's arithmetic), they differ only in speed, and which is
// fastest depends on precision, integrator, width and level count. A candidate launch
// reads the current state and writes the next-state buffer, which the real step then
// overwrites, so tuning leaves no trace in the results.
template <typename T>
static void autotune_time(ws_sim* s) {
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
    const int fixed_kernel = s->kernel;
    // multi-step launches only where a run can use them (slab blocks of >= tb steps)
    for (int k : {kKernDppLdsY, kKernX2Y, kKernPc, kKernPc2, kKernLds})
      for (int tb : {1, 2, 4, 8}) {
        if (s->kernel_fixed && k != fixed_kernel) continue;  // pinned kernel: tune the rest for it
        if (tb > 1 && s->nranks > 1 && s->block < tb) continue;
        // (the split variants are two-step launches only: their one-step launches are dppy's /
        // x2y's; four steps: Euler / RK2 on the one-wave march, eight: Euler; ws::fused_tb_ok)
        if (k == kKernLds ? tb != 1 : !ws::fused_tb_ok(k, tb, nst, (int)elem_size(s->dtype))) continue;
        if (s->tb_fixed && k != kKernLds) {  // a pinned 4 means 2 where this kernel / integrator takes no 4
            int t = fixed_tb;
            while (t > 1 && !ws::fused_tb_ok(k, t, nst, (int)elem_size(s->dtype))) t /= 2;
            if (tb != t) continue;
        }
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
                const int wave_per_block = k == kKernLds ? 4 : ws::fused_split(k) ? 2 : 1;
                for (int64_t waves : {1024, 2048, 3072, 4096, 6144})
                    segs.push_back(s->seg_for_blocks(nst, waves / wave_per_block, 5 * nst));
                if (ws::fused_is_dppy(k)) {  // more waves per SIMD fit: shorter segments pay
                    for (int64_t waves : {8192, 12288}) segs.push_back(s->seg_for_blocks(nst, waves, 5 * nst));
                    // the chain schedule: 1, 2, 3, 4 or 6 chains (waves) per SIMD
                    for (int r : {1, 2, 3, 4, 6}) segs.push_back(seg_chains(r));
                }
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
    // (around the best candidate of the two fastest kernel variants: dppy and pc at C2 are within
    // a few % of each other, each at its own segment length)
    if (!s->seg_fixed) {
        std::vector<Cand> best2;
        for (const Cand& c : cands) {
            auto it = std::find_if(best2.begin(), best2.end(), [&](const Cand& b) { return b.kernel == c.kernel; });
            if (it == best2.end()) best2.push_back(c);
            else if (c.ms < it->ms) *it = c;
        }
        std::sort(best2.begin(), best2.end(), [](const Cand& x, const Cand& y) { return x.ms < y.ms; });
        if (best2.size() > 2) best2.resize(2);
        for (const Cand& b : best2)
            for (int d : {-16, -8, 8, 16}) {
                if (chain_rounds(b.seg) > 0) break;  // a chain schedule has no row neighbours
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
    // the new neighbours (ms = 0) sort first; keep them, the three fastest timed ones, and the
    // fastest of every other kernel variant (variants within a few % of each other -- dppy /
    // pc at C2 -- were decided by one short window's noise)
    size_t keep = 0;
    while (keep < top.size() && top[keep]->ms == 0.f) ++keep;
    if (top.size() > keep + 3) {
        std::vector<Cand*> rest(top.begin() + keep + 3, top.end());
        top.resize(keep + 3);
        for (Cand* c : rest)
            if (std::none_of(top.begin(), top.end(), [&](const Cand* t) { return t->kernel == c->kernel; }))
                top.push_back(c);
    }
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
    if (env_int("WS_AUTOTUNE", 1) >= 2)
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
    int32_t W, H, L, dtype, model, nst, numerics, top, bot, block, device;
    bool operator<(const TuneKey& o) const {
        return std::memcmp(this, &o, sizeof(TuneKey)) < 0;
    }
};
struct TuneChoice {
    int32_t kernel, seg, align, tb;
};
static std::mutex g_tune_mu;
static std::map<TuneKey, TuneChoice> g_tune_cache;
static bool g_tune_file_loaded = false;

static TuneKey tune_key(const ws_sim* s) {
    const ws_grid* g = s->slot[0];
    TuneKey k;
    std::memset(&k, 0, sizeof(k));
    k.W = g->W; k.H = g->H; k.L = g->L; k.dtype = s->dtype; k.model = s->cfg.model; k.nst = fused_stages(s);
    k.numerics = s->numerics; k.top = g->top_clamp; k.bot = g->bot_clamp; k.block = s->block;
    k.device = s->device;
    return k;
}

// The cache file: a version line, then one line of 15 integers per entry (the key, then the
// choice). Read line by line; a file without the version line (an older build's format), a line
// with any other field count or a choice out of range is ignored, never read across lines.
static constexpr const char* kTuneCacheVersion = "ws-tune-cache v2 W H L dtype model nst numerics top bot block "
                                                 "device kernel seg align tb";

static void tune_file_load_locked() {
    if (g_tune_file_loaded) return;
    g_tune_file_loaded = true;
    const char* path = std::getenv("WS_TUNE_CACHE");
    if (!path) return;
    FILE* f = std::fopen(path, "r");
    if (!f) return;
    char line[512];
    bool versioned = false;
    if (std::fgets(line, sizeof line, f)) {
        line[std::strcspn(line, "\r\n")] = 0;
        versioned = std::strcmp(line, kTuneCacheVersion) == 0;
    }
    while (versioned && std::fgets(line, sizeof line, f)) {
        TuneKey k;
        TuneChoice c;
        std::memset(&k, 0, sizeof(k));
        int used = 0;
        const int n = std::sscanf(line, "%d %d %d %d %d %d %d %d %d %d %d %d %d %d %d %n", &k.W, &k.H, &k.L, &k.dtype,
                                  &k.model, &k.nst, &k.numerics, &k.top, &k.bot, &k.block, &k.device, &c.kernel, &c.seg,
                                  &c.align, &c.tb, &used);
        if (n != 15 || line[used] != 0) continue;  // exactly 15 fields
        const bool kernel_ok = c.kernel == kKernLds || ws::fused_is_dppy(c.kernel);
        const bool tb_ok = c.kernel == kKernLds ? c.tb == 1
                                                : ws::fused_tb_ok(c.kernel, c.tb, k.nst, (int)elem_size(k.dtype));
        const bool seg_ok = (c.seg > 0 && c.seg <= k.H) ||
                            (ws::fused_is_dppy(c.kernel) && chain_rounds(c.seg) > 0 && chain_rounds(c.seg) <= kMaxChainRounds);
        if (kernel_ok && tb_ok && seg_ok && (c.align == 0 || c.align == 1) && k.W > 0 && k.H > 0 && k.L > 0)
            g_tune_cache[k] = c;
    }
    std::fclose(f);
}

static void tune_file_append_locked(const TuneKey& k, const TuneChoice& c) {
    const char* path = std::getenv("WS_TUNE_CACHE");
    if (!path) return;
    // a missing, empty or old-format file is (re)started with the version line
    bool fresh = true;
    if (FILE* r = std::fopen(path, "r")) {
        char line[512];
        if (std::fgets(line, sizeof line, r)) {
            line[std::strcspn(line, "\r\n")] = 0;
            fresh = std::strcmp(line, kTuneCacheVersion) != 0;
        }
        std::fclose(r);
    }
    if (FILE* f = std::fopen(path, fresh ? "w" : "a")) {
        if (fresh) std::fprintf(f, "%s\n", kTuneCacheVersion);
        std::fprintf(f, "%d %d %d %d %d %d %d %d %d %d %d %d %d %d %d\n", k.W, k.H, k.L, k.dtype, k.model, k.nst,
                     k.numerics, k.top, k.bot, k.block, k.device, c.kernel, c.seg, c.align, c.tb);
        std::fclose(f);
    }
}

// Pick the variant for this simulation: from the cache, or by timing (autotune_time). A slab
// of a multi-rank decomposition takes rank 0's choice (one broadcast), so every rank runs the
// same kernel and segment length and no rank runs behind on a different pick.
template <typename T>
static void autotune_t(ws_sim* s) {
    s->tuned = true;
    if (!use_fused(s)) return;
    const bool lead = !s->comm || s->comm->rank() == 0;
    if (lead && s->tune_free()) {
        const TuneKey key = tune_key(s);
        bool hit = false;
        {
            std::lock_guard<std::mutex> lk(g_tune_mu);
            tune_file_load_locked();
            auto it = g_tune_cache.find(key);
            if (it != g_tune_cache.end() && !s->kernel_fixed && !s->seg_fixed && !s->align_fixed && !s->tb_fixed) {
                s->kernel = it->second.kernel;
                s->seg_override = it->second.seg;
                s->align = it->second.align != 0;
                s->tb = it->second.tb;
                hit = true;
            }
        }
        if (!hit) {
            autotune_time<T>(s);
            if (!s->kernel_fixed && !s->seg_fixed && !s->align_fixed && !s->tb_fixed) {
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

void autotune(ws_sim* s) {
    if (s->dtype == WS_F64) autotune_t<double>(s);
    else autotune_t<float>(s);
}

// Overlap or stream-ordered slab blocks, decided by MEASURING both: the
// overlap schedule's edge bands cost extra stencil work (their warm-up rows) and two cross-stream
// waits per block, which hiding the exchange repays only when the exchange takes long enough --
// and where that break-even lies depends on the slab's rows, the kernel and the link. Here rank 0
// times the block-depth exchange of the current state (RCCL on the compute stream, one warm-up +
// the mean of three; reported by ws_sim_slab_exchange_us), and where the slabs have an interior
// to overlap (>= three block depths) the next run of >= sixteen blocks times each schedule's steady
// blocks (four-block segments, alternating, the last three blocks of each timed) and keeps the faster (run_steps, ws_schedule.cpp: the slowest rank's times decide,
// so every rank runs the same schedule).
void choose_slab_schedule(ws_sim* s) {
    const int nst = fused_stages(s);
    const int depth = s->block * nst;
    const int thin = s->cfg.grid_height / std::max(1, s->nranks);
    const bool room = use_fused(s) && thin >= 3 * depth;
    double us = 0.0;
    if (room && (s->comm || s->emu_xfer_us >= 0)) {
        hipEvent_t e0 = nullptr, e1 = nullptr;
        WS_HIP_CHECK(hipEventCreate(&e0));
        WS_HIP_CHECK(hipEventCreate(&e1));
        ws_grid* c = s->slot[s->cur];
        slab_exchange(s, c, 3, depth, s->stream);  // warm-up (RCCL connects lazily)
        WS_HIP_CHECK(hipEventRecord(e0, s->stream));
        for (int i = 0; i < 3; ++i) slab_exchange(s, c, 3, depth, s->stream);
        WS_HIP_CHECK(hipEventRecord(e1, s->stream));
        WS_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        WS_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        us = ms * 1000.0 / 3.0;
    }
    int32_t v[2] = {room ? 1 : 0, (int32_t)std::lround(us * 1000.0)};  // ns
    if (s->comm && s->comm->nranks() > 1) s->comm->broadcast_i32(v, 2, 0, s->stream);
    s->overlap = false;  // stream-ordered until the trial decides
    s->overlap_trial = v[0] != 0;
    if (s->overlap_trial)
        for (auto& e : s->ev_trial)
            if (!e) WS_HIP_CHECK(hipEventCreate(&e));
    s->xfer_us = v[1] / 1000.0;
}

}  // namespace wsr
