// Multi-GPU simulation in ONE process ("a single process ... that fits the
// single-object Python API"; the reference's simulation object takes one device,
// weather_sim.hpp:180, and has no distributed path at all).
//
// ws_multi_create(cfg, devices, n): the y-slab decomposition of cfg's global grid, slab r on
// devices[r]. Distinct devices: every slab is a full rank of the RCCL decomposition
// (ws_slab.cpp create_slab: its own communicator, streams, autotune broadcast, exchange plan
// and overlap schedule), driven by a host thread of its own that keeps that device current.
// Every collective call (run, step, CFL) is posted to all threads at once, so each thread runs
// exactly the code a process-per-GPU rank runs (torchrun + ws_sim_create_slab), RCCL included.
// All devices equal: the slabs share that device and a ws_group (device-copy halos) runs them.
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>

#include "ws_sim.h"

using namespace wsr;

struct ws_multi {
    std::vector<int> devices;
    std::vector<ws_sim*> slabs;
    ws_group_t* group = nullptr;  // every device the same: the one-device slab group
    // one worker thread per slab (distinct devices)
    std::vector<std::thread> workers;
    std::mutex m;
    std::condition_variable cv_go, cv_done;
    std::function<int(int)> task;
    uint64_t gen = 0;
    int pending = 0;
    bool stop = false;
    std::vector<int> status;
    std::vector<std::string> errors;
};

namespace {

void worker_main(ws_multi* mu, int r) {
    uint64_t seen = 0;
    const bool dev_ok = hipSetDevice(mu->devices[r]) == hipSuccess;
    for (;;) {
        std::function<int(int)> f;
        {
            std::unique_lock<std::mutex> l(mu->m);
            mu->cv_go.wait(l, [&] { return mu->stop || mu->gen != seen; });
            if (mu->stop) return;
            seen = mu->gen;
            f = mu->task;
        }
        int st = WS_ERR_DEVICE;
        std::string err = "hipSetDevice failed on the worker thread";
        if (dev_ok) {
            st = f(r);
            err = st == WS_OK ? std::string() : std::string(ws_last_error());
        }
        std::lock_guard<std::mutex> l(mu->m);
        mu->status[r] = st;
        mu->errors[r] = err;
        if (--mu->pending == 0) mu->cv_done.notify_all();
    }
}

// f(r) on every slab's thread at once; the first failing rank's status and message are
// rethrown on the caller's thread.
void run_all(ws_multi* mu, std::function<int(int)> f) {
    const int n = (int)mu->workers.size();
    std::unique_lock<std::mutex> l(mu->m);
    mu->task = std::move(f);
    mu->status.assign(n, WS_OK);
    mu->errors.assign(n, std::string());
    mu->pending = n;
    ++mu->gen;
    mu->cv_go.notify_all();
    mu->cv_done.wait(l, [&] { return mu->pending == 0; });
    for (int r = 0; r < n; ++r)
        if (mu->status[r] != WS_OK) throw WsError(mu->status[r], "rank " + std::to_string(r) + ": " + mu->errors[r]);
}

void stop_workers(ws_multi* mu) {
    {
        std::lock_guard<std::mutex> l(mu->m);
        mu->stop = true;
    }
    mu->cv_go.notify_all();
    for (std::thread& t : mu->workers)
        if (t.joinable()) t.join();
    mu->workers.clear();
}

void destroy(ws_multi* mu) {
    if (mu->group) {
        (void)ws_group_destroy(mu->group);
    } else if (!mu->workers.empty()) {
        // each slab is freed on its own thread (its device current; ncclCommDestroy per rank)
        try {
            run_all(mu, [mu](int r) {
                return guarded([&] {
                    if (mu->slabs[r]) sim_free(mu->slabs[r]);
                    mu->slabs[r] = nullptr;
                });
            });
        } catch (...) {
        }
        stop_workers(mu);
    }
    delete mu;
}

ws_multi* checked(ws_multi_t* m) {
    require(m != nullptr, WS_ERR_INVALID, "null multi-GPU simulation");
    return m;
}

// Steps run_until(max_time) asks for (weather_simulation.cpp:105-115, in scalar_t): 0 when
// max_time <= t, else int((max_time - t) / dt) + 1 (before run()'s own max_time cap).
int until_request(const ws_sim* s, double max_time) {
    if (s->dtype == WS_F64) {
        const double mt = max_time, t = s->time;
        return mt <= t ? 0 : (int)((mt - t) / s->dt) + 1;
    }
    const float mt = (float)max_time, t = (float)s->time;
    return mt <= t ? 0 : (int)((mt - t) / (float)s->dt) + 1;
}

}  // namespace

extern "C" {

int ws_multi_create(const ws_config_t* cfg, const int32_t* devices, int32_t ndevices, ws_multi_t** out) {
    return guarded([&] {
        require(cfg && devices && out, WS_ERR_INVALID, "null pointer");
        require(ndevices >= 1, WS_ERR_INVALID, "need at least one device");
        require(cfg->grid_height >= 4 * ndevices, WS_ERR_INVALID, "a slab needs at least 4 rows per device");
        const int nd = device_count();
        require(nd > 0, WS_ERR_DEVICE, "no HIP device available (MI355X build has no CPU path)");
        bool same = true;
        for (int r = 0; r < ndevices; ++r) {
            require(devices[r] >= 0 && devices[r] < nd, WS_ERR_DEVICE, "device id out of range");
            same = same && devices[r] == devices[0];
            for (int q = 0; q < r; ++q)
                require(ndevices == 1 || same || devices[q] != devices[r], WS_ERR_INVALID,
                        "devices must be all distinct (one slab per GPU, RCCL) or all equal (slabs sharing one GPU)");
        }
        ws_multi* mu = new ws_multi;
        mu->devices.assign(devices, devices + ndevices);
        mu->slabs.assign(ndevices, nullptr);
        if (same && ndevices > 1) {
            ws_config_t c = *cfg;
            c.device_id = devices[0];
            const int st = ws_group_create(&c, ndevices, &mu->group);
            if (st != WS_OK) {
                const std::string msg = ws_last_error();
                delete mu;
                throw WsError(st, msg);
            }
            for (int r = 0; r < ndevices; ++r) (void)ws_group_slab(mu->group, r, &mu->slabs[r], nullptr, nullptr);
            *out = mu;
            return;
        }
        // every device is made current once on the caller's thread first: a rank whose device
        // fails on its worker thread would return before joining the communicator, and the
        // other ranks would wait in ncclCommInitRank for it forever. (What create_slab checks
        // before the join -- rank, rows, config -- is the same on every rank, so it fails on
        // all of them alike; after the join a failing rank cannot block the others.)
        for (int r = 0; r < ndevices; ++r) set_device(devices[r]);
        try {
            uint8_t id[WS_COMM_ID_BYTES];
            set_device(devices[0]);
            ws::SlabComm::unique_id(id);
            for (int r = 0; r < ndevices; ++r) mu->workers.emplace_back(worker_main, mu, r);
            // every rank joins the communicator at once (ncclCommInitRank blocks until all have)
            run_all(mu, [&](int r) {
                ws_config_t c = *cfg;
                c.device_id = mu->devices[r];
                return ws_sim_create_slab(&c, r, ndevices, id, &mu->slabs[r], nullptr, nullptr);
            });
        } catch (...) {
            destroy(mu);
            throw;
        }
        *out = mu;
    });
}

int ws_multi_destroy(ws_multi_t* m) {
    return guarded([&] {
        if (m) destroy(m);
    });
}

int ws_multi_size(const ws_multi_t* m, int32_t* nslabs, int32_t* shared_device) {
    return guarded([&] {
        require(m != nullptr && nslabs != nullptr, WS_ERR_INVALID, "null pointer");
        *nslabs = (int32_t)m->slabs.size();
        if (shared_device) *shared_device = m->group ? 1 : 0;
    });
}

int ws_multi_slab(ws_multi_t* m, int32_t rank, ws_sim_t** sim, int32_t* row0, int32_t* rows) {
    return guarded([&] {
        ws_multi* mu = checked(m);
        require(sim && rank >= 0 && rank < (int)mu->slabs.size(), WS_ERR_INVALID, "bad argument");
        ws_sim* s = mu->slabs[rank];
        *sim = s;
        if (row0) *row0 = s->row0;
        if (rows) *rows = s->slot[0]->H;
    });
}

// run(n) / step() / run_until(T) of the whole decomposition (ws_sim_run semantics per slab;
// every slab takes the same steps)
static void multi_run(ws_multi* mu, int n, int32_t* taken) {
    if (mu->group) {
        int32_t k = 0;
        const int st = ws_group_run(mu->group, n, &k);
        if (st != WS_OK) throw WsError(st, ws_last_error());
        if (taken) *taken = k;
        return;
    }
    std::vector<int32_t> k(mu->slabs.size(), 0);
    run_all(mu, [&](int r) { return ws_sim_run(mu->slabs[r], n, &k[r]); });
    for (int32_t x : k) require(x == k[0], WS_ERR_COMM, "slabs took different step counts");
    if (taken) *taken = k[0];
}

int ws_multi_run(ws_multi_t* m, int32_t num_steps, int32_t* steps_taken) {
    return guarded([&] {
        ws_multi* mu = checked(m);
        if (steps_taken) *steps_taken = 0;
        if (num_steps > 0) multi_run(mu, num_steps, steps_taken);
    });
}

int ws_multi_step(ws_multi_t* m) {
    // run(1) == step(): run() always takes its first step (weather_simulation.cpp:68-103)
    return guarded([&] { multi_run(checked(m), 1, nullptr); });
}

int ws_multi_run_until(ws_multi_t* m, double max_time, int32_t* steps_taken) {
    return guarded([&] {
        ws_multi* mu = checked(m);
        const int n = until_request(mu->slabs[0], max_time);
        if (steps_taken) *steps_taken = 0;
        if (n > 0) multi_run(mu, n, steps_taken);
    });
}

int ws_multi_cfl(ws_multi_t* m, double* cfl, double* per_level, int32_t nlevels, double* ms) {
    return guarded([&] {
        ws_multi* mu = checked(m);
        require(cfl != nullptr, WS_ERR_INVALID, "null pointer");
        const int n = (int)mu->slabs.size();
        const int L = mu->slabs[0]->slot[0]->L;
        require(per_level == nullptr || nlevels >= L, WS_ERR_INVALID, "per_level needs num_levels entries");
        std::vector<double> c(n, 0.0), t(n, 0.0), lv((size_t)n * L, 0.0);
        if (mu->group) {  // no communicator: each slab's maxima, combined here
            for (int r = 0; r < n; ++r) {
                const int st = ws_sim_cfl(mu->slabs[r], &c[r], &lv[(size_t)r * L], L, &t[r]);
                if (st != WS_OK) throw WsError(st, ws_last_error());
            }
        } else {  // a collective: every rank's ws_sim_cfl max-reduces over RCCL
            run_all(mu, [&](int r) { return ws_sim_cfl(mu->slabs[r], &c[r], &lv[(size_t)r * L], L, &t[r]); });
        }
        double best = c[0], tm = t[0];
        for (int r = 1; r < n; ++r) {
            // NaN (a broken state) wins, as in the device reduction's bit ordering
            if (std::isnan(c[r]) || c[r] > best) best = c[r];
            tm = std::max(tm, t[r]);
        }
        *cfl = best;
        if (per_level)
            for (int l = 0; l < L; ++l) {
                double v = lv[l];
                for (int r = 1; r < n; ++r)
                    if (std::isnan(lv[(size_t)r * L + l]) || lv[(size_t)r * L + l] > v) v = lv[(size_t)r * L + l];
                per_level[l] = v;
            }
        if (ms) *ms = tm;
    });
}

int ws_multi_exchange_diag_halo(ws_multi_t* m) {
    return guarded([&] {
        ws_multi* mu = checked(m);
        if (mu->group) {
            group_diag_halo(mu->group);
            return;
        }
        run_all(mu, [mu](int r) {
            return guarded([&] {
                ws_sim* s = mu->slabs[r];
                set_device(s->device);
                ws_grid* c = s->slot[s->cur];
                if (s->comm) s->comm->exchange(c->f, 2, (int)elem_size(s->dtype), c->geom(), 1, s->stream);
                c->diag_pending = true;
                WS_HIP_CHECK(hipStreamSynchronize(s->stream));
            });
        });
    });
}

int ws_multi_synchronize(ws_multi_t* m) {
    return guarded([&] {
        ws_multi* mu = checked(m);
        for (ws_sim* s : mu->slabs) {
            const int st = ws_sim_synchronize(s);
            if (st != WS_OK) throw WsError(st, ws_last_error());
        }
    });
}

}  // extern "C"
