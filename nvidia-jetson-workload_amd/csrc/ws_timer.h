// Per-kernel device timing with HIP events on the launching stream (opt-in; bench.py
// turns it on for the timed region so the roofline figure comes from live launches).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace ws {

class KernelTimer {
public:
    static constexpr int kKinds = 8;
    struct Stat {
        int64_t launches = 0;
        double total_ms = 0.0;
        double bytes_per_launch = 0.0;  // algorithmic bytes
    };

    ~KernelTimer() {
        for (hipEvent_t e : pool_) (void)hipEventDestroy(e);
    }
    void enable(bool on) { on_ = on; }
    // pre-create events for n timed launches (hipEventCreate inside a timed run would
    // stall the host between launches)
    void reserve(size_t n) {
        while (pool_.size() < 2 * n) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) break;
            pool_.push_back(e);
        }
    }
    bool enabled() const { return on_; }
    void reset() {
        for (auto& s : stats_) s = Stat{};
        for (auto& n : seen_) n = 0;
        used_ = 0;
        pending_.clear();
    }
    void begin(int kind, double bytes, hipStream_t s) {
        if (!on_ || suspended_) return;
        if (period_ > 1 && (seen_[kind]++ % period_) != 0) return;  // sampled launches only
        hipEvent_t e = get();
        (void)hipEventRecord(e, s);
        pending_.push_back({kind, bytes, e, nullptr});
    }
    void end(hipStream_t s) {
        if (!on_ || suspended_ || pending_.empty() || pending_.back().e1) return;
        hipEvent_t e = get();
        (void)hipEventRecord(e, s);
        pending_.back().e1 = e;
    }
    // after the stream has been synchronised
    void collect() {
        for (auto& p : pending_) {
            float ms = 0.f;
            if (p.e1 && hipEventElapsedTime(&ms, p.e0, p.e1) == hipSuccess) {
                Stat& st = stats_[p.kind];
                st.launches++;
                st.total_ms += ms;
                st.bytes_per_launch = p.bytes;
            }
        }
        pending_.clear();
        used_ = 0;
    }
    // Whole-run attribution: `launches` back-to-back launches of one kernel were the only
    // work on the stream between two events `ms` apart (per-launch events would put two
    // timestamp packets between consecutive kernels of the run they measure).
    void add_span(int kind, double bytes, int64_t launches, double ms) {
        if (!on_ || launches <= 0) return;
        Stat& st = stats_[kind];
        st.launches += launches;
        st.total_ms += ms;
        st.bytes_per_launch = bytes;
    }
    // suspend per-launch events (begin/end become no-ops) while a span is measured
    void suspend(bool off) { suspended_ = off; }
    // time one launch in `p` per kind (every launch: 1); the mean over the sampled launches
    // stands for all of them, and the other launches run without timestamp packets
    void sample_period(int p) { period_ = p > 1 ? p : 1; }
    const Stat& stat(int kind) const { return stats_[kind]; }

private:
    struct Pending {
        int kind;
        double bytes;
        hipEvent_t e0, e1;
    };
    hipEvent_t get() {
        if (used_ == pool_.size()) {
            hipEvent_t e;
            (void)hipEventCreate(&e);
            pool_.push_back(e);
        }
        return pool_[used_++];
    }
    bool on_ = false;
    bool suspended_ = false;
    int period_ = 1;
    int64_t seen_[kKinds] = {};
    std::vector<hipEvent_t> pool_;
    size_t used_ = 0;
    std::vector<Pending> pending_;
    Stat stats_[kKinds];
};

}  // namespace ws
