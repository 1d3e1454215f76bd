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
        used_ = 0;
        pending_.clear();
    }
    void begin(int kind, double bytes, hipStream_t s) {
        if (!on_) return;
        hipEvent_t e = get();
        (void)hipEventRecord(e, s);
        pending_.push_back({kind, bytes, e, nullptr});
    }
    void end(hipStream_t s) {
        if (!on_) return;
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
    std::vector<hipEvent_t> pool_;
    size_t used_ = 0;
    std::vector<Pending> pending_;
    Stat stats_[kKinds];
};

}  // namespace ws
