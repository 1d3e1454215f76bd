// Host-side initial-condition generation (ws_initial_conditions.cpp).
#pragma once

#include <cstddef>
#include <string>
#include <vector>

namespace ws {

enum IcMask : unsigned { kU = 1, kV = 2, kH = 4, kP = 8, kT = 16, kQ = 32 };

// Fields of rows [y0, y0 + rows) of a global W x H grid (a y-slab; y0 = 0, rows = H for a
// whole grid). The IC formulas use the global W, H.
template <typename T>
struct IcFields {
    int W = 0, H = 0, y0 = 0, rows = 0;
    std::vector<T> u, v, h, p, t, q;
    unsigned wrote = 0;  // IcMask bits of the fields the IC wrote
    IcFields(int w, int global_h, int row0, int nrows) : W(w), H(global_h), y0(row0), rows(nrows) {
        const size_t n = (size_t)w * nrows;
        u.resize(n); v.resize(n); h.resize(n); p.resize(n); t.resize(n); q.resize(n);
    }
    int y1() const { return y0 + rows; }
    size_t idx(int x, int y) const { return (size_t)(y - y0) * W + x; }
    size_t n() const { return (size_t)W * rows; }
};

template <typename T>
bool compute_initial_condition(const std::string& name, const double* params, int nparams, const std::string& sparam,
                               IcFields<T>& f);

}  // namespace ws
