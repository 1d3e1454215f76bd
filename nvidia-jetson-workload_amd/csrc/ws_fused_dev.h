// Device helpers shared by the fused step kernels (ws_fused.hip, ws_fused_dppy_kernel.h):
// buffer-descriptor memory access, DPP lane shifts, and the SWE tendency
// written once for scalar and 2-wide (ext_vector) cell values, per spacing / numerics mode.
#pragma once

#include "ws_fused.h"

namespace ws {
namespace dev {

// ---- buffer descriptors: wave-uniform base (SGPRs) + 32-bit per-lane voffset ----------
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

using U2 = unsigned int __attribute__((ext_vector_type(2)));
using U4 = unsigned int __attribute__((ext_vector_type(4)));
// cache policy bit of the output stores: nontemporal (streamed output; cached stores measured
// -5 % at C3 and +3 % at C2)
constexpr int kNT = 2;
constexpr uint32_t kDropped = 0x80000000u;  // voffset past every descriptor's range: op dropped

// V is any 4-, 8- or 16-byte value type (float, double, float2, double2)
template <typename V>
__device__ __forceinline__ V buf_load(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    if constexpr (sizeof(V) == 16)
        return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0));
    else if constexpr (sizeof(V) == 8)
        return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0));
    else
        return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0));
}
template <typename V, int POL = kNT>
__device__ __forceinline__ void buf_store_nt(V v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    // 16-byte stores take the row offset in voffset, soffset = 0: a dwordx4 store's data
    // VGPRs rewritten by the next VALU instruction need one wait state, and the compiler only
    // inserts it when soffset is not a register -- with an SGPR soffset it scheduled
    // `v_add v0, ...` straight after `buffer_store_dwordx4 v[0:3], ..., s10` and corrupted
    // the pair's first element (found on gfx950 at large grids). kDropped + soff stays past
    // every range (soff < 2^31), so dropped stores stay dropped.
    if constexpr (sizeof(V) == 16)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(U4, v), r, (int)(voff + soff), 0, POL);
    else if constexpr (sizeof(V) == 8)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(U2, v), r, (int)voff, (int)soff, POL);
    else
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, (int)voff, (int)soff, POL);
}

// LDS-DMA: 16 bytes per lane from the buffer into LDS at lds + 16 * lane (wave-uniform base;
// buffer_load_dwordx4 ... lds). Completion is counted by vmcnt; the compiler does not order
// later LDS reads after it, callers wait explicitly. (A device function, not a lambda: the
// builtin inside a kernel-local lambda silently drops the kernel's host launch stub.)
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t voff) {
    typedef __attribute__((address_space(3))) void* lds_ptr;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr)lds, 16, (int)voff, 0, 0, 0);
}

// ---- DPP lane shifts -------------------------------------------------------------------
// lane i <- lane i-1 (wave_shr:1) / lane i <- lane i+1 (wave_shl:1). Lanes without a source
// read 0 (bound_ctrl): a strip's edge lanes, whose results lie in the discarded margin.
// (Keeping the lane's own value instead costs a v_mov per shift to pre-load the destination.)
__device__ __forceinline__ int shr1(int v) { return __builtin_amdgcn_mov_dpp(v, 0x138, 0xF, 0xF, true); }
__device__ __forceinline__ int shl1(int v) { return __builtin_amdgcn_mov_dpp(v, 0x130, 0xF, 0xF, true); }

__device__ __forceinline__ float from_left(float v) { return __builtin_bit_cast(float, shr1(__builtin_bit_cast(int, v))); }
__device__ __forceinline__ float from_right(float v) { return __builtin_bit_cast(float, shl1(__builtin_bit_cast(int, v))); }
__device__ __forceinline__ double from_left(double v) {
    const U2 b = __builtin_bit_cast(U2, v);
    U2 o;
    o.x = (unsigned)shr1((int)b.x);
    o.y = (unsigned)shr1((int)b.y);
    return __builtin_bit_cast(double, o);
}
__device__ __forceinline__ double from_right(double v) {
    const U2 b = __builtin_bit_cast(U2, v);
    U2 o;
    o.x = (unsigned)shl1((int)b.x);
    o.y = (unsigned)shl1((int)b.y);
    return __builtin_bit_cast(double, o);
}

// ---- the SWE tendency (weather_simulation.cpp:521-537), same evaluation order ---------
// VT is T or a 2-wide ext_vector of T: every operation below is element-wise IEEE (the
// build has -ffp-contract=off), so each element gets exactly the reference's arithmetic.
template <typename VT>
struct V3 {
    VT u, v, h;
};

// Central difference, per spacing mode (ws_fused.h): the reference's (ar - al) / (2.0f * d);
// the same times the exact reciprocal when 2d is a power of two; or, for fast numerics, the
// raw difference (the 1/(2d) factor rides on the constants).
template <int MODE, typename VT, typename T>
__device__ __forceinline__ VT cdiff(VT ar, VT al, T two_d, T inv) {
    if constexpr (MODE >= kSpFast) return ar - al;
    else if constexpr (MODE == kSpMul) return (ar - al) * inv;  // exact: inv is a power of two
    else return (ar - al) / two_d;
}

// fused multiply-add a * b + c, element-wise for ext_vector values (one rounding)
template <typename VT>
__device__ __forceinline__ VT fmadd(VT a, VT b, VT c) {
    return __builtin_elementwise_fma(a, b, c);
}

// the tendency from the cell (c), its x-derivatives X = (u_x, v_x, h_x) (cdiff of its right
// and left neighbours) and its top / bottom neighbours: the x-derivatives depend only on the
// cell's row, so a march may form them ahead of the rest (ws_fused_dppy_kernel.h)
template <int MODE, typename VT, typename T>
__device__ __forceinline__ V3<VT> tend_x(const V3<VT>& c, const V3<VT>& X, const V3<VT>& t, const V3<VT>& b,
                                         const Spacing<T>& sp, T g, T f) {
    const VT u_x = X.u;
    const VT u_y = cdiff<MODE>(b.u, t.u, sp.two_dy, sp.inv2dy);
    const VT v_x = X.v;
    const VT v_y = cdiff<MODE>(b.v, t.v, sp.two_dy, sp.inv2dy);
    const VT h_x = X.h;
    const VT h_y = cdiff<MODE>(b.h, t.h, sp.two_dy, sp.inv2dy);
    V3<VT> k;
    if constexpr (MODE >= kSpFast) {
        // fast numerics: k / s = -u D_x u - v D_y u - g D_x h + (f / s) v, ... (ws_fused.h)
        const VT ng = (VT)(-g);
        k.u = fmadd(-c.v, u_y, fmadd(ng, h_x, -c.u * u_x));
        k.v = fmadd(-c.v, v_y, fmadd(ng, h_y, -c.u * v_x));
        k.h = fmadd(-c.v, h_y, fmadd(-c.u, h_x, -c.h * (u_x + v_y)));
        if constexpr (MODE == kSpFast) {
            k.u = fmadd((VT)f, c.v, k.u);
            k.v = fmadd((VT)(-f), c.u, k.v);
        }
    } else {
        // the reference's order (weather_simulation.cpp:535-537); no contraction in this build
        k.u = -c.u * u_x - c.v * u_y - g * h_x + f * c.v;
        k.v = -c.u * v_x - c.v * v_y - g * h_y - f * c.u;
        k.h = -c.h * (u_x + v_y) - c.u * h_x - c.v * h_y;
    }
    return k;
}

// x-derivatives (u_x, v_x, h_x) from the left / right neighbours
template <int MODE, typename VT, typename T>
__device__ __forceinline__ V3<VT> xdiffs(const V3<VT>& l, const V3<VT>& r, const Spacing<T>& sp) {
    return V3<VT>{cdiff<MODE>(r.u, l.u, sp.two_dx, sp.inv2dx), cdiff<MODE>(r.v, l.v, sp.two_dx, sp.inv2dx),
                  cdiff<MODE>(r.h, l.h, sp.two_dx, sp.inv2dx)};
}

template <int MODE, typename VT, typename T>
__device__ __forceinline__ V3<VT> tend(const V3<VT>& c, const V3<VT>& l, const V3<VT>& r, const V3<VT>& t,
                                       const V3<VT>& b, const Spacing<T>& sp, T g, T f) {
    return tend_x<MODE>(c, xdiffs<MODE>(l, r, sp), t, b, sp, g, f);
}

// stage update y + c k (fast numerics: one fused multiply-add)
template <int MODE, typename VT, typename T>
__device__ __forceinline__ V3<VT> axpy(const V3<VT>& y, T c, const V3<VT>& k) {
    if constexpr (MODE >= kSpFast) return {fmadd((VT)c, k.u, y.u), fmadd((VT)c, k.v, y.v), fmadd((VT)c, k.h, y.h)};
    else return {y.u + c * k.u, y.v + c * k.v, y.h + c * k.h};
}

// RK4-as-implemented: what the stage-3 ring keeps for the final combination -- k3 (exact), or
// the running sum k2 + k3 (fast numerics). (Round 3 measured an accumulator y + dt/3 (k2 + k3)
// kept instead, which frees the y ring one row earlier: 1.5-2 % faster, but v of the C2 case
// drifted to 3.2e-11 relative L2 from the exact run after 13 steps against 1.3e-16 -- not kept.)
template <int MODE, typename VT>
__device__ __forceinline__ V3<VT> rk4_keep3(const V3<VT>& k2, const V3<VT>& k3) {
    if constexpr (MODE >= kSpFast) return {k2.u + k3.u, k2.v + k3.v, k2.h + k3.h};
    else return k3;
}

// The final combination (k1 aliases k4, weather_simulation.cpp:437-451):
// exact: y + dt/6 * (((k4 + 2 k2) + 2 k3) + k4); fast: y + dt/3 * (kept + k4), kept = k2 + k3
// (c = a.c_dt6, which prepare_fast turns into dt/3 * s)
template <int MODE, typename VT, typename T>
__device__ __forceinline__ V3<VT> rk4_final(const V3<VT>& y, T c, const V3<VT>& k4, const V3<VT>& k2,
                                            const V3<VT>& kept3) {
    if constexpr (MODE >= kSpFast) {
        const VT cv = (VT)c;
        return {fmadd(cv, kept3.u + k4.u, y.u), fmadd(cv, kept3.v + k4.v, y.v), fmadd(cv, kept3.h + k4.h, y.h)};
    } else {
        const T two = T(2);
        V3<VT> o;
        o.u = y.u + c * (((k4.u + two * k2.u) + two * kept3.u) + k4.u);
        o.v = y.v + c * (((k4.v + two * k2.v) + two * kept3.v) + k4.v);
        o.h = y.h + c * (((k4.h + two * k2.h) + two * kept3.h) + k4.h);
        return o;
    }
}

// launch a fused kernel template instantiated per spacing mode: GO(MODE) for the runtime mode
#define WS_SP_DISPATCH(mode, GO)           \
    switch (mode) {                        \
        case kSpFast0: GO(kSpFast0); break; \
        case kSpFast: GO(kSpFast); break;   \
        case kSpMul: GO(kSpMul); break;     \
        default: GO(kSpDiv); break;         \
    }

// XCD-aware work mapping: consecutive work items (neighbouring strips of one segment,
// which share halo columns) go to blocks b, b+8, ... that the dispatcher places on the
// same XCD (same L2). Bijective for any block count. Speed only, never correctness.
__device__ __forceinline__ int xcd_work_item() {
    const int nb = gridDim.x;
    const int b = blockIdx.x;
    const int q = nb / 8, rr = nb % 8, xcd = b % 8;
    return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + b / 8;
}

}  // namespace dev
}  // namespace ws
