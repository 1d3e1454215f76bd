// Fused multi-stage time step, wave-independent, TWO columns per lane ("x2").
//
// The march of ws_fused_dpp.hip (one kernel per time step; y read once, y' written once;
// stage s = 1..NST computes row R - s while row R is taken; register rings indexed by a
// compile-time phase), with each lane owning an adjacent column pair: a 64-lane wave covers
// a 128-column strip, every load/store moves 16 B (fp64) or 8 B (fp32) per lane, and of a
// pair's four horizontal neighbours two are the lane's own values -- only two DPP shifts
// per field and stage instead of four. The halo margin shrinks to 2*M of 128 columns
// (M = NST rounded up to even; RK4 6.3 % redundant instead of 12.5 %), and the pair's two
// columns are independent dependency chains (ILP 2). fp32 pairs run as packed VALU.
//
// Arithmetic per cell is the reference's, in the reference's order
// (weather_simulation.cpp:160-455, 473-540), element-wise on the pair: results are
// bit-for-bit those of the CPU solver.
#include <type_traits>
#include <utility>

#include "ws_fused_dev.h"

namespace ws {
namespace {

using namespace dev;

constexpr int kWave = 64;
constexpr int kCols = 2 * kWave;  // columns per strip
#ifndef WS_X2_PF
#define WS_X2_PF 2
#endif
constexpr int kPf = WS_X2_PF;              // rows of y loads in flight per lane
#ifndef WS_X2_LDS
#define WS_X2_LDS 1  // RK4: keep K2, K3 and the two oldest y rows in LDS instead of VGPRs
#endif
constexpr int kUMax = 2 * (5 + kPf);  // upper bound of any instantiation's march unroll

// y ring length (rows R - past + 1 .. R + kPf in VGPRs) and march unroll (a multiple of
// the ring length and of the stage rings' period 2)
constexpr int ring_rows(int nst) {
    return (nst == 4 && WS_X2_LDS ? 3 : (nst + 1 < 3 ? 3 : nst + 1)) + kPf;
}
constexpr int unroll(int nst) { return ring_rows(nst) % 2 ? 2 * ring_rows(nst) : ring_rows(nst); }

template <typename T>
using P2 = T __attribute__((ext_vector_type(2)));

// margin columns on each side of a strip: the dependency cone (NST), rounded up to even
// so margins cover whole lanes
constexpr int margin(int nst) { return (nst + 1) / 2 * 2; }

// Per-lane column facts for the edge strips (XCLAMP): the reference clamps the neighbour
// index to the cell itself at x = 0 and x = W-1 (weather_simulation.cpp:510-511).
struct EdgeCols {
    bool lo0;        // column 0 of the pair is x = 0 (column 1 never is: the pair starts even)
    bool hi0, hi1;   // column 0 / 1 of the pair is x = W - 1
};

// One stage at row j from rows j-1 (up), j (mid), j+1 (down) of the previous stage.
template <int POW2, bool XCLAMP, bool YCLAMP, typename T>
__device__ __forceinline__ V3<P2<T>> stage_tend(const EdgeCols& e, int j, const Geom& g, const V3<P2<T>>& up,
                                                const V3<P2<T>>& mid, const V3<P2<T>>& down, const Spacing<T>& sp,
                                                T grav, T cor) {
    using VT = P2<T>;
    // left neighbours of (c0, c1) = (lane-1's c1, own c0); right = (own c1, lane+1's c0)
    V3<VT> l{VT{from_left(mid.u.y), mid.u.x}, VT{from_left(mid.v.y), mid.v.x}, VT{from_left(mid.h.y), mid.h.x}};
    V3<VT> r{VT{mid.u.y, from_right(mid.u.x)}, VT{mid.v.y, from_right(mid.v.x)}, VT{mid.h.y, from_right(mid.h.x)}};
    if constexpr (XCLAMP) {
        if (e.lo0) { l.u.x = mid.u.x; l.v.x = mid.v.x; l.h.x = mid.h.x; }
        if (e.hi0) { r.u.x = mid.u.x; r.v.x = mid.v.x; r.h.x = mid.h.x; }
        if (e.hi1) { r.u.y = mid.u.y; r.v.y = mid.v.y; r.h.y = mid.h.y; }
    }
    if constexpr (YCLAMP) {
        const bool ytop = (j == 0) && g.top_clamp;
        const bool ybot = (j == g.H - 1) && g.bot_clamp;
        const V3<VT> t{ytop ? mid.u : up.u, ytop ? mid.v : up.v, ytop ? mid.h : up.h};
        const V3<VT> b{ybot ? mid.u : down.u, ybot ? mid.v : down.v, ybot ? mid.h : down.h};
        return tend<POW2>(mid, l, r, t, b, sp, grav, cor);
    } else {
        return tend<POW2>(mid, l, r, up, down, sp, grav, cor);
    }
}

#ifndef WS_X2_MINW
#define WS_X2_MINW 1
#endif

template <typename T, int NST, int POW2>
__global__ __launch_bounds__(kWave, WS_X2_MINW) void fused_x2_kernel(FusedArgs<T> a, Geom g, int nstrips,
                                                                      int nsegs) {
    using VT = P2<T>;
    constexpr int kNY = ring_rows(NST);
    constexpr int kU = unroll(NST);
    constexpr bool kLds = NST == 4 && WS_X2_LDS;
    constexpr int kM = margin(NST);
    const int out_w = a.out_w;  // even: the window starts on a pair

    const int w = xcd_work_item();
    const int strip = w % nstrips;
    int y0, y1;
    fused_rows(a, (w / nstrips) % nsegs, y0, y1);
    const int level = w / (nstrips * nsegs);

    const int lane = threadIdx.x;
    const int base = strip * out_w - kM;  // global column of the strip's first column (even)
    const int cx0 = base + 2 * lane;      // this lane's columns: cx0, cx0 + 1
    const bool pair_out = 2 * lane >= kM && 2 * lane < kM + out_w;
    EdgeCols e;
    e.lo0 = cx0 == 0;
    e.hi0 = cx0 == g.W - 1;
    e.hi1 = cx0 + 1 == g.W - 1;

    const int row_lo = g.top_clamp ? 0 : -g.halo;  // rows that exist in memory (halo rows in slabs)
    const int row_hi = g.bot_clamp ? g.H : g.H + g.halo;

    // Buffer addressing (as ws_fused_dpp.hip): per-field descriptors based at this wave's
    // first row, the row as a scalar byte offset, the lane's column(s) as fixed voffsets;
    // stores of non-output columns get an out-of-range voffset and are dropped.
    const int64_t lofs = (int64_t)level * g.lstride;
    const int rbase = max(y0 - NST, row_lo);
    const int rtop = min(row_hi, y1 + NST + kU + kPf);  // past the last row the march loads
    const uint32_t in_bytes = (uint32_t)((int64_t)(rtop - rbase) * g.pitch * sizeof(T));
    const uint32_t out_bytes = (uint32_t)((int64_t)(y1 - y0) * g.pitch * sizeof(T));
    const int64_t ib = lofs + (int64_t)rbase * g.pitch, ob = lofs + (int64_t)y0 * g.pitch;
    const auto ru = make_rsrc(a.in_u + ib, in_bytes), rv = make_rsrc(a.in_v + ib, in_bytes),
               rh = make_rsrc(a.in_h + ib, in_bytes);
    const auto wu = make_rsrc(a.out_u + ob, out_bytes), wv = make_rsrc(a.out_v + ob, out_bytes),
               wh = make_rsrc(a.out_h + ob, out_bytes);
    const uint32_t row_bytes = (uint32_t)g.pitch * sizeof(T);

    // interior strips: one vector access per field; edge strips: per-column clamped loads
    // and per-column store masks
    const uint32_t lpair = (uint32_t)max(cx0, 0) * sizeof(T);
    const uint32_t l0 = (uint32_t)min(max(cx0, 0), g.W - 1) * sizeof(T);
    const uint32_t l1 = (uint32_t)min(max(cx0 + 1, 0), g.W - 1) * sizeof(T);
    const uint32_t spair = pair_out ? lpair : kDropped;
    const uint32_t s0 = pair_out && cx0 >= 0 && cx0 < g.W ? (uint32_t)cx0 * sizeof(T) : kDropped;
    const uint32_t s1 = pair_out && cx0 + 1 >= 0 && cx0 + 1 < g.W ? (uint32_t)(cx0 + 1) * sizeof(T) : kDropped;

    auto load_f = [&](auto Xc, __amdgpu_buffer_rsrc_t r, uint32_t so) -> VT {
        if constexpr (decltype(Xc)::value) return VT{buf_load<T>(r, l0, so), buf_load<T>(r, l1, so)};
        else return buf_load<VT>(r, lpair, so);
    };
    auto load_row = [&](auto Xc, int R) -> V3<VT> {
        const int rr = min(max(R, row_lo), row_hi - 1);
        const uint32_t so = (uint32_t)(rr - rbase) * row_bytes;
        return V3<VT>{load_f(Xc, ru, so), load_f(Xc, rv, so), load_f(Xc, rh, so)};
    };
    // Stores are issued for every row, unconditionally: rows outside [y0, y1) (warm-up and
    // round-up rows) are dropped by the range check through the voffset. A branch around
    // them would make the compiler's vmcnt bookkeeping merge the taken / not-taken paths
    // and wait for nearly every outstanding load at each row -- draining the prefetch.
    auto store_f = [&](auto Xc, VT v, __amdgpu_buffer_rsrc_t r, bool row_ok, uint32_t so) {
        if constexpr (decltype(Xc)::value) {
            buf_store_nt<T>(v.x, r, row_ok ? s0 : kDropped, so);
            buf_store_nt<T>(v.y, r, row_ok ? s1 : kDropped, so);
        } else {
            buf_store_nt<VT>(v, r, row_ok ? spair : kDropped, so);
        }
    };
    auto store_row = [&](auto Xc, int j, const V3<VT>& o) {
        const bool row_ok = j >= y0 && j < y1;
        const uint32_t so = row_ok ? (uint32_t)(j - y0) * row_bytes : 0u;
        store_f(Xc, o.u, wu, row_ok, so);
        store_f(Xc, o.v, wv, row_ok, so);
        store_f(Xc, o.h, wh, row_ok, so);
    };

    // LDS (RK4): per wave, slots of one row x 3 fields x 64 lanes; [slot][field][lane] so a
    // wave's access is 64 consecutive 8/16-byte words (conflict-free)
    constexpr int kSlotY = 0, kSlotK2 = 2, kSlotK3 = 4, kSlots = kLds ? 5 : 1;
    __shared__ VT lds[kSlots][3][kWave];
    auto lds_put = [&](int slot, const V3<VT>& v) {
        lds[slot][0][lane] = v.u;
        lds[slot][1][lane] = v.v;
        lds[slot][2][lane] = v.h;
    };
    auto lds_get = [&](int slot) -> V3<VT> { return V3<VT>{lds[slot][0][lane], lds[slot][1][lane], lds[slot][2][lane]}; };

    const VT zero = VT{T(0), T(0)};
    const V3<VT> Z{zero, zero, zero};
    V3<VT> Y[kNY];               // Y[(r - R0) % kNY] = y row r
    V3<VT> S1[2], S2[2], S3[2];  // [r % 2] = stage output at row r
    V3<VT> K2[2], K3;            // RK4 stage-2 tendency at row r ([r % 2]); stage-3 at the previous row
#pragma unroll
    for (int i = 0; i < kNY; ++i) Y[i] = Z;
#pragma unroll
    for (int i = 0; i < 2; ++i) S1[i] = S2[i] = S3[i] = K2[i] = Z;
    K3 = Z;

    const int R0 = y0 - NST;
    const int R1 = R0 + (y1 + NST - R0 + kU - 1) / kU * kU;  // rounded up to the unroll

    // Warm-up (the first kU bodies, Wc = true) skips stage s while R - R0 < 2s: those rows
    // lie outside the segment's dependency cone (see ws_fused_dpp.hip). A skipped final
    // stage still issues its (dropped) store row: every body keeps one load/store pattern.
    auto body = [&](auto Pc, auto Xc, auto Yc, auto Wc, int R) {
        constexpr int P = decltype(Pc)::value;
        constexpr bool XC = decltype(Xc)::value;
        constexpr bool YC = decltype(Yc)::value;
        constexpr bool WARM = decltype(Wc)::value;
        constexpr auto on = [](int st) { return !WARM || P >= 2 * st; };
        constexpr auto yi = [](int d) { return ((P + d) % kNY + kNY) % kNY; };
        constexpr auto r2 = [](int d) { return ((P + d) % 2 + 2) % 2; };
        Y[yi(kPf)] = load_row(Xc, R + kPf);  // its slot held row R + kPf - kNY: dead
        // keep the row's loads at the head of the body: the scheduler would otherwise sink
        // them below the stencil math, shortening the prefetch distance
#if WS_SCHED_BARRIER
        __builtin_amdgcn_sched_barrier(0);
#endif
#ifdef WS_ABLATE
        if constexpr (WS_ABLATE == 2) {  // measurement build: memory stream only, no stencil math
            store_row(Xc, R - NST, Y[yi(-NST < -2 ? -2 : -NST)]);
            return;
        }
#endif
        // RK4 with LDS rings: y row R-2 leaves the VGPR ring after this body (it is the s3
        // base at R+1 and the output base at R+2); its LDS slot is row R-4's, so it is
        // written after the final combination read that (a wave's LDS ops run in order)
        auto put_y = [&] {
            if constexpr (kLds) lds_put(kSlotY + r2(-2), Y[yi(-2)]);
        };
        if constexpr (!on(1)) {
            store_row(Xc, y0 - 1, Z);
            if constexpr (NST == 4) put_y();
            return;
        }
        const V3<VT> k1 = stage_tend<POW2, XC, YC>(e, R - 1, g, Y[yi(-2)], Y[yi(-1)], Y[yi(0)], a.sp1, a.gravity,
                                                   a.coriolis_f);
        if constexpr (NST == 1) {
            store_row(Xc, R - 1, axpy(Y[yi(-1)], a.c_dt, k1));  // Euler: y + dt k
        } else {
            const V3<VT> s1 = axpy(Y[yi(-1)], a.c_half, k1);  // y + (0.5f dt) k
            if constexpr (on(2)) {
                const V3<VT> k2 = stage_tend<POW2, XC, YC>(e, R - 2, g, S1[r2(-3)], S1[r2(-2)], s1, a.sp2,
                                                           a.gravity, a.coriolis_f);
                if constexpr (NST == 2) {
                    store_row(Xc, R - 2, axpy(Y[yi(-2)], a.c_dt, k2));  // RK2: y + dt k2
                } else {
                    const V3<VT> s2 = axpy(Y[yi(-2)], a.c_half, k2);
                    if constexpr (on(3)) {
                        const V3<VT> k3 = stage_tend<POW2, XC, YC>(e, R - 3, g, S2[r2(-4)], S2[r2(-3)], s2, a.sp2,
                                                                   a.gravity, a.coriolis_f);
                        const V3<VT> y3 = kLds ? lds_get(kSlotY + r2(-3)) : Y[yi(-3)];
                        const V3<VT> s3 = axpy(y3, a.c_dt, k3);
                        if constexpr (on(4)) {
                            const V3<VT> k4 = stage_tend<POW2, XC, YC>(e, R - 4, g, S3[r2(-5)], S3[r2(-4)], s3,
                                                                       a.sp2, a.gravity, a.coriolis_f);
                            // y + dt/6 * (((k4 + 2 k2) + 2 k3) + k4)   (k1 aliases k4, :437-451)
                            const T two = T(2);
                            const V3<VT> y4 = kLds ? lds_get(kSlotY + r2(-4)) : Y[yi(-4)];
                            const V3<VT> kk2 = kLds ? lds_get(kSlotK2 + r2(-4)) : K2[r2(-4)];
                            const V3<VT> kk3 = kLds ? lds_get(kSlotK3) : K3;
                            V3<VT> o;
                            o.u = y4.u + a.c_dt6 * (((k4.u + two * kk2.u) + two * kk3.u) + k4.u);
                            o.v = y4.v + a.c_dt6 * (((k4.v + two * kk2.v) + two * kk3.v) + k4.v);
                            o.h = y4.h + a.c_dt6 * (((k4.h + two * kk2.h) + two * kk3.h) + k4.h);
                            store_row(Xc, R - 4, o);
                        } else {
                            store_row(Xc, y0 - 1, Z);
                        }
                        S3[r2(-3)] = s3;  // after k4 read S3[r2(-5)] (same slot)
                        if constexpr (kLds) lds_put(kSlotK3, k3);
                        else K3 = k3;
                    } else {
                        store_row(Xc, y0 - 1, Z);
                    }
                    S2[r2(-2)] = s2;  // after k3 read S2[r2(-4)] (same slot)
                    if constexpr (kLds) lds_put(kSlotK2 + r2(-2), k2);  // after the final read K2[r2(-4)]
                    else K2[r2(-2)] = k2;
                    put_y();
                }
            } else {
                store_row(Xc, y0 - 1, Z);
                if constexpr (NST == 4) put_y();
            }
            S1[r2(-1)] = s1;  // after k2 read S1[r2(-3)] (same slot)
        }
    };

    auto march = [&](auto Xc, auto Yc) {
        // prologue: the first kPf rows, each followed by a (dropped) store row like every
        // march body, so the loop is entered with the same outstanding-op pattern from the
        // prologue as from its back edge and the compiler's vmcnt waits stay partial
#pragma unroll
        for (int i = 0; i < kPf; ++i) {
            Y[i] = load_row(Xc, R0 + i);
            store_row(Xc, y0 - 1, Z);
        }
        auto period = [&](auto Wc, int R) {
            [&]<int... Ps>(std::integer_sequence<int, Ps...>) {
                (body(std::integral_constant<int, Ps>{}, Xc, Yc, Wc, R + Ps), ...);
            }(std::make_integer_sequence<int, kU>{});
        };
        period(std::true_type{}, R0);  // R1 - R0 >= kU: the march spans >= 2 NST rows
        for (int R = R0 + kU; R < R1; R += kU) period(std::false_type{}, R);
    };
    // global edges matter only to strips / segments within reach of them
    const bool xclamp = base < 0 || base + kCols > g.W;
    const bool yclamp = (g.top_clamp && y0 < NST) || (g.bot_clamp && y1 > g.H - NST);
    if (xclamp) {
        if (yclamp) march(std::true_type{}, std::true_type{});
        else march(std::true_type{}, std::false_type{});
    } else {
        if (yclamp) march(std::false_type{}, std::true_type{});
        else march(std::false_type{}, std::false_type{});
    }
}

}  // namespace

template <typename T>
hipError_t launch_fused_step_x2(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s) {
    const int out_w = a.out_w;
    if (out_w < 2 || out_w % 2 || out_w > kCols - 2 * margin(nstages)) return hipErrorInvalidValue;
    const int nstrips = (g.W + out_w - 1) / out_w;
    const int nsegs = a.seg_n;
    if (nsegs <= 0) return hipSuccess;
    const int64_t nblocks = (int64_t)nstrips * nsegs * g.L;
    if (nblocks > 0x7fffffff) return hipErrorInvalidValue;
    // buffer descriptors span one segment's rows (+ margins); offsets are 32-bit and the
    // dropped-store voffset is 2^31
    const int64_t span = (int64_t)(a.seg_rows + 2 * nstages + 2 * kUMax + kPf) * g.pitch * (int64_t)sizeof(T);
    if (span >= 0x7fffffff) return hipErrorInvalidValue;
    if (g.pitch % 2 != 0) return hipErrorInvalidValue;  // column pairs stay 2-element aligned
    const dim3 grid((unsigned)nblocks), block(kWave);
    const int sp_mode = fused_sp_mode(a);  // spacing mode (ws_fused.h)
#define WS_X2_LAUNCH(N)                                                                                   \
    if (sp_mode == kSpScaled)                                                                              \
        hipLaunchKernelGGL((fused_x2_kernel<T, N, kSpScaled>), grid, block, 0, s, a, g, nstrips, nsegs);   \
    else if (sp_mode == kSpMul)                                                                            \
        hipLaunchKernelGGL((fused_x2_kernel<T, N, kSpMul>), grid, block, 0, s, a, g, nstrips, nsegs);      \
    else hipLaunchKernelGGL((fused_x2_kernel<T, N, kSpDiv>), grid, block, 0, s, a, g, nstrips, nsegs);
    switch (nstages) {
        case 1: WS_X2_LAUNCH(1) break;
        case 2: WS_X2_LAUNCH(2) break;
        case 4: WS_X2_LAUNCH(4) break;
        default: return hipErrorInvalidValue;
    }
#undef WS_X2_LAUNCH
    return hipGetLastError();
}

template hipError_t launch_fused_step_x2<float>(int, const FusedArgs<float>&, const Geom&, hipStream_t);
template hipError_t launch_fused_step_x2<double>(int, const FusedArgs<double>&, const Geom&, hipStream_t);

}  // namespace ws
