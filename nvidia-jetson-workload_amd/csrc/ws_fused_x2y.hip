// Fused multi-stage time step: column pairs per lane with LDS-resident y rows ("x2y").
//
// The march of ws_fused_dppy.hip (one kernel per time step; y read
// once, y' written once; stage s = 1..NST computes row R - s while row R arrives) with the
// column-pair lane layout: each lane owns an adjacent column pair, a 64-lane wave a
// 128-column strip, so of a pair's four horizontal neighbours two are the lane's own values
// (half the DPP moves per cell) and the strip overlap is 2 * 4 of 128 columns (RK4: 6 %
// recomputed instead of 12.5 %). The y rows arrive by LDS-DMA (buffer_load_dwordx4 ... lds,
// 16 bytes = one pair per lane) into a 6-row ring and are read from it in place (rows R-2,
// R-1, R each body); only rows R-3 and R-4 are held in VGPRs. Stores are one 16-byte pair
// store per field and row (a pair never straddles the row's end: pitch is a multiple of 64
// elements, so the column after an odd W is row padding, whose content is unspecified).
//
// Arithmetic per cell, element-wise on the pair: the reference's, in the reference's order
// (weather_simulation.cpp:160-455, 473-540) -- bit-for-bit those of the CPU solver -- or
// fast numerics (ws_fused.h), by spacing mode.
#include <type_traits>
#include <utility>

#include "ws_fused_dev.h"

namespace ws {
namespace {

using namespace dev;

constexpr int kWave = 64;
constexpr int kCols = 2 * kWave;  // columns per strip

template <typename T>
using P2 = T __attribute__((ext_vector_type(2)));

// margin columns on each side of a strip: the dependency cone (NST) rounded up to whole
// 16-byte DMA chunks (2 fp64 / 4 fp32 columns; both even, so margins are whole pairs)
template <typename T>
constexpr int margin(int nst) {
    return (nst + 16 / (int)sizeof(T) - 1) / (16 / (int)sizeof(T)) * (16 / (int)sizeof(T));
}

struct EdgeCols {
    bool lo0;        // column 0 of the pair is x = 0 (column 1 never is: pairs start even)
    bool hi0, hi1;   // column 0 / 1 of the pair is x = W - 1
};

// One stage at row j from rows j-1 (up), j (mid), j+1 (down) of the previous stage; the
// reference's clamp-to-self at global edges (weather_simulation.cpp:510-513).
template <int MODE, bool XCLAMP, bool YCLAMP, typename T>
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
        return tend<MODE>(mid, l, r, t, b, sp, grav, cor);
    } else {
        return tend<MODE>(mid, l, r, up, down, sp, grav, cor);
    }
}

constexpr int waitcnt_vm(int n) { return (n & 0xF) | ((n >> 4) << 14) | (0x7 << 4) | (0xF << 8); }

#ifndef WS_X2Y_MINW
#define WS_X2Y_MINW 1
#endif

template <typename T, int NST, int MODE>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(WS_X2Y_MINW))) void fused_x2y_kernel(FusedArgs<T> a, Geom g, int nstrips,
                                                                        int nsegs) {
    using VT = P2<T>;
    constexpr int kG = 16 / (2 * (int)sizeof(T));  // rows per DMA instruction (fp64 1, fp32 2)
    constexpr int kD = 2;                          // DMA rows in flight
    constexpr int kNR = 6;                         // LDS ring rows: R-2 .. R+kD+kG-1 fit
    constexpr int kU = kNR;                        // march unroll: ring slot == phase
    static_assert(kNR >= kD + kG + 2 && kU % kG == 0 && kU % 2 == 0 && kD % kG == 0, "ring");
    // wait until at most the younger DMA loads are outstanding (the DMAs issued since the
    // group, incl. the reading body's): loads complete in order, stores do not (a younger
    // store can retire before an older load), so stores are not counted -- see
    // ws_fused_dppy.hip
    constexpr int kWaitN = 3 * (kD / kG);
    constexpr int kM = margin<T>(NST);
    const int out_w = a.out_w;

    const int w = xcd_work_item();
    const int strip = w % nstrips;
    int y0, y1;
    fused_rows(a, (w / nstrips) % nsegs, y0, y1);
    const int level = w / (nstrips * nsegs);

    const int lane = threadIdx.x;
    const int base = strip * out_w - kM;  // global column of the strip's first column (even)
    const int cx0 = base + 2 * lane;      // this lane's columns: cx0, cx0 + 1
    const bool pair_out = 2 * lane >= kM && 2 * lane < kM + out_w && cx0 >= 0 && cx0 < g.W;
    EdgeCols e;
    e.lo0 = cx0 == 0;
    e.hi0 = cx0 == g.W - 1;
    e.hi1 = cx0 + 1 == g.W - 1;

    const int row_lo = g.top_clamp ? 0 : -g.halo;
    const int row_hi = g.bot_clamp ? g.H : g.H + g.halo;

    const int64_t lofs = (int64_t)level * g.lstride;
    const int rbase = max(y0 - NST, row_lo);
    const int rtop = min(row_hi, y1 + NST + kU + kD + kG);  // past the last row the march fetches
    const uint32_t in_bytes = (uint32_t)((int64_t)(rtop - rbase) * g.pitch * sizeof(T));
    const uint32_t out_bytes = (uint32_t)((int64_t)(y1 - y0) * g.pitch * sizeof(T));
    const int64_t ib = lofs + (int64_t)rbase * g.pitch, ob = lofs + (int64_t)y0 * g.pitch;
    const auto ru = make_rsrc(a.in_u + ib, in_bytes), rv = make_rsrc(a.in_v + ib, in_bytes),
               rh = make_rsrc(a.in_h + ib, in_bytes);
    const auto wu = make_rsrc(a.out_u + ob, out_bytes), wv = make_rsrc(a.out_v + ob, out_bytes),
               wh = make_rsrc(a.out_h + ob, out_bytes);
    const uint32_t row_bytes = (uint32_t)g.pitch * sizeof(T);
    const uint32_t soff = pair_out ? (uint32_t)cx0 * sizeof(T) : kDropped;

    // stores for every row; rows outside [y0, y1) dropped through the voffset (one store
    // pattern per body keeps the explicit vmcnt waits exact)
    auto store_row = [&](int j, const V3<VT>& o) {
        const bool row_ok = j >= y0 && j < y1;
        const uint32_t so = row_ok ? (uint32_t)(j - y0) * row_bytes : 0u;
        const uint32_t vo = row_ok ? soff : kDropped;
        buf_store_nt<VT>(o.u, wu, vo, so);
        buf_store_nt<VT>(o.v, wv, vo, so);
        buf_store_nt<VT>(o.h, wh, vo, so);
    };

    // ring[field][slot][lane] = the lane's pair of row (slot); one DMA per field fills kG
    // consecutive slots (64 lanes x 16 B)
    __shared__ __attribute__((aligned(16))) VT ring[3][kNR][kWave];
    const int dk = lane / (kWave / kG);  // row of the group this lane fetches
    const int dcol = base * (int)sizeof(T) + (lane % (kWave / kG)) * 16;
    auto dma = [&](int q, int slot) {
        const int r = min(max(q + dk, row_lo), row_hi - 1);
        // chunks left of column 0 wrap to huge offsets (dropped: zeros), chunks past the row's
        // end read the next row or padding: margin lanes only, never an output column's input
        const uint32_t vo = (uint32_t)((r - rbase) * (int)row_bytes + dcol);
        lds_dma16(ru, &ring[0][slot][0], vo);
        lds_dma16(rv, &ring[1][slot][0], vo);
        lds_dma16(rh, &ring[2][slot][0], vo);
    };
    auto read_row = [&](int slot) -> V3<VT> {
        return V3<VT>{ring[0][slot][lane], ring[1][slot][lane], ring[2][slot][lane]};
    };

    const VT zero = VT{T(0), T(0)};
    const V3<VT> Z{zero, zero, zero};
    V3<VT> Y[2];                 // [r % 2] = y row r, r <= R-3
    V3<VT> S1[2], S2[2], S3[2];  // [r % 2] = stage output at row r
    V3<VT> K2[2], K3[2];         // RK4 stage-2 / stage-3 tendencies at row r
#pragma unroll
    for (int i = 0; i < 2; ++i) Y[i] = S1[i] = S2[i] = S3[i] = K2[i] = K3[i] = Z;

    const int R0 = y0 - NST;
    const int R1 = R0 + (y1 + NST - R0 + kU - 1) / kU * kU;

    auto body = [&](auto Pc, auto Xc, auto Yc, auto Wc, int R) {
        constexpr int P = decltype(Pc)::value;
        constexpr bool XC = decltype(Xc)::value;
        constexpr bool YC = decltype(Yc)::value;
        constexpr bool WARM = decltype(Wc)::value;
        constexpr auto on = [](int st) { return !WARM || P >= 2 * st; };
        constexpr auto r2 = [](int d) { return ((P + d) % 2 + 2) % 2; };
        constexpr auto sl = [](int d) { return ((P + d) % kNR + kNR) % kNR; };
        if constexpr (P % kG == 0) {
            dma(R + kD, sl(kD));  // into the slots of rows <= R-4 (read in earlier bodies)
            __builtin_amdgcn_s_waitcnt(waitcnt_vm(kWaitN));  // rows R .. R+kG-1 have landed
        }
        const V3<VT> yR0 = read_row(sl(0)), yR1 = read_row(sl(-1)), yR2 = read_row(sl(-2));
#if WS_SCHED_BARRIER
        __builtin_amdgcn_sched_barrier(0);
#endif
        if constexpr (!on(1)) {
            store_row(y0 - 1, Z);
            return;
        }
        const V3<VT> k1 = stage_tend<MODE, XC, YC>(e, R - 1, g, yR2, yR1, yR0, a.sp1, a.gravity, a.coriolis_f);
        if constexpr (NST == 1) {
            store_row(R - 1, axpy<MODE>(yR1, a.c_dt, k1));  // Euler: y + dt k
        } else {
            const V3<VT> s1 = axpy<MODE>(yR1, a.c_half, k1);  // y + (0.5f dt) k
            if constexpr (on(2)) {
                const V3<VT> k2 = stage_tend<MODE, XC, YC>(e, R - 2, g, S1[r2(-3)], S1[r2(-2)], s1, a.sp2,
                                                           a.gravity, a.coriolis_f);
                if constexpr (NST == 2) {
                    store_row(R - 2, axpy<MODE>(yR2, a.c_dt, k2));  // RK2: y + dt k2
                } else {
                    const V3<VT> s2 = axpy<MODE>(yR2, a.c_half, k2);
                    if constexpr (on(3)) {
                        const V3<VT> k3 = stage_tend<MODE, XC, YC>(e, R - 3, g, S2[r2(-4)], S2[r2(-3)], s2, a.sp2,
                                                                   a.gravity, a.coriolis_f);
                        const V3<VT> s3 = axpy<MODE>(Y[r2(-3)], a.c_dt, k3);
                        if constexpr (on(4)) {
                            const V3<VT> k4 = stage_tend<MODE, XC, YC>(e, R - 4, g, S3[r2(-5)], S3[r2(-4)], s3,
                                                                       a.sp2, a.gravity, a.coriolis_f);
                            // y + dt/6 * (((k4 + 2 k2) + 2 k3) + k4)   (k1 aliases k4, :437-451)
                            const V3<VT> o = rk4_final<MODE>(Y[r2(-4)], a.c_dt6, k4, K2[r2(-4)], K3[r2(-4)]);
                            store_row(R - 4, o);
                        } else {
                            store_row(y0 - 1, Z);
                        }
                        S3[r2(-3)] = s3;
                        K3[r2(-3)] = rk4_keep3<MODE>(K2[r2(-3)], k3);
                    } else {
                        store_row(y0 - 1, Z);
                    }
                    S2[r2(-2)] = s2;
                    K2[r2(-2)] = k2;
                }
            } else {
                store_row(y0 - 1, Z);
            }
            S1[r2(-1)] = s1;
        }
        Y[r2(-2)] = yR2;  // row R-2 is R-3 / R-4 of the next bodies (its slot held R-4, read above)
    };

    auto march = [&](auto Xc, auto Yc) {
        // the kD virtual bodies before R0: DMAs for rows R0 .. R0+kD-1 and (dropped) stores,
        // the same outstanding-op pattern the loop's back edge has
        [&]<int... Vs>(std::integer_sequence<int, Vs...>) {
            ([&] {
                constexpr int v = Vs - kD;
                if constexpr (((v % kG) + kG) % kG == 0) dma(R0 + v + kD, v + kD);
                store_row(y0 - 1, Z);
            }(), ...);
        }(std::make_integer_sequence<int, kD>{});
        auto period = [&](auto Wc, int R) {
            [&]<int... Ps>(std::integer_sequence<int, Ps...>) {
                (body(std::integral_constant<int, Ps>{}, Xc, Yc, Wc, R + Ps), ...);
            }(std::make_integer_sequence<int, kU>{});
        };
        period(std::true_type{}, R0);
        for (int R = R0 + kU; R < R1; R += kU) period(std::false_type{}, R);
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));  // no DMA into LDS after exit
    };
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
hipError_t launch_fused_step_x2y(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s) {
    const int out_w = a.out_w;
    const int chunk = 16 / (int)sizeof(T);
    if (out_w < chunk || out_w % chunk || out_w > kCols - 2 * margin<T>(nstages)) return hipErrorInvalidValue;
    if (g.pitch % 64 != 0) return hipErrorInvalidValue;  // pair stores stay inside the row
    const int nstrips = (g.W + out_w - 1) / out_w;
    const int nsegs = a.seg_n;
    if (nsegs <= 0) return hipSuccess;
    const int64_t nblocks = (int64_t)nstrips * nsegs * g.L;
    if (nblocks > 0x7fffffff) return hipErrorInvalidValue;
    const int64_t span = (int64_t)(a.seg_rows + 2 * nstages + 12 + 8) * g.pitch * (int64_t)sizeof(T);
    if (span >= 0x7fffffff) return hipErrorInvalidValue;
    const dim3 grid((unsigned)nblocks), block(kWave);
#define WS_X2Y_GO(N, M) hipLaunchKernelGGL((fused_x2y_kernel<T, N, M>), grid, block, 0, s, a, g, nstrips, nsegs)
#define WS_X2Y_G1(M) WS_X2Y_GO(1, M)
#define WS_X2Y_G2(M) WS_X2Y_GO(2, M)
#define WS_X2Y_G4(M) WS_X2Y_GO(4, M)
    switch (nstages) {
        case 1: WS_SP_DISPATCH(a.sp_mode, WS_X2Y_G1) break;
        case 2: WS_SP_DISPATCH(a.sp_mode, WS_X2Y_G2) break;
        case 4: WS_SP_DISPATCH(a.sp_mode, WS_X2Y_G4) break;
        default: return hipErrorInvalidValue;
    }
#undef WS_X2Y_G1
#undef WS_X2Y_G2
#undef WS_X2Y_G4
#undef WS_X2Y_GO
    return hipGetLastError();
}

template hipError_t launch_fused_step_x2y<float>(int, const FusedArgs<float>&, const Geom&, hipStream_t);
template hipError_t launch_fused_step_x2y<double>(int, const FusedArgs<double>&, const Geom&, hipStream_t);

}  // namespace ws
