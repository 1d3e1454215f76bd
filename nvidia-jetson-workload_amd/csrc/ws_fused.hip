// Fused multi-stage time step: one kernel per time step (Euler: 1 stage, RK2: 2, RK4: 4).
//
// Why: the unfused stage kernels move 6w / 15w / 45w bytes per cell per step (Euler /
// RK2 / RK4-as-implemented); this kernel moves ~6w for every integrator --
// y = (u, v, h) is read once and y' written once -- and keeps every intermediate stage
// (tmp, K2, K3) on chip. Arithmetic per cell is identical to the reference, in the same
// order (weather_simulation.cpp:160-218, 220-323, 325-455, 473-540), so results stay
// bit-for-bit equal to the CPU solver; redundantly recomputed halo cells are discarded.
//
// Decomposition (CDNA4): a workgroup of kFusedCols lanes owns a column strip (one column
// per lane) and marches down a segment of rows. At march step R it takes input row R
// (loaded kPf rows ahead into registers) and stage s = 1..NST computes row R - s (a skewed
// wavefront). Vertical neighbours come from per-lane register rings; horizontal neighbours
// come from the LDS copy of the previous stage's row, published one march step earlier, so
// the whole pipeline needs ONE workgroup barrier per row. Each stage invalidates one column
// at each strip edge: a strip outputs kFusedCols - 2*NST columns and neighbouring strips
// overlap by 2*NST columns. A segment of S output rows marches S + 2*NST rows (warm-up +
// drain), rounded up to the unroll length.
#include <type_traits>
#include <utility>

#include "ws_fused_dev.h"

namespace ws {
namespace {

using namespace dev;

// LDS image, column-major: column c (= lane + 1; columns 0 and kFusedCols + 1 are pads)
// holds, for every published quantity q = 2 * stage + (row parity), the three fields at
// [c][q][field]. The column stride kCs = 6*NST + 1 elements (odd in dwords for fp32,
// 2 mod 4 for fp64) spreads the 32 / 64 lanes of one access over distinct banks, and a
// lane's left and right neighbours (columns lane, lane + 2) sit within one ds_read2's
// offset range of a single per-lane base address, so every LDS access uses one address
// register plus immediate offsets.
//
// Clamp-to-self at the global x edges (weather_simulation.cpp:510-511) is done on the
// WRITE side (XCLAMP strips only): the lane at x = 0 also writes its value into its left
// column, the lane at x = W-1 into its right column, and lanes outside [0, W) publish
// into pad column 0 (never read by a live output).
template <typename T, int NST>
struct Lds {
    static constexpr int kCs = 6 * NST + 1;
    T a[(kFusedCols + 2) * kCs];
    __device__ __forceinline__ T* col(int c) { return a + c * kCs; }
};

template <int NST, int Q, typename T>
__device__ __forceinline__ void publish(T* colp, const V3<T>& v) {
    colp[Q * 3 + 0] = v.u;
    colp[Q * 3 + 1] = v.v;
    colp[Q * 3 + 2] = v.h;
}

// One stage at row j: the tendency of (prev stage) at row j from rows j-1 (up), j (mid),
// j+1 (down) and the published row j (x-neighbours, quantity Q). YCLAMP: the segment
// touches a global y edge, where the reference clamps j-1 / j+1 to j
// (weather_simulation.cpp:512-513).
template <int MODE, bool YCLAMP, int NST, int Q, typename T>
__device__ __forceinline__ V3<T> stage_tend(const T* lcol, int j, const Geom& g, const V3<T>& up, const V3<T>& mid,
                                            const V3<T>& down, const Spacing<T>& sp, T grav, T cor) {
    constexpr int kCs = Lds<T, NST>::kCs;
    const T* rcol = lcol + 2 * kCs;
    const V3<T> l{lcol[Q * 3 + 0], lcol[Q * 3 + 1], lcol[Q * 3 + 2]};
    const V3<T> r{rcol[Q * 3 + 0], rcol[Q * 3 + 1], rcol[Q * 3 + 2]};
    if constexpr (YCLAMP) {
        const bool ytop = (j == 0) && g.top_clamp;
        const bool ybot = (j == g.H - 1) && g.bot_clamp;
        // select by value (a ?: on two lvalues selects an address and spills to scratch)
        const V3<T> t{ytop ? mid.u : up.u, ytop ? mid.v : up.v, ytop ? mid.h : up.h};
        const V3<T> b{ybot ? mid.u : down.u, ybot ? mid.v : down.v, ybot ? mid.h : down.h};
        return tend<MODE>(mid, l, r, t, b, sp, grav, cor);
    } else {
        return tend<MODE>(mid, l, r, up, down, sp, grav, cor);
    }
}

constexpr int kPf = 3;  // rows of y loads in flight per lane
constexpr int kU = 8;   // march unroll = y ring length

#ifndef WS_FUSED_MINW
#define WS_FUSED_MINW 1
#endif

template <typename T, int NST, int MODE>
__global__ __launch_bounds__(kFusedCols, WS_FUSED_MINW) void fused_step_kernel(FusedArgs<T> a, Geom g) {
    // All per-lane state lives in rotating register rings indexed by the march phase P
    // (compile-time): the body is instantiated for P = 0..kU-1, so ring "shifts" are renames,
    // not moves (hipcc will not runtime-unroll a loop that contains a barrier). The march
    // starts on an even row, so the LDS double-buffer parity is compile-time too.
    constexpr int kYb = NST + 1 < 3 ? 3 : NST + 1;  // past y rows used: R-kYb+1 .. R
    static_assert(kYb + kPf <= kU, "y ring too short");
    __shared__ Lds<T, NST> lds;

    const int lane = threadIdx.x;
    const int out_w = a.out_w;
    const int x = blockIdx.x * out_w - NST + lane;  // this lane's global column
    const bool xlive = x >= 0 && x < g.W;
    const bool xout = xlive && lane >= NST && lane < NST + out_w;
    T* const mycol = lds.col(xlive ? lane + 1 : 0);
    T* const clampcol = lds.col(x == 0 ? lane : (x == g.W - 1 ? lane + 2 : (xlive ? lane + 1 : 0)));
    const T* const lcol = lds.col(lane);  // left neighbour column; right = lcol + 2 kCs

    int y0, y1;
    fused_rows(a, blockIdx.y, y0, y1);
    const int row_lo = g.top_clamp ? 0 : -g.halo;  // rows that exist in memory (halo rows in slabs)
    const int row_hi = g.bot_clamp ? g.H : g.H + g.halo;

    // buffer addressing as in ws_fused_dppy.hip: per-field descriptors based at this
    // workgroup's first row, row = scalar offset, column = fixed voffset; stores of
    // non-output lanes / rows go to an out-of-range voffset and are dropped (no branch)
    const int64_t lofs = (int64_t)blockIdx.z * g.lstride;
    const int R0 = (y0 - NST) & ~1;  // march rows [R0, R1): R0 even (LDS parity), length a multiple of kU
    const int R1 = R0 + (y1 + NST - R0 + kU - 1) / kU * kU;
    const int rbase = max(R0, row_lo);
    const int rtop = min(row_hi, R1 + kPf);
    const uint32_t in_bytes = (uint32_t)((int64_t)(rtop - rbase) * g.pitch * sizeof(T));
    const uint32_t out_bytes = (uint32_t)((int64_t)(y1 - y0) * g.pitch * sizeof(T));
    const int64_t ib = lofs + (int64_t)rbase * g.pitch, ob = lofs + (int64_t)y0 * g.pitch;
    const auto ru = make_rsrc(a.in_u + ib, in_bytes), rv = make_rsrc(a.in_v + ib, in_bytes),
               rh = make_rsrc(a.in_h + ib, in_bytes);
    const auto wu = make_rsrc(a.out_u + ob, out_bytes), wv = make_rsrc(a.out_v + ob, out_bytes),
               wh = make_rsrc(a.out_h + ob, out_bytes);
    const uint32_t row_bytes = (uint32_t)g.pitch * sizeof(T);
    const uint32_t loff = (uint32_t)min(max(x, 0), g.W - 1) * sizeof(T);
    const uint32_t soff = xout ? (uint32_t)x * sizeof(T) : kDropped;

    // Always-issued loads at clamped (allocated) rows: dead rows / columns hold real data
    // that no live output reads, and no branch splits the load stream.
    auto load_row = [&](int R) -> V3<T> {
        const int r = min(max(R, row_lo), row_hi - 1);
        const uint32_t so = (uint32_t)(r - rbase) * row_bytes;
        return V3<T>{buf_load<T>(ru, loff, so), buf_load<T>(rv, loff, so), buf_load<T>(rh, loff, so)};
    };
    auto store_row = [&](int j, const V3<T>& o) {
        const bool row_ok = j >= y0 && j < y1;
        const uint32_t so = row_ok ? (uint32_t)(j - y0) * row_bytes : 0u;
        const uint32_t vo = row_ok ? soff : kDropped;
        buf_store_nt<T>(o.u, wu, vo, so);
        buf_store_nt<T>(o.v, wv, vo, so);
        buf_store_nt<T>(o.h, wh, vo, so);
    };

    V3<T> Y[kU];                // Y[r % kU] = y row r (rows R-kYb+1 .. R+kPf live)
    V3<T> S1[2], S2[2], S3[2];  // [r % 2] = stage output at row r
    V3<T> K2[2], K3[2];         // RK4 stage-2 / stage-3 tendencies at row r
    const V3<T> Z{T(0), T(0), T(0)};
#pragma unroll
    for (int i = 0; i < kU; ++i) Y[i] = Z;
#pragma unroll
    for (int i = 0; i < 2; ++i) S1[i] = S2[i] = S3[i] = K2[i] = K3[i] = Z;

    // prologue: each row followed by a (dropped) store row like every march body, so the
    // loop is entered with the same outstanding-op pattern from here as from its back edge
#pragma unroll
    for (int i = 0; i < kPf; ++i) {
        Y[i] = load_row(R0 + i);
        store_row(y0 - 1, Z);
    }

    // Warm-up (the first kU bodies, Wc = true) skips stage s while R - R0 < 2s (outside the
    // segment's dependency cone; R0 may sit one row above y0 - NST, which only makes the
    // test conservative). Skipped stages publish nothing: the next stage to read that LDS
    // quantity is itself inactive until a body after the first active one. A skipped final
    // stage still issues its (dropped) store row: one load/store pattern for every body.
    auto body = [&](auto Pc, auto Xc, auto Yc, auto Wc, int R) {
        constexpr int P = decltype(Pc)::value;
        constexpr bool XC = decltype(Xc)::value;
        constexpr bool YC = decltype(Yc)::value;
        constexpr bool WARM = decltype(Wc)::value;
        constexpr auto on = [](int st) { return !WARM || P >= 2 * st; };
        constexpr int cur = P & 1, prv = cur ^ 1;  // R0 even => parity of R is parity of P
        constexpr auto yi = [](int d) { return ((P + d) % kU + kU) % kU; };
        constexpr auto r2 = [](int d) { return ((P + d) % 2 + 2) % 2; };
        auto pub = [&](auto Qc, const V3<T>& v) {
            constexpr int Q = decltype(Qc)::value;
            publish<NST, Q>(mycol, v);
            if constexpr (XC) publish<NST, Q>(clampcol, v);
        };
        using Q0c = std::integral_constant<int, 0 + cur>;
        using Q1c = std::integral_constant<int, 2 + cur>;
        using Q2c = std::integral_constant<int, 4 + cur>;
        using Q3c = std::integral_constant<int, 6 + cur>;

        Y[yi(kPf)] = load_row(R + kPf);  // its slot held row R + kPf - kU: dead
        __builtin_amdgcn_sched_barrier(0);  // keep the loads at the head of the body
        pub(Q0c{}, Y[yi(0)]);

        if constexpr (on(1)) {
            // stage 1 at row R-1 from y rows R-2, R-1, R
            const V3<T> k1 = stage_tend<MODE, YC, NST, 0 + prv>(lcol, R - 1, g, Y[yi(-2)], Y[yi(-1)], Y[yi(0)],
                                                                a.sp1, a.gravity, a.coriolis_f);
            if constexpr (NST == 1) {
                store_row(R - 1, axpy<MODE>(Y[yi(-1)], a.c_dt, k1));  // Euler: y + dt k
            } else {
                const V3<T> s1 = axpy<MODE>(Y[yi(-1)], a.c_half, k1);  // y + (0.5f dt) k
                if constexpr (on(2)) {
                    // stage 2 at row R-2 from s1 rows R-3, R-2, R-1
                    const V3<T> k2 = stage_tend<MODE, YC, NST, 2 + prv>(lcol, R - 2, g, S1[r2(-3)], S1[r2(-2)], s1,
                                                                        a.sp2, a.gravity, a.coriolis_f);
                    if constexpr (NST == 2) {
                        store_row(R - 2, axpy<MODE>(Y[yi(-2)], a.c_dt, k2));  // RK2: y + dt k2
                    } else {
                        const V3<T> s2 = axpy<MODE>(Y[yi(-2)], a.c_half, k2);
                        if constexpr (on(3)) {
                            // stage 3 at row R-3
                            const V3<T> k3 = stage_tend<MODE, YC, NST, 4 + prv>(lcol, R - 3, g, S2[r2(-4)],
                                                                                S2[r2(-3)], s2, a.sp2, a.gravity,
                                                                                a.coriolis_f);
                            const V3<T> s3 = axpy<MODE>(Y[yi(-3)], a.c_dt, k3);
                            if constexpr (on(4)) {
                                // stage 4 at row R-4
                                const V3<T> k4 = stage_tend<MODE, YC, NST, 6 + prv>(lcol, R - 4, g, S3[r2(-5)],
                                                                                    S3[r2(-4)], s3, a.sp2,
                                                                                    a.gravity, a.coriolis_f);
                                // y + dt/6 * (((k4 + 2 k2) + 2 k3) + k4)   (k1 aliases k4, :437-451)
                                const V3<T> o = rk4_final<MODE>(Y[yi(-4)], a.c_dt6, k4, K2[r2(-4)], K3[r2(-4)]);
                                store_row(R - 4, o);
                            } else {
                                store_row(y0 - 1, Z);
                            }
                            pub(Q3c{}, s3);
                            S3[r2(-3)] = s3;
                            K3[r2(-3)] = rk4_keep3<MODE>(K2[r2(-3)], k3);
                        } else {
                            store_row(y0 - 1, Z);
                        }
                        pub(Q2c{}, s2);
                        S2[r2(-2)] = s2;
                        K2[r2(-2)] = k2;
                    }
                } else {
                    store_row(y0 - 1, Z);
                }
                pub(Q1c{}, s1);
                S1[r2(-1)] = s1;
            }
        } else {
            store_row(y0 - 1, Z);
        }
        __syncthreads();
    };

    auto march = [&](auto Xc, auto Yc) {
        auto period = [&](auto Wc, int R) {
            [&]<int... Ps>(std::integer_sequence<int, Ps...>) {
                (body(std::integral_constant<int, Ps>{}, Xc, Yc, Wc, R + Ps), ...);
            }(std::make_integer_sequence<int, kU>{});
        };
        period(std::true_type{}, R0);  // R1 - R0 >= kU: the march spans >= 2 NST rows
        for (int R = R0 + kU; R < R1; R += kU) period(std::false_type{}, R);
    };
    // Global edges matter only to strips / segments within NST cells of them; every other
    // workgroup runs the clamp-free body.
    const bool xclamp = blockIdx.x == 0 || (int)(blockIdx.x + 1) * out_w >= g.W - NST;
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
hipError_t launch_fused_step(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s) {
    if (g.W < 2) return hipErrorInvalidValue;  // x = 0 == W-1 needs two clamp copies: use the stage kernels
    const int out_w = a.out_w;
    if (out_w < 1 || out_w > kFusedCols - 2 * nstages) return hipErrorInvalidValue;
    if (a.seg_n <= 0) return hipSuccess;
    // buffer descriptors span one segment's rows (+ margins); 32-bit offsets, dropped-store
    // voffset 2^31
    if ((int64_t)(a.seg_rows + 2 * nstages + 2 * kU + kPf + 2) * g.pitch * (int64_t)sizeof(T) >= 0x7fffffff)
        return hipErrorInvalidValue;
    const dim3 grid((g.W + out_w - 1) / out_w, a.seg_n, g.L);
    const dim3 block(kFusedCols);
#define WS_FUSED_GO(N, M) hipLaunchKernelGGL((fused_step_kernel<T, N, M>), grid, block, 0, s, a, g)
#define WS_FUSED_G1(M) WS_FUSED_GO(1, M)
#define WS_FUSED_G2(M) WS_FUSED_GO(2, M)
#define WS_FUSED_G4(M) WS_FUSED_GO(4, M)
    switch (nstages) {
        case 1: WS_SP_DISPATCH(a.sp_mode, WS_FUSED_G1) break;
        case 2: WS_SP_DISPATCH(a.sp_mode, WS_FUSED_G2) break;
        case 4: WS_SP_DISPATCH(a.sp_mode, WS_FUSED_G4) break;
        default: return hipErrorInvalidValue;
    }
#undef WS_FUSED_G1
#undef WS_FUSED_G2
#undef WS_FUSED_G4
#undef WS_FUSED_GO
    return hipGetLastError();
}

template hipError_t launch_fused_step<float>(int, const FusedArgs<float>&, const Geom&, hipStream_t);
template hipError_t launch_fused_step<double>(int, const FusedArgs<double>&, const Geom&, hipStream_t);

}  // namespace ws
