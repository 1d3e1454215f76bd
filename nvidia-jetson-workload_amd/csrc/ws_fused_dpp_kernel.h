// Fused multi-stage time step, wave-independent variant: one 64-lane wave per column strip,
// horizontal neighbours by DPP lane shifts (wave_shr:1 / wave_shl:1) -- no LDS, no barrier.
//
// Same march as ws_fused.hip (one kernel per time step; y read once, y' written once;
// stage s = 1..NST computes row R - s while row R is taken; register rings indexed by a
// compile-time phase), but every wave runs free: nothing synchronises it with any other
// wave, so a wave waiting on HBM never holds its neighbours back. The price is halo
// redundancy: a 64-column strip outputs 64 - 2*NST columns (RK4: 56, 14% recomputed).
// Arithmetic per cell is the reference's, in the reference's order
// (weather_simulation.cpp:160-455, 473-540): results are bit-for-bit those of the CPU solver.
#include <type_traits>
#include <utility>

#pragma once

#include "ws_fused_dev.h"

namespace ws {
namespace {

using namespace dev;

constexpr int kWave = 64;
#ifndef WS_DPP_PF
#define WS_DPP_PF 3
#endif
// rows of y loads in flight per lane (template parameter PF; 3 measured best at C2 -- a
// 6-row variant did not help even on grids too small to fill the chip)
constexpr int unroll_for(int pf) { return (5 + pf + 1) / 2 * 2; }  // y ring length (>= 5 past rows + pf, even)
constexpr int kUMax = unroll_for(WS_DPP_PF) > 16 ? unroll_for(WS_DPP_PF) : 16;

// One stage at row j from rows j-1 (up), j (mid), j+1 (down) of the previous stage.
// XCLAMP / YCLAMP: the strip / segment touches a global edge, where the reference clamps
// the neighbour index to the cell itself (weather_simulation.cpp:510-513).
template <int POW2, bool XCLAMP, bool YCLAMP, typename T>
__device__ __forceinline__ V3<T> stage_tend(bool xlo, bool xhi, int j, const Geom& g, const V3<T>& up,
                                            const V3<T>& mid, const V3<T>& down, const Spacing<T>& sp, T grav,
                                            T cor) {
    V3<T> l{from_left(mid.u), from_left(mid.v), from_left(mid.h)};
    V3<T> r{from_right(mid.u), from_right(mid.v), from_right(mid.h)};
    if constexpr (XCLAMP) {
        l = V3<T>{xlo ? mid.u : l.u, xlo ? mid.v : l.v, xlo ? mid.h : l.h};
        r = V3<T>{xhi ? mid.u : r.u, xhi ? mid.v : r.v, xhi ? mid.h : r.h};
    }
    if constexpr (YCLAMP) {
        const bool ytop = (j == 0) && g.top_clamp;
        const bool ybot = (j == g.H - 1) && g.bot_clamp;
        const V3<T> t{ytop ? mid.u : up.u, ytop ? mid.v : up.v, ytop ? mid.h : up.h};
        const V3<T> b{ybot ? mid.u : down.u, ybot ? mid.v : down.v, ybot ? mid.h : down.h};
        return tend<POW2>(mid, l, r, t, b, sp, grav, cor);
    } else {
        return tend<POW2>(mid, l, r, up, down, sp, grav, cor);
    }
}

#ifndef WS_DPP_MINW
#define WS_DPP_MINW 1
#endif
#ifndef WS_DPPY_MINW
#define WS_DPPY_MINW 1  // LDS-resident y: 133 VGPRs (RK4 fp64) fit 3 waves per SIMD unforced
#endif
#ifndef WS_DPP_WPB
#define WS_DPP_WPB 1  // waves per workgroup: >1 puts adjacent strips on one CU (shared L1 for the overlap)
#endif
constexpr int kWpb = WS_DPP_WPB;
#ifndef WS_SCHED_EVERY
#define WS_SCHED_EVERY 1
#endif
#ifndef WS_DPPY_GROUPS
#define WS_DPPY_GROUPS 1  // LDS-resident y: DMA groups in flight (ring 6 rows fp64 / 12 fp32 at 1)
#endif

// s_waitcnt immediate for "vmcnt <= n" alone (gfx9 encoding: vmcnt[3:0], expcnt[6:4],
// lgkmcnt[11:8], vmcnt[15:14]); the other counters at their maxima = not waited on
constexpr int waitcnt_vm(int n) { return (n & 0xF) | ((n >> 4) << 14) | (0x7 << 4) | (0xF << 8); }

// PF > 0: y rows loaded PF rows ahead into VGPRs (buffer_load, 8 or 4 bytes per lane).
// PF == 0 ("DMA"): y rows staged through an LDS ring by LDS-DMA -- buffer_load_dwordx4 ...
// lds, 16 bytes per lane, one instruction per field moves kG = 16 / sizeof(T) rows of the
// strip -- kD rows ahead, with no VGPR held by a load in flight; each group of kG rows is
// copied LDS -> VGPR ring one body before its first row is needed. The compiler does not
// order LDS reads after LDS-DMA writes, so the kernel waits itself: every body issues
// exactly 3 stores and every kG-th body 3 DMAs, hence a fixed count of younger vector-
// memory ops at each wait (kWaitN below).
// PF < 0 ("LDS-resident y"): as PF == 0, but the y rows stay in the LDS ring and each body
// reads the three it needs for stage 1 (rows R-2, R-1, R) straight from it; only rows R-3
// and R-4 (for the late stage updates) are kept in VGPRs. The ring is shorter (the DMA runs
// one group ahead) and the VGPR ring of y rows is gone, which is what lets the kernel fit
// three waves per SIMD (<= 168 VGPRs) where the others fit two.
template <typename T, int NST, int POW2, int PF>
__global__ __launch_bounds__(kWave * kWpb, PF < 0 ? WS_DPPY_MINW : WS_DPP_MINW) void fused_dpp_kernel(FusedArgs<T> a, Geom g, int nstrips,
                                                                        int nsegs) {
    constexpr bool kDma = PF <= 0;
    constexpr bool kLdsY = PF < 0;
    constexpr int kG = 16 / (int)sizeof(T);                    // rows per DMA instruction
    // DMA rows in flight; LDS ring rows (LDS-resident y: rows R-2 .. R+kD+kG-1, rounded up
    // to whole groups)
    constexpr int kD = !kDma ? 0 : kLdsY ? kG * WS_DPPY_GROUPS : ((int)sizeof(T) == 8 ? 6 : 8);
    constexpr int kNR = kLdsY ? (kD + kG + 2 + kG - 1) / kG * kG : ((int)sizeof(T) == 8 ? 8 : 16);
    constexpr int kPf = kDma ? 0 : PF;
    constexpr int kU = kDma ? kNR : unroll_for(PF);            // DMA: ring slot == y ring index
    constexpr int kYb = NST + 1 < 3 ? 3 : NST + 1;  // past y rows used: R-kYb+1 .. R
    static_assert(kDma || kYb + kPf <= kU, "y ring too short");
    // a group's DMA may overwrite only slots whose rows were consumed (compiler lgkmcnt wait) in
    // an earlier body: kNR >= kD + kG (VGPR copy one body ahead) / kD + kG + 2 (LDS-resident
    // rows R-2 .. R read in the body itself)
    static_assert(!kDma || (kU % kG == 0 && kU % 2 == 0 && kNR >= kD + kG + (kLdsY ? 2 : 0) && kD % kG == 0 &&
                            (kLdsY || kU > kG + 4)),
                  "DMA ring");
    // Wait for a group's DMAs before reading it: vmcnt <= the number of vector-memory ops
    // issued after them that are LOADS (the DMAs issued in between, including the reading
    // body's own). Stores are not counted: a store may complete before an older load, so an
    // outstanding count that includes them can drop below the threshold while the group is
    // still in flight (seen as stale rows at 4096^2). Loads complete in order, so at most
    // kWaitN outstanding ops means every older load -- the group -- has landed.
    constexpr int kWaitN = kLdsY ? 3 * (kD / kG) : 3 * ((kD - 1) / (kG > 0 ? kG : 1));

    // XCD-aware: neighbouring strips share an L2 (and with kWpb > 1 a CU)
    const int w = xcd_work_item() * kWpb + (int)threadIdx.x / kWave;
    if (w >= nstrips * nsegs * g.L) return;  // the last workgroup's spare waves (no barriers)
    const int strip = w % nstrips;
    int y0, y1;
    fused_rows(a, (w / nstrips) % nsegs, y0, y1);
    const int level = w / (nstrips * nsegs);

    const int lane = (int)threadIdx.x % kWave;
    const int wave_id = (int)threadIdx.x / kWave;  // wave within the workgroup (its LDS ring)
    // left margin: the cone (NST), for DMA rounded up to whole 16-byte chunks
    constexpr int kM = kDma ? (NST + kG - 1) / kG * kG : NST;
    const int out_w = a.out_w;
    const int x = strip * out_w - kM + lane;  // this lane's global column
    const bool xout = x >= 0 && x < g.W && lane >= kM && lane < kM + out_w;
    const bool xlo = x == 0, xhi = x == g.W - 1;

    const int row_lo = g.top_clamp ? 0 : -g.halo;  // rows that exist in memory (halo rows in slabs)
    const int row_hi = g.bot_clamp ? g.H : g.H + g.halo;

    // Buffer addressing: one descriptor per field, based at this wave's first row (all
    // wave-uniform, SGPRs), the row as a scalar byte offset, the lane's column as a fixed
    // 32-bit voffset -- no per-row VALU address arithmetic. Stores of lanes outside the
    // strip's output columns get an out-of-range voffset: the buffer range check drops them
    // (no exec-mask branch). launch_fused_step_dpp checks the byte ranges fit.
    const int64_t lofs = (int64_t)level * g.lstride;
    const int rbase = max(y0 - NST, row_lo);
    const int rtop = min(row_hi, y1 + NST + kU + (kDma ? kD + kG : kPf));  // past the last row the march loads
    const uint32_t in_bytes = (uint32_t)((int64_t)(rtop - rbase) * g.pitch * sizeof(T));
    const uint32_t out_bytes = (uint32_t)((int64_t)(y1 - y0) * g.pitch * sizeof(T));
    const int64_t ib = lofs + (int64_t)rbase * g.pitch, ob = lofs + (int64_t)y0 * g.pitch;
    const auto ru = make_rsrc(a.in_u + ib, in_bytes), rv = make_rsrc(a.in_v + ib, in_bytes),
               rh = make_rsrc(a.in_h + ib, in_bytes);
    const auto wu = make_rsrc(a.out_u + ob, out_bytes), wv = make_rsrc(a.out_v + ob, out_bytes),
               wh = make_rsrc(a.out_h + ob, out_bytes);
    const uint32_t row_bytes = (uint32_t)g.pitch * sizeof(T);

    const int xc = min(max(x, 0), g.W - 1);
    const uint32_t loff = (uint32_t)xc * sizeof(T);
    const uint32_t soff = xout ? (uint32_t)x * sizeof(T) : kDropped;
#ifndef WS_ABLATE
#define WS_ABLATE 0  // measurement builds only: 1 = no loads (compute only), 2 = no compute
#endif
    auto load_row = [&](int R) -> V3<T> {
        const int r = min(max(R, row_lo), row_hi - 1);
        if constexpr (WS_ABLATE == 1) {
            const T q = T(r & 7) * T(0.125) + T(xc & 3);
            return V3<T>{q, q * T(0.5), T(10) + q};
        } else {
            const uint32_t so = (uint32_t)(r - rbase) * row_bytes;
            return V3<T>{buf_load<T>(ru, loff, so), buf_load<T>(rv, loff, so), buf_load<T>(rh, loff, so)};
        }
    };
    // Stores are issued for every row, unconditionally: rows outside [y0, y1) are dropped by
    // the range check through the voffset (a branch around them makes the compiler's vmcnt
    // bookkeeping merge both paths and drain the load prefetch at every row).
    auto store_row = [&](int j, const V3<T>& o) {
        const bool row_ok = j >= y0 && j < y1;
        const uint32_t so = row_ok ? (uint32_t)(j - y0) * row_bytes : 0u;
        uint32_t vo = row_ok ? soff : kDropped;
        if (WS_ABLATE == 1 && o.u != T(12345.678)) vo = kDropped;
        buf_store_nt<T>(o.u, wu, vo, so);
        buf_store_nt<T>(o.v, wv, vo, so);
        buf_store_nt<T>(o.h, wh, vo, so);
    };

    // LDS-DMA ring: ring[field][slot][lane], slot = (row - R0) % kNR; one DMA fills kG
    // consecutive slots (64 lanes x 16 B = kG rows of 64 columns)
    __shared__ __attribute__((aligned(16))) T rings[kWpb][kDma ? 3 : 1][kDma ? kNR : 1][kWave];
    auto& ring = rings[wave_id];
    const int dk = lane / (kWave / kG);                          // row of the group this lane fetches
    const int dcol = (strip * out_w - kM) * (int)sizeof(T) + (lane % (kWave / kG)) * 16;  // byte column (16-B aligned)
    auto dma = [&](int q, int slot) {  // rows q .. q + kG - 1 into slots slot .. slot + kG - 1
        const int r = min(max(q + dk, row_lo), row_hi - 1);
        // chunks left of column 0 (whole chunks: kM is chunk-aligned) wrap to huge offsets or
        // read the previous row, chunks past the row end read the next row: margin lanes
        // only, never read by an output lane
        const uint32_t vo = (uint32_t)((r - rbase) * (int)row_bytes + dcol);
        lds_dma16(ru, &ring[0][slot][0], vo);
        lds_dma16(rv, &ring[1 % (kDma ? 3 : 1)][slot][0], vo);
        lds_dma16(rh, &ring[2 % (kDma ? 3 : 1)][slot][0], vo);
    };
    auto read_row = [&](int slot) -> V3<T> {
        return V3<T>{ring[0][slot][lane], ring[1 % (kDma ? 3 : 1)][slot][lane], ring[2 % (kDma ? 3 : 1)][slot][lane]};
    };

    const V3<T> Z{T(0), T(0), T(0)};
    V3<T> Y[kLdsY ? 2 : kU];     // Y[r % kU] = y row r (LDS-resident y: Y[r % 2] = row r, r <= R-3)
    V3<T> S1[2], S2[2], S3[2];   // [r % 2] = stage output at row r
    V3<T> K2[2], K3[2];          // RK4 stage-2 / stage-3 tendencies at row r
#pragma unroll
    for (int i = 0; i < (kLdsY ? 2 : kU); ++i) Y[i] = Z;
#pragma unroll
    for (int i = 0; i < 2; ++i) S1[i] = S2[i] = S3[i] = K2[i] = K3[i] = Z;

    const int R0 = y0 - NST;
    const int R1 = R0 + (y1 + NST - R0 + kU - 1) / kU * kU;  // rounded up to the unroll
    // prologue: each row followed by a (dropped) store row like every march body, so the
    // loop is entered with the same outstanding-op pattern from here as from its back edge
    if constexpr (kDma) {
        // the kD virtual bodies before R0: DMAs for rows R0 .. R0 + kD - 1, stores, and the
        // copy of the first group into the y ring
        [&]<int... Vs>(std::integer_sequence<int, Vs...>) {
            ([&] {
                constexpr int v = Vs - kD;  // -kD .. -1
                if constexpr (((v % kG) + kG) % kG == 0) dma(R0 + v + kD, v + kD);
                store_row(y0 - 1, Z);
                if constexpr (v == -1 && !kLdsY) {
                    __builtin_amdgcn_s_waitcnt(waitcnt_vm(kWaitN));
#pragma unroll
                    for (int k = 0; k < kG; ++k) Y[k] = read_row(k);
                }
            }(), ...);
        }(std::make_integer_sequence<int, kD>{});
    } else {
#pragma unroll
        for (int i = 0; i < kPf; ++i) {
            Y[i] = load_row(R0 + i);
            store_row(y0 - 1, Z);
        }
    }

    // Warm-up (the first kU bodies of a segment, Wc = true): stage s at row R - s is needed
    // for the segment's outputs only from R - R0 >= 2s on (its cone above y0 is NST - s rows
    // deep), so earlier bodies skip it -- NST(NST+1) stage-rows less per segment (RK4: 20).
    // A skipped final stage still issues its (dropped) store row, keeping every body's
    // load/store pattern identical for the compiler's vmcnt bookkeeping.
    // y row R+d inside a body: LDS-resident rows R-2..R from this body's reads, older ones
    // from the 2-row VGPR ring; otherwise the y VGPR ring
#define YROW(d) yrow.template operator()<d>()
    auto body = [&](auto Pc, auto Xc, auto Yc, auto Wc, int R) {
        constexpr int P = decltype(Pc)::value;
        constexpr bool XC = decltype(Xc)::value;
        constexpr bool YC = decltype(Yc)::value;
        constexpr bool WARM = decltype(Wc)::value;
        constexpr auto on = [](int st) { return !WARM || P >= 2 * st; };
        constexpr auto yi = [](int d) { return ((P + d) % kU + kU) % kU; };
        constexpr auto r2 = [](int d) { return ((P + d) % 2 + 2) % 2; };
        constexpr auto sl = [](int d) { return ((P + d) % kNR + kNR) % kNR; };  // LDS ring slot of row R+d
        V3<T> yR0, yR1, yR2;  // LDS-resident y: rows R, R-1, R-2
        const auto yrow = [&]<int d>() -> V3<T> {
            if constexpr (!kLdsY) return Y[yi(d)];
            else if constexpr (d == 0) return yR0;
            else if constexpr (d == -1) return yR1;
            else if constexpr (d == -2) return yR2;
            else return Y[r2(d)];
        };
        if constexpr (kLdsY) {
            if constexpr (P % kG == 0) {
                dma(R + kD, sl(kD));  // slots of rows R+kD-kNR.. (<= R-4): read in earlier bodies
                // rows R .. R+kG-1 (issued kD bodies ago) have landed
                __builtin_amdgcn_s_waitcnt(waitcnt_vm(kWaitN));
            }
            yR0 = read_row(sl(0));
            yR1 = read_row(sl(-1));
            yR2 = read_row(sl(-2));
        } else if constexpr (kDma) {
            if constexpr (P % kG == 0) dma(R + kD, (P + kD) % kNR);  // slots of rows R+kD-kNR..: read
            if constexpr ((P + 1) % kG == 0) {  // rows R+1 .. R+kG: LDS -> y ring, needed from R+1 on
                __builtin_amdgcn_s_waitcnt(waitcnt_vm(kWaitN));
#pragma unroll
                for (int k = 1; k <= kG; ++k) Y[yi(k)] = read_row((P + k) % kNR);
            }
        } else {
            Y[yi(kPf)] = load_row(R + kPf);  // its slot held row R + kPf - kU: dead
        }
        // keep the row's loads at the head of the body: the scheduler would otherwise sink
        // them below the stencil math, shortening the prefetch distance
#if WS_SCHED_BARRIER
        // (every WS_SCHED_EVERY-th body: between barriers the scheduler may interleave
        // consecutive rows' stage chains)
        if constexpr (P % WS_SCHED_EVERY == 0) __builtin_amdgcn_sched_barrier(0);
#endif
        if constexpr (WS_ABLATE == 2) {
            store_row(R - NST, YROW(-NST));
            return;
        }
        if constexpr (!on(1)) {
            store_row(y0 - 1, Z);
            return;
        }
        const V3<T> k1 = stage_tend<POW2, XC, YC>(xlo, xhi, R - 1, g, YROW(-2), YROW(-1), YROW(0), a.sp1,
                                                  a.gravity, a.coriolis_f);
        if constexpr (NST == 1) {
            store_row(R - 1, axpy(YROW(-1), a.c_dt, k1));  // Euler: y + dt k
        } else {
            const V3<T> s1 = axpy(YROW(-1), a.c_half, k1);  // y + (0.5f dt) k
            if constexpr (on(2)) {
                const V3<T> k2 = stage_tend<POW2, XC, YC>(xlo, xhi, R - 2, g, S1[r2(-3)], S1[r2(-2)], s1, a.sp2,
                                                          a.gravity, a.coriolis_f);
                if constexpr (NST == 2) {
                    store_row(R - 2, axpy(YROW(-2), a.c_dt, k2));  // RK2: y + dt k2
                } else {
                    const V3<T> s2 = axpy(YROW(-2), a.c_half, k2);
                    if constexpr (on(3)) {
                        const V3<T> k3 = stage_tend<POW2, XC, YC>(xlo, xhi, R - 3, g, S2[r2(-4)], S2[r2(-3)], s2,
                                                                  a.sp2, a.gravity, a.coriolis_f);
                        const V3<T> s3 = axpy(YROW(-3), a.c_dt, k3);
                        if constexpr (on(4)) {
                            const V3<T> k4 = stage_tend<POW2, XC, YC>(xlo, xhi, R - 4, g, S3[r2(-5)], S3[r2(-4)],
                                                                      s3, a.sp2, a.gravity, a.coriolis_f);
                            // y + dt/6 * (((k4 + 2 k2) + 2 k3) + k4)   (k1 aliases k4, :437-451)
                            const T two = T(2);
                            const V3<T> y4 = YROW(-4);
                            const V3<T>& kk2 = K2[r2(-4)];
                            const V3<T>& kk3 = K3[r2(-4)];
                            V3<T> o;
                            o.u = y4.u + a.c_dt6 * (((k4.u + two * kk2.u) + two * kk3.u) + k4.u);
                            o.v = y4.v + a.c_dt6 * (((k4.v + two * kk2.v) + two * kk3.v) + k4.v);
                            o.h = y4.h + a.c_dt6 * (((k4.h + two * kk2.h) + two * kk3.h) + k4.h);
                            store_row(R - 4, o);
                        } else {
                            store_row(y0 - 1, Z);
                        }
                        S3[r2(-3)] = s3;  // after k4 read S3[r2(-5)] (same slot)
                        K3[r2(-3)] = k3;
                    } else {
                        store_row(y0 - 1, Z);
                    }
                    S2[r2(-2)] = s2;  // after k3 read S2[r2(-4)] (same slot)
                    K2[r2(-2)] = k2;  // after the final combination read K2[r2(-4)]
                }
            } else {
                store_row(y0 - 1, Z);
            }
            S1[r2(-1)] = s1;  // after k2 read S1[r2(-3)] (same slot)
        }
        // LDS-resident y: row R-2 becomes R-3 / R-4 of the next bodies (its slot held row
        // R-4, read above)
        if constexpr (kLdsY) Y[r2(-2)] = yR2;
    };

#undef YROW
    auto march = [&](auto Xc, auto Yc) {
        auto period = [&](auto Wc, int R) {
            [&]<int... Ps>(std::integer_sequence<int, Ps...>) {
                (body(std::integral_constant<int, Ps>{}, Xc, Yc, Wc, R + Ps), ...);
            }(std::make_integer_sequence<int, kU>{});
        };
        period(std::true_type{}, R0);  // R1 - R0 >= kU: the march spans >= 2 NST rows
        for (int R = R0 + kU; R < R1; R += kU) period(std::false_type{}, R);
        if constexpr (kDma) __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));  // no DMA into LDS after exit
    };
    // global edges matter only to strips / segments within NST cells of them
    const bool xclamp = strip == 0 || (strip + 1) * out_w >= g.W - NST;
    const bool yclamp = (g.top_clamp && y0 < NST) || (g.bot_clamp && y1 > g.H - NST);
    if (xclamp) {
        if (yclamp) march(std::true_type{}, std::true_type{});
        else march(std::true_type{}, std::false_type{});
    } else {
        if (yclamp) march(std::false_type{}, std::true_type{});
        else march(std::false_type{}, std::false_type{});
    }
}

// Launch one y-row mode (PF: > 0 VGPR prefetch, 0 LDS-DMA, < 0 LDS-resident y) of the DPP
// kernel: each mode's instantiations are compiled in a translation unit of their own
// (ws_fused_dpp.hip, ws_fused_dpp_dma.hip, ws_fused_dpp_ldsy.hip) so the build runs them in
// parallel.
template <typename T, int PF>
hipError_t launch_dpp_impl(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s) {
    const int out_w = a.out_w;
    constexpr bool dma = PF <= 0;
    if (out_w < 1 || out_w > kWave - 2 * fused_margin(dma ? kFusedDppDma : kFusedDpp, nstages, (int)sizeof(T)))
        return hipErrorInvalidValue;
    if (dma && out_w % (16 / (int)sizeof(T)) != 0) return hipErrorInvalidValue;  // chunk-aligned strips
    const int nstrips = (g.W + out_w - 1) / out_w;
    const int nsegs = a.seg_n;
    if (nsegs <= 0) return hipSuccess;
    const int64_t nblocks = (int64_t)nstrips * nsegs * g.L;
    if (nblocks > 0x7fffffff) return hipErrorInvalidValue;
    // buffer descriptors span one segment's rows (+ margins); offsets are 32-bit and the
    // dropped-store voffset is 2^31
    const int64_t span = (int64_t)(a.seg_rows + 2 * nstages + 3 * kUMax) * g.pitch * (int64_t)sizeof(T);
    if (span >= 0x7fffffff) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((nblocks + kWpb - 1) / kWpb)), block(kWave * kWpb);
    const int sp_mode = fused_sp_mode(a);  // spacing mode (ws_fused.h)
#define WS_DPP_GO(N, P2) hipLaunchKernelGGL((fused_dpp_kernel<T, N, P2, PF>), grid, block, 0, s, a, g, nstrips, nsegs)
#define WS_DPP_LAUNCH(N)                                  \
    if (sp_mode == kSpScaled) WS_DPP_GO(N, kSpScaled);    \
    else if (sp_mode == kSpMul) WS_DPP_GO(N, kSpMul);     \
    else WS_DPP_GO(N, kSpDiv);
    switch (nstages) {
        case 1: WS_DPP_LAUNCH(1) break;
        case 2: WS_DPP_LAUNCH(2) break;
        case 4: WS_DPP_LAUNCH(4) break;
        default: return hipErrorInvalidValue;
    }
#undef WS_DPP_LAUNCH
#undef WS_DPP_GO
    return hipGetLastError();
}

}  // namespace
}  // namespace ws
