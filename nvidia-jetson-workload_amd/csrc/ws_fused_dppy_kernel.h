// Fused multi-stage time step, wave-independent variant ("dppy"): one 64-lane wave per
// column strip, horizontal neighbours by DPP lane shifts (wave_shr:1 / wave_shl:1) -- no
// workgroup barrier -- and the y rows staged by LDS-DMA and read from LDS in place.
//
// Lane width CPL: one column per lane (64-column strips, variant "dppy"), or an adjacent
// column pair per lane (128-column strips, variant "x2y"). With pairs, of a cell's two
// horizontal neighbours one is the lane's own other column -- half the DPP moves per cell --
// the strip overlap is 2 * margin of 128 columns instead of 64, and fp32 pairs run as packed
// fp32 (v_pk_*) instructions. Every operation is element-wise, so both widths give the
// same bits.
//
// Same march as ws_fused.hip (one kernel per time step; y read once, y' written once;
// stage s = 1..NST computes row R - s while row R arrives; register rings indexed by a
// compile-time phase), but every wave runs free: nothing synchronises it with any other
// wave, so a wave waiting on HBM never holds its neighbours back. The price is halo
// redundancy: a 64-column strip outputs 64 - 2*margin columns.
//
// y rows: LDS-DMA (buffer_load_dwordx4 ... lds, 16 bytes per lane: one instruction per
// field moves kG = 16 / (CPL sizeof(T)) rows of the strip) into a ring kD rows ahead; each
// body reads the three rows stage 1 needs (R-2, R-1, R) straight from the ring, only rows R-3
// and R-4 (the late stage updates) live in VGPRs.
// The compiler does not order LDS reads after LDS-DMA writes, so the kernel waits itself:
// every body issues exactly 3 stores and every kG-th body 3 DMAs, a fixed count of younger
// vector-memory ops at each wait (kWaitN).
//
// Temporal blocking (NSTEP = 2): one launch advances two time steps. The march chains the
// second step's stages behind the first's: the first step's output row (R - NST) is the
// second step's "arriving" row, its last two rows sit in a register ring, and only the
// second step's output is stored -- y_n is read once and y_{n+2} written once, halving the
// HBM bytes per step, for a dependency cone twice as deep (margins of 2 NST columns, 4 NST
// warm-up rows per segment).
//
// Arithmetic per cell: the reference's, in the reference's order
// (weather_simulation.cpp:160-455, 473-540), or fast numerics (ws_fused.h) by spacing mode.
#pragma once

#include <type_traits>
#include <utility>

#include "ws_fused_dev.h"
#include "ws_knobs.h"

namespace ws {
namespace {  // kernels: internal to each translation unit

using namespace dev;

constexpr int kWave = 64;

template <typename T>
using P2 = T __attribute__((ext_vector_type(2)));

// A lane's cells at a global x edge: its (first) column is x = 0 (lo) / x = W - 1 (hi); a
// pair's second column is x = W - 1 (hi1; it is never x = 0: pairs start on even columns).
struct XEdge {
    bool lo, hi, hi1;
};

// A stage's x-derivatives (u_x, v_x, h_x) of its mid row from the mid row's left / right
// neighbours l / r (DPP lane shifts, or LDS reads: see kLdsStages below). XCLAMP: the strip
// touches a global x edge, where the reference clamps the neighbour index to the cell itself
// (weather_simulation.cpp:510-513). VT = T, or P2<T> for a column pair (element-wise).
template <int MODE, bool XCLAMP, typename VT, typename T>
__device__ __forceinline__ V3<VT> stage_x(const XEdge& e, const V3<VT>& mid, V3<VT> l, V3<VT> r, const Spacing<T>& sp) {
    if constexpr (XCLAMP) {
        if constexpr (std::is_same_v<VT, T>) {
            l = V3<VT>{e.lo ? mid.u : l.u, e.lo ? mid.v : l.v, e.lo ? mid.h : l.h};
            r = V3<VT>{e.hi ? mid.u : r.u, e.hi ? mid.v : r.v, e.hi ? mid.h : r.h};
        } else {
            // a pair's inner neighbours are its own columns; only the outer ones clamp
            if (e.lo) { l.u.x = mid.u.x; l.v.x = mid.v.x; l.h.x = mid.h.x; }
            if (e.hi) { r.u.x = mid.u.x; r.v.x = mid.v.x; r.h.x = mid.h.x; }
            if (e.hi1) { r.u.y = mid.u.y; r.v.y = mid.v.y; r.h.y = mid.h.y; }
        }
    }
    return xdiffs<MODE>(l, r, sp);
}

// One stage at row j from rows j-1 (up), j (mid), j+1 (down) of the previous stage and the mid
// row's x-derivatives X (stage_x). YCLAMP: the segment touches a global y edge (clamp-to-self).
template <int MODE, bool YCLAMP, typename VT, typename T>
__device__ __forceinline__ V3<VT> stage_tend_x(int j, const Geom& g, const V3<VT>& up, const V3<VT>& mid,
                                               const V3<VT>& down, const V3<VT>& X, const Spacing<T>& sp, T grav,
                                               T cor) {
    if constexpr (YCLAMP) {
        const bool ytop = (j == 0) && g.top_clamp;
        const bool ybot = (j == g.H - 1) && g.bot_clamp;
        const V3<VT> t = ytop ? mid : up;
        const V3<VT> b = ybot ? mid : down;
        return tend_x<MODE>(mid, X, t, b, sp, grav, cor);
    } else {
        return tend_x<MODE>(mid, X, up, down, sp, grav, cor);
    }
}

// left / right neighbours by DPP lane shifts: one column per lane -- the neighbouring
// lanes' values; a column pair (x, y) -- (left lane's y, own x) and (own y, right lane's x)
template <typename T>
__device__ __forceinline__ void dpp_lr(const T& m, T& l, T& r) {
    l = from_left(m);
    r = from_right(m);
}
template <typename T>
__device__ __forceinline__ void dpp_lr(const P2<T>& m, P2<T>& l, P2<T>& r) {
    l = P2<T>{from_left(m.y), m.x};
    r = P2<T>{m.y, from_right(m.x)};
}
template <typename VT>
__device__ __forceinline__ void dpp_lr3(const V3<VT>& m, V3<VT>& l, V3<VT>& r) {
    dpp_lr(m.u, l.u, r.u);
    dpp_lr(m.v, l.v, r.v);
    dpp_lr(m.h, l.h, r.h);
}
// the same from an LDS row of the values (row[lane] = this lane's): lanes 0 / 63 read past
// the row -- margin lanes only (the previous / next row, or outside the array: LDS returns 0)
template <typename T>
__device__ __forceinline__ void lds_lr(const T* row, int lane, const T& m, T& l, T& r) {
    l = row[lane - 1];
    r = row[lane + 1];
}
template <typename T>
__device__ __forceinline__ void lds_lr(const P2<T>* row, int lane, const P2<T>& m, P2<T>& l, P2<T>& r) {
    // whole neighbouring pairs (lane-contiguous reads, no bank conflicts; reading the single
    // columns 2 lane - 1 / 2 lane + 2 strides the banks by two)
    l = P2<T>{row[lane - 1].y, m.x};
    r = P2<T>{m.y, row[lane + 1].x};
}

// Stages of the launch's cone (bit gs - 1 for stage gs = q NST + s) that take their
// horizontal neighbours from LDS instead of DPP lane shifts: an fp64 neighbour is two 32-bit
// DPP moves (VALU), an LDS read is not VALU. Stage 1's mid row is already in the LDS-DMA
// ring (two extra ds_read per field); a later stage's mid row is the previous body's output
// of the stage before, which that body writes to a per-wave LDS row (double-buffered by body
// parity: three ds_write + six ds_read per stage and body). LDS bandwidth and capacity bound
// how many stages can move (measured). Default (-1): stage 1 for one column
// per lane; none for column pairs, whose DPP moves are already halved (C3 fp32 pairs: 0.0183
// -> 0.0167 ms/step without the LDS reads, C4 0.145 -> 0.133).
// LDS-DMA prefetch distance in groups of kG rows; 0 = by precision (see kPF). Round 1 (one
// step per launch, exact fp64): 2 or 3 groups measured -3 / -8 %; round 2 (two steps per
// launch, fast fp64: bodies twice as long, so one group gave the DMA ~1000 cycles): 2 groups
// +9 %, 3 groups +0 %.

// Workgroup barrier ordering LDS traffic only (no global-memory fence: the DMA prefetch stays
// in flight across it)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// s_waitcnt immediate for "vmcnt <= n" alone (gfx9 encoding: vmcnt[3:0], expcnt[6:4],
// lgkmcnt[11:8], vmcnt[15:14]); the other counters at their maxima = not waited on
constexpr int waitcnt_vm(int n) { return (n & 0xF) | ((n >> 4) << 14) | (0x7 << 4) | (0xF << 8); }

// Per time step of a launch: the march's register rings (parity-indexed by row)
template <typename VT>
struct StepRings {
    V3<VT> Y[2];                  // Y[r % 2] = the step's input row r, r <= R-3
    V3<VT> S1[2], S2[2], S3[2];   // [r % 2] = stage output at row r
    V3<VT> K2[2], K3[2];          // RK4 stage-2 tendency / stage-3 keep (rk4_keep3) at row r
    V3<VT> O[2];                  // the step's last output rows (the next step's input), NSTEP > 1
};

// SPLIT (two steps per launch, one column per lane; variant "pc"): a workgroup of two waves on
// one strip and segment, wave 0 the producer of the first time step (LDS-DMA of y_n, its four
// stages, its output rows into an LDS ring), wave 1 the consumer (the second step's stages from
// that ring, the stores of y_{n+2}). Each wave holds one step's register rings, so the kernel
// fits 4 waves per SIMD where the one-wave two-step march (221 VGPRs) fits 2. The consumer runs
// kLag = 2 march bodies behind the producer; an LDS-only workgroup barrier every 2 bodies hands
// the rows over (the consumer reads rows the producer finished before the last barrier, the
// producer overwrites slots the consumer finished before it: kU >= 6 ring slots).
constexpr int kLag = 2;  // the consumer's lag = the barrier interval, in bodies (1 measured 1 % slower)

// the producer / consumer kernel: 4 waves per SIMD (128 VGPRs), fp64 pairs 2
constexpr int pc_min_waves(int cpl, int elem) { return cpl == 2 && elem == 8 ? 2 : 4; }

// Diagnostic builds only (tools/wave_timeline.py, -DWS_WAVE_STAMPS): each workgroup's first lane
// records its start / end time (100 MHz real-time counter and shader clock), its hardware
// placement (HW_ID: wave slot, SIMD, CU, SE; XCC id) and work item -- into a buffer no other code
// reads, via ordinary vector stores. Not part of the product library.
#ifdef WS_WAVE_STAMPS
constexpr int kStampWords = 8;
constexpr int kStampMax = 1 << 16;
__device__ unsigned long long g_wave_stamps[kStampMax * kStampWords];
#endif
template <typename T, int NST, int NSTEP, int MODE, int CPL, bool SPLIT = false>
__global__ __launch_bounds__(SPLIT ? 2 * kWave : kWave, SPLIT ? pc_min_waves(CPL, (int)sizeof(T)) : 1) void fused_dppy_kernel(FusedArgs<T> a, Geom g, int nstrips, int nsegs) {
    static_assert(CPL == 1 || CPL == 2, "one column or a column pair per lane");
    static_assert(!SPLIT || NSTEP == 2, "producer / consumer: a two-step launch");
    using VT = std::conditional_t<CPL == 1, T, P2<T>>;     // a lane's cells of one row
    constexpr int kG = 16 / (int)sizeof(VT);               // rows per DMA instruction
    // DMA rows in flight: WS_DPPY_PF groups ahead (0 = 4 rows; C2 two-step fp64: 0.1272 ->
    // 0.1162 ms/step at 4 rows against 2; C3 fp32 pairs: 0.0260 -> 0.0222 at 4 rows
    // against 2, 0.0256 at 6). The producer's bodies are one step long: at least 2 rows ahead
    // (fp64 / fp32 pairs: one group; fp64 pairs: two).
    constexpr int kPF = SPLIT ? (2 / kG > 1 ? 2 / kG : 1) : WS_DPPY_PF > 0 ? WS_DPPY_PF : (4 / kG > 1 ? 4 / kG : 1);
    constexpr int kD = kG * kPF;
    constexpr int kR = kG > 2 ? kG : 2;                     // ring granule: whole groups, even
    constexpr int kNR = (kD + kG + 2 + kR - 1) / kR * kR;   // ring: rows R-2 .. R+kD+kG-1
    // march unroll: ring slot == phase (SPLIT: >= 6, the handover ring's slots, see above)
    // SPLIT: between two barriers (every kLag bodies) the consumer reads the rows produced before
    // the first of them while the producer writes its newest kLag slots, so the handover ring
    // needs >= 2 kLag + 2 slots, and the barrier intervals must tile the unrolled period
    constexpr int kHandover = 2 * kLag + 2;
    constexpr int kUlcm = kNR % kLag == 0 ? kNR : kNR * kLag;  // a multiple of kNR and of kLag (kLag <= 2 divides kNR)
    constexpr int kU = SPLIT ? (kHandover + kUlcm - 1) / kUlcm * kUlcm : kNR;
    static_assert(!SPLIT || (kU % kLag == 0 && kU >= 2 * kLag + 2 && kU % kNR == 0), "handover ring vs barrier interval");
    constexpr int kNS = NST * NSTEP;                        // stages per launch (the cone depth)
    // warm-up periods: stage gs (1..kNS) is needed from march row R - R0 >= 2 gs on (the
    // consumer's bodies lag kLag rows). At most three are peeled: a stage computed before it
    // enters the cone only reaches rows that are never stored (skipping it saves work only).
    constexpr int kWarm = 2 * kNS + (SPLIT ? kLag : 0);
    constexpr int kNW = (kWarm + kU - 1) / kU < 3 ? (kWarm + kU - 1) / kU : 3;
    // a group's DMA may overwrite only slots whose rows were read in an earlier body
    static_assert(kU % kG == 0 && kU % 2 == 0 && kU % kNR == 0 && kNR >= kD + kG + 2 && kD % kG == 0, "DMA ring");
    static_assert(NSTEP == 1 || NSTEP == 2 || ((NSTEP == 4 || NSTEP == 8) && !SPLIT), "1, 2, 4 or 8 steps per launch");
    // Wait for a group's DMAs before reading it: vmcnt <= the number of vector-memory LOADS
    // issued after them (the DMAs in between, incl. the reading body's own). Stores are not
    // counted: a store may complete before an older load, so a count that includes them can
    // drop below the threshold while the group is still in flight (seen as stale rows at
    // 4096^2). Loads complete in order.
    constexpr int kWaitN = 3 * (kD / kG);
    constexpr unsigned kLdsX = ((WS_DPPY_LDSX >= 0 ? (unsigned)(WS_DPPY_LDSX) : CPL == 1 ? 0x1u : 0x0u) |
                                (SPLIT ? 1u << NST : 0u)) & ((1u << kNS) - 1u);
    constexpr auto ldsx = [](int gs) { return ((kLdsX >> (gs - 1)) & 1u) != 0; };
    // LDS row slots of the stages (other than stage 1) that read neighbours from LDS
    // (SPLIT: the consumer's first stage reads the handover ring, no LDS row of its own)
    constexpr unsigned kXRow = kLdsX & ~1u & ~(SPLIT ? 1u << NST : 0u);
    constexpr auto xslot = [](int gs) { return __builtin_popcount(kXRow & ((1u << (gs - 1)) - 1u)); };
    constexpr int kNX = __builtin_popcount(kXRow);

#ifdef WS_WAVE_STAMPS
    const unsigned long long st_r0 = __builtin_amdgcn_s_memrealtime(), st_c0 = __builtin_amdgcn_s_memtime();
#endif
    if (a.prio > 0) __builtin_amdgcn_s_setprio(3);  // (wave-uniform: a kernel argument)
    const int w = xcd_work_item();  // XCD-aware: neighbouring strips share an L2
    int strip, y0, y1, level;
    if (a.chains) {  // chain schedule: this workgroup's march from the host's table
        const ChainSeg c = a.chains[w];
        strip = c.unit % nstrips;
        level = c.unit / nstrips;
        y0 = c.y0;
        y1 = c.y1;
    } else {
        strip = w % nstrips;
        fused_rows(a, (w / nstrips) % nsegs, y0, y1);
        level = w / (nstrips * nsegs);
    }

    const int lane = (int)threadIdx.x % kWave;
    // SPLIT: wave 0 produces the first time step, wave 1 consumes it (wave-uniform)
    const bool producer = !SPLIT || __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave) == 0;
    // left margin: the cone (kNS) rounded up to whole 16-byte chunks, so a strip's DMA chunks
    // never straddle column 0 (a partly negative chunk is dropped whole by the range check)
    constexpr int kC = 16 / (int)sizeof(T);  // columns per chunk
    constexpr int kM = (kNS + kC - 1) / kC * kC;
    const int out_w = a.out_w;
    // the strip's window and output columns (edge-aware layout, ws_fused.h strip_geom)
    const StripGeom sg = strip_geom(strip, nstrips, g.W, kWave * CPL, kM, kC, out_w);
    const int x = sg.xs + CPL * lane;  // this lane's (first) global column
    // a pair is stored whole: its second column is x + 1 < W, or row padding (x < W <= pitch,
    // both even), whose content is unspecified
    const bool xout = x >= sg.o0 && x < sg.o1;
    const XEdge xe{x == 0, x == g.W - 1, CPL == 2 && x + 1 == g.W - 1};

    const int row_lo = g.top_clamp ? 0 : -g.halo;  // rows that exist in memory (halo rows in slabs)
    const int row_hi = g.bot_clamp ? g.H : g.H + g.halo;

    // Buffer addressing: one descriptor per field, based at this wave's first row (all
    // wave-uniform, SGPRs), the row as a scalar byte offset, the lane's column as a fixed
    // 32-bit voffset -- no per-row VALU address arithmetic. Stores of lanes outside the
    // strip's output columns get an out-of-range voffset: the buffer range check drops them
    // (no exec-mask branch). launch_fused_step_dppy checks the byte ranges fit.
    const int64_t lofs = (int64_t)level * g.lstride;
    const int rbase = max(y0 - kNS, row_lo);
    // past the last input row the output rows [y0, y1) depend on (their cone: y1 + kNS - 1).
    // The march's prefetch runs further -- kD rows ahead, rounded up to its unroll, SPLIT's
    // lag -- but rows past the cone feed only rows that are never stored, so their DMAs are
    // left out of range: the buffer range check drops them without a memory access (round 4:
    // up to kU + kD + kG + kLag rows of HBM reads per segment or chain saved)
    const int rtop = min(row_hi, y1 + kNS);
    const uint32_t in_bytes = (uint32_t)((int64_t)(rtop - rbase) * g.pitch * sizeof(T));
    const uint32_t out_bytes = (uint32_t)((int64_t)(y1 - y0) * g.pitch * sizeof(T));
    const int64_t ib = lofs + (int64_t)rbase * g.pitch, ob = lofs + (int64_t)y0 * g.pitch;
    const auto ru = make_rsrc(a.in_u + ib, in_bytes), rv = make_rsrc(a.in_v + ib, in_bytes),
               rh = make_rsrc(a.in_h + ib, in_bytes);
    const auto wu = make_rsrc(a.out_u + ob, out_bytes), wv = make_rsrc(a.out_v + ob, out_bytes),
               wh = make_rsrc(a.out_h + ob, out_bytes);
    const uint32_t row_bytes = (uint32_t)g.pitch * sizeof(T);
    const uint32_t soff = xout ? (uint32_t)x * sizeof(T) : kDropped;

    // Stores are issued for every row, unconditionally: rows outside [y0, y1) are dropped by
    // the range check through the voffset (a branch around them makes the compiler's vmcnt
    // bookkeeping merge both paths and drain the prefetch at every row).
    auto store_row = [&](int j, const V3<VT>& o) {
        const bool row_ok = j >= y0 && j < y1;
        const uint32_t so = row_ok ? (uint32_t)(j - y0) * row_bytes : 0u;
        const uint32_t vo = row_ok ? soff : kDropped;
        // (a.cached is a kernel argument: wave-uniform, both arms issue the same three stores)
        if (a.cached) {
            buf_store_nt<VT, 0>(o.u, wu, vo, so);
            buf_store_nt<VT, 0>(o.v, wv, vo, so);
            buf_store_nt<VT, 0>(o.h, wh, vo, so);
        } else {
            buf_store_nt<VT>(o.u, wu, vo, so);
            buf_store_nt<VT>(o.v, wv, vo, so);
            buf_store_nt<VT>(o.h, wh, vo, so);
        }
    };

    // LDS-DMA ring: ring[field][slot][lane], slot = (row - R0) % kNR; one DMA fills kG
    // consecutive slots (64 lanes x 16 B = kG rows of the strip)
    __shared__ __attribute__((aligned(16))) VT ring[3][kNR][kWave];
    const int dk = lane / (kWave / kG);  // row of the group this lane fetches
    const int dcol = sg.xs * (int)sizeof(T) + (lane % (kWave / kG)) * 16;  // 16-B aligned
    auto dma = [&](int q, int slot) {  // rows q .. q + kG - 1 into slots slot .. slot + kG - 1
        const int r = min(max(q + dk, row_lo), row_hi - 1);
        // chunks left of column 0 (whole chunks: kM is chunk-aligned) wrap to huge offsets or
        // read the previous row, chunks past the row end read the next row: margin lanes
        // only, never read by an output lane
        const uint32_t vo = (uint32_t)((r - rbase) * (int)row_bytes + dcol);
        lds_dma16(ru, &ring[0][slot][0], vo);
        lds_dma16(rv, &ring[1][slot][0], vo);
        lds_dma16(rh, &ring[2][slot][0], vo);
    };
    auto read_row = [&](int slot) -> V3<VT> { return V3<VT>{ring[0][slot][lane], ring[1][slot][lane], ring[2][slot][lane]}; };
    // SPLIT: the handover ring of the first step's output rows, hring[field][slot][lane], slot =
    // the producing body's march phase (row R - NST of the body at phase P goes to slot P)
    __shared__ VT hring[3][SPLIT ? kU : 1][kWave];
    // per-wave LDS rows of the LDS-neighbour stages: xrow[parity][slot][field][lane]
    __shared__ VT xrow[2][kNX > 0 ? kNX : 1][3][kWave];
    auto xput = [&](auto Pc, auto GSc, const V3<VT>& v) {
        constexpr int P = decltype(Pc)::value, gs = decltype(GSc)::value;
        if constexpr (gs > 1 && ldsx(gs) && !(SPLIT && gs == NST + 1)) {
            auto& b = xrow[P % 2][xslot(gs)];
            b[0][lane] = v.u;
            b[1][lane] = v.v;
            b[2][lane] = v.h;
        }
    };
    // neighbours of stage gs's mid row `mid` (its ring slot `rs` for stage 1)
    auto nbrs = [&](auto Pc, auto GSc, const V3<VT>& mid, int rs, V3<VT>& l, V3<VT>& r) {
        constexpr int P = decltype(Pc)::value, gs = decltype(GSc)::value;
        if constexpr (!ldsx(gs)) {
            dpp_lr3(mid, l, r);
        } else {
            // stage 1: the mid row's ring slot; the consumer's first stage: the mid row's
            // handover slot; later stages: the previous body's LDS row
            if constexpr (SPLIT && gs == NST + 1) {
                lds_lr(hring[0][rs], lane, mid.u, l.u, r.u);
                lds_lr(hring[1][rs], lane, mid.v, l.v, r.v);
                lds_lr(hring[2][rs], lane, mid.h, l.h, r.h);
            } else if constexpr (gs == 1) {
                lds_lr(ring[0][rs], lane, mid.u, l.u, r.u);
                lds_lr(ring[1][rs], lane, mid.v, l.v, r.v);
                lds_lr(ring[2][rs], lane, mid.h, l.h, r.h);
            } else {
                auto& b = xrow[(P + 1) % 2][xslot(gs)];
                lds_lr(b[0], lane, mid.u, l.u, r.u);
                lds_lr(b[1], lane, mid.v, l.v, r.v);
                lds_lr(b[2], lane, mid.h, l.h, r.h);
            }
        }
    };

    // stage gs's x-derivatives of its mid row (neighbours by nbrs)
    auto xderiv = [&](auto Pc, auto GSc, auto Xc, const V3<VT>& mid, int rs, const Spacing<T>& sp) __attribute__((always_inline)) -> V3<VT> {
        V3<VT> l, r;
        nbrs(Pc, GSc, mid, rs, l, r);
        return stage_x<MODE, decltype(Xc)::value>(xe, mid, l, r, sp);
    };

    const V3<VT> Z{VT{}, VT{}, VT{}};
    StepRings<VT> st[NSTEP];
#pragma unroll
    for (int q = 0; q < NSTEP; ++q)
#pragma unroll
        for (int i = 0; i < 2; ++i) st[q].Y[i] = st[q].S1[i] = st[q].S2[i] = st[q].S3[i] = st[q].K2[i] = st[q].K3[i] = st[q].O[i] = Z;

    const int R0 = y0 - kNS;
    // the first march row no stored output depends on: the body at row R stores row R - kNS
    // (SPLIT: the consumer's bodies lag kLag rows behind the march). The march runs whole
    // unrolled periods of kU bodies up to the last period that reaches it, and that period only
    // as far as Rstop (a wave-uniform test per body): a chain of ~22 rows plus its 16 warm-up rows
    // rounded up to whole periods ran 3.5 bodies past its cone on average
    // (Only the one-column fp64 march -- C2, its slab shares -- and the fp32 pair march -- C3,
    // C4 -- end at Rstop; the others keep whole periods, R1 rounded up: the guarded period made
    // the split kernels spill at their register caps, and in the fp64-pair and one-column fp32
    // instantiations the compiler merged the guarded bodies' stores into blocks that
    // tests/test_isa_hazards.py rule 2 cannot prove address-defined.)
    constexpr bool kTail = !SPLIT && ((CPL == 1 && sizeof(T) == 8) || (CPL == 2 && sizeof(T) == 4));
    const int Rstop = kTail ? y1 + kNS : R0 + (y1 + kNS + (SPLIT ? kLag : 0) - R0 + kU - 1) / kU * kU;

    // One time step's stages at march row Rq of its input (rows Rq, Rq-1, Rq-2 = i0, i1, i2):
    // stage s computes row Rq - s; the step's output row Rq - NST goes to `out`. Stage s of
    // step q is stage gs = q NST + s of the launch's cone; `ON(gs)` says whether this body
    // needs it (warm-up: the first bodies of a segment skip stages outside the segment's
    // cone; whatever a body computes beyond the cone only ever reaches rows that are not
    // stored). Ring slots are indexed by the parity of the body phase P.
    auto step = [&](auto Qc, auto Pc, auto Xc, auto Yc, auto ONc, StepRings<VT>& S, const V3<VT>& i0,
                    const V3<VT>& i1, const V3<VT>& i2, int Rq, V3<VT>& out) __attribute__((always_inline)) {
        constexpr int q = decltype(Qc)::value;
        constexpr int P = decltype(Pc)::value;
                constexpr bool YC = decltype(Yc)::value;
        constexpr auto on = [](int s) { return decltype(ONc){}(q * NST + s); };
        constexpr auto r2 = [](int d) { return ((P + d) % 2 + 2) % 2; };
        auto gsc = [](auto sc) { return std::integral_constant<int, q * NST + decltype(sc)::value>{}; };
        using S1c = std::integral_constant<int, 1>;
        using S2c = std::integral_constant<int, 2>;
        using S3c = std::integral_constant<int, 3>;
        using S4c = std::integral_constant<int, 4>;
        // ring slot of row R-1 (step 1's stage-1 mid); the consumer's: the handover slot of the
        // row produced one body before the one arriving (bodies lag kLag phases)
        constexpr int rs1 = SPLIT && q == 1 ? ((P - kLag - 1) % kU + kU) % kU : ((P - 1) % kNR + kNR) % kNR;
        // stage 1's mid row next body (written even while stage 1 is outside the cone: the
        // next body may need it)
        xput(Pc, gsc(S1c{}), i0);
        if constexpr (on(1)) {
            // stage 1 of the launch reads the current grid (its spacing sp1); every later stage
            // a temp / next grid (the config's spacing sp2; the host launches two steps at once
            // only when sp1 == sp2)
            const Spacing<T>& sp_in = q == 0 ? a.sp1 : a.sp2;
            const V3<VT> k1 = stage_tend_x<MODE, YC>(Rq - 1, g, i2, i1, i0, xderiv(Pc, gsc(S1c{}), Xc, i1, rs1, sp_in),
                                                     sp_in, a.gravity, a.coriolis_f);
            if constexpr (NST == 1) {
                out = axpy<MODE>(i1, a.c_dt, k1);  // Euler: y + dt k
            } else {
                const V3<VT> s1 = axpy<MODE>(i1, a.c_half, k1);  // y + (0.5f dt) k
                xput(Pc, gsc(S2c{}), s1);
                if constexpr (on(2)) {
                    const V3<VT> k2 = stage_tend_x<MODE, YC>(Rq - 2, g, S.S1[r2(-3)], S.S1[r2(-2)], s1,
                                                             xderiv(Pc, gsc(S2c{}), Xc, S.S1[r2(-2)], 0, a.sp2), a.sp2,
                                                             a.gravity, a.coriolis_f);
                    if constexpr (NST == 2) {
                        out = axpy<MODE>(i2, a.c_dt, k2);  // RK2: y + dt k2
                    } else {
                        const V3<VT> s2 = axpy<MODE>(i2, a.c_half, k2);
                        xput(Pc, gsc(S3c{}), s2);
                        if constexpr (on(3)) {
                            const V3<VT> k3 = stage_tend_x<MODE, YC>(Rq - 3, g, S.S2[r2(-4)], S.S2[r2(-3)], s2,
                                                                     xderiv(Pc, gsc(S3c{}), Xc, S.S2[r2(-3)], 0, a.sp2),
                                                                     a.sp2, a.gravity, a.coriolis_f);
                            const V3<VT> s3 = axpy<MODE>(S.Y[r2(-3)], a.c_dt, k3);
                            xput(Pc, gsc(S4c{}), s3);
                            if constexpr (on(4)) {
                                const V3<VT> k4 = stage_tend_x<MODE, YC>(
                                    Rq - 4, g, S.S3[r2(-5)], S.S3[r2(-4)], s3,
                                    xderiv(Pc, gsc(S4c{}), Xc, S.S3[r2(-4)], 0, a.sp2), a.sp2, a.gravity, a.coriolis_f);
                                // y + dt/6 * (((k4 + 2 k2) + 2 k3) + k4)   (k1 aliases k4, :437-451)
                                out = rk4_final<MODE>(S.Y[r2(-4)], a.c_dt6, k4, S.K2[r2(-4)], S.K3[r2(-4)]);
                            }
                            S.S3[r2(-3)] = s3;  // after k4 read S3[r2(-5)] (same slot)
                            S.K3[r2(-3)] = rk4_keep3<MODE>(S.K2[r2(-3)], k3);
                        }
                        S.S2[r2(-2)] = s2;  // after k3 read S2[r2(-4)] (same slot)
                        S.K2[r2(-2)] = k2;  // after the final combination read K2[r2(-4)]
                    }
                }
                S.S1[r2(-1)] = s1;  // after k2 read S1[r2(-3)] (same slot)
            }
            S.Y[r2(-2)] = i2;  // row Rq-2 is Rq-3 / Rq-4 of the next bodies (its slot held Rq-4, read above)
        }
    };

    // One march body at row R: DMA / wait, the y rows from the LDS ring, the steps' stages, and
    // one stored row (the last step's output, or a dropped store while it is outside the
    // cone, keeping every body's store pattern the same). KW = warm-up period index (-1 =
    // steady state): the body's march position is R - R0 = KW kU + P.
    auto body = [&](auto Pc, auto Xc, auto Yc, auto KWc, int R) __attribute__((always_inline)) {
        constexpr int P = decltype(Pc)::value;
        constexpr int KW = decltype(KWc)::value;
        struct On {
            constexpr bool operator()(int gs) const { return KW < 0 || KW * kU + P >= 2 * gs; }
        };
        constexpr auto r2 = [](int d) { return ((P + d) % 2 + 2) % 2; };
        constexpr auto sl = [](int d) { return ((P + d) % kNR + kNR) % kNR; };  // ring slot of row R+d
        if constexpr (P % kG == 0) {
            dma(R + kD, sl(kD));  // slots of rows R+kD-kNR.. (<= R-4): read in earlier bodies
            __builtin_amdgcn_s_waitcnt(waitcnt_vm(kWaitN));  // rows R .. R+kG-1 have landed
        }
        const V3<VT> yR0 = read_row(sl(0)), yR1 = read_row(sl(-1)), yR2 = read_row(sl(-2));
        // keep the row's DMA at the head of the body: the scheduler would otherwise sink it
        // below the stencil math, shortening the prefetch distance
        __builtin_amdgcn_sched_barrier(0);
        V3<VT> o = Z;
        step(std::integral_constant<int, 0>{}, Pc, Xc, Yc, On{}, st[0], yR0, yR1, yR2, R, o);
        // step q's input rows R-qNST (step q-1's output, just computed), R-qNST-1, R-qNST-2
        // (step q-1's output ring)
        [&]<int... Qs>(std::integer_sequence<int, Qs...>) {
            ([&] {
                constexpr int q = Qs + 1;
                const V3<VT> i1 = st[q - 1].O[r2(-q * NST - 1)], i2 = st[q - 1].O[r2(-q * NST - 2)];
                if constexpr (On{}(q * NST)) st[q - 1].O[r2(-q * NST)] = o;  // the slot of row R-qNST-2, read above
                V3<VT> oq = Z;
                step(std::integral_constant<int, q>{}, Pc, Xc, Yc, On{}, st[q], o, i1, i2, R - q * NST, oq);
                o = oq;
            }(), ...);
        }(std::make_integer_sequence<int, NSTEP - 1>{});
        if constexpr (On{}(NSTEP * NST)) store_row(R - NSTEP * NST, o);
        else store_row(y0 - 1, Z);
    };

    // SPLIT: the producer's body -- the first step at march row R, its output row R - NST into
    // handover slot P (no store)
    auto pbody = [&](auto Pc, auto Xc, auto Yc, auto KWc, int R) __attribute__((always_inline)) {
        constexpr int P = decltype(Pc)::value;
        constexpr int KW = decltype(KWc)::value;
        struct On {
            constexpr bool operator()(int gs) const { return KW < 0 || KW * kU + P >= 2 * gs; }
        };
        constexpr auto sl = [](int d) { return ((P + d) % kNR + kNR) % kNR; };
        if constexpr (P % kG == 0) {
            dma(R + kD, sl(kD));
            __builtin_amdgcn_s_waitcnt(waitcnt_vm(kWaitN));
        }
        const V3<VT> yR0 = read_row(sl(0)), yR1 = read_row(sl(-1)), yR2 = read_row(sl(-2));
        __builtin_amdgcn_sched_barrier(0);
        V3<VT> o0 = Z;
        step(std::integral_constant<int, 0>{}, Pc, Xc, Yc, On{}, st[0], yR0, yR1, yR2, R, o0);
        hring[0][P][lane] = o0.u;
        hring[1][P][lane] = o0.v;
        hring[2][P][lane] = o0.h;
    };
    // SPLIT: the consumer's body at the same phase -- march row R - kLag of the second step: its
    // input rows from the handover slots the producer filled kLag .. kLag + 2 bodies ago, its
    // output row stored
    auto cbody = [&](auto Pc, auto Xc, auto Yc, auto KWc, int R) __attribute__((always_inline)) {
        constexpr int P = decltype(Pc)::value;
        constexpr int KW = decltype(KWc)::value;
        struct On {
            constexpr bool operator()(int gs) const { return KW < 0 || KW * kU + P - kLag >= 2 * gs; }
        };
        constexpr auto hs = [](int d) { return ((P - kLag + d) % kU + kU) % kU; };
        const V3<VT> i0{hring[0][hs(0)][lane], hring[1][hs(0)][lane], hring[2][hs(0)][lane]};
        const V3<VT> i1{hring[0][hs(-1)][lane], hring[1][hs(-1)][lane], hring[2][hs(-1)][lane]};
        const V3<VT> i2{hring[0][hs(-2)][lane], hring[1][hs(-2)][lane], hring[2][hs(-2)][lane]};
        const int Rc = R - kLag;
        V3<VT> o1 = Z;
        step(std::integral_constant<int, 1>{}, Pc, Xc, Yc, On{}, st[1], i0, i1, i2, Rc - NST, o1);
        if constexpr (On{}(2 * NST)) store_row(Rc - 2 * NST, o1);
        else store_row(y0 - 1, Z);
    };

    // ROLE (SPLIT): the producer's or the consumer's march -- two loops, each carrying only its
    // own step's register rings, passing the same barriers (the same periods)
    auto march_role = [&](auto Xc, auto Yc, auto ROLEc) {
        constexpr bool kProd = decltype(ROLEc)::value;
        // the kD virtual bodies before R0: DMAs for rows R0 .. R0 + kD - 1 and (dropped)
        // stores, the same outstanding-op pattern the loop's back edge has (SPLIT: the
        // producer's DMAs only)
        if constexpr (kProd) {
            [&]<int... Vs>(std::integer_sequence<int, Vs...>) {
                ([&] {
                    constexpr int v = Vs - kD;  // -kD .. -1
                    if constexpr (((v % kG) + kG) % kG == 0) dma(R0 + v + kD, v + kD);
                    if constexpr (!SPLIT) store_row(y0 - 1, Z);
                }(), ...);
            }(std::make_integer_sequence<int, kD>{});
        }
        // a period of kU bodies; GUARD: only the bodies before Rstop (the march's last period)
        auto period = [&](auto KWc, int R, auto GUARDc) __attribute__((always_inline)) {
            [&]<int... Ps>(std::integer_sequence<int, Ps...>) {
                ([&] {
                    constexpr int P = Ps;
                    const bool run = !(kTail && decltype(GUARDc)::value) || R + P < Rstop;
                    if constexpr (!SPLIT) {
                        if (run) body(std::integral_constant<int, P>{}, Xc, Yc, KWc, R + P);
                    } else {
                        // both waves pass every barrier: the branch is below it
                        if constexpr (P % kLag == 0) lds_barrier();
                        if (run) {
                            if constexpr (kProd) pbody(std::integral_constant<int, P>{}, Xc, Yc, KWc, R + P);
                            else cbody(std::integral_constant<int, P>{}, Xc, Yc, KWc, R + P);
                        }
                    }
                }(), ...);
            }(std::make_integer_sequence<int, kU>{});
        };
        // warm-up periods (Rstop - R0 > 2 kNS: the first runs; a short march may end in one),
        // then the steady march: whole periods, and the last one guarded
        [&]<int... Ks>(std::integer_sequence<int, Ks...>) {
            ([&] {
                if (Ks == 0 || R0 + Ks * kU < Rstop) period(std::integral_constant<int, Ks>{}, R0 + Ks * kU, std::true_type{});
            }(), ...);
        }(std::make_integer_sequence<int, kNW>{});
        int R = R0 + kNW * kU;
        for (; R + kU <= Rstop; R += kU) period(std::integral_constant<int, -1>{}, R, std::false_type{});
        if constexpr (kTail) {
            if (R < Rstop) period(std::integral_constant<int, -1>{}, R, std::true_type{});
        }
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));  // no DMA into LDS after exit
    };
    auto march = [&](auto Xc, auto Yc) {
        if constexpr (!SPLIT) march_role(Xc, Yc, std::true_type{});
        else if (producer) march_role(Xc, Yc, std::true_type{});
        else march_role(Xc, Yc, std::false_type{});
    };
    // global edges matter only to strips / segments whose outputs' cone (kNS cells) reaches them
    const bool xclamp = sg.o0 <= kNS || sg.o1 + kNS >= g.W;
    const bool yclamp = (g.top_clamp && y0 < kNS) || (g.bot_clamp && y1 > g.H - kNS);
    if (xclamp) {
        if (yclamp) march(std::true_type{}, std::true_type{});
        else march(std::true_type{}, std::false_type{});
    } else {
        if (yclamp) march(std::false_type{}, std::true_type{});
        else march(std::false_type{}, std::false_type{});
    }
#ifdef WS_WAVE_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < (unsigned)kStampMax) {
        const unsigned long long st_r1 = __builtin_amdgcn_s_memrealtime(), st_c1 = __builtin_amdgcn_s_memtime();
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID, all 32 bits
        const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20); // XCC_ID
        unsigned long long* p = g_wave_stamps + (size_t)blockIdx.x * kStampWords;
        p[0] = st_r0; p[1] = st_r1; p[2] = st_c0; p[3] = st_c1;
        p[4] = hw; p[5] = xcc;
        p[6] = (unsigned long long)(unsigned)w | ((unsigned long long)(unsigned)(level * nstrips + strip) << 32);
        p[7] = (unsigned long long)(unsigned)y0 | ((unsigned long long)(unsigned)y1 << 32);
    }
#endif
}

#ifdef WS_WAVE_STAMPS
}  // namespace
// diagnostic export (built into variant libraries only): copy the stamps of the last launch
extern "C" int ws_diag_wave_stamps(void* dst, size_t bytes) {
    if (bytes > sizeof(g_wave_stamps)) bytes = sizeof(g_wave_stamps);
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_wave_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int ws_diag_wave_stamps_reset() {  // zero the records (before the recorded launch)
    void* p = nullptr;
    const hipError_t e = hipGetSymbolAddress(&p, HIP_SYMBOL(g_wave_stamps));
    if (e != hipSuccess) return (int)e;
    return (int)hipMemset(p, 0, sizeof(g_wave_stamps));
}
namespace {
#endif

}  // namespace

// Launch fused_dppy_kernel<T, nstages, NSTEP, mode, CPL> (one translation unit per (T,
// NSTEP, CPL): ws_fused_dppy{,2}_<t>_<n>.hip, compiled in parallel).

// Workgroups of fused_dppy_kernel<T, nstages, NSTEP, mode, CPL, SPLIT> one CU holds at once
// (the chain schedule's round size is this times the CU count).
template <typename T, int NSTEP, int CPL, bool SPLIT = false>
int dppy_blocks_per_cu_impl(int nstages, int sp_mode) {
    int nb = 0;
    const int threads = SPLIT ? 2 * kWave : kWave;
#define WS_DPPY_OCC(N, M)                                                                                            \
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)fused_dppy_kernel<T, N, NSTEP, M, CPL, SPLIT>, \
                                                       threads, 0)
#define WS_DPPY_O1(M) WS_DPPY_OCC(1, M)
#define WS_DPPY_O2(M) WS_DPPY_OCC(2, M)
#define WS_DPPY_O4(M) WS_DPPY_OCC(4, M)
    switch (nstages) {
        case 1: WS_SP_DISPATCH(sp_mode, WS_DPPY_O1) break;
        case 2:  // (eight-step launches: Euler only)
            if constexpr (NSTEP < 8) { WS_SP_DISPATCH(sp_mode, WS_DPPY_O2) }
            break;
        case 4:  // (four-step launches: Euler / RK2 only -- an RK4 cone of 16)
            if constexpr (NSTEP < 4) { WS_SP_DISPATCH(sp_mode, WS_DPPY_O4) }
            break;
        default: return 0;
    }
#undef WS_DPPY_O1
#undef WS_DPPY_O2
#undef WS_DPPY_O4
#undef WS_DPPY_OCC
    return nb;
}

template <typename T, int NSTEP, int CPL, bool SPLIT = false>
hipError_t launch_dppy_impl(int nstages, const FusedArgs<T>& a, const Geom& g, hipStream_t s, int nstrips, int nsegs) {
    const dim3 grid((unsigned)(a.chains ? (int64_t)a.nchains : (int64_t)nstrips * nsegs * g.L)),
        block(SPLIT ? 2 * kWave : kWave);
#define WS_DPPY_GO(N, M) \
    hipLaunchKernelGGL((fused_dppy_kernel<T, N, NSTEP, M, CPL, SPLIT>), grid, block, 0, s, a, g, nstrips, nsegs)
#define WS_DPPY_G1(M) WS_DPPY_GO(1, M)
#define WS_DPPY_G2(M) WS_DPPY_GO(2, M)
#define WS_DPPY_G4(M) WS_DPPY_GO(4, M)
    switch (nstages) {
        case 1: WS_SP_DISPATCH(a.sp_mode, WS_DPPY_G1) break;
        case 2:
            if constexpr (NSTEP < 8) { WS_SP_DISPATCH(a.sp_mode, WS_DPPY_G2) }
            else return hipErrorInvalidValue;
            break;
        case 4:
            if constexpr (NSTEP < 4) { WS_SP_DISPATCH(a.sp_mode, WS_DPPY_G4) }
            else return hipErrorInvalidValue;
            break;
        default: return hipErrorInvalidValue;
    }
#undef WS_DPPY_G1
#undef WS_DPPY_G2
#undef WS_DPPY_G4
#undef WS_DPPY_GO
    return hipGetLastError();
}

}  // namespace ws
