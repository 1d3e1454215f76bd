// Physics-mode layered primitive-equation model (BASELINE config C4's "3D
// stencil, vertical columns in LDS"). The reference has no such model -- its
// PrimitiveEquations model steps every level with the 2-D shallow-water tendencies
// (weather_simulation.cpp:542-560), which WeatherSimulation reproduces bit for bit -- so this
// is a new model with its own oracle (oracle/layered_pe_oracle.py, pinned to properties of
// the discrete system): hydrostatic primitive equations in isopycnal coordinates, L stacked
// constant-density layers (k = 0 on top) over a flat bottom, doubly periodic:
//     eta_k = sum_{j >= k} h_j,   M_0 = g eta_0,   M_k = M_{k-1} + g' eta_k
//     du/dt = -u u_x - v u_y - M_x + f v,  dv/dt = -u v_x - v v_y - M_y - f u,
//     dh/dt = -(h u)_x - (h v)_y
//
// One kernel per RK stage. A kTX x kTY (128 x 4) tile of columns plus a 1-column halo
// computes the Montgomery potential of every column by a vertical scan, chunk by chunk of
// levels (each chunk's M profiles, and the h values the scan loaded, in LDS), and after each
// chunk every thread walks its own column through those levels, taking M's and h's
// horizontal neighbours from LDS and u's, v's from global memory (L1/L2), and applies the
// stage update (and the RK4 accumulator) in the same pass.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>

#include <string>
#include <vector>

#include "ws_abi.h"
#include "ws_comm.h"
#include "ws_hip.h"

namespace ws {
namespace {

#ifndef WS_LPE_TX
#define WS_LPE_TX 128  // c4p RK4 fp32 tile sweep 32x8 / 64x8 / 64x16 / 128x4 / 128x8 -> 15.5 / 18.1 / 18.2 / 18.4 / 18.6 Gcell/s
#endif
#ifndef WS_LPE_TY
#define WS_LPE_TY 4  // 128x4 (2 waves per SIMD) so the 80-VGPR fp32 kernel runs 3 workgroups per CU
#endif
constexpr int kTX = WS_LPE_TX, kTY = WS_LPE_TY;  // output tile (workgroup = kTX x kTY threads)
constexpr int kCX = kTX + 2, kCY = kTY + 2;  // tile + halo columns

template <typename T>
struct LpeArgs {
    const T *u, *v, *h;     // stage input (stencils)
    const T *bu, *bv, *bh;  // state at the start of the step
    T *ou, *ov, *oh;        // base + c * k
    T *au, *av, *ah;        // RK4 accumulator
    const T* tin;           // total thickness sum_k h_k of the input (H x W), or null: summed here
    T* tout;                // total thickness of the output h (summed in the walk), or null
    int W, H, L;
    int64_t lstride;        // H * W; a slab: (H + 2) * W
    int halo;               // 0: y wraps around H (the whole periodic domain); 1: a slab -- rows
                            // -1 and H of every level are halo rows (the neighbours' edge rows)
    T c, w;
    int acc_mode;           // 0 none, 1 acc = w k, 2 acc += w k, 3 out = base + c (acc + k)
    T ix, iy;               // 1 / (2 dx), 1 / (2 dy)
    T g, gp, f;
};

__device__ __forceinline__ int wrapi(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }

// Levels are processed in chunks of kChunk: the column scan's running state (total
// thickness, prefix, M of the level above) stays in registers, each chunk's M profile goes
// to LDS (Ms: kChunk x kCY x kCX = 8 x 6 x 130 values, 25 KB fp32 / 50 KB fp64) next to
// the chunk's h tile (Hs, the same size with WS_LPE_HLDS): 50 KB fp32 lets 3 workgroups
// share a CU (160 KB of LDS), the fp64 kernel's 100 KB one; the column walk of one chunk
// overlaps the other workgroups' loads.
#ifndef WS_LPE_CHUNK
#define WS_LPE_CHUNK 8
#endif
constexpr int kChunk = WS_LPE_CHUNK;
// the level walk is not unrolled (`#pragma unroll 1` below; a literal: -save-temps does not
// expand macros inside pragmas): 1024^2 x 32 fp32 RK4: 32x8 tile 1 / 2 / 4 / 8 -> 15.2 / 16.2 /
// 14.2 / 15.5; 128x8 tile 1 / 2 -> 18.8 / 17.6 Gcell/s
constexpr int kColsPerThread = (kCX * kCY + kTX * kTY - 1) / (kTX * kTY);

#ifndef WS_LPE_HLDS
#define WS_LPE_HLDS 1  // the walk takes h's neighbours from an LDS copy of the scan's loads (0: from L1/L2; c4p 20.5 -> 21.2 Gcell/s)
#endif
#define WS_LPE_HLDS_ON (WS_LPE_HLDS ? 1 : 0)
// static LDS of the stage kernel (Ms, and Hs with WS_LPE_HLDS) must fit the CDNA4 CU's 160 KB
template <typename T>
constexpr int lpe_lds_bytes() { return (1 + WS_LPE_HLDS_ON) * kChunk * kCY * kCX * (int)sizeof(T); }
static_assert(lpe_lds_bytes<double>() <= 160 * 1024, "layered PE tile + chunk exceed the gfx950 LDS (160 KB)");
#ifndef WS_LPE_WAVES
#define WS_LPE_WAVES 6  // fp32: VGPRs capped at 80 -> 6 waves/SIMD (128x4 tile: 18.5 -> 19.1-19.3 Gcell/s; 8 waves spills: 14.5); fp64 unconstrained
#endif

template <typename T>
__global__ __launch_bounds__(kTX* kTY) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 4 ? WS_LPE_WAVES : 1)))
void lpe_stage_kernel(LpeArgs<T> a) {
    __shared__ T Ms[kChunk][kCY][kCX];
#if WS_LPE_HLDS
    __shared__ T Hs[kChunk][kCY][kCX];  // the chunk's h tile + halo, loaded once by the scan
#endif
    const int x0 = blockIdx.x * kTX, y0 = blockIdx.y * kTY;
    const int tid = threadIdx.y * kTX + threadIdx.x;
    // scan state of this thread's columns of the tile + halo (oracle order: total = h_0 +
    // h_1 + ...; eta_k = total - (h_0 + ... + h_{k-1}); M_0 = g eta_0, M_k = M_{k-1} + g' eta_k)
    const T* hc[kColsPerThread];
    T total[kColsPerThread], prefix[kColsPerThread], Mprev[kColsPerThread];
#pragma unroll
    for (int i = 0; i < kColsPerThread; ++i) {
        const int c = tid + i * kTX * kTY;
        const int cc = c < kCX * kCY ? c : 0;
        const int lx = cc % kCX, ly = cc / kCX;
        int gx = (x0 + lx - 1) % a.W;
        if (gx < 0) gx += a.W;
        int gy = y0 + ly - 1;
        if (a.halo) {
            gy = gy > a.H ? a.H : gy;  // rows below the bottom halo row only feed cells outside the slab
        } else {
            gy %= a.H;
            if (gy < 0) gy += a.H;
        }
        hc[i] = a.h + (int64_t)gy * a.W + gx;
        T t = T(0);
        if (c < kCX * kCY) {
            if (a.tin && gy >= 0 && gy < a.H) {
                // the producing stage summed the levels in the same order (bitwise the same);
                // a slab's halo rows have no total here: summed below, in the same order
                t = a.tin[(int64_t)gy * a.W + gx];
            } else {
#pragma unroll 8
                for (int k = 0; k < a.L; ++k) t = t + hc[i][(int64_t)k * a.lstride];
            }
        }
        total[i] = t;
        prefix[i] = T(0);
        Mprev[i] = T(0);
    }
    const int x = x0 + threadIdx.x, y = y0 + threadIdx.y;
    const bool inside = x < a.W && y < a.H;
    const int lx = threadIdx.x + 1, ly = threadIdx.y + 1;
    const int xc = inside ? x : 0, yc = inside ? y : 0;
    const int64_t oc = (int64_t)yc * a.W + xc;
    const int64_t oe = (int64_t)yc * a.W + wrapi(xc + 1, a.W), ow = (int64_t)yc * a.W + wrapi(xc - 1, a.W);
    const int yn = a.halo ? yc + 1 : wrapi(yc + 1, a.H), ys = a.halo ? yc - 1 : wrapi(yc - 1, a.H);
    const int64_t on = (int64_t)yn * a.W + xc, os = (int64_t)ys * a.W + xc;
    T tsum = T(0);  // total thickness of the output column, levels in order (as the scan sums)
    for (int k0 = 0; k0 < a.L; k0 += kChunk) {
        const int nk = a.L - k0 < kChunk ? a.L - k0 : kChunk;
#pragma unroll
        for (int i = 0; i < kColsPerThread; ++i) {
            const int c = tid + i * kTX * kTY;
            if (c >= kCX * kCY) continue;
            const int lxc = c % kCX, lyc = c / kCX;
            // the chunk's thicknesses first (independent loads in flight together), then the scan
            T hv[kChunk];
#pragma unroll
            for (int j = 0; j < kChunk; ++j) hv[j] = j < nk ? hc[i][(int64_t)(k0 + j) * a.lstride] : T(0);
#pragma unroll
            for (int j = 0; j < kChunk; ++j) {
                if (j >= nk) break;
                const int k = k0 + j;
                const T eta = total[i] - prefix[i];
                Mprev[i] = k == 0 ? a.g * eta : Mprev[i] + a.gp * eta;
                Ms[j][lyc][lxc] = Mprev[i];
#if WS_LPE_HLDS
                Hs[j][lyc][lxc] = hv[j];
#endif
                prefix[i] = prefix[i] + hv[j];
            }
        }
        __syncthreads();
        if (inside) {
#pragma unroll 1
            for (int j = 0; j < nk; ++j) {
                const int64_t lo = (int64_t)(k0 + j) * a.lstride;
                const T* U = a.u + lo;
                const T* V = a.v + lo;
                const T* Hh = a.h + lo;
                const T u = U[oc], v = V[oc];
                const T ue = U[oe], uw = U[ow], un = U[on], us = U[os];
                const T ve = V[oe], vw = V[ow], vn = V[on], vs = V[os];
#if WS_LPE_HLDS
                (void)Hh;
                const T he = Hs[j][ly][lx + 1], hw = Hs[j][ly][lx - 1];
                const T hn = Hs[j][ly + 1][lx], hs = Hs[j][ly - 1][lx];
#else
                const T he = Hh[oe], hw = Hh[ow], hn = Hh[on], hs = Hh[os];
#endif
                const T Me = Ms[j][ly][lx + 1], Mw = Ms[j][ly][lx - 1];
                const T Mn = Ms[j][ly + 1][lx], Mso = Ms[j][ly - 1][lx];
                const T u_x = (ue - uw) * a.ix, u_y = (un - us) * a.iy;
                const T v_x = (ve - vw) * a.ix, v_y = (vn - vs) * a.iy;
                const T M_x = (Me - Mw) * a.ix, M_y = (Mn - Mso) * a.iy;
                const T du = -u * u_x - v * u_y - M_x + a.f * v;
                const T dv = -u * v_x - v * v_y - M_y - a.f * u;
                const T dh = -((he * ue - hw * uw) * a.ix) - (hn * vn - hs * vs) * a.iy;
                const int64_t o = lo + oc;
                const T b0 = a.bu[o], b1 = a.bv[o], b2 = a.bh[o];
                if (a.acc_mode == 3) {
                    a.ou[o] = b0 + a.c * (a.au[o] + du);
                    a.ov[o] = b1 + a.c * (a.av[o] + dv);
                    const T hnew = b2 + a.c * (a.ah[o] + dh);
                    a.oh[o] = hnew;
                    tsum = tsum + hnew;
                    continue;
                }
                a.ou[o] = b0 + a.c * du;
                a.ov[o] = b1 + a.c * dv;
                const T hnew = b2 + a.c * dh;
                a.oh[o] = hnew;
                tsum = tsum + hnew;
                if (a.acc_mode == 1) {
                    a.au[o] = a.w * du;
                    a.av[o] = a.w * dv;
                    a.ah[o] = a.w * dh;
                } else if (a.acc_mode == 2) {
                    a.au[o] = a.au[o] + a.w * du;
                    a.av[o] = a.av[o] + a.w * dv;
                    a.ah[o] = a.ah[o] + a.w * dh;
                }
            }
        }
        __syncthreads();  // the next chunk overwrites Ms
    }
    if (a.tout && inside) a.tout[oc] = tsum;
}

// The halo rows of one slab of a one-process decomposition, pulled from its neighbours'
// memory (same device, or a peer over xGMI): row -1 of every level of u, v, h <- the upper
// neighbour's last row, row H <- the lower neighbour's row 0. grid (W / 256, L, 3 fields x 2).
template <typename T>
struct LpePull {
    T* dst[3];
    const T* up[3];
    const T* dn[3];
    int W, H, up_rows;
    int64_t lstride, up_lstride, dn_lstride;
};

template <typename T>
__global__ __launch_bounds__(256) void lpe_pull_kernel(LpePull<T> a) {
    const int x = blockIdx.x * 256 + threadIdx.x;
    if (x >= a.W) return;
    const int l = blockIdx.y, f = blockIdx.z % 3, side = blockIdx.z / 3;
    const T* src = side == 0 ? a.up[f] + (int64_t)l * a.up_lstride + (int64_t)(a.up_rows - 1) * a.W
                             : a.dn[f] + (int64_t)l * a.dn_lstride;
    T* dst = a.dst[f] + (int64_t)l * a.lstride + (side == 0 ? -(int64_t)a.W : (int64_t)a.H * a.W);
    dst[x] = src[x];
}

void hck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw AbiError(WS_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace
}  // namespace ws
struct ws_lpe {
    int W = 0, H = 0, L = 0, dtype = WS_F32, device = 0, method = WS_RK4;
    double dx = 1, dy = 1, dt = 0.01, g = 9.81, gp = 0.05, f = 0;
    double time = 0;
    int32_t step = 0;
    hipStream_t stream = nullptr;
    // state slots, stage buffers A / B and the RK4 accumulator: 3 fields each, [L][H][W]
    // (a slab: [L][H + 2][W], the pointers at row 0 of level 0, rows -1 and H the halo)
    void* S[2][3] = {};
    void* A[3] = {};
    void* B[3] = {};
    void* acc[3] = {};
    // total thickness (sum over levels of h, H x W) of S[0], S[1], A, B, written by the stage
    // that produces the set, so the next stage's column scan skips its pre-pass over h;
    // tot_ok[i] false (initial / set_field state) = the stage sums it itself
    void* tot[4] = {};
    bool tot_ok[4] = {};
    int cur = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_ms = 0;
    int64_t launches = 0;
    // y-slab decomposition around the periodic ring (ws_lpe_create_multi / _create_slab): this
    // model owns global rows [row0, row0 + H) of Hg; halo = 1 gives every level a halo row
    // above and below, refreshed before every RK stage -- from the neighbours' memory by the
    // process's own kernels (parts of a one-process decomposition) or over RCCL (comm)
    int Hg = 0, row0 = 0, halo = 0;
    int rank = 0, nranks = 1;
    ws::SlabComm* comm = nullptr;
    std::vector<ws_lpe*> parts;     // a one-process decomposition: its slabs (it holds no buffers itself)
    hipEvent_t ev_stage = nullptr;  // a part: recorded after its latest stage kernel
    bool pull_direct = true;        // a part: the pull kernel may read both neighbours' memory
    size_t es() const { return dtype == WS_F64 ? 8 : 4; }
    size_t cells() const { return (size_t)L * H * W; }
    int64_t lstride() const { return (int64_t)(H + 2 * halo) * W; }
    size_t alloc_bytes() const { return (size_t)L * lstride() * es(); }
    size_t halo_bytes() const { return (size_t)halo * W * es(); }
};

namespace ws {
namespace {

void lpe_free(ws_lpe* m) {
    for (ws_lpe* p : m->parts) {
        (void)hipSetDevice(p->device);
        lpe_free(p);
    }
    m->parts.clear();
    if (m->stream) (void)hipStreamSynchronize(m->stream);  // nothing queued may touch freed memory
    auto field_free = [&](void* p) {
        if (p) (void)hipFree((char*)p - m->halo_bytes());
    };
    for (int s = 0; s < 2; ++s)
        for (void* p : m->S[s]) field_free(p);
    for (void** grp : {m->A, m->B, m->acc})
        for (int i = 0; i < 3; ++i) field_free(grp[i]);
    for (void* p : m->tot)
        if (p) (void)hipFree(p);
    for (hipEvent_t e : {m->ev0, m->ev1, m->ev_stage})
        if (e) (void)hipEventDestroy(e);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m->comm;
    delete m;
}

// the model parameters of cfg (no buffers)
void lpe_params(ws_lpe* m, const ws_config_t* cfg, double gp) {
    m->W = cfg->grid_width;
    m->H = m->Hg = cfg->grid_height;
    m->L = cfg->num_levels;
    m->dtype = cfg->double_precision ? WS_F64 : WS_F32;
    m->device = cfg->device_id;
    m->method = cfg->integration_method == WS_RK2 ? WS_RK2 : cfg->integration_method == WS_RK4 ? WS_RK4 : WS_EULER;
    m->dx = cfg->dx;
    m->dy = cfg->dy;
    m->dt = cfg->dt;
    m->g = cfg->gravity;
    m->f = cfg->coriolis_f;
    m->gp = gp;
}

void lpe_check_config(const ws_config_t* cfg) {
    if (cfg->grid_width < 3 || cfg->grid_height < 3 || cfg->num_levels < 1)
        throw AbiError(WS_ERR_INVALID, "layered model needs a grid of at least 3 x 3 and one layer");
    if (!(cfg->dx > 0 && cfg->dy > 0)) throw AbiError(WS_ERR_INVALID, "Grid spacing must be positive");
}

// stream, events and zeroed buffers of a model whose geometry (W, H, L, halo) is set; the
// device is current
void lpe_alloc(ws_lpe* m) {
    hck(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking), "hipStreamCreate");
    hck(hipEventCreate(&m->ev0), "hipEventCreate");
    hck(hipEventCreate(&m->ev1), "hipEventCreate");
    hck(hipEventCreateWithFlags(&m->ev_stage, hipEventDisableTiming), "hipEventCreate");
    auto field = [&](void*& p) {
        void* a = nullptr;
        hck(hipMalloc(&a, m->alloc_bytes()), "hipMalloc");
        p = (char*)a + m->halo_bytes();
        hck(hipMemsetAsync(a, 0, m->alloc_bytes(), m->stream), "hipMemsetAsync");
    };
    for (int s = 0; s < 2; ++s)
        for (void*& p : m->S[s]) field(p);
    for (void** grp : {m->A, m->B, m->acc})
        for (int i = 0; i < 3; ++i) field(grp[i]);
    for (void*& p : m->tot) hck(hipMalloc(&p, (size_t)m->H * m->W * m->es()), "hipMalloc");
    // the field uploads (ws_lpe_set_field) use hipMemcpy, which is not ordered with the
    // model's non-blocking stream: the zeroing must be complete first
    hck(hipStreamSynchronize(m->stream), "hipStreamSynchronize");
}

// field sets by id: 0 the current state, 1 the next, 2 A, 3 B
void* const* set_of(ws_lpe* m, int id) {
    switch (id) {
        case 0: return m->S[m->cur];
        case 1: return m->S[1 - m->cur];
        case 2: return m->A;
        default: return m->B;
    }
}

// index of a field set's total-thickness buffer: S[0], S[1], A, B
int tot_index(const ws_lpe* m, void* const* set) {
    if (set == m->S[0]) return 0;
    if (set == m->S[1]) return 1;
    return set == m->A ? 2 : 3;
}

template <typename T>
void stage(ws_lpe* m, void* const* in, void* const* out, T c, T w, int acc_mode) {
    LpeArgs<T> a{};
    const int ti = tot_index(m, in), to = tot_index(m, out);
    // the input's total thickness when the producing stage wrote it (else the scan sums it)
    a.tin = m->tot_ok[ti] ? (const T*)m->tot[ti] : nullptr;
    a.tout = (T*)m->tot[to];
    m->tot_ok[to] = true;
    a.u = (const T*)in[0];
    a.v = (const T*)in[1];
    a.h = (const T*)in[2];
    void* const* base = m->S[m->cur];
    a.bu = (const T*)base[0];
    a.bv = (const T*)base[1];
    a.bh = (const T*)base[2];
    a.ou = (T*)out[0];
    a.ov = (T*)out[1];
    a.oh = (T*)out[2];
    a.au = (T*)m->acc[0];
    a.av = (T*)m->acc[1];
    a.ah = (T*)m->acc[2];
    a.W = m->W;
    a.H = m->H;
    a.L = m->L;
    a.lstride = m->lstride();
    a.halo = m->halo;
    a.c = c;
    a.w = w;
    a.acc_mode = acc_mode;
    a.ix = (T)(1.0 / (2.0 * m->dx));
    a.iy = (T)(1.0 / (2.0 * m->dy));
    a.g = (T)m->g;
    a.gp = (T)m->gp;
    a.f = (T)m->f;
    const dim3 grid((m->W + kTX - 1) / kTX, (m->H + kTY - 1) / kTY), block(kTX, kTY);
    hipLaunchKernelGGL((lpe_stage_kernel<T>), grid, block, 0, m->stream, a);
    hck(hipGetLastError(), "lpe_stage_kernel");
    m->launches += 1;
}

// part p's halo rows of field set `sid` from its ring neighbours (one-process decomposition),
// on p's stream once the neighbours' previous stages are done
template <typename T>
void pull_halo(ws_lpe* m, int p, int sid) {
    const int n = (int)m->parts.size();
    ws_lpe* me = m->parts[p];
    ws_lpe* up = m->parts[(p + n - 1) % n];
    ws_lpe* dn = m->parts[(p + 1) % n];
    hck(hipStreamWaitEvent(me->stream, up->ev_stage, 0), "hipStreamWaitEvent");
    if (dn != up) hck(hipStreamWaitEvent(me->stream, dn->ev_stage, 0), "hipStreamWaitEvent");
    void* const* d = set_of(me, sid);
    void* const* u = set_of(up, sid);
    void* const* w = set_of(dn, sid);
    if (me->pull_direct) {
        LpePull<T> a{};
        for (int f = 0; f < 3; ++f) {
            a.dst[f] = (T*)d[f];
            a.up[f] = (const T*)u[f];
            a.dn[f] = (const T*)w[f];
        }
        a.W = me->W;
        a.H = me->H;
        a.up_rows = up->H;
        a.lstride = me->lstride();
        a.up_lstride = up->lstride();
        a.dn_lstride = dn->lstride();
        hipLaunchKernelGGL((lpe_pull_kernel<T>), dim3((me->W + 255) / 256, me->L, 6), dim3(256), 0, me->stream, a);
        hck(hipGetLastError(), "lpe_pull_kernel");
        me->launches += 1;
        return;
    }
    // no peer access between the devices: the runtime's 2-D copies (L rows of W each)
    const size_t row = (size_t)me->W * sizeof(T);
    for (int f = 0; f < 3; ++f) {
        hck(hipMemcpy2DAsync((char*)d[f] - row, me->lstride() * sizeof(T), (const char*)u[f] + (up->H - 1) * row,
                             up->lstride() * sizeof(T), row, me->L, hipMemcpyDefault, me->stream),
            "hipMemcpy2DAsync");
        hck(hipMemcpy2DAsync((char*)d[f] + me->H * row, me->lstride() * sizeof(T), w[f], dn->lstride() * sizeof(T),
                             row, me->L, hipMemcpyDefault, me->stream),
            "hipMemcpy2DAsync");
    }
}

// one RK stage of the model -- every part of a one-process decomposition (halo pulls for all
// of them first: a part's pull must not see a neighbour's event of this same stage), or a
// process's slab after its RCCL exchange, or the whole domain
template <typename T>
void stage_all(ws_lpe* m, int in_id, int out_id, T c, T w, int acc_mode) {
    if (m->parts.empty()) {
        if (m->comm && m->nranks > 1) {
            Geom g{};
            g.W = m->W; g.H = m->H; g.L = m->L;
            g.pitch = m->W;
            g.lstride = m->lstride();
            g.halo = 1;
            m->comm->exchange(set_of(m, in_id), 3, (int)sizeof(T), g, 1, m->stream, /*periodic=*/true);
        }
        stage<T>(m, set_of(m, in_id), set_of(m, out_id), c, w, acc_mode);
        return;
    }
    const int n = (int)m->parts.size();
    for (int p = 0; p < n; ++p) {
        hck(hipSetDevice(m->parts[p]->device), "hipSetDevice");
        pull_halo<T>(m, p, in_id);
    }
    for (ws_lpe* p : m->parts) {
        hck(hipSetDevice(p->device), "hipSetDevice");
        stage<T>(p, set_of(p, in_id), set_of(p, out_id), c, w, acc_mode);
        hck(hipEventRecord(p->ev_stage, p->stream), "hipEventRecord");
    }
}

template <typename T>
void enqueue_step(ws_lpe* m) {
    const T dt = (T)m->dt;
    switch (m->method) {
        case WS_RK2:
            stage_all<T>(m, 0, 2, T(0.5) * dt, T(0), 0);
            stage_all<T>(m, 2, 1, dt, T(0), 0);
            break;
        case WS_RK4:
            stage_all<T>(m, 0, 2, T(0.5) * dt, T(1), 1);
            stage_all<T>(m, 2, 3, T(0.5) * dt, T(2), 2);
            stage_all<T>(m, 3, 2, dt, T(2), 2);
            stage_all<T>(m, 2, 1, dt / T(6), T(0), 3);
            break;
        default:
            stage_all<T>(m, 0, 1, dt, T(0), 0);
            break;
    }
    m->cur = 1 - m->cur;
    for (ws_lpe* p : m->parts) p->cur = 1 - p->cur;
}

void check_field_call(const ws_lpe* m, const void* host, int32_t field, int32_t levels, int32_t height, int32_t width,
                      int32_t dtype) {
    if (!m || !host) throw AbiError(WS_ERR_INVALID, "null argument");
    if (field < 0 || field > 2) throw AbiError(WS_ERR_INVALID, "bad field id");
    if (levels != m->L || height != m->H || width != m->W) throw AbiError(WS_ERR_SHAPE, "array shape mismatch");
    if (dtype != m->dtype) throw AbiError(WS_ERR_INVALID, "dtype must match the model precision");
}

// host (L, rows, W) rows [r0, r0 + p->H) of every level <-> part p's own rows
void copy_field(ws_lpe* p, int32_t field, void* host, int host_rows, int r0, bool upload) {
    abi_set_device(p->device);
    hck(hipStreamSynchronize(p->stream), "hipStreamSynchronize");
    const size_t row = (size_t)p->W * p->es();
    char* h = (char*)host + (size_t)r0 * row;
    char* d = (char*)p->S[p->cur][field];
    const size_t hpitch = (size_t)host_rows * row, dpitch = (size_t)p->lstride() * p->es();
    if (upload) {
        hck(hipMemcpy2D(d, dpitch, h, hpitch, p->H * row, p->L, hipMemcpyHostToDevice), "hipMemcpy2D");
        p->tot_ok[p->cur] = false;  // the next stage sums the new thickness itself
    } else {
        hck(hipMemcpy2D(h, hpitch, d, dpitch, p->H * row, p->L, hipMemcpyDeviceToHost), "hipMemcpy2D");
    }
}

void transfer(ws_lpe* m, int32_t field, void* host, bool upload) {
    if (m->parts.empty()) {
        copy_field(m, field, host, m->H, 0, upload);
        return;
    }
    for (ws_lpe* p : m->parts) copy_field(p, field, host, m->H, p->row0, upload);
}

// one slab of the ring: rows [row0, row0 + rows) of cfg's grid, halo rows when nranks > 1
ws_lpe* lpe_make(const ws_config_t* cfg, double gp, int device, int rank, int nranks) {
    ws_lpe* m = new ws_lpe;
    lpe_params(m, cfg, gp);
    m->device = device;
    m->rank = rank;
    m->nranks = nranks;
    slab_rows(m->Hg, rank, nranks, &m->row0, &m->H);
    m->halo = nranks > 1 ? 1 : 0;
    try {
        abi_set_device(device);
        lpe_alloc(m);
    } catch (...) {
        lpe_free(m);
        throw;
    }
    return m;
}

// peer access from `dev` to `peer` (already enabled counts); false where the devices cannot
bool enable_peer(int dev, int peer) {
    if (dev == peer) return true;
    int ok = 0;
    if (hipDeviceCanAccessPeer(&ok, dev, peer) != hipSuccess || !ok) {
        (void)hipGetLastError();  // (no sticky error for the next launch check to report)
        return false;
    }
    hck(hipSetDevice(dev), "hipSetDevice");
    const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
    if (e != hipSuccess) (void)hipGetLastError();  // already enabled, or the runtime's copies instead
    return e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled;
}

}  // namespace
}  // namespace ws

using ws::AbiError;

extern "C" {

int ws_lpe_create(const ws_config_t* cfg, double reduced_gravity, ws_lpe_t** out) {
    return ws::abi_guarded([&] {
        if (!cfg || !out) throw AbiError(WS_ERR_INVALID, "null argument");
        ws::lpe_check_config(cfg);
        *out = ws::lpe_make(cfg, reduced_gravity, cfg->device_id, 0, 1);
    });
}

int ws_lpe_create_multi(const ws_config_t* cfg, double reduced_gravity, const int32_t* devices, int32_t ndevices,
                        ws_lpe_t** out) {
    return ws::abi_guarded([&] {
        if (!cfg || !out || !devices) throw AbiError(WS_ERR_INVALID, "null argument");
        ws::lpe_check_config(cfg);
        if (ndevices < 1 || ndevices > cfg->grid_height)
            throw AbiError(WS_ERR_INVALID, "need 1 <= slabs <= grid_height");
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
        for (int i = 0; i < ndevices; ++i)
            if (devices[i] < 0 || devices[i] >= count) throw AbiError(WS_ERR_DEVICE, "no such device");
        if (ndevices == 1) {
            *out = ws::lpe_make(cfg, reduced_gravity, devices[0], 0, 1);
            return;
        }
        ws_lpe* m = new ws_lpe;
        ws::lpe_params(m, cfg, reduced_gravity);
        m->device = devices[0];
        m->nranks = ndevices;
        try {
            for (int r = 0; r < ndevices; ++r)
                m->parts.push_back(ws::lpe_make(cfg, reduced_gravity, devices[r], r, ndevices));
            for (int r = 0; r < ndevices; ++r) {
                ws_lpe* p = m->parts[r];
                const int up = devices[(r + ndevices - 1) % ndevices], dn = devices[(r + 1) % ndevices];
                p->pull_direct = ws::enable_peer(p->device, up) && ws::enable_peer(p->device, dn);
            }
        } catch (...) {
            ws::lpe_free(m);
            throw;
        }
        *out = m;
    });
}

int ws_lpe_create_slab(const ws_config_t* cfg, double reduced_gravity, int32_t rank, int32_t nranks,
                       const uint8_t id[WS_COMM_ID_BYTES], ws_lpe_t** out, int32_t* row0, int32_t* rows) {
    return ws::abi_guarded([&] {
        if (!cfg || !out || !id) throw AbiError(WS_ERR_INVALID, "null argument");
        ws::lpe_check_config(cfg);
        if (nranks < 1 || rank < 0 || rank >= nranks || nranks > cfg->grid_height)
            throw AbiError(WS_ERR_INVALID, "bad rank / nranks");
        ws_lpe* m = ws::lpe_make(cfg, reduced_gravity, cfg->device_id, rank, nranks);
        try {
            // a 1-rank slab gets its communicator too (the exchanges are no-ops): the RCCL
            // bootstrap runs on one GPU
            m->comm = new ws::SlabComm(rank, nranks, id);
        } catch (const std::exception& e) {
            ws::lpe_free(m);
            throw AbiError(WS_ERR_DEVICE, e.what());
        }
        *out = m;
        if (row0) *row0 = m->row0;
        if (rows) *rows = m->H;
    });
}

int ws_lpe_layout(const ws_lpe_t* m, int32_t* nslabs, int32_t* row0, int32_t* rows) {
    return ws::abi_guarded([&] {
        if (!m) throw AbiError(WS_ERR_INVALID, "null model");
        if (nslabs) *nslabs = m->nranks;
        if (row0) *row0 = m->row0;
        if (rows) *rows = m->H;
    });
}

int ws_lpe_exchange_plan(int32_t width, int32_t rows, int32_t levels, int32_t dtype, int32_t rank, int32_t nranks,
                         ws_xfer_t* out, int32_t capacity, int32_t* count, int64_t* level_stride) {
    return ws::abi_guarded([&] {
        if (width < 1 || rows < 1 || levels < 1) throw AbiError(WS_ERR_INVALID, "Grid dimensions must be positive");
        if (dtype != WS_F32 && dtype != WS_F64) throw AbiError(WS_ERR_INVALID, "bad dtype");
        if (nranks < 1 || rank < 0 || rank >= nranks) throw AbiError(WS_ERR_INVALID, "bad rank / nranks");
        // a slab's layout (lpe_alloc): unpadded rows, one halo row above and below every level
        ws::Geom g{};
        g.W = width; g.H = rows; g.L = levels;
        g.pitch = width;
        g.lstride = (int64_t)(rows + 2) * width;
        g.halo = 1;
        const auto x = ws::make_halo_plan(g, dtype == WS_F64 ? 8 : 4, rank, nranks, 3, 1, true).xfers();
        if (count) *count = (int32_t)x.size();
        if (level_stride) *level_stride = g.lstride;
        if (out) {
            if (capacity < (int32_t)x.size()) throw AbiError(WS_ERR_INVALID, "plan capacity too small");
            for (size_t i = 0; i < x.size(); ++i) {
                out[i].peer = x[i].peer; out[i].kind = x[i].kind; out[i].field = x[i].field;
                out[i].level = x[i].level; out[i].offset = x[i].offset; out[i].bytes = x[i].bytes;
                out[i].msg_offset = x[i].msg_offset;
            }
        }
    });
}

int ws_lpe_destroy(ws_lpe_t* m) {
    return ws::abi_guarded([&] {
        if (!m) return;
        (void)hipSetDevice(m->device);
        ws::lpe_free(m);
    });
}

int ws_lpe_set_field(ws_lpe_t* m, int32_t field, const void* host, int32_t levels, int32_t height, int32_t width,
                     int32_t dtype) {
    return ws::abi_guarded([&] {
        ws::check_field_call(m, host, field, levels, height, width, dtype);
        ws::transfer(m, field, const_cast<void*>(host), true);
    });
}

int ws_lpe_get_field(ws_lpe_t* m, int32_t field, void* host, int32_t levels, int32_t height, int32_t width,
                     int32_t dtype) {
    return ws::abi_guarded([&] {
        ws::check_field_call(m, host, field, levels, height, width, dtype);
        ws::transfer(m, field, host, false);
    });
}

int ws_lpe_run(ws_lpe_t* m, int32_t n) {
    return ws::abi_guarded([&] {
        if (!m) throw AbiError(WS_ERR_INVALID, "null model");
        if (n <= 0) return;
        m->launches = 0;
        for (ws_lpe* p : m->parts) p->launches = 0;
        // one-process decomposition: host time from the first enqueue to the last part's end
        const auto t0 = std::chrono::steady_clock::now();
        if (m->parts.empty()) {
            ws::abi_set_device(m->device);
            ws::hck(hipEventRecord(m->ev0, m->stream), "hipEventRecord");
        }
        for (int i = 0; i < n; ++i) {
            if (m->dtype == WS_F64) {
                ws::enqueue_step<double>(m);
                m->time += m->dt;
            } else {
                ws::enqueue_step<float>(m);
                m->time = (double)((float)m->time + (float)m->dt);
            }
            m->step++;
        }
        if (m->parts.empty()) {
            ws::hck(hipEventRecord(m->ev1, m->stream), "hipEventRecord");
            ws::hck(hipEventSynchronize(m->ev1), "hipEventSynchronize");
            float ms = 0.f;
            ws::hck(hipEventElapsedTime(&ms, m->ev0, m->ev1), "hipEventElapsedTime");
            m->last_ms = ms;
            return;
        }
        for (ws_lpe* p : m->parts) {
            ws::hck(hipSetDevice(p->device), "hipSetDevice");
            ws::hck(hipStreamSynchronize(p->stream), "hipStreamSynchronize");
            m->launches += p->launches;
        }
        m->last_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    });
}

int ws_lpe_get_state(const ws_lpe_t* m, double* time, int32_t* step, double* last_run_ms,
                     int64_t* last_run_launches) {
    return ws::abi_guarded([&] {
        if (!m) throw AbiError(WS_ERR_INVALID, "null model");
        if (time) *time = m->time;
        if (step) *step = m->step;
        if (last_run_ms) *last_run_ms = m->last_ms;
        if (last_run_launches) *last_run_launches = m->launches;
    });
}

}  // extern "C"
