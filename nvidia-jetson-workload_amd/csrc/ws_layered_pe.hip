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

#include <cstdlib>

#include <string>

#include "ws_abi.h"
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
    int64_t lstride;        // H * W
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
        int gy = (y0 + ly - 1) % a.H;
        if (gy < 0) gy += a.H;
        hc[i] = a.h + (int64_t)gy * a.W + gx;
        T t = T(0);
        if (c < kCX * kCY) {
            if (a.tin) {
                // the producing stage summed the levels in the same order (bitwise the same)
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
    const int64_t on = (int64_t)wrapi(yc + 1, a.H) * a.W + xc, os = (int64_t)wrapi(yc - 1, a.H) * a.W + xc;
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
    size_t es() const { return dtype == WS_F64 ? 8 : 4; }
    size_t cells() const { return (size_t)L * H * W; }
};

namespace ws {
namespace {

void lpe_free(ws_lpe* m) {
    if (m->stream) (void)hipStreamSynchronize(m->stream);  // nothing queued may touch freed memory
    for (int s = 0; s < 2; ++s)
        for (void* p : m->S[s])
            if (p) (void)hipFree(p);
    for (void** grp : {m->A, m->B, m->acc})
        for (int i = 0; i < 3; ++i)
            if (grp[i]) (void)hipFree(grp[i]);
    for (void* p : m->tot)
        if (p) (void)hipFree(p);
    for (hipEvent_t e : {m->ev0, m->ev1})
        if (e) (void)hipEventDestroy(e);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
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
    a.lstride = (int64_t)m->H * m->W;
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

template <typename T>
void enqueue_step(ws_lpe* m) {
    const T dt = (T)m->dt;
    void* const* y0 = m->S[m->cur];
    void* const* y1 = m->S[1 - m->cur];
    switch (m->method) {
        case WS_RK2:
            stage<T>(m, y0, m->A, T(0.5) * dt, T(0), 0);
            stage<T>(m, m->A, y1, dt, T(0), 0);
            break;
        case WS_RK4:
            stage<T>(m, y0, m->A, T(0.5) * dt, T(1), 1);
            stage<T>(m, m->A, m->B, T(0.5) * dt, T(2), 2);
            stage<T>(m, m->B, m->A, dt, T(2), 2);
            stage<T>(m, m->A, y1, dt / T(6), T(0), 3);
            break;
        default:
            stage<T>(m, y0, y1, dt, T(0), 0);
            break;
    }
    m->cur = 1 - m->cur;
}

void check_field_call(const ws_lpe* m, const void* host, int32_t field, int32_t levels, int32_t height, int32_t width,
                      int32_t dtype) {
    if (!m || !host) throw AbiError(WS_ERR_INVALID, "null argument");
    if (field < 0 || field > 2) throw AbiError(WS_ERR_INVALID, "bad field id");
    if (levels != m->L || height != m->H || width != m->W) throw AbiError(WS_ERR_SHAPE, "array shape mismatch");
    if (dtype != m->dtype) throw AbiError(WS_ERR_INVALID, "dtype must match the model precision");
}

}  // namespace
}  // namespace ws

using ws::AbiError;

extern "C" {

int ws_lpe_create(const ws_config_t* cfg, double reduced_gravity, ws_lpe_t** out) {
    return ws::abi_guarded([&] {
        if (!cfg || !out) throw AbiError(WS_ERR_INVALID, "null argument");
        if (cfg->grid_width < 3 || cfg->grid_height < 3 || cfg->num_levels < 1)
            throw AbiError(WS_ERR_INVALID, "layered model needs a grid of at least 3 x 3 and one layer");
        if (!(cfg->dx > 0 && cfg->dy > 0)) throw AbiError(WS_ERR_INVALID, "Grid spacing must be positive");
        ws::abi_set_device(cfg->device_id);
        ws_lpe* m = new ws_lpe;
        m->W = cfg->grid_width;
        m->H = cfg->grid_height;
        m->L = cfg->num_levels;
        m->dtype = cfg->double_precision ? WS_F64 : WS_F32;
        m->device = cfg->device_id;
        m->method = cfg->integration_method == WS_RK2 ? WS_RK2 : cfg->integration_method == WS_RK4 ? WS_RK4 : WS_EULER;
        m->dx = cfg->dx;
        m->dy = cfg->dy;
        m->dt = cfg->dt;
        m->g = cfg->gravity;
        m->f = cfg->coriolis_f;
        m->gp = reduced_gravity;
        try {
            ws::hck(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking), "hipStreamCreate");
            ws::hck(hipEventCreate(&m->ev0), "hipEventCreate");
            ws::hck(hipEventCreate(&m->ev1), "hipEventCreate");
            const size_t fb = m->cells() * m->es();
            for (int s = 0; s < 2; ++s)
                for (void*& p : m->S[s]) {
                    ws::hck(hipMalloc(&p, fb), "hipMalloc");
                    ws::hck(hipMemsetAsync(p, 0, fb, m->stream), "hipMemsetAsync");
                }
            // the field uploads (ws_lpe_set_field) use hipMemcpy, which is not ordered with the
            // model's non-blocking stream: the zeroing must be complete first
            ws::hck(hipStreamSynchronize(m->stream), "hipStreamSynchronize");
            for (void** grp : {m->A, m->B, m->acc})
                for (int i = 0; i < 3; ++i) ws::hck(hipMalloc(&grp[i], fb), "hipMalloc");
            for (void*& p : m->tot) ws::hck(hipMalloc(&p, (size_t)m->H * m->W * m->es()), "hipMalloc");
        } catch (...) {
            ws::lpe_free(m);
            throw;
        }
        *out = m;
    });
}

int ws_lpe_destroy(ws_lpe_t* m) {
    return ws::abi_guarded([&] {
        if (!m) return;
        (void)hipSetDevice(m->device);
        (void)hipStreamSynchronize(m->stream);
        ws::lpe_free(m);
    });
}

int ws_lpe_set_field(ws_lpe_t* m, int32_t field, const void* host, int32_t levels, int32_t height, int32_t width,
                     int32_t dtype) {
    return ws::abi_guarded([&] {
        ws::check_field_call(m, host, field, levels, height, width, dtype);
        ws::abi_set_device(m->device);
        ws::hck(hipStreamSynchronize(m->stream), "hipStreamSynchronize");
        ws::hck(hipMemcpy(m->S[m->cur][field], host, m->cells() * m->es(), hipMemcpyHostToDevice), "hipMemcpy");
        m->tot_ok[m->cur] = false;  // the next stage sums the new thickness itself
    });
}

int ws_lpe_get_field(ws_lpe_t* m, int32_t field, void* host, int32_t levels, int32_t height, int32_t width,
                     int32_t dtype) {
    return ws::abi_guarded([&] {
        ws::check_field_call(m, host, field, levels, height, width, dtype);
        ws::abi_set_device(m->device);
        ws::hck(hipStreamSynchronize(m->stream), "hipStreamSynchronize");
        ws::hck(hipMemcpy(host, m->S[m->cur][field], m->cells() * m->es(), hipMemcpyDeviceToHost), "hipMemcpy");
    });
}

int ws_lpe_run(ws_lpe_t* m, int32_t n) {
    return ws::abi_guarded([&] {
        if (!m) throw AbiError(WS_ERR_INVALID, "null model");
        if (n <= 0) return;
        ws::abi_set_device(m->device);
        m->launches = 0;
        ws::hck(hipEventRecord(m->ev0, m->stream), "hipEventRecord");
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
        ws::hck(hipEventRecord(m->ev1, m->stream), "hipEventRecord");
        ws::hck(hipEventSynchronize(m->ev1), "hipEventSynchronize");
        float ms = 0.f;
        ws::hck(hipEventElapsedTime(&ms, m->ev0, m->ev1), "hipEventElapsedTime");
        m->last_ms = ms;
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
