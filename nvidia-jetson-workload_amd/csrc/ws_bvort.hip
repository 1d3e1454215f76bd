// Physics-mode barotropic vorticity model (BASELINE config C3's "Jacobian +
// Laplacian stencil"). The reference has no such model -- its Barotropic model runs the
// shallow-water tendencies (weather_simulation.cpp:542-560) -- so this is a new model with
// its own oracle (oracle/bvort_oracle.py, pinned against analytic solutions of the discrete
// system). Doubly periodic W x H grid:
//     d(zeta)/dt = -J(psi, zeta) - beta d(psi)/dx + nu lap(zeta),   lap(psi) = zeta
// J = Arakawa (1966) 9-point Jacobian; the Poisson inverse is spectral (hipFFT R2C / C2R
// around a diagonal scale by the 5-point Laplacian's eigenvalues); the config fields
// `beta` and `viscosity` (weather_sim.hpp:176-178, never read by the reference) are the
// parameters. Euler, RK2 midpoint and classical RK4.
//
// Per RK stage: R2C(zeta_s) -> scale -> C2R -> psi_s, then one fused stencil kernel computes
// the tendency at every cell from LDS tiles of psi_s and zeta_s (1-cell periodic halo) and
// applies the stage update (and the RK4 accumulator) in the same pass.
#include <hip/hip_runtime.h>
#include <hipfft/hipfft.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ws_abi.h"
#include "ws_hip.h"

namespace ws {
namespace {

constexpr int kTX = 64;  // tile columns (one wave wide)
constexpr int kTY = 16;  // tile rows (4 per thread, 4 waves)
constexpr int kBY = 4;

template <typename T>
struct BvArgs {
    const T* zin;   // stage input zeta (stencil)
    const T* psi;   // its streamfunction
    const T* z0;    // zeta at the start of the step
    T* zout;        // z0 + c * k
    T* acc;         // RK4: sum of weighted tendencies
    int W, H;
    T c;            // stage coefficient
    T w;            // accumulator weight
    int acc_mode;   // 0 none, 1 acc = w k, 2 acc += w k, 3 final: zout = z0 + c (acc + k)
    T inv12dxdy, inv2dx, idx2, idy2, beta, nu;
};

__device__ __forceinline__ int wrap(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }

template <typename T>
__global__ __launch_bounds__(kTX* kBY) void bv_stage_kernel(BvArgs<T> a) {
    __shared__ T P[kTY + 2][kTX + 2];
    __shared__ T Z[kTY + 2][kTX + 2];
    const int x0 = blockIdx.x * kTX, y0 = blockIdx.y * kTY;
    const int tid = threadIdx.y * kTX + threadIdx.x;
    const int x = x0 + threadIdx.x;
    const bool xin = x < a.W;
    // This thread's rows of z0 and of the accumulator, loaded ahead of the tile fill so their
    // latency overlaps it (indices clamped to a valid cell for threads outside the grid, whose
    // values are never used). The epilogue below then stores through fixed pointers only: one
    // zout store per row, the accumulator store under a wave-uniform mode test. (Round 3's
    // register-array form of these loads ended in a `switch` of stores whose default case --
    // RK4's final combination -- hipcc compiled to a store through an undefined SGPR pair, an
    // illegal address at the next row: DESIGN.md §10.)
    T z0v[kTY / kBY], accv[kTY / kBY];
#pragma unroll
    for (int r = 0; r < kTY / kBY; ++r) {
        const int y = y0 + threadIdx.y + r * kBY;
        const int64_t o = xin && y < a.H ? (int64_t)y * a.W + x : 0;
        z0v[r] = a.z0[o];
        accv[r] = a.acc_mode >= 2 ? a.acc[o] : T(0);
    }
    // (x0 + lx - 1) lies in [-1, W + kTX], (y0 + ly - 1) in [-1, H + kTY]: one wrap step
    // covers grids at least a tile (+ halo) wide and tall (a wave-uniform test); narrower
    // grids reduce fully (an integer division per element: the fill's dominant VALU cost)
    const bool wide = a.W >= kTX + 2 && a.H >= kTY + 2;
    for (int i = tid; i < (kTY + 2) * (kTX + 2); i += kTX * kBY) {
        const int ly = i / (kTX + 2), lx = i - ly * (kTX + 2);
        int gx = x0 + lx - 1, gy = y0 + ly - 1;
        if (wide) {
            gx = gx < 0 ? gx + a.W : (gx >= a.W ? gx - a.W : gx);
            gy = gy < 0 ? gy + a.H : (gy >= a.H ? gy - a.H : gy);
        } else {
            gx %= a.W;
            if (gx < 0) gx += a.W;
            gy %= a.H;
            if (gy < 0) gy += a.H;
        }
        const int64_t o = (int64_t)gy * a.W + gx;
        P[ly][lx] = a.psi[o];
        Z[ly][lx] = a.zin[o];
    }
    __syncthreads();
    const int lx = threadIdx.x + 1;
    if (!xin) return;
    const bool keep_acc = a.acc_mode == 1 || a.acc_mode == 2;  // wave-uniform
#pragma unroll
    for (int r = 0; r < kTY / kBY; ++r) {
        const int ly = threadIdx.y + r * kBY + 1;
        const int y = y0 + ly - 1;
        if (y >= a.H) break;
        // e / w = x +- 1, n / s = y +- 1 (n = the next row in memory, as oracle/bvort_oracle.py)
        const T pe = P[ly][lx + 1], pw = P[ly][lx - 1], pn = P[ly + 1][lx], ps = P[ly - 1][lx];
        const T pne = P[ly + 1][lx + 1], pnw = P[ly + 1][lx - 1], pse = P[ly - 1][lx + 1], psw = P[ly - 1][lx - 1];
        const T zc = Z[ly][lx], ze = Z[ly][lx + 1], zw = Z[ly][lx - 1], zn = Z[ly + 1][lx], zs = Z[ly - 1][lx];
        const T zne = Z[ly + 1][lx + 1], znw = Z[ly + 1][lx - 1], zse = Z[ly - 1][lx + 1], zsw = Z[ly - 1][lx - 1];
        const T jpp = (pe - pw) * (zn - zs) - (pn - ps) * (ze - zw);
        const T jpx = pe * (zne - zse) - pw * (znw - zsw) - pn * (zne - znw) + ps * (zse - zsw);
        const T jxp = zn * (pne - pnw) - zs * (pse - psw) - ze * (pne - pse) + zw * (pnw - psw);
        T k = -((jpp + jpx + jxp) * a.inv12dxdy);
        k = k - a.beta * ((pe - pw) * a.inv2dx);
        k = k + a.nu * ((ze + zw - T(2) * zc) * a.idx2 + (zn + zs - T(2) * zc) * a.idy2);
        const int64_t o = (int64_t)y * a.W + x;
        // modes 0-2: zout = z0 + c k; 3 (RK4's final): zout = z0 + c (acc + k)
        a.zout[o] = z0v[r] + a.c * (a.acc_mode == 3 ? accv[r] + k : k);
        // mode 1: acc = w k; 2: acc += w k
        if (keep_acc) a.acc[o] = a.acc_mode == 2 ? accv[r] + a.w * k : a.w * k;
    }
}

// spec[l][k] *= norm / lambda(k, l), lambda = ax[k] + ay[l]; the (0, 0) mode (lambda = 0,
// the domain mean) is set to 0.
template <typename T, typename C>
__global__ __launch_bounds__(256) void bv_spectral_kernel(C* spec, const T* ax, const T* ay, int nk, int H, T norm) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    const int l = blockIdx.y;
    if (k >= nk) return;
    const int64_t o = (int64_t)l * nk + k;
    const T lam = ax[k] + ay[l];
    const T m = (k == 0 && l == 0) ? T(0) : norm / lam;
    C v = spec[o];
    v.x *= m;
    v.y *= m;
    spec[o] = v;
}

// u = -d(psi)/dy, v = d(psi)/dx (centred, periodic)
template <typename T>
__global__ __launch_bounds__(256) void bv_velocity_kernel(const T* psi, T* u, T* v, int W, int H, T inv2dx,
                                                          T inv2dy) {
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= W) return;
    const int64_t o = (int64_t)y * W + x;
    const T pn = psi[(int64_t)wrap(y + 1, H) * W + x], ps = psi[(int64_t)wrap(y - 1, H) * W + x];
    const T pe = psi[(int64_t)y * W + wrap(x + 1, W)], pw = psi[(int64_t)y * W + wrap(x - 1, W)];
    u[o] = -((pn - ps) * inv2dy);
    v[o] = (pe - pw) * inv2dx;
}

// ---- Poisson solve by LDS-resident FFTs (power-of-two W, H <= 4096) --------------------
// Three passes, each reading and writing the field once (hipFFT's 2-D plan is eight kernels
// per R2C / C2R pair, two of them transposes):
//   1. bv_rowfft_fwd: two real rows a, b as one complex FFT z = a + i b (radix-2 DIT in
//      LDS), split into the half spectra A(k), B(k), k = 0..W/2 -> spec[l][k];
//   2. bv_colsolve:  CW adjacent spectrum columns: forward FFT along y (DIT), scale by
//      norm / lambda(k, l) (the (0, 0) mode -> 0), inverse FFT along y (DIF, bit-reversed
//      result written back in natural order);
//   3. bv_rowfft_inv: Z = A + i B over the full Hermitian extension, inverse FFT (DIF),
//      real part -> row a of psi, imaginary part -> row b.
// Twiddles tw[j] = exp(-2 pi i j / N), j < N/2, computed on the host in double.
template <typename T>
struct Cx {
    T x, y;
};

// LDS index swizzle: element i lives at slot i ^ (((i >> 3) ^ (i >> 4) ^ (i >> 9)) & 31) -- a
// permutation inside each aligned block of 32 elements (256 B, every bank once for 8-byte
// elements). Chosen by a GF(2) search over shift-xor maps (tools/lds_swizzle.py): every
// 32-lane ds_read_b64 group of the FFT passes (radix-8 groups at strides 1 / 8 / 64..., the
// bit-reversed row / column gathers, 4-column blocks at stride H) touches 32 distinct slots,
// and every 16-lane ds_write_b64 group at most 2 per bank (modelled at 2048: 32 + 831 extra
// LDS cycles where the round-2 "+1 per 16" padding had 6 912 + 9 920).
__device__ __forceinline__ int P(int i) { return i ^ (((i >> 3) ^ (i >> 4) ^ (i >> 9)) & 31); }
__host__ __device__ constexpr size_t padded(size_t n) { return (n + 31) / 32 * 32; }
// Twiddle table slots: a pass reads tw[k * tstep] with k following the lanes, at strides of
// 2 .. 128 entries -- with a plain table 8 to 16 lanes of a 32-lane group share a bank. Entry
// k lives at k ^ ((k >> 5) & 31): for every stride 2^a (a = 1..7) the 32 lanes' slots are
// distinct modulo 32 (their low index bits pass through, the bits shifted out of the low
// five come back in by the xor). A permutation inside each aligned block of 32 entries.
__device__ __forceinline__ int TW(int k) { return k ^ ((k >> 5) & 31); }

__device__ __forceinline__ int bitrev(int i, int logn) { return (int)(__builtin_bitreverse32((uint32_t)i) >> (32 - logn)); }

// Workgroup barrier ordering LDS traffic only (the FFT passes exchange data through LDS; no
// global-memory fence needed between them)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Radix-2 stages taken R at a time in registers (one LDS pass and one barrier per R stages):
// a thread owns the 2^R elements base + j + m h (m < 2^R, j < h) that those stages combine.
// DIT: stages s .. s+R-1 (h = 2^(s-1)); input bit-reversed, output natural after all passes.
template <typename T, bool INV, int R>
__device__ __forceinline__ void dit_pass(Cx<T>* a, const Cx<T>* tw, int n, int logn, int s, int ncol) {
    constexpr int M = 1 << R;
    const int h = 1 << (s - 1);
    const int lg = logn - R;  // log2(groups per column)
    for (int g = threadIdx.x; g < (ncol << lg); g += blockDim.x) {
        const int c = g >> lg, gg = g & ((1 << lg) - 1);
        const int j = gg & (h - 1);
        const int base = c * n + ((gg >> (s - 1)) << (s - 1 + R)) + j;
        Cx<T> x[M];
#pragma unroll
        for (int m = 0; m < M; ++m) x[m] = a[P(base + m * h)];
#pragma unroll
        for (int t = 0; t < R; ++t) {
            const int hs = 1 << t;
            const int tstep = n >> (s + t);
#pragma unroll
            for (int m = 0; m < M; ++m) {
                if (m & hs) continue;
                Cx<T> w = tw[TW((j + (m & (hs - 1)) * h) * tstep)];
                if (INV) w.y = -w.y;
                const Cx<T> v = x[m + hs];
                const Cx<T> p{v.x * w.x - v.y * w.y, v.x * w.y + v.y * w.x};
                x[m + hs] = Cx<T>{x[m].x - p.x, x[m].y - p.y};
                x[m] = Cx<T>{x[m].x + p.x, x[m].y + p.y};
            }
        }
#pragma unroll
        for (int m = 0; m < M; ++m) a[P(base + m * h)] = x[m];
    }
    lds_barrier();
}

// DIF: stages s, s-1, .., s-R+1 (h = 2^(s-R), the smallest half); input natural, output
// bit-reversed after all passes.
template <typename T, bool INV, int R>
__device__ __forceinline__ void dif_pass(Cx<T>* a, const Cx<T>* tw, int n, int logn, int s, int ncol) {
    constexpr int M = 1 << R;
    const int lh = s - R;
    const int h = 1 << lh;
    const int lg = logn - R;
    for (int g = threadIdx.x; g < (ncol << lg); g += blockDim.x) {
        const int c = g >> lg, gg = g & ((1 << lg) - 1);
        const int j = gg & (h - 1);
        const int base = c * n + ((gg >> lh) << (lh + R)) + j;
        Cx<T> x[M];
#pragma unroll
        for (int m = 0; m < M; ++m) x[m] = a[P(base + m * h)];
#pragma unroll
        for (int t = R - 1; t >= 0; --t) {
            const int hs = 1 << t;
            const int tstep = n >> (lh + 1 + t);
#pragma unroll
            for (int m = 0; m < M; ++m) {
                if (m & hs) continue;
                Cx<T> w = tw[TW((j + (m & (hs - 1)) * h) * tstep)];
                if (INV) w.y = -w.y;
                const Cx<T> u = x[m], v = x[m + hs];
                const Cx<T> d{u.x - v.x, u.y - v.y};
                x[m] = Cx<T>{u.x + v.x, u.y + v.y};
                x[m + hs] = Cx<T>{d.x * w.x - d.y * w.y, d.x * w.y + d.y * w.x};
            }
        }
#pragma unroll
        for (int m = 0; m < M; ++m) a[P(base + m * h)] = x[m];
    }
    lds_barrier();
}

// radix-2 decimation in time over ncol columns of length n (column c at a + c * n), input in
// bit-reversed order, output natural; forward (INV = false) or unscaled inverse
template <typename T, bool INV>
__device__ void fft_dit(Cx<T>* a, const Cx<T>* tw, int n, int logn, int ncol) {
    int s = 1;
    for (; logn - s + 1 >= 3; s += 3) dit_pass<T, INV, 3>(a, tw, n, logn, s, ncol);
    if (logn - s + 1 == 2) dit_pass<T, INV, 2>(a, tw, n, logn, s, ncol);
    else if (logn - s + 1 == 1) dit_pass<T, INV, 1>(a, tw, n, logn, s, ncol);
}

// radix-2 decimation in frequency: input natural, output bit-reversed
template <typename T, bool INV>
__device__ void fft_dif(Cx<T>* a, const Cx<T>* tw, int n, int logn, int ncol) {
    int s = logn;
    for (; s >= 3; s -= 3) dif_pass<T, INV, 3>(a, tw, n, logn, s, ncol);
    if (s == 2) dif_pass<T, INV, 2>(a, tw, n, logn, s, ncol);
    else if (s == 1) dif_pass<T, INV, 1>(a, tw, n, logn, s, ncol);
}

constexpr int kRowThreads = 256;
constexpr int kColPer = 8;  // column pass: elements per thread, cw H <= 8 kColThreads (one radix-8 group per pass)
template <typename T>
constexpr int kColThreads = sizeof(T) == 8 ? 512 : 1024;

// One pair of rows per workgroup. (Persistent workgroups walking several pairs with the next
// pair's loads in flight during the FFT measured slower: 16.4-17.1 us against 14.5 at 2048^2
// fp32 -- the prefetch registers cost a wave per SIMD of occupancy.)
template <typename T>
__global__ __launch_bounds__(kRowThreads) void bv_rowfft_fwd(const T* z, Cx<T>* spec, const Cx<T>* tw, int W, int logw) {
    extern __shared__ __align__(16) unsigned char smem[];
    Cx<T>* a = (Cx<T>*)smem;
    Cx<T>* twl = a + padded(W);  // twiddles staged in LDS: every pass reads them
    const int nk = W / 2;        // spectrum columns: k = 1 .. W/2-1, plus the packed real bins in column 0
    const int64_t r0 = 2 * (int64_t)blockIdx.x, r1 = r0 + 1;
    for (int i = threadIdx.x; i < W / 2; i += kRowThreads) twl[TW(i)] = tw[i];
    for (int i = threadIdx.x; i < W; i += kRowThreads) a[P(bitrev(i, logw))] = Cx<T>{z[r0 * W + i], z[r1 * W + i]};
    lds_barrier();
    fft_dit<T, false>(a, twl, W, logw, 1);
    const T h = T(0.5);
    for (int k = threadIdx.x; k < nk; k += kRowThreads) {
        const Cx<T> zk = a[P(k)];
        if (k == 0) {
            // the real bins A(0) = Re Z(0), A(W/2) = Re Z(W/2) (B: the imaginary parts) share
            // column 0 as A(0) + i A(W/2): the column pass transforms both real columns at once
            const Cx<T> zn = a[P(W / 2)];
            spec[r0 * nk] = Cx<T>{zk.x, zn.x};
            spec[r1 * nk] = Cx<T>{zk.y, zn.y};
            continue;
        }
        const Cx<T> zm = a[P(W - k)];  // Z(W - k)
        // A = (Z(k) + conj Z(W-k)) / 2, B = (Z(k) - conj Z(W-k)) / 2i
        spec[r0 * nk + k] = Cx<T>{(zk.x + zm.x) * h, (zk.y - zm.y) * h};
        spec[r1 * nk + k] = Cx<T>{(zk.y + zm.y) * h, (zm.x - zk.x) * h};
    }
}

// nk = W/2 spectrum columns (column 0 = the packed real bins, see bv_rowfft_fwd), cw per
// workgroup; the grid is mapped XCD-major (workgroup b runs on XCD b % 8) so the workgroups
// that share the 128-byte lines of a spectrum row segment share one L2. (Persistent
// workgroups with a register prefetch of the next block measured slower, 27.4 against 25.1 us.)
template <typename T>
__global__ __launch_bounds__(kColThreads<T>) void bv_colsolve(Cx<T>* spec, const Cx<T>* tw, const T* ax, const T* ay,
                                                               int nk, int H, int logh, int logcw, T norm) {
    extern __shared__ __align__(16) unsigned char smem[];
    Cx<T>* a = (Cx<T>*)smem;
    const int cw = 1 << logcw;
    Cx<T>* twl = a + padded((size_t)cw * H);
    const int nblk = gridDim.x;
    const int blk = (nblk & 7) ? (int)blockIdx.x : (int)((blockIdx.x & 7) * (nblk >> 3) + (blockIdx.x >> 3));
    const int k0 = blk * cw;
    const int ncol = min(cw, nk - k0);
    const int t = threadIdx.x, nt = blockDim.x;
    for (int i = t; i < H / 2; i += nt) twl[TW(i)] = tw[i];
    for (int i = t; i < H * cw; i += nt) {
        const int l = i >> logcw, c = i & (cw - 1);
        if (c < ncol) a[P((c << logh) + bitrev(l, logh))] = spec[(int64_t)l * nk + k0 + c];
    }
    lds_barrier();
    fft_dit<T, false>(a, twl, H, logh, ncol);
    for (int i = t; i < H * ncol; i += nt) {
        const int c = i >> logh, l = i & (H - 1);
        const int k = k0 + c;
        if (k == 0) {
            // packed column Z = C0 + i CN (C0, CN: spectra of the real bins' columns, both
            // Hermitian); scaled separately by s0 = norm / lambda(0, l) (0 at l = 0) and
            // sN = norm / lambda(W/2, l), recombined: Z'(l) = (s0 + sN)/2 Z(l) + (s0 - sN)/2 conj Z(-l)
            if (l > H / 2) continue;  // the pair (l, H - l) is done by the thread of l
            const int n = (H - l) & (H - 1);
            const T s0 = l == 0 ? T(0) : norm / (ax[0] + ay[l]);
            const T sN = norm / (ax[nk] + ay[l]);
            const T p = (s0 + sN) * T(0.5), q = (s0 - sN) * T(0.5);
            const Cx<T> zl = a[P(l)], zn = a[P(n)];
            a[P(l)] = Cx<T>{p * zl.x + q * zn.x, p * zl.y - q * zn.y};
            if (n != l) a[P(n)] = Cx<T>{p * zn.x + q * zl.x, p * zn.y - q * zl.y};
            continue;
        }
        const T m = norm / (ax[k] + ay[l]);
        a[P(i)].x *= m;
        a[P(i)].y *= m;
    }
    lds_barrier();
    fft_dif<T, true>(a, twl, H, logh, ncol);
    for (int i = t; i < H * cw; i += nt) {
        const int l = i >> logcw, c = i & (cw - 1);
        if (c < ncol) spec[(int64_t)l * nk + k0 + c] = a[P((c << logh) + bitrev(l, logh))];
    }
}

template <typename T>
__global__ __launch_bounds__(kRowThreads) void bv_rowfft_inv(const Cx<T>* spec, T* psi, const Cx<T>* tw, int W, int logw) {
    extern __shared__ __align__(16) unsigned char smem[];
    Cx<T>* a = (Cx<T>*)smem;
    Cx<T>* twl = a + padded(W);
    const int nk = W / 2;  // column 0 packs the real bins: A(0) + i A(W/2)
    const int64_t r0 = 2 * (int64_t)blockIdx.x, r1 = r0 + 1;
    for (int i = threadIdx.x; i < W / 2; i += kRowThreads) twl[TW(i)] = tw[i];
    // Z = A + i B over the Hermitian extension: bin k < W/2 gives Z(k) and Z(W - k); the real
    // bins (C2R: their imaginary parts are ignored) give Z(0) and Z(W/2). Each bin read once.
    for (int k = threadIdx.x; k < nk; k += kRowThreads) {
        const Cx<T> A = spec[r0 * nk + k], B = spec[r1 * nk + k];
        if (k == 0) {
            a[P(0)] = Cx<T>{A.x, B.x};
            a[P(nk)] = Cx<T>{A.y, B.y};
        } else {
            a[P(k)] = Cx<T>{A.x - B.y, A.y + B.x};
            a[P(W - k)] = Cx<T>{A.x + B.y, B.x - A.y};
        }
    }
    lds_barrier();
    fft_dif<T, true>(a, twl, W, logw, 1);
    for (int i = threadIdx.x; i < W; i += kRowThreads) {
        const Cx<T> v = a[P(bitrev(i, logw))];
        psi[r0 * W + i] = v.x;
        psi[r1 * W + i] = v.y;
    }
}

void hck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw AbiError(WS_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}
void fck(hipfftResult r, const char* what) {
    if (r != HIPFFT_SUCCESS) throw AbiError(WS_ERR_DEVICE, std::string(what) + ": hipFFT error " + std::to_string((int)r));
}

}  // namespace
}  // namespace ws

struct ws_bvort {
    int W = 0, H = 0, dtype = WS_F32, device = 0, method = WS_RK4;
    double dx = 1, dy = 1, dt = 0.01, beta = 0, nu = 0;
    double time = 0;
    int32_t step = 0;
    hipStream_t stream = nullptr;
    hipfftHandle r2c = 0, c2r = 0;
    bool have_r2c = false, have_c2r = false;
    void* z[2] = {nullptr, nullptr};
    void *A = nullptr, *B = nullptr, *psi = nullptr, *acc = nullptr, *spec = nullptr, *ax = nullptr, *ay = nullptr;
    void *u = nullptr, *v = nullptr;
    // LDS-FFT Poisson path (power-of-two W, H; WS_POISSON_HIPFFT at creation selects the library)
    bool lds_fft = false;
    void *twW = nullptr, *twH = nullptr;
    int logw = 0, logh = 0, cw = 1;
    int cur = 0;
    bool psi_current = false;  // psi holds the streamfunction of z[cur]
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_ms = 0;
    int64_t launches = 0;

    size_t es() const { return dtype == WS_F64 ? 8 : 4; }
    size_t cells() const { return (size_t)W * H; }
};

namespace ws {
namespace {

void bv_free(ws_bvort* b) {
    if (b->stream) (void)hipStreamSynchronize(b->stream);  // nothing queued may touch freed memory
    for (void* p : {b->z[0], b->z[1], b->A, b->B, b->psi, b->acc, b->spec, b->ax, b->ay, b->u, b->v, b->twW, b->twH})
        if (p) (void)hipFree(p);
    if (b->have_r2c) hipfftDestroy(b->r2c);
    if (b->have_c2r) hipfftDestroy(b->c2r);
    for (hipEvent_t e : {b->ev0, b->ev1})
        if (e) (void)hipEventDestroy(e);
    if (b->stream) (void)hipStreamDestroy(b->stream);
    delete b;
}

template <typename T>
void upload_eigen(ws_bvort* b) {
    const int nk = b->W / 2 + 1;
    std::vector<T> ax(nk), ay(b->H);
    const double pi = 3.14159265358979323846;
    for (int k = 0; k < nk; ++k) ax[k] = (T)((2.0 * std::cos(2.0 * pi * k / b->W) - 2.0) / (b->dx * b->dx));
    for (int l = 0; l < b->H; ++l) ay[l] = (T)((2.0 * std::cos(2.0 * pi * l / b->H) - 2.0) / (b->dy * b->dy));
    hck(hipMemcpy(b->ax, ax.data(), nk * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy");
    hck(hipMemcpy(b->ay, ay.data(), b->H * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy");
    if (b->lds_fft) {
        auto twiddles = [&](int n, void* dst) {
            std::vector<T> t((size_t)n);  // n / 2 complex
            for (int j = 0; j < n / 2; ++j) {
                t[2 * j] = (T)std::cos(2.0 * pi * j / n);
                t[2 * j + 1] = (T)-std::sin(2.0 * pi * j / n);
            }
            hck(hipMemcpy(dst, t.data(), t.size() * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy");
        };
        twiddles(b->W, b->twW);
        twiddles(b->H, b->twH);
    }
}

template <typename T>
void poisson_lds(ws_bvort* b, const void* zin) {
    const size_t cs = 2 * sizeof(T);
    const int nk = b->W / 2;  // spectrum columns of the LDS path (real bins packed in column 0)
    Cx<T>* spec = (Cx<T>*)b->spec;
    const size_t row_lds = (padded(b->W) + b->W / 2) * cs, col_lds = (padded((size_t)b->cw * b->H) + b->H / 2) * cs;
    hipLaunchKernelGGL((bv_rowfft_fwd<T>), dim3(b->H / 2), dim3(kRowThreads), row_lds, b->stream, (const T*)zin, spec,
                       (const Cx<T>*)b->twW, b->W, b->logw);
    hck(hipGetLastError(), "bv_rowfft_fwd");
    // one radix-8 group per thread and pass
    const int col_threads = std::min(kColThreads<T>, std::max(64, b->cw * b->H / 8));
    hipLaunchKernelGGL((bv_colsolve<T>), dim3((nk + b->cw - 1) / b->cw), dim3(col_threads), col_lds, b->stream, spec,
                       (const Cx<T>*)b->twH, (const T*)b->ax, (const T*)b->ay, nk, b->H, b->logh,
                       __builtin_ctz((unsigned)b->cw), (T)(1.0 / ((double)b->W * b->H)));
    hck(hipGetLastError(), "bv_colsolve");
    hipLaunchKernelGGL((bv_rowfft_inv<T>), dim3(b->H / 2), dim3(kRowThreads), row_lds, b->stream, (const Cx<T>*)spec,
                       (T*)b->psi, (const Cx<T>*)b->twW, b->W, b->logw);
    hck(hipGetLastError(), "bv_rowfft_inv");
    b->launches += 3;
}

// psi = lap^-1 zin (spectral), on the model's stream
template <typename T>
void poisson(ws_bvort* b, const void* zin) {
    if (b->lds_fft) return poisson_lds<T>(b, zin);
    const int nk = b->W / 2 + 1;
    if constexpr (sizeof(T) == 8) {
        fck(hipfftExecD2Z(b->r2c, (hipfftDoubleReal*)const_cast<void*>(zin), (hipfftDoubleComplex*)b->spec), "D2Z");
        hipLaunchKernelGGL((bv_spectral_kernel<double, double2>), dim3((nk + 255) / 256, b->H), dim3(256), 0,
                           b->stream, (double2*)b->spec, (const double*)b->ax, (const double*)b->ay, nk, b->H,
                           1.0 / ((double)b->W * b->H));
        hck(hipGetLastError(), "bv_spectral_kernel");
        fck(hipfftExecZ2D(b->c2r, (hipfftDoubleComplex*)b->spec, (hipfftDoubleReal*)b->psi), "Z2D");
    } else {
        fck(hipfftExecR2C(b->r2c, (hipfftReal*)const_cast<void*>(zin), (hipfftComplex*)b->spec), "R2C");
        hipLaunchKernelGGL((bv_spectral_kernel<float, float2>), dim3((nk + 255) / 256, b->H), dim3(256), 0,
                           b->stream, (float2*)b->spec, (const float*)b->ax, (const float*)b->ay, nk, b->H,
                           (float)(1.0 / ((double)b->W * b->H)));
        hck(hipGetLastError(), "bv_spectral_kernel");
        fck(hipfftExecC2R(b->c2r, (hipfftComplex*)b->spec, (hipfftReal*)b->psi), "C2R");
    }
    b->launches += 3;
}

template <typename T>
void stage(ws_bvort* b, const void* zin, void* zout, T c, T w, int acc_mode) {
    poisson<T>(b, zin);
    BvArgs<T> a{};
    a.zin = (const T*)zin;
    a.psi = (const T*)b->psi;
    a.z0 = (const T*)b->z[b->cur];
    a.zout = (T*)zout;
    a.acc = (T*)b->acc;
    a.W = b->W;
    a.H = b->H;
    a.c = c;
    a.w = w;
    a.acc_mode = acc_mode;
    a.inv12dxdy = (T)(1.0 / (12.0 * b->dx * b->dy));
    a.inv2dx = (T)(1.0 / (2.0 * b->dx));
    a.idx2 = (T)(1.0 / (b->dx * b->dx));
    a.idy2 = (T)(1.0 / (b->dy * b->dy));
    a.beta = (T)b->beta;
    a.nu = (T)b->nu;
    const dim3 grid((b->W + kTX - 1) / kTX, (b->H + kTY - 1) / kTY), block(kTX, kBY);
    hipLaunchKernelGGL((bv_stage_kernel<T>), grid, block, 0, b->stream, a);
    hck(hipGetLastError(), "bv_stage_kernel");
    b->launches += 1;
}

template <typename T>
void enqueue_step(ws_bvort* b) {
    const T dt = (T)b->dt;
    void* z0 = b->z[b->cur];
    void* z1 = b->z[1 - b->cur];
    switch (b->method) {
        case WS_RK2:
            stage<T>(b, z0, b->A, T(0.5) * dt, T(0), 0);
            stage<T>(b, b->A, z1, dt, T(0), 0);
            break;
        case WS_RK4:
            stage<T>(b, z0, b->A, T(0.5) * dt, T(1), 1);
            stage<T>(b, b->A, b->B, T(0.5) * dt, T(2), 2);
            stage<T>(b, b->B, b->A, dt, T(2), 2);
            stage<T>(b, b->A, z1, dt / T(6), T(0), 3);
            break;
        default:  // Euler
            stage<T>(b, z0, z1, dt, T(0), 0);
            break;
    }
    b->cur = 1 - b->cur;
    b->psi_current = false;
}

template <typename T>
void convert_copy(void* dst, int dst_dtype, const void* src, int src_dtype, size_t n) {
    (void)dst_dtype;
    T* d = (T*)dst;
    if (src_dtype == WS_F64) {
        const double* s = (const double*)src;
        for (size_t i = 0; i < n; ++i) d[i] = (T)s[i];
    } else {
        const float* s = (const float*)src;
        for (size_t i = 0; i < n; ++i) d[i] = (T)s[i];
    }
}

}  // namespace
}  // namespace ws

using ws::AbiError;

extern "C" {

int ws_bvort_create(const ws_config_t* cfg, ws_bvort_t** out) { return ws_bvort_create_poisson(cfg, WS_POISSON_AUTO, out); }

int ws_bvort_create_poisson(const ws_config_t* cfg, int32_t poisson, ws_bvort_t** out) {
    return ws::abi_guarded([&] {
        if (!cfg || !out) throw AbiError(WS_ERR_INVALID, "null argument");
        if (cfg->grid_width < 3 || cfg->grid_height < 3)
            throw AbiError(WS_ERR_INVALID, "barotropic vorticity model needs a grid of at least 3 x 3");
        if (!(cfg->dx > 0 && cfg->dy > 0)) throw AbiError(WS_ERR_INVALID, "Grid spacing must be positive");
        ws::abi_set_device(cfg->device_id);
        ws_bvort* b = new ws_bvort;
        b->W = cfg->grid_width;
        b->H = cfg->grid_height;
        b->dtype = cfg->double_precision ? WS_F64 : WS_F32;
        b->device = cfg->device_id;
        b->method = cfg->integration_method == WS_RK2 ? WS_RK2 : cfg->integration_method == WS_RK4 ? WS_RK4 : WS_EULER;
        b->dx = cfg->dx;
        b->dy = cfg->dy;
        b->dt = cfg->dt;
        b->beta = cfg->beta;
        b->nu = cfg->viscosity;
        try {
            ws::hck(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking), "hipStreamCreate");
            ws::hck(hipEventCreate(&b->ev0), "hipEventCreate");
            ws::hck(hipEventCreate(&b->ev1), "hipEventCreate");
            const size_t fb = b->cells() * b->es();
            for (void** p : {&b->z[0], &b->z[1], &b->A, &b->B, &b->psi, &b->acc})
                ws::hck(hipMalloc(p, fb), "hipMalloc");
            const int nk = b->W / 2 + 1;
            ws::hck(hipMalloc(&b->spec, (size_t)nk * b->H * 2 * b->es()), "hipMalloc");
            ws::hck(hipMalloc(&b->ax, (size_t)nk * b->es()), "hipMalloc");
            ws::hck(hipMalloc(&b->ay, (size_t)b->H * b->es()), "hipMalloc");
            for (void* p : {b->z[0], b->z[1], b->A, b->B, b->psi, b->acc})
                ws::hck(hipMemsetAsync(p, 0, fb, b->stream), "hipMemsetAsync");
            // the field uploads (ws_bvort_set_vorticity) use hipMemcpy, which is not ordered
            // with the model's non-blocking stream: the zeroing must be complete first
            ws::hck(hipStreamSynchronize(b->stream), "hipStreamSynchronize");
            const bool f64 = b->dtype == WS_F64;
            auto pow2 = [](int n) { return n >= 16 && n <= 4096 && (n & (n - 1)) == 0; };
            if (poisson != WS_POISSON_AUTO && poisson != WS_POISSON_HIPFFT) throw AbiError(WS_ERR_INVALID, "bad poisson mode");
            b->lds_fft = pow2(b->W) && pow2(b->H) && poisson != WS_POISSON_HIPFFT;
            if (b->lds_fft) {
                while ((1 << b->logw) < b->W) ++b->logw;
                while ((1 << b->logh) < b->H) ++b->logh;
                // adjacent spectrum columns per column-pass workgroup: <= 64 KB of LDS (1 / 2 / 8
                // columns measured no better than the 4 this gives at 2048^2 fp32)
                const size_t col_budget = 65536;
                while (b->cw < 16 && (size_t)2 * b->cw * b->H * 2 * b->es() <= col_budget) b->cw *= 2;
                // at most kColPer elements per thread of the column pass
                while (b->cw > 1 && (size_t)b->cw * b->H > (size_t)(f64 ? 512 : 1024) * ws::kColPer) b->cw /= 2;
                // data + twiddles can pass the 64 KB default of dynamic LDS (fp64 rows of 4096)
                const int lds_max = 160 * 1024;
                if (f64) {
                    ws::hck(hipFuncSetAttribute((const void*)ws::bv_rowfft_fwd<double>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max), "hipFuncSetAttribute");
                    ws::hck(hipFuncSetAttribute((const void*)ws::bv_rowfft_inv<double>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max), "hipFuncSetAttribute");
                    ws::hck(hipFuncSetAttribute((const void*)ws::bv_colsolve<double>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max), "hipFuncSetAttribute");
                } else {
                    ws::hck(hipFuncSetAttribute((const void*)ws::bv_rowfft_fwd<float>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max), "hipFuncSetAttribute");
                    ws::hck(hipFuncSetAttribute((const void*)ws::bv_rowfft_inv<float>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max), "hipFuncSetAttribute");
                    ws::hck(hipFuncSetAttribute((const void*)ws::bv_colsolve<float>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max), "hipFuncSetAttribute");
                }
                ws::hck(hipMalloc(&b->twW, (size_t)b->W * b->es()), "hipMalloc");
                ws::hck(hipMalloc(&b->twH, (size_t)b->H * b->es()), "hipMalloc");
            } else {
                ws::fck(hipfftPlan2d(&b->r2c, b->H, b->W, f64 ? HIPFFT_D2Z : HIPFFT_R2C), "hipfftPlan2d");
                b->have_r2c = true;
                ws::fck(hipfftPlan2d(&b->c2r, b->H, b->W, f64 ? HIPFFT_Z2D : HIPFFT_C2R), "hipfftPlan2d");
                b->have_c2r = true;
                ws::fck(hipfftSetStream(b->r2c, b->stream), "hipfftSetStream");
                ws::fck(hipfftSetStream(b->c2r, b->stream), "hipfftSetStream");
            }
            if (f64) ws::upload_eigen<double>(b);
            else ws::upload_eigen<float>(b);
        } catch (...) {
            ws::bv_free(b);
            throw;
        }
        *out = b;
    });
}

int ws_bvort_destroy(ws_bvort_t* b) {
    return ws::abi_guarded([&] {
        if (!b) return;
        (void)hipSetDevice(b->device);
        (void)hipStreamSynchronize(b->stream);
        ws::bv_free(b);
    });
}

int ws_bvort_set_vorticity(ws_bvort_t* b, const void* host, int32_t height, int32_t width, int32_t dtype) {
    return ws::abi_guarded([&] {
        if (!b || !host) throw AbiError(WS_ERR_INVALID, "null argument");
        if (height != b->H || width != b->W) throw AbiError(WS_ERR_SHAPE, "vorticity array shape mismatch");
        if (dtype != WS_F32 && dtype != WS_F64) throw AbiError(WS_ERR_INVALID, "bad dtype");
        ws::abi_set_device(b->device);
        std::vector<char> buf(b->cells() * b->es());
        if (b->dtype == WS_F64) ws::convert_copy<double>(buf.data(), b->dtype, host, dtype, b->cells());
        else ws::convert_copy<float>(buf.data(), b->dtype, host, dtype, b->cells());
        ws::hck(hipStreamSynchronize(b->stream), "hipStreamSynchronize");
        ws::hck(hipMemcpy(b->z[b->cur], buf.data(), buf.size(), hipMemcpyHostToDevice), "hipMemcpy");
        b->psi_current = false;
    });
}

// which: 0 vorticity, 1 streamfunction, 2 u, 3 v (of the current state)
int ws_bvort_get_field(ws_bvort_t* b, int32_t which, void* host, int32_t height, int32_t width, int32_t dtype) {
    return ws::abi_guarded([&] {
        if (!b || !host) throw AbiError(WS_ERR_INVALID, "null argument");
        if (which < 0 || which > 3) throw AbiError(WS_ERR_INVALID, "bad field id");
        if (height != b->H || width != b->W) throw AbiError(WS_ERR_SHAPE, "array shape mismatch");
        if (dtype != b->dtype) throw AbiError(WS_ERR_INVALID, "dtype must match the model precision");
        ws::abi_set_device(b->device);
        const void* src = b->z[b->cur];
        if (which >= 1) {
            if (!b->psi_current) {
                if (b->dtype == WS_F64) ws::poisson<double>(b, b->z[b->cur]);
                else ws::poisson<float>(b, b->z[b->cur]);
                b->psi_current = true;
            }
            src = b->psi;
            if (which >= 2) {
                const size_t fb = b->cells() * b->es();
                if (!b->u) ws::hck(hipMalloc(&b->u, fb), "hipMalloc");
                if (!b->v) ws::hck(hipMalloc(&b->v, fb), "hipMalloc");
                const dim3 grid((b->W + 255) / 256, b->H);
                if (b->dtype == WS_F64)
                    hipLaunchKernelGGL((ws::bv_velocity_kernel<double>), grid, dim3(256), 0, b->stream,
                                       (const double*)b->psi, (double*)b->u, (double*)b->v, b->W, b->H,
                                       1.0 / (2.0 * b->dx), 1.0 / (2.0 * b->dy));
                else
                    hipLaunchKernelGGL((ws::bv_velocity_kernel<float>), grid, dim3(256), 0, b->stream,
                                       (const float*)b->psi, (float*)b->u, (float*)b->v, b->W, b->H,
                                       (float)(1.0 / (2.0 * b->dx)), (float)(1.0 / (2.0 * b->dy)));
                ws::hck(hipGetLastError(), "bv_velocity_kernel");
                src = which == 2 ? b->u : b->v;
            }
        }
        ws::hck(hipStreamSynchronize(b->stream), "hipStreamSynchronize");
        ws::hck(hipMemcpy(host, src, b->cells() * b->es(), hipMemcpyDeviceToHost), "hipMemcpy");
    });
}

int ws_bvort_run(ws_bvort_t* b, int32_t n) {
    return ws::abi_guarded([&] {
        if (!b) throw AbiError(WS_ERR_INVALID, "null model");
        if (n <= 0) return;
        ws::abi_set_device(b->device);
        b->launches = 0;
        ws::hck(hipEventRecord(b->ev0, b->stream), "hipEventRecord");
        for (int i = 0; i < n; ++i) {
            if (b->dtype == WS_F64) {
                ws::enqueue_step<double>(b);
                b->time += b->dt;
            } else {
                ws::enqueue_step<float>(b);
                b->time = (double)((float)b->time + (float)b->dt);
            }
            b->step++;
        }
        ws::hck(hipEventRecord(b->ev1, b->stream), "hipEventRecord");
        ws::hck(hipEventSynchronize(b->ev1), "hipEventSynchronize");
        float ms = 0.f;
        ws::hck(hipEventElapsedTime(&ms, b->ev0, b->ev1), "hipEventElapsedTime");
        b->last_ms = ms;
    });
}

int ws_bvort_get_state(const ws_bvort_t* b, double* time, int32_t* step, double* last_run_ms,
                       int64_t* last_run_launches) {
    return ws::abi_guarded([&] {
        if (!b) throw AbiError(WS_ERR_INVALID, "null model");
        if (time) *time = b->time;
        if (step) *step = b->step;
        if (last_run_ms) *last_run_ms = b->last_ms;
        if (last_run_launches) *last_run_launches = b->launches;
    });
}

}  // extern "C"
