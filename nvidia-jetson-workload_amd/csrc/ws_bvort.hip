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
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ws_abi.h"
#include "ws_comm.h"
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
    int halo;       // 0: y wraps around H; 1: a slab -- rows -1 and H are halo rows (the ring neighbours')
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
    // (a slab reads its halo rows -1 / H directly; tile rows past the bottom halo row only feed
    // cells outside the slab and read that row)
    const bool wide = a.W >= kTX + 2 && (a.halo || a.H >= kTY + 2);
    for (int i = tid; i < (kTY + 2) * (kTX + 2); i += kTX * kBY) {
        const int ly = i / (kTX + 2), lx = i - ly * (kTX + 2);
        int gx = x0 + lx - 1, gy = y0 + ly - 1;
        if (wide) {
            gx = gx < 0 ? gx + a.W : (gx >= a.W ? gx - a.W : gx);
            if (a.halo) gy = gy > a.H ? a.H : gy;
            else gy = gy < 0 ? gy + a.H : (gy >= a.H ? gy - a.H : gy);
        } else {
            gx %= a.W;
            if (gx < 0) gx += a.W;
            if (a.halo) {
                gy = gy > a.H ? a.H : gy;
            } else {
                gy %= a.H;
                if (gy < 0) gy += a.H;
            }
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
                                                          T inv2dy, int halo) {
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= W) return;
    const int64_t o = (int64_t)y * W + x;
    // (a slab: rows -1 and H are psi's halo rows)
    const int yn = halo ? y + 1 : wrap(y + 1, H), ys = halo ? y - 1 : wrap(y - 1, H);
    const T pn = psi[(int64_t)yn * W + x], ps = psi[(int64_t)ys * W + x];
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

// Spectrum layout of the row passes: spectrum row r, column k at sidx(r, k) -- blocks of
// 2^lognc columns, each block holding all `rows` rows contiguously (block-major). One block
// (2^lognc = W/2) is the plain [row][k] layout of the single domain; a slab of a decomposition
// over n ranks uses n blocks, block q being what it sends to rank q in the transpose.
__device__ __forceinline__ int64_t sidx(int64_t r, int k, int rows, int lognc) {
    return (((int64_t)(k >> lognc) * rows + r) << lognc) + (k & ((1 << lognc) - 1));
}

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
__global__ __launch_bounds__(kRowThreads) void bv_rowfft_fwd(const T* z, Cx<T>* spec, const Cx<T>* tw, int W, int logw,
                                                              int rows, int lognc) {
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
            spec[sidx(r0, 0, rows, lognc)] = Cx<T>{zk.x, zn.x};
            spec[sidx(r1, 0, rows, lognc)] = Cx<T>{zk.y, zn.y};
            continue;
        }
        const Cx<T> zm = a[P(W - k)];  // Z(W - k)
        // A = (Z(k) + conj Z(W-k)) / 2, B = (Z(k) - conj Z(W-k)) / 2i
        spec[sidx(r0, k, rows, lognc)] = Cx<T>{(zk.x + zm.x) * h, (zk.y - zm.y) * h};
        spec[sidx(r1, k, rows, lognc)] = Cx<T>{(zk.y + zm.y) * h, (zm.x - zk.x) * h};
    }
}

// nk = W/2 spectrum columns (column 0 = the packed real bins, see bv_rowfft_fwd), cw per
// workgroup; the grid is mapped XCD-major (workgroup b runs on XCD b % 8) so the workgroups
// that share the 128-byte lines of a spectrum row segment share one L2. (Persistent
// workgroups with a register prefetch of the next block measured slower, 27.4 against 25.1 us.)
template <typename T>
// (a slab's column block: nk = its columns, global column kofs + c; nkg = W / 2, the global
// count, whose real bin A(W/2) is packed into global column 0)
__global__ __launch_bounds__(kColThreads<T>) void bv_colsolve(Cx<T>* spec, const Cx<T>* tw, const T* ax, const T* ay,
                                                               int nk, int H, int logh, int logcw, T norm, int kofs,
                                                               int nkg) {
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
        const int k = kofs + k0 + c;  // the global column
        if (k == 0) {
            // packed column Z = C0 + i CN (C0, CN: spectra of the real bins' columns, both
            // Hermitian); scaled separately by s0 = norm / lambda(0, l) (0 at l = 0) and
            // sN = norm / lambda(W/2, l), recombined: Z'(l) = (s0 + sN)/2 Z(l) + (s0 - sN)/2 conj Z(-l)
            if (l > H / 2) continue;  // the pair (l, H - l) is done by the thread of l
            const int n = (H - l) & (H - 1);
            const T s0 = l == 0 ? T(0) : norm / (ax[0] + ay[l]);
            const T sN = norm / (ax[nkg] + ay[l]);
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
__global__ __launch_bounds__(kRowThreads) void bv_rowfft_inv(const Cx<T>* spec, T* psi, const Cx<T>* tw, int W, int logw,
                                                              int rows, int lognc) {
    extern __shared__ __align__(16) unsigned char smem[];
    Cx<T>* a = (Cx<T>*)smem;
    Cx<T>* twl = a + padded(W);
    const int nk = W / 2;  // column 0 packs the real bins: A(0) + i A(W/2)
    const int64_t r0 = 2 * (int64_t)blockIdx.x, r1 = r0 + 1;
    for (int i = threadIdx.x; i < W / 2; i += kRowThreads) twl[TW(i)] = tw[i];
    // Z = A + i B over the Hermitian extension: bin k < W/2 gives Z(k) and Z(W - k); the real
    // bins (C2R: their imaginary parts are ignored) give Z(0) and Z(W/2). Each bin read once.
    for (int k = threadIdx.x; k < nk; k += kRowThreads) {
        const Cx<T> A = spec[sidx(r0, k, rows, lognc)], B = spec[sidx(r1, k, rows, lognc)];
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

// The copies of a one-process decomposition in one launch per slab and exchange: segment i
// moves n16[i] 16-byte units from src[i] (another slab's memory: the same device, or a peer)
// to dst[i] -- the blocks of a spectrum transpose, or the four halo rows of psi and zeta.
constexpr int kMaxSeg = 64;
struct BvSegments {
    const void* src[kMaxSeg];
    void* dst[kMaxSeg];
    int64_t n16[kMaxSeg];
};

__global__ __launch_bounds__(256) void bv_copy_segments(BvSegments a) {
    using V4 = unsigned int __attribute__((ext_vector_type(4)));
    const int seg = blockIdx.y;
    const V4* src = (const V4*)a.src[seg];
    V4* dst = (V4*)a.dst[seg];
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < a.n16[seg]; i += (int64_t)gridDim.x * 256)
        dst[i] = src[i];
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
    // fields: [H][W] (a slab: [H + 2][W], the pointer at row 0, rows -1 and H the halo)
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
    // y-slab decomposition around the periodic ring (ws_bvort_create_multi / _create_slab): this
    // model owns rows [row0, row0 + H) of Hg. The row FFTs stay local; the column pass needs
    // whole columns, so the spectrum is transposed in blocks of nc = (W/2) / nranks columns --
    // block q of every slab's spectrum rows (spec, block-major) to slab q's column block specc
    // ([Hg][nc]) and back -- and the stencils read one halo row of psi and zeta from the ring
    // neighbours. Transports: the process's own copies between the slabs of a one-process
    // decomposition (parts), or RCCL between processes (comm: send / receive per block; the
    // periodic halo plan).
    int Hg = 0, row0 = 0, halo = 0, rank = 0, nranks = 1;
    int nc = 0, lognc = 0;
    void* specc = nullptr;
    ws::SlabComm* comm = nullptr;
    std::vector<ws_bvort*> parts;
    hipEvent_t ev_phase = nullptr;  // a part: after its latest phase of a stage
    bool copy_kernel = true;        // parts: every slab may read every other's memory (same device / peer access)

    size_t es() const { return dtype == WS_F64 ? 8 : 4; }
    size_t cells() const { return (size_t)W * H; }
    size_t alloc_bytes() const { return (size_t)W * (H + 2 * halo) * es(); }
    size_t halo_bytes() const { return (size_t)halo * W * es(); }
};

namespace ws {
namespace {

void bv_free(ws_bvort* b) {
    for (ws_bvort* p : b->parts) {
        (void)hipSetDevice(p->device);
        bv_free(p);
    }
    b->parts.clear();
    if (b->stream) (void)hipStreamSynchronize(b->stream);  // nothing queued may touch freed memory
    for (void* p : {b->z[0], b->z[1], b->A, b->B, b->psi, b->acc, b->u, b->v})
        if (p) (void)hipFree((char*)p - b->halo_bytes());
    for (void* p : {b->spec, b->specc, b->ax, b->ay, b->twW, b->twH})
        if (p) (void)hipFree(p);
    if (b->have_r2c) hipfftDestroy(b->r2c);
    if (b->have_c2r) hipfftDestroy(b->c2r);
    for (hipEvent_t e : {b->ev0, b->ev1, b->ev_phase})
        if (e) (void)hipEventDestroy(e);
    if (b->stream) (void)hipStreamDestroy(b->stream);
    delete b->comm;
    delete b;
}

template <typename T>
void upload_eigen(ws_bvort* b) {
    const int nk = b->W / 2 + 1;
    std::vector<T> ax(nk), ay(b->Hg);
    const double pi = 3.14159265358979323846;
    for (int k = 0; k < nk; ++k) ax[k] = (T)((2.0 * std::cos(2.0 * pi * k / b->W) - 2.0) / (b->dx * b->dx));
    for (int l = 0; l < b->Hg; ++l) ay[l] = (T)((2.0 * std::cos(2.0 * pi * l / b->Hg) - 2.0) / (b->dy * b->dy));
    hck(hipMemcpy(b->ax, ax.data(), nk * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy");
    hck(hipMemcpy(b->ay, ay.data(), b->Hg * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy");
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
        twiddles(b->Hg, b->twH);
    }
}

// the row pass (forward: zeta rows -> spectrum rows; inverse: spectrum rows -> psi rows)
template <typename T>
void rowfft(ws_bvort* b, const void* zin, bool inverse) {
    const size_t row_lds = (padded(b->W) + b->W / 2) * 2 * sizeof(T);
    if (!inverse)
        hipLaunchKernelGGL((bv_rowfft_fwd<T>), dim3(b->H / 2), dim3(kRowThreads), row_lds, b->stream, (const T*)zin,
                           (Cx<T>*)b->spec, (const Cx<T>*)b->twW, b->W, b->logw, b->H, b->lognc);
    else
        hipLaunchKernelGGL((bv_rowfft_inv<T>), dim3(b->H / 2), dim3(kRowThreads), row_lds, b->stream,
                           (const Cx<T>*)b->spec, (T*)b->psi, (const Cx<T>*)b->twW, b->W, b->logw, b->H, b->lognc);
    hck(hipGetLastError(), inverse ? "bv_rowfft_inv" : "bv_rowfft_fwd");
    b->launches += 1;
}

// the column pass over a column block: the whole spectrum (single domain) or a slab's block
template <typename T>
void colsolve(ws_bvort* b, Cx<T>* cols, int nk, int kofs) {
    const size_t col_lds = (padded((size_t)b->cw * b->Hg) + b->Hg / 2) * 2 * sizeof(T);
    // one radix-8 group per thread and pass
    const int col_threads = std::min(kColThreads<T>, std::max(64, b->cw * b->Hg / 8));
    hipLaunchKernelGGL((bv_colsolve<T>), dim3((nk + b->cw - 1) / b->cw), dim3(col_threads), col_lds, b->stream, cols,
                       (const Cx<T>*)b->twH, (const T*)b->ax, (const T*)b->ay, nk, b->Hg, b->logh,
                       __builtin_ctz((unsigned)b->cw), (T)(1.0 / ((double)b->W * b->Hg)), kofs, b->W / 2);
    hck(hipGetLastError(), "bv_colsolve");
    b->launches += 1;
}

// RCCL slab: psi of this rank's rows of zin -- row pass, block transpose to the column blocks,
// column pass, transpose back, inverse row pass (every rank at once: collective)
template <typename T>
void poisson_comm(ws_bvort* b, const void* zin) {
    const size_t blk = (size_t)b->H * b->nc * 2 * sizeof(T);  // one block: my rows x nc columns
    rowfft<T>(b, zin, false);
    auto transpose = [&](bool back) {
        std::vector<SlabComm::Block> send, recv;
        for (int q = 0; q < b->nranks; ++q) {
            char* rows_blk = (char*)b->spec + (size_t)q * blk;       // my rows, q's columns
            char* cols_blk = (char*)b->specc + (size_t)q * blk;      // q's rows, my columns
            send.push_back({back ? cols_blk : rows_blk, blk, q});
            recv.push_back({back ? rows_blk : cols_blk, blk, q});
        }
        b->comm->alltoall(send, recv, b->stream);
    };
    transpose(false);
    colsolve<T>(b, (Cx<T>*)b->specc, b->nc, b->rank * b->nc);
    transpose(true);
    rowfft<T>(b, nullptr, true);
}

// psi = lap^-1 zin (spectral), on the model's stream (a single domain)
template <typename T>
void poisson(ws_bvort* b, const void* zin) {
    if (b->comm && b->nranks > 1) return poisson_comm<T>(b, zin);
    if (b->lds_fft) {
        rowfft<T>(b, zin, false);
        colsolve<T>(b, (Cx<T>*)b->spec, b->W / 2, 0);
        rowfft<T>(b, nullptr, true);
        return;
    }
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

// field of a model by id: 0 z[cur], 1 z[1 - cur], 2 A, 3 B, 4 psi
void* field_of(ws_bvort* b, int id) {
    switch (id) {
        case 0: return b->z[b->cur];
        case 1: return b->z[1 - b->cur];
        case 2: return b->A;
        case 3: return b->B;
        default: return b->psi;
    }
}

// One phase of a stage over the parts of a one-process decomposition: first, on every part's
// stream, the waits (for every part's previous phase, or only the ring neighbours') and the
// copies that read the other parts' memory; then every part's own kernels and its phase event
// -- so no wait of this phase can see an event of this same phase.
template <class Pull, class Work>
void phase(ws_bvort* m, bool all, Pull pull, Work work) {
    const int n = (int)m->parts.size();
    for (int q = 0; q < n; ++q) {
        ws_bvort* me = m->parts[q];
        hck(hipSetDevice(me->device), "hipSetDevice");
        for (int p = 0; p < n; ++p) {
            const bool nbr = p == (q + 1) % n || p == (q + n - 1) % n;
            if (p != q && (all || nbr)) hck(hipStreamWaitEvent(me->stream, m->parts[p]->ev_phase, 0), "hipStreamWaitEvent");
        }
        pull(q, me);
    }
    for (ws_bvort* me : m->parts) {
        hck(hipSetDevice(me->device), "hipSetDevice");
        work(me);
        hck(hipEventRecord(me->ev_phase, me->stream), "hipEventRecord");
    }
}

// copies (dst, src, bytes) on `me`'s stream: one bv_copy_segments launch when the slabs can
// read each other's memory and every piece is whole 16-byte units, else the runtime's copies
struct Piece {
    void* dst;
    const void* src;
    size_t bytes;
};
void copy_pieces(const ws_bvort* m, ws_bvort* me, const std::vector<Piece>& pieces) {
    bool kernel = m->copy_kernel && (int)pieces.size() <= kMaxSeg;
    size_t most = 0;
    for (const Piece& p : pieces) {
        kernel = kernel && p.bytes % 16 == 0 && (uintptr_t)p.dst % 16 == 0 && (uintptr_t)p.src % 16 == 0;
        most = std::max(most, p.bytes);
    }
    if (!kernel) {
        for (const Piece& p : pieces)
            hck(hipMemcpyAsync(p.dst, p.src, p.bytes, hipMemcpyDefault, me->stream), "hipMemcpyAsync");
        return;
    }
    BvSegments a{};
    for (size_t i = 0; i < pieces.size(); ++i) {
        a.src[i] = pieces[i].src;
        a.dst[i] = pieces[i].dst;
        a.n16[i] = (int64_t)(pieces[i].bytes / 16);
    }
    const unsigned bx = (unsigned)std::min<size_t>((most / 16 + 255) / 256, 1024);
    hipLaunchKernelGGL(bv_copy_segments, dim3(std::max(1u, bx), (unsigned)pieces.size()), dim3(256), 0, me->stream, a);
    hck(hipGetLastError(), "bv_copy_segments");
    me->launches += 1;
}

// psi of field `zid` on every part (one-process decomposition)
template <typename T>
void poisson_parts(ws_bvort* m, int zid) {
    const int n = (int)m->parts.size();
    phase(m, true, [](int, ws_bvort*) {}, [&](ws_bvort* me) { rowfft<T>(me, field_of(me, zid), false); });
    // block q of slab p's spectrum rows -> rows [row0_p, ...) of slab q's column block
    phase(m, true,
          [&](int q, ws_bvort* me) {
              std::vector<Piece> pieces;
              for (int p = 0; p < n; ++p) {
                  const ws_bvort* src = m->parts[p];
                  const size_t blk = (size_t)src->H * src->nc * 2 * sizeof(T);
                  pieces.push_back({(char*)me->specc + (size_t)src->row0 * me->nc * 2 * sizeof(T),
                                    (const char*)src->spec + (size_t)q * blk, blk});
              }
              copy_pieces(m, me, pieces);
          },
          [&](ws_bvort* me) { colsolve<T>(me, (Cx<T>*)me->specc, me->nc, me->rank * me->nc); });
    // and back: rows [row0_p, ...) of slab q's column block -> block q of slab p's spectrum rows
    phase(m, true,
          [&](int, ws_bvort* me) {
              std::vector<Piece> pieces;
              for (int q = 0; q < n; ++q) {
                  const ws_bvort* src = m->parts[q];
                  const size_t blk = (size_t)me->H * me->nc * 2 * sizeof(T);
                  pieces.push_back({(char*)me->spec + (size_t)q * blk,
                                    (const char*)src->specc + (size_t)me->row0 * src->nc * 2 * sizeof(T), blk});
              }
              copy_pieces(m, me, pieces);
          },
          [&](ws_bvort* me) { rowfft<T>(me, nullptr, true); });
}

// one halo row above and below of the given fields of every part, from its ring neighbours
void pull_halos(ws_bvort* m, int q, ws_bvort* me, std::initializer_list<int> ids) {
    const int n = (int)m->parts.size();
    ws_bvort* up = m->parts[(q + n - 1) % n];
    ws_bvort* dn = m->parts[(q + 1) % n];
    const size_t row = (size_t)me->W * me->es();
    std::vector<Piece> pieces;
    for (int id : ids) {
        char* f = (char*)field_of(me, id);
        pieces.push_back({f - row, (const char*)field_of(up, id) + (size_t)(up->H - 1) * row, row});
        pieces.push_back({f + (size_t)me->H * row, field_of(dn, id), row});
    }
    copy_pieces(m, me, pieces);
}

// an RCCL slab's halo rows of the given fields (the periodic plan; collective)
template <typename T>
void exchange_halos(ws_bvort* b, std::initializer_list<int> ids) {
    if (!b->comm || b->nranks < 2) return;
    void* f[4];
    int n = 0;
    for (int id : ids) f[n++] = field_of(b, id);
    Geom g{};
    g.W = b->W; g.H = b->H; g.L = 1;
    g.pitch = b->W;
    g.lstride = (int64_t)(b->H + 2) * b->W;
    g.halo = 1;
    b->comm->exchange(f, n, (int)sizeof(T), g, 1, b->stream, /*periodic=*/true);
}

template <typename T>
void stage_kernel(ws_bvort* b, const void* zin, void* zout, T c, T w, int acc_mode) {
    BvArgs<T> a{};
    a.zin = (const T*)zin;
    a.psi = (const T*)b->psi;
    a.z0 = (const T*)b->z[b->cur];
    a.zout = (T*)zout;
    a.acc = (T*)b->acc;
    a.W = b->W;
    a.H = b->H;
    a.halo = b->halo;
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

// one RK stage: field in_id -> field out_id (ids of field_of)
template <typename T>
void stage(ws_bvort* b, int in_id, int out_id, T c, T w, int acc_mode) {
    if (b->parts.empty()) {
        poisson<T>(b, field_of(b, in_id));
        exchange_halos<T>(b, {in_id, 4});
        stage_kernel<T>(b, field_of(b, in_id), field_of(b, out_id), c, w, acc_mode);
        return;
    }
    poisson_parts<T>(b, in_id);
    phase(b, false, [&](int q, ws_bvort* me) { pull_halos(b, q, me, {in_id, 4}); },
          [&](ws_bvort* me) { stage_kernel<T>(me, field_of(me, in_id), field_of(me, out_id), c, w, acc_mode); });
}

template <typename T>
void enqueue_step(ws_bvort* b) {
    const T dt = (T)b->dt;
    switch (b->method) {
        case WS_RK2:
            stage<T>(b, 0, 2, T(0.5) * dt, T(0), 0);
            stage<T>(b, 2, 1, dt, T(0), 0);
            break;
        case WS_RK4:
            stage<T>(b, 0, 2, T(0.5) * dt, T(1), 1);
            stage<T>(b, 2, 3, T(0.5) * dt, T(2), 2);
            stage<T>(b, 3, 2, dt, T(2), 2);
            stage<T>(b, 2, 1, dt / T(6), T(0), 3);
            break;
        default:  // Euler
            stage<T>(b, 0, 1, dt, T(0), 0);
            break;
    }
    b->cur = 1 - b->cur;
    for (ws_bvort* p : b->parts) p->cur = 1 - p->cur;
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

// a model's buffers, stream, events and Poisson path (its geometry and parameters set; the
// device current); slabs (halo = 1) take the LDS-FFT path only
void bv_alloc(ws_bvort* b, int32_t poisson) {
    hck(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking), "hipStreamCreate");
    hck(hipEventCreate(&b->ev0), "hipEventCreate");
    hck(hipEventCreate(&b->ev1), "hipEventCreate");
    hck(hipEventCreateWithFlags(&b->ev_phase, hipEventDisableTiming), "hipEventCreate");
    for (void** p : {&b->z[0], &b->z[1], &b->A, &b->B, &b->psi, &b->acc}) {
        void* a = nullptr;
        hck(hipMalloc(&a, b->alloc_bytes()), "hipMalloc");
        hck(hipMemsetAsync(a, 0, b->alloc_bytes(), b->stream), "hipMemsetAsync");
        *p = (char*)a + b->halo_bytes();
    }
    const int nk = b->W / 2 + 1;
    hck(hipMalloc(&b->spec, (size_t)nk * b->H * 2 * b->es()), "hipMalloc");
    hck(hipMalloc(&b->ax, (size_t)nk * b->es()), "hipMalloc");
    hck(hipMalloc(&b->ay, (size_t)b->Hg * b->es()), "hipMalloc");
    // the field uploads (ws_bvort_set_vorticity) use hipMemcpy, which is not ordered with the
    // model's non-blocking stream: the zeroing must be complete first
    hck(hipStreamSynchronize(b->stream), "hipStreamSynchronize");
    const bool f64 = b->dtype == WS_F64;
    auto pow2 = [](int n) { return n >= 16 && n <= 4096 && (n & (n - 1)) == 0; };
    if (poisson != WS_POISSON_AUTO && poisson != WS_POISSON_HIPFFT) throw AbiError(WS_ERR_INVALID, "bad poisson mode");
    b->lds_fft = pow2(b->W) && pow2(b->Hg) && poisson != WS_POISSON_HIPFFT;
    if (b->nranks > 1 && !b->lds_fft)
        throw AbiError(WS_ERR_INVALID, "a decomposed vorticity model needs power-of-two width and height "
                                       "(16..4096) and the LDS-FFT Poisson path");
    if (b->lds_fft) {
        while ((1 << b->logw) < b->W) ++b->logw;
        while ((1 << b->logh) < b->Hg) ++b->logh;
        b->nc = b->W / 2 / b->nranks;
        while ((1 << b->lognc) < b->nc) ++b->lognc;
        if (b->nranks > 1) hck(hipMalloc(&b->specc, (size_t)b->Hg * b->nc * 2 * b->es()), "hipMalloc");
        // adjacent spectrum columns per column-pass workgroup: <= 64 KB of LDS (1 / 2 / 8
        // columns measured no better than the 4 this gives at 2048^2 fp32)
        const size_t col_budget = 65536;
        while (b->cw < 16 && (size_t)2 * b->cw * b->Hg * 2 * b->es() <= col_budget) b->cw *= 2;
        // at most kColPer elements per thread of the column pass
        while (b->cw > 1 && (size_t)b->cw * b->Hg > (size_t)(f64 ? 512 : 1024) * kColPer) b->cw /= 2;
        // data + twiddles can pass the 64 KB default of dynamic LDS (fp64 rows of 4096)
        const int lds_max = 160 * 1024;
        if (f64) {
            hck(hipFuncSetAttribute((const void*)bv_rowfft_fwd<double>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max), "hipFuncSetAttribute");
            hck(hipFuncSetAttribute((const void*)bv_rowfft_inv<double>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max), "hipFuncSetAttribute");
            hck(hipFuncSetAttribute((const void*)bv_colsolve<double>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max), "hipFuncSetAttribute");
        } else {
            hck(hipFuncSetAttribute((const void*)bv_rowfft_fwd<float>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max), "hipFuncSetAttribute");
            hck(hipFuncSetAttribute((const void*)bv_rowfft_inv<float>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max), "hipFuncSetAttribute");
            hck(hipFuncSetAttribute((const void*)bv_colsolve<float>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max), "hipFuncSetAttribute");
        }
        hck(hipMalloc(&b->twW, (size_t)b->W * b->es()), "hipMalloc");
        hck(hipMalloc(&b->twH, (size_t)b->Hg * b->es()), "hipMalloc");
    } else {
        fck(hipfftPlan2d(&b->r2c, b->H, b->W, f64 ? HIPFFT_D2Z : HIPFFT_R2C), "hipfftPlan2d");
        b->have_r2c = true;
        fck(hipfftPlan2d(&b->c2r, b->H, b->W, f64 ? HIPFFT_Z2D : HIPFFT_C2R), "hipfftPlan2d");
        b->have_c2r = true;
        fck(hipfftSetStream(b->r2c, b->stream), "hipfftSetStream");
        fck(hipfftSetStream(b->c2r, b->stream), "hipfftSetStream");
    }
    if (f64) upload_eigen<double>(b);
    else upload_eigen<float>(b);
}

void bv_params(ws_bvort* b, const ws_config_t* cfg) {
    b->W = cfg->grid_width;
    b->H = b->Hg = cfg->grid_height;
    b->dtype = cfg->double_precision ? WS_F64 : WS_F32;
    b->device = cfg->device_id;
    b->method = cfg->integration_method == WS_RK2 ? WS_RK2 : cfg->integration_method == WS_RK4 ? WS_RK4 : WS_EULER;
    b->dx = cfg->dx;
    b->dy = cfg->dy;
    b->dt = cfg->dt;
    b->beta = cfg->beta;
    b->nu = cfg->viscosity;
}

void bv_check(const ws_config_t* cfg, int nranks) {
    if (cfg->grid_width < 3 || cfg->grid_height < 3)
        throw AbiError(WS_ERR_INVALID, "barotropic vorticity model needs a grid of at least 3 x 3");
    if (!(cfg->dx > 0 && cfg->dy > 0)) throw AbiError(WS_ERR_INVALID, "Grid spacing must be positive");
    if (nranks > 1) {
        // equal slabs of whole row pairs (the row passes pair rows 2i, 2i+1) and equal column blocks
        if ((nranks & (nranks - 1)) != 0 || cfg->grid_height % (2 * nranks) != 0 || (cfg->grid_width / 2) % nranks != 0)
            throw AbiError(WS_ERR_INVALID, "a decomposed vorticity model needs a power-of-two slab count that splits "
                                           "the rows into equal even slabs and width / 2 into equal column blocks");
    }
}

// slab r of n (n = 1: the whole domain)
ws_bvort* bv_make(const ws_config_t* cfg, int32_t poisson, int device, int rank, int nranks) {
    ws_bvort* b = new ws_bvort;
    bv_params(b, cfg);
    b->device = device;
    b->rank = rank;
    b->nranks = nranks;
    slab_rows(b->Hg, rank, nranks, &b->row0, &b->H);
    b->halo = nranks > 1 ? 1 : 0;
    try {
        abi_set_device(device);
        bv_alloc(b, poisson);
    } catch (...) {
        bv_free(b);
        throw;
    }
    return b;
}

// host (height, W) rows [r0, r0 + p->H) <-> part p's own rows of a device field
void copy_rows(ws_bvort* p, void* dev, void* host, int r0, bool upload) {
    abi_set_device(p->device);
    hck(hipStreamSynchronize(p->stream), "hipStreamSynchronize");
    const size_t bytes = p->cells() * p->es();
    char* h = (char*)host + (size_t)r0 * p->W * p->es();
    if (upload) hck(hipMemcpy(dev, h, bytes, hipMemcpyHostToDevice), "hipMemcpy");
    else hck(hipMemcpy(h, dev, bytes, hipMemcpyDeviceToHost), "hipMemcpy");
}

template <typename T>
void velocity(ws_bvort* b) {
    const size_t fb = b->alloc_bytes();
    for (void** p : {&b->u, &b->v})
        if (!*p) {
            void* a = nullptr;
            hck(hipMalloc(&a, fb), "hipMalloc");
            *p = (char*)a + b->halo_bytes();
        }
    const dim3 grid((b->W + 255) / 256, b->H);
    hipLaunchKernelGGL((bv_velocity_kernel<T>), grid, dim3(256), 0, b->stream, (const T*)b->psi, (T*)b->u, (T*)b->v,
                       b->W, b->H, (T)(1.0 / (2.0 * b->dx)), (T)(1.0 / (2.0 * b->dy)), b->halo);
    hck(hipGetLastError(), "bv_velocity_kernel");
}

// psi (and, which >= 2, u / v) of the current state, on every part
template <typename T>
void diagnose(ws_bvort* b, int which) {
    if (!b->psi_current) {
        if (b->parts.empty()) poisson<T>(b, b->z[b->cur]);
        else poisson_parts<T>(b, 0);
        b->psi_current = true;
    }
    if (which < 2) return;
    if (b->parts.empty()) {
        exchange_halos<T>(b, {4});
        velocity<T>(b);
        return;
    }
    phase(b, false, [&](int q, ws_bvort* me) { pull_halos(b, q, me, {4}); }, [&](ws_bvort* me) { velocity<T>(me); });
}

}  // namespace
}  // namespace ws

using ws::AbiError;

extern "C" {

int ws_bvort_create(const ws_config_t* cfg, ws_bvort_t** out) { return ws_bvort_create_poisson(cfg, WS_POISSON_AUTO, out); }

int ws_bvort_create_poisson(const ws_config_t* cfg, int32_t poisson, ws_bvort_t** out) {
    return ws::abi_guarded([&] {
        if (!cfg || !out) throw AbiError(WS_ERR_INVALID, "null argument");
        ws::bv_check(cfg, 1);
        *out = ws::bv_make(cfg, poisson, cfg->device_id, 0, 1);
    });
}

int ws_bvort_create_multi(const ws_config_t* cfg, int32_t poisson, const int32_t* devices, int32_t ndevices,
                          ws_bvort_t** out) {
    return ws::abi_guarded([&] {
        if (!cfg || !out || !devices) throw AbiError(WS_ERR_INVALID, "null argument");
        if (ndevices < 1) throw AbiError(WS_ERR_INVALID, "need at least one slab");
        ws::bv_check(cfg, ndevices);
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
        for (int i = 0; i < ndevices; ++i)
            if (devices[i] < 0 || devices[i] >= count) throw AbiError(WS_ERR_DEVICE, "no such device");
        if (ndevices == 1) {
            *out = ws::bv_make(cfg, poisson, devices[0], 0, 1);
            return;
        }
        ws_bvort* m = new ws_bvort;
        ws::bv_params(m, cfg);
        m->device = devices[0];
        m->nranks = ndevices;
        try {
            for (int r = 0; r < ndevices; ++r) m->parts.push_back(ws::bv_make(cfg, poisson, devices[r], r, ndevices));
            // the copies read the other slabs' memory (peer access between distinct devices
            // where the devices allow it; the runtime stages the copy otherwise)
            for (int r = 0; r < ndevices; ++r)
                for (int p = 0; p < ndevices; ++p) {
                    const int a = devices[r], c = devices[p];
                    if (a == c) continue;
                    int ok = 0;
                    if (hipDeviceCanAccessPeer(&ok, a, c) != hipSuccess || !ok) {
                        m->copy_kernel = false;  // the runtime's copies (staged) instead
                        continue;
                    }
                    ws::hck(hipSetDevice(a), "hipSetDevice");
                    const hipError_t e = hipDeviceEnablePeerAccess(c, 0);
                    if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
                    else if (e != hipSuccess) {
                        (void)hipGetLastError();
                        m->copy_kernel = false;
                    }
                }
        } catch (...) {
            ws::bv_free(m);
            throw;
        }
        *out = m;
    });
}

int ws_bvort_create_slab(const ws_config_t* cfg, int32_t poisson, int32_t rank, int32_t nranks,
                         const uint8_t id[WS_COMM_ID_BYTES], ws_bvort_t** out, int32_t* row0, int32_t* rows) {
    return ws::abi_guarded([&] {
        if (!cfg || !out || !id) throw AbiError(WS_ERR_INVALID, "null argument");
        if (nranks < 1 || rank < 0 || rank >= nranks) throw AbiError(WS_ERR_INVALID, "bad rank / nranks");
        ws::bv_check(cfg, nranks);
        ws_bvort* b = ws::bv_make(cfg, poisson, cfg->device_id, rank, nranks);
        try {
            // a 1-rank slab gets its communicator too (the RCCL bootstrap runs on one GPU)
            b->comm = new ws::SlabComm(rank, nranks, id);
        } catch (const std::exception& e) {
            ws::bv_free(b);
            throw AbiError(WS_ERR_DEVICE, e.what());
        }
        *out = b;
        if (row0) *row0 = b->row0;
        if (rows) *rows = b->H;
    });
}

int ws_bvort_layout(const ws_bvort_t* b, int32_t* nslabs, int32_t* row0, int32_t* rows) {
    return ws::abi_guarded([&] {
        if (!b) throw AbiError(WS_ERR_INVALID, "null model");
        if (nslabs) *nslabs = b->nranks;
        if (row0) *row0 = b->row0;
        if (rows) *rows = b->H;
    });
}

int ws_bvort_destroy(ws_bvort_t* b) {
    return ws::abi_guarded([&] {
        if (!b) return;
        (void)hipSetDevice(b->device);
        ws::bv_free(b);
    });
}

int ws_bvort_set_vorticity(ws_bvort_t* b, const void* host, int32_t height, int32_t width, int32_t dtype) {
    return ws::abi_guarded([&] {
        if (!b || !host) throw AbiError(WS_ERR_INVALID, "null argument");
        if (height != b->H || width != b->W) throw AbiError(WS_ERR_SHAPE, "vorticity array shape mismatch");
        if (dtype != WS_F32 && dtype != WS_F64) throw AbiError(WS_ERR_INVALID, "bad dtype");
        std::vector<char> buf(b->cells() * b->es());
        if (b->dtype == WS_F64) ws::convert_copy<double>(buf.data(), b->dtype, host, dtype, b->cells());
        else ws::convert_copy<float>(buf.data(), b->dtype, host, dtype, b->cells());
        if (b->parts.empty()) ws::copy_rows(b, b->z[b->cur], buf.data(), 0, true);
        for (ws_bvort* p : b->parts) ws::copy_rows(p, p->z[p->cur], buf.data(), p->row0, true);
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
        if (which >= 1) {
            if (b->dtype == WS_F64) ws::diagnose<double>(b, which);
            else ws::diagnose<float>(b, which);
        }
        auto src = [&](ws_bvort* p) -> void* {
            return which == 0 ? p->z[p->cur] : which == 1 ? p->psi : which == 2 ? p->u : p->v;
        };
        if (b->parts.empty()) ws::copy_rows(b, src(b), host, 0, false);
        for (ws_bvort* p : b->parts) ws::copy_rows(p, src(p), host, p->row0, false);
    });
}

int ws_bvort_run(ws_bvort_t* b, int32_t n) {
    return ws::abi_guarded([&] {
        if (!b) throw AbiError(WS_ERR_INVALID, "null model");
        if (n <= 0) return;
        ws::abi_set_device(b->device);
        b->launches = 0;
        for (ws_bvort* p : b->parts) p->launches = 0;
        const auto t0 = std::chrono::steady_clock::now();  // a one-process decomposition: host time
        if (b->parts.empty()) ws::hck(hipEventRecord(b->ev0, b->stream), "hipEventRecord");
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
        if (b->parts.empty()) {
            ws::hck(hipEventRecord(b->ev1, b->stream), "hipEventRecord");
            ws::hck(hipEventSynchronize(b->ev1), "hipEventSynchronize");
            float ms = 0.f;
            ws::hck(hipEventElapsedTime(&ms, b->ev0, b->ev1), "hipEventElapsedTime");
            b->last_ms = ms;
            return;
        }
        for (ws_bvort* p : b->parts) {
            ws::hck(hipSetDevice(p->device), "hipSetDevice");
            ws::hck(hipStreamSynchronize(p->stream), "hipStreamSynchronize");
            b->launches += p->launches;
        }
        b->last_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
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
