// Bandwidth probe 2 (measurement tool, not product): does the ADDRESS PATTERN of the fused
// stencil's stream (every wave marching down its own 512 B / 1 KB wide column strip of
// row-major fields: each row access touches one 32 KB-strided chunk) cost HBM efficiency
// against (a) the same bytes with each wave's strip stored contiguously (a strip-major
// "tiled" layout) and (b) workgroups of adjacent strips marching in lockstep (wide
// contiguous row spans)? 3 fields in, 3 out, 4096 x 4096 fp64, 16 B per lane, nt stores.
//   hipcc -O3 --offload-arch=gfx950 -std=c++20 tools/bw_probe2.hip -o tools/bw_probe2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                    \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

constexpr int W = 4096, H = 4096;
using D2 = double __attribute__((ext_vector_type(2)));

__global__ void copy3(const D2* __restrict__ a, const D2* __restrict__ b, const D2* __restrict__ c, D2* __restrict__ x,
                      D2* __restrict__ y, D2* __restrict__ z, long n2) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (long)gridDim.x * blockDim.x) {
        const D2 va = a[i], vb = b[i], vc = c[i];
        __builtin_nontemporal_store(va, x + i);
        __builtin_nontemporal_store(vb, y + i);
        __builtin_nontemporal_store(vc, z + i);
    }
}

// one wave per (strip of 128 columns, segment of seg rows). TILED: element (row, col) of
// strip s at s * H * 128 + row * 128 + (col - 128 s) (each strip contiguous); else row-major.
// WPB waves per workgroup on adjacent strips; SYNC: a workgroup barrier every row (lockstep).
template <bool TILED, int WPB, bool SYNC, int PF>
__global__ __launch_bounds__(64 * WPB) void march(const D2* __restrict__ a, const D2* __restrict__ b,
                                                  const D2* __restrict__ c, D2* __restrict__ x, D2* __restrict__ y,
                                                  D2* __restrict__ z, int seg, int xcd) {
    constexpr int nstrips = W / 128;
    int blk = blockIdx.x;
    if (xcd) {  // consecutive work items on one XCD (blocks b, b+8, ...)
        const int nb = gridDim.x, q = nb / 8, rr = nb % 8, k = blk % 8;
        blk = (k < rr ? k * (q + 1) : rr * (q + 1) + (k - rr) * q) + blk / 8;
    }
    const int w = blk * WPB + threadIdx.x / 64;
    const int strip = w % nstrips, s = w / nstrips;
    const int lane = threadIdx.x % 64;
    const int r0 = s * seg, r1 = min(r0 + seg, H);
    auto idx = [&](int r) -> long {
        return TILED ? ((long)strip * H + r) * 64 + lane : (long)r * (W / 2) + strip * 64 + lane;
    };
    D2 ra[PF], rb[PF], rc[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        const long i = idx(min(r0 + k, H - 1));
        ra[k] = a[i]; rb[k] = b[i]; rc[k] = c[i];
    }
    for (int r = r0; r < r1; r += PF) {
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const D2 va = ra[k], vb = rb[k], vc = rc[k];
            const long j = idx(min(r + k + PF, H - 1));
            ra[k] = a[j]; rb[k] = b[j]; rc[k] = c[j];
            if (r + k < r1) {
                const long i = idx(r + k);
                __builtin_nontemporal_store(va, x + i);
                __builtin_nontemporal_store(vb, y + i);
                __builtin_nontemporal_store(vc, z + i);
            }
            if constexpr (SYNC) __syncthreads();
        }
    }
}

int main() {
    const long n = (long)W * H;
    D2* d[6];
    for (auto& p : d) {
        CK(hipMalloc(&p, n * 8));
        CK(hipMemset(p, 0, n * 8));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 5; ++w) launch();
        CK(hipDeviceSynchronize());
        const int reps = 30;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("%-52s %8.1f GB/s  %.4f ms\n", name, 6.0 * 8 * n / (ms / reps * 1e-3) / 1e9, ms / reps);
    };
    run("copy3 16B nt grid-stride", [&] { copy3<<<256 * 8, 256>>>(d[0], d[1], d[2], d[3], d[4], d[5], n / 2); });
    for (int seg : {40, 80, 160, 320}) {
        const int waves = (W / 128) * ((H + seg - 1) / seg);
        char nm[128];
#define GO(T, WPB, S, PF, X)                                                                                     \
    std::snprintf(nm, sizeof nm, "seg%-3d %s wpb%d %s pf%d %s (%d waves)", seg, T ? "tiled" : "rowmj", WPB,      \
                  S ? "sync" : "free", PF, X ? "xcd" : "lin", waves);                                            \
    run(nm, [&] { march<T, WPB, S, PF><<<waves / WPB, 64 * WPB>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg, X); });
        GO(false, 1, false, 2, 1)
        GO(false, 1, false, 4, 1)
        GO(true, 1, false, 2, 1)
        GO(true, 1, false, 4, 1)
        GO(false, 4, true, 2, 0)
        GO(false, 8, true, 2, 0)
        GO(false, 8, true, 4, 0)
        GO(false, 16, true, 2, 0)
        GO(false, 4, false, 2, 0)
#undef GO
    }
    return 0;
}
