// Bandwidth probe (measurement tool, not product): what HBM rate does a 3-field
// read + 3-field write stream reach on this MI355X for the access shapes the fused
// stencil uses? Prints GB/s per variant (bytes = 6 words per cell).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                    \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

constexpr int W = 4096, H = 4096;

// grid-stride elementwise, VEC elements per lane, nt or plain stores
template <int VEC, bool NT>
__global__ void copy3(const double* __restrict__ a, const double* __restrict__ b, const double* __restrict__ c,
                      double* __restrict__ x, double* __restrict__ y, double* __restrict__ z, long n) {
    long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * VEC;
    const long stride = (long)gridDim.x * blockDim.x * VEC;
    for (; i < n; i += stride) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const double va = a[i + k], vb = b[i + k], vc = c[i + k];
            if (NT) {
                __builtin_nontemporal_store(va + 1.0, x + i + k);
                __builtin_nontemporal_store(vb + 1.0, y + i + k);
                __builtin_nontemporal_store(vc + 1.0, z + i + k);
            } else {
                x[i + k] = va + 1.0;
                y[i + k] = vb + 1.0;
                z[i + k] = vc + 1.0;
            }
        }
    }
}

// row-march: one wave per 64-column strip, marching a segment of rows (the fused pattern)
template <bool NT>
__global__ void march3(const double* __restrict__ a, const double* __restrict__ b, const double* __restrict__ c,
                       double* __restrict__ x, double* __restrict__ y, double* __restrict__ z, int seg) {
    const int nstrips = W / 64;
    const int strip = blockIdx.x % nstrips, s = blockIdx.x / nstrips;
    const int col = strip * 64 + threadIdx.x;
    for (int r = s * seg; r < (s + 1) * seg && r < H; ++r) {
        const long i = (long)r * W + col;
        const double va = a[i], vb = b[i], vc = c[i];
        if (NT) {
            __builtin_nontemporal_store(va + 1.0, x + i);
            __builtin_nontemporal_store(vb + 1.0, y + i);
            __builtin_nontemporal_store(vc + 1.0, z + i);
        } else {
            x[i] = va + 1.0;
            y[i] = vb + 1.0;
            z[i] = vc + 1.0;
        }
    }
}

int main() {
    const long n = (long)W * H;
    double* d[6];
    for (auto& p : d) {
        CK(hipMalloc(&p, n * 8));
        CK(hipMemset(p, 0, n * 8));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        CK(hipDeviceSynchronize());
        const int reps = 20;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double gbs = 6.0 * 8 * n / (ms / reps * 1e-3) / 1e9;
        std::printf("%-40s %8.1f GB/s  %.4f ms\n", name, gbs, ms / reps);
    };
    const int blocks = 256 * 8;
    run("copy3 vec1 plain", [&] { copy3<1, false><<<blocks, 256>>>(d[0], d[1], d[2], d[3], d[4], d[5], n); });
    run("copy3 vec1 nt", [&] { copy3<1, true><<<blocks, 256>>>(d[0], d[1], d[2], d[3], d[4], d[5], n); });
    run("copy3 vec2 plain", [&] { copy3<2, false><<<blocks, 256>>>(d[0], d[1], d[2], d[3], d[4], d[5], n); });
    run("copy3 vec2 nt", [&] { copy3<2, true><<<blocks, 256>>>(d[0], d[1], d[2], d[3], d[4], d[5], n); });
    for (int seg : {32, 64, 128, 256}) {
        char nm[64];
        const int nb = (W / 64) * ((H + seg - 1) / seg);
        std::snprintf(nm, sizeof nm, "march3 seg%d plain (%d waves)", seg, nb);
        run(nm, [&] { march3<false><<<nb, 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
        std::snprintf(nm, sizeof nm, "march3 seg%d nt", seg);
        run(nm, [&] { march3<true><<<nb, 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
    }
    return 0;
}
