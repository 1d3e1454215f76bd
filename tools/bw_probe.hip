// Bandwidth probe (measurement tool, not product): what HBM rate does a 3-field read +
// 3-field write stream reach on this MI355X for the access shapes the fused stencil uses?
// Prints GB/s per variant (bytes = 6 words of 8 B per cell, 4096 x 4096 fp64 fields).
//   hipcc -O3 --offload-arch=gfx950 -std=c++20 tools/bw_probe.hip -o tools/bw_probe
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
using D2 = double __attribute__((ext_vector_type(2)));

// one field, grid-stride, 16 B per lane (the guide's float4-copy reference shape)
__global__ void copy1(const D2* __restrict__ a, D2* __restrict__ x, long n2) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (long)gridDim.x * blockDim.x)
        x[i] = a[i];
}

// three fields, grid-stride, VEC doubles per lane (8 or 16 B accesses)
template <int VEC, bool NT>
__global__ void copy3(const double* __restrict__ a, const double* __restrict__ b, const double* __restrict__ c,
                      double* __restrict__ x, double* __restrict__ y, double* __restrict__ z, long n) {
    long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * VEC;
    const long stride = (long)gridDim.x * blockDim.x * VEC;
    using V = std::conditional_t<VEC == 2, D2, double>;
    for (; i < n; i += stride) {
        const V va = *(const V*)(a + i), vb = *(const V*)(b + i), vc = *(const V*)(c + i);
        if (NT) {
            __builtin_nontemporal_store(va, (V*)(x + i));
            __builtin_nontemporal_store(vb, (V*)(y + i));
            __builtin_nontemporal_store(vc, (V*)(z + i));
        } else {
            *(V*)(x + i) = va;
            *(V*)(y + i) = vb;
            *(V*)(z + i) = vc;
        }
    }
}

// row march: one 64-lane wave per strip of 64*VEC columns, PF rows of loads in flight
template <int VEC, bool NT, int PF>
__global__ void march3(const double* __restrict__ a, const double* __restrict__ b, const double* __restrict__ c,
                       double* __restrict__ x, double* __restrict__ y, double* __restrict__ z, int seg) {
    using V = std::conditional_t<VEC == 2, D2, double>;
    constexpr int cols = 64 * VEC;
    const int nstrips = W / cols;
    const int strip = blockIdx.x % nstrips, s = blockIdx.x / nstrips;
    const int col = strip * cols + threadIdx.x * VEC;
    const int r0 = s * seg, r1 = min(r0 + seg, H);
    V ra[PF], rb[PF], rc[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        const long i = (long)min(r0 + k, H - 1) * W + col;
        ra[k] = *(const V*)(a + i); rb[k] = *(const V*)(b + i); rc[k] = *(const V*)(c + i);
    }
    for (int r = r0; r < r1; r += PF) {
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const long i = (long)(r + k) * W + col;
            const V va = ra[k], vb = rb[k], vc = rc[k];
            const long j = (long)min(r + k + PF, H - 1) * W + col;
            ra[k] = *(const V*)(a + j); rb[k] = *(const V*)(b + j); rc[k] = *(const V*)(c + j);
            if (r + k < r1) {
                if (NT) {
                    __builtin_nontemporal_store(va, (V*)(x + i));
                    __builtin_nontemporal_store(vb, (V*)(y + i));
                    __builtin_nontemporal_store(vc, (V*)(z + i));
                } else {
                    *(V*)(x + i) = va; *(V*)(y + i) = vb; *(V*)(z + i) = vc;
                }
            }
        }
    }
}

// the fused kernels' shape: strips of 64*VEC columns overlapping by 2*M, each storing
// only its middle 64*VEC - 2*M columns (unaligned to cache lines unless M == 0)
template <int VEC, bool NT, int M>
__global__ void strip3(const double* __restrict__ a, const double* __restrict__ b, const double* __restrict__ c,
                       double* __restrict__ x, double* __restrict__ y, double* __restrict__ z, int seg) {
    using V = std::conditional_t<VEC == 2, D2, double>;
    constexpr int cols = 64 * VEC, outw = cols - 2 * M;
    const int nstrips = (W + outw - 1) / outw;
    const int strip = blockIdx.x % nstrips, s = blockIdx.x / nstrips;
    const int col = strip * outw - M + threadIdx.x * VEC;
    const int cl = min(max(col, 0), W - VEC);
    const bool out = threadIdx.x * VEC >= M && threadIdx.x * VEC < cols - M && col >= 0 && col + VEC <= W;
    const int r0 = s * seg, r1 = min(r0 + seg, H);
    V ra[2], rb[2], rc[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const long i = (long)min(r0 + k, H - 1) * W + cl;
        ra[k] = *(const V*)(a + i); rb[k] = *(const V*)(b + i); rc[k] = *(const V*)(c + i);
    }
    for (int r = r0; r < r1; r += 2) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const long i = (long)(r + k) * W + cl;
            const V va = ra[k], vb = rb[k], vc = rc[k];
            const long j = (long)min(r + k + 2, H - 1) * W + cl;
            ra[k] = *(const V*)(a + j); rb[k] = *(const V*)(b + j); rc[k] = *(const V*)(c + j);
            if (out && r + k < r1) {
                if (NT) {
                    __builtin_nontemporal_store(va, (V*)(x + i));
                    __builtin_nontemporal_store(vb, (V*)(y + i));
                    __builtin_nontemporal_store(vc, (V*)(z + i));
                } else {
                    *(V*)(x + i) = va; *(V*)(y + i) = vb; *(V*)(z + i) = vc;
                }
            }
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
    auto run = [&](const char* name, double bytes, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        CK(hipDeviceSynchronize());
        const int reps = 20;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("%-46s %8.1f GB/s  %.4f ms\n", name, bytes / (ms / reps * 1e-3) / 1e9, ms / reps);
    };
    const double b6 = 6.0 * 8 * n;
    run("copy1 16B/lane (1 field in, 1 out)", 2.0 * 8 * n,
        [&] { copy1<<<256 * 16, 256>>>((const D2*)d[0], (D2*)d[3], n / 2); });
    run("copy3 8B/lane plain", b6, [&] { copy3<1, false><<<256 * 8, 256>>>(d[0], d[1], d[2], d[3], d[4], d[5], n); });
    run("copy3 8B/lane nt", b6, [&] { copy3<1, true><<<256 * 8, 256>>>(d[0], d[1], d[2], d[3], d[4], d[5], n); });
    run("copy3 16B/lane plain", b6, [&] { copy3<2, false><<<256 * 8, 256>>>(d[0], d[1], d[2], d[3], d[4], d[5], n); });
    run("copy3 16B/lane nt", b6, [&] { copy3<2, true><<<256 * 8, 256>>>(d[0], d[1], d[2], d[3], d[4], d[5], n); });
    for (int seg : {32, 64, 128}) {
        char nm[96];
        int nb = (W / 64) * ((H + seg - 1) / seg);
        std::snprintf(nm, sizeof nm, "march3 8B pf2 seg%d plain (%d waves)", seg, nb);
        run(nm, b6, [&] { march3<1, false, 2><<<nb, 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
        std::snprintf(nm, sizeof nm, "march3 8B pf2 seg%d nt", seg);
        run(nm, b6, [&] { march3<1, true, 2><<<nb, 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
        std::snprintf(nm, sizeof nm, "march3 8B pf4 seg%d nt", seg);
        run(nm, b6, [&] { march3<1, true, 4><<<nb, 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
        nb = (W / 128) * ((H + seg - 1) / seg);
        std::snprintf(nm, sizeof nm, "march3 16B pf2 seg%d plain (%d waves)", seg, nb);
        run(nm, b6, [&] { march3<2, false, 2><<<nb, 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
        std::snprintf(nm, sizeof nm, "march3 16B pf2 seg%d nt", seg);
        run(nm, b6, [&] { march3<2, true, 2><<<nb, 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
        std::snprintf(nm, sizeof nm, "march3 16B pf4 seg%d nt", seg);
        run(nm, b6, [&] { march3<2, true, 4><<<nb, 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
    }
    for (int seg : {64}) {
        char nm[96];
        auto strips = [&](int outw) { return ((W + outw - 1) / outw) * ((H + seg - 1) / seg); };
        std::snprintf(nm, sizeof nm, "strip3 16B M0 seg%d nt", seg);
        run(nm, b6, [&] { strip3<2, true, 0><<<strips(128), 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
        std::snprintf(nm, sizeof nm, "strip3 16B M2 seg%d nt", seg);
        run(nm, b6, [&] { strip3<2, true, 2><<<strips(124), 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
        std::snprintf(nm, sizeof nm, "strip3 16B M2 seg%d plain", seg);
        run(nm, b6, [&] { strip3<2, false, 2><<<strips(124), 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
        std::snprintf(nm, sizeof nm, "strip3 16B M4 seg%d nt", seg);
        run(nm, b6, [&] { strip3<2, true, 4><<<strips(120), 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
        std::snprintf(nm, sizeof nm, "strip3 16B M4 seg%d plain", seg);
        run(nm, b6, [&] { strip3<2, false, 4><<<strips(120), 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
        std::snprintf(nm, sizeof nm, "strip3 16B M8 seg%d nt", seg);
        run(nm, b6, [&] { strip3<2, true, 8><<<strips(112), 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
        std::snprintf(nm, sizeof nm, "strip3 8B M4 seg%d nt", seg);
        run(nm, b6, [&] { strip3<1, true, 4><<<strips(56), 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
        std::snprintf(nm, sizeof nm, "strip3 8B M4 seg%d plain", seg);
        run(nm, b6, [&] { strip3<1, false, 4><<<strips(56), 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
        std::snprintf(nm, sizeof nm, "strip3 8B M8 seg%d nt", seg);
        run(nm, b6, [&] { strip3<1, true, 8><<<strips(48), 64>>>(d[0], d[1], d[2], d[3], d[4], d[5], seg); });
    }
    return 0;
}
