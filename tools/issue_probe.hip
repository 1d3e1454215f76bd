// VALU issue probe (measurement tool, not product): how many SIMD cycles does a wave64 fp64 FMA,
// a 32-bit DPP lane move, and the fused C2 kernel's mix of the two (164 fp64 : 91 32-bit per
// march body) cost on one MI355X SIMD with 1, 2, 3 or 4 resident waves? Independent chains (8
// accumulators per wave), no memory traffic; the grid puts `w` waves on every SIMD (one-wave
// workgroups, 256 CUs x 4 SIMDs x w). Prints cycles per instruction per SIMD at the measured
// clock (s_memtime / s_memrealtime inside the kernel).
//   hipcc -O3 --offload-arch=gfx950 -std=c++20 tools/issue_probe.hip -o tools/issue_probe && tools/issue_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                 \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

constexpr int kIters = 4096;

__device__ __forceinline__ int shr1(int v) { return __builtin_amdgcn_mov_dpp(v, 0x138, 0xF, 0xF, true); }

// MODE 0: fp64 FMAs only; 1: DPP moves only; 2: the fused kernel's mix (per unrolled group:
// 16 fp64 FMAs + 9 DPP moves ~ 164 : 91)
template <int MODE>
__global__ __launch_bounds__(64) void probe(double* out, unsigned long long* clk, double seed) {
    double a[8];
    int b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = seed + threadIdx.x + i;
        b[i] = (int)threadIdx.x + i;
    }
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < kIters; ++it) {
        if constexpr (MODE == 0 || MODE == 2) {
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int i = 0; i < 8; ++i) a[i] = __builtin_fma(a[i], 1.0000001, 0.5);
        }
        if constexpr (MODE == 1) {
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int i = 0; i < 8; ++i) b[i] = shr1(b[i]);
        }
        if constexpr (MODE == 2) {
#pragma unroll
            for (int i = 0; i < 8; ++i) b[i] = shr1(b[i]);
            b[0] = shr1(b[0]);
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i] + b[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = c1 - c0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int MODE>
void run(int waves_per_simd, int cus) {
    const int blocks = cus * 4 * waves_per_simd;
    double* out;
    unsigned long long* clk;
    CK(hipMalloc(&out, (size_t)blocks * 64 * sizeof(double)));
    CK(hipMalloc(&clk, (size_t)blocks * 2 * sizeof(unsigned long long)));
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(64), 0, 0, out, clk, 1.0);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h((size_t)blocks * 2);
    CK(hipMemcpy(h.data(), clk, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    double cyc = 0, real = 0;
    for (int b = 0; b < blocks; ++b) {
        cyc += (double)h[2 * b];
        real += (double)h[2 * b + 1];
    }
    cyc /= blocks;
    real /= blocks;
    const double ghz = cyc / real / 10.0;  // memrealtime: 100 MHz
    // instructions per wave in the loop
    const double f64 = MODE == 1 ? 0 : 16.0 * kIters, dpp = MODE == 0 ? 0 : (MODE == 1 ? 16.0 : 9.0) * kIters;
    const double per_simd = cyc / (waves_per_simd * (f64 + dpp));  // SIMD cycles per instruction
    std::printf("mode %d (%s) waves/SIMD %d: %.2f GHz, %.3f SIMD cycles per instruction (%.0f fp64 + %.0f dpp per wave)\n",
                MODE, MODE == 0 ? "fp64 fma" : MODE == 1 ? "dpp mov " : "mix 16:9", waves_per_simd, ghz, per_simd, f64,
                dpp);
    CK(hipFree(out));
    CK(hipFree(clk));
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int w : {1, 2, 3, 4}) {
        run<0>(w, cus);
        run<1>(w, cus);
        run<2>(w, cus);
    }
    return 0;
}
