// x after n steps of x <- fl(x + c), every step rounded to nearest-even as the reference's
// per-step `T_ += dt_ * tendency` rounds it (weather_simulation.cpp:201-214, the PE T / P drift
// of a run; ws_schedule.cpp tp_flush) -- in O(binades crossed) instead of O(n) additions.
//
// Inside one binade [2^(e-1), 2^e) the representable numbers are the multiples of u = ulp, so
// for z a multiple of u and an exact sum z + c <= 2^e - u, fl(z + c) = z + d with the constant
// d = u * round(c / u) -- unless c / u is a tie (fraction exactly 1/2), where round-to-even
// makes the increment alternate with z's parity. So after one real step y = fl(x + c), the
// steps that keep the sum in y's binade are taken at once (integer arithmetic in units of u);
// ties, non-positive values or increments, non-finite values and subnormal ranges take single
// real steps. Bit-identical to the loop (tests/test_repeat_add.py checks it on the host).
// Shared by the device kernel (ws_kernels.hip affine2_kernel) and the host test.
#pragma once

#include <cmath>
#include <cstdint>
#include <type_traits>

#ifndef WS_HD
#if defined(__HIPCC__)
#define WS_HD __host__ __device__
#else
#define WS_HD
#endif
#endif

namespace ws {

template <typename T>
WS_HD inline T repeat_add(T x, T c, int n) {
    constexpr int kDigits = sizeof(T) == 4 ? 24 : 53;                 // significand bits
    // integer arithmetic in units of the ulp: every quantity is below 2^(kDigits + 1), so
    // fp32 runs it in 32-bit integers (single conversions and a 32-bit division on the GPU,
    // where 64-bit ones are long software sequences)
    using I = std::conditional_t<sizeof(T) == 4, int32_t, int64_t>;
    constexpr I kTop = (I)1 << kDigits;                                // 2^e / u
    const T kMinBulk = sizeof(T) == 4 ? T(1e-30) : T(1e-290);          // well inside the normal range
    while (n > 0) {
        const T y = x + c;  // one real step
        --n;
        x = y;
        if (n == 0 || !(y >= kMinBulk) || !(c > T(0)) || !std::isfinite(y)) continue;
        int e = 0;
        (void)std::frexp(y, &e);                        // y in [2^(e-1), 2^e), ulp u = 2^(e - kDigits)
        // scalings by powers of two (exact; no divisions: the device pass runs this per value)
        const T q = std::ldexp(c, kDigits - e);         // c / u
        if (!(q < T(kTop))) continue;                   // c spans the binade: single steps
        const T qf = std::floor(q);
        const T fr = q - qf;
        if (fr == T(0.5)) continue;                     // a tie: the parity decides, single steps
        const I D = (I)qf + (fr > T(0.5) ? 1 : 0);      // increment in units of u
        if (D == 0) return y;                           // c rounds away: y never moves again
        const I Y = (I)std::ldexp(y, kDigits - e);      // y / u: an integer < 2^kDigits
        const I Cc = (I)std::ceil(q);
        // bulk steps j = 0 .. m-1 from z_j = y + j d need z_j + c <= 2^e - u
        const I room = kTop - 1 - Y - Cc;
        if (room < 0) continue;
        const I steps = room / D + 1;
        const I m = steps < (I)n ? steps : (I)n;
        x = std::ldexp(T(Y + m * D), e - kDigits);      // exact: a multiple of u below 2^e
        n -= (int)m;
    }
    return x;
}

}  // namespace ws
