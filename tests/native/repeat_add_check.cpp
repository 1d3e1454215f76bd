// Host check of ws::repeat_add (csrc/ws_repeat_add.h) against the plain loop of rounded
// additions, fp32 and fp64: random starts / increments / step counts around the PE T / P drift
// (T ~ 300 + k dt 288.15, P ~ 1013 + k dt 1013.25), binade crossings, ties, tiny and huge
// increments, signs, zero, subnormal, inf / nan. Prints "mismatches N cases M". Built and run by
// tests/test_repeat_add.py (g++ -O2 -ffp-contract=off: IEEE round-to-nearest SSE arithmetic).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <random>

#include "ws_repeat_add.h"

template <typename T>
static T loop(T x, T c, int n) {
    for (int i = 0; i < n; ++i) x = x + c;
    return x;
}

template <typename T>
static bool same(T a, T b) {
    return std::memcmp(&a, &b, sizeof(T)) == 0 || (std::isnan(a) && std::isnan(b));
}

template <typename T>
static long check(std::mt19937_64& g, long cases, long* bad) {
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::uniform_int_distribution<int> N(0, 700);
    long done = 0;
    const T specials[] = {T(0), -T(0), std::numeric_limits<T>::denorm_min(), std::numeric_limits<T>::min(),
                          std::numeric_limits<T>::infinity(), std::numeric_limits<T>::quiet_NaN(), T(1), T(-1)};
    for (long i = 0; i < cases; ++i) {
        T x, c;
        const int kind = i % 8;
        if (kind == 0) {  // the PE drift: T / P starts, dt * constant increments
            x = T(U(g) < 0.5 ? 280.0 + 40 * U(g) : 900.0 + 200 * U(g));
            c = T(std::pow(10.0, -4 + 4 * U(g))) * T(U(g) < 0.5 ? 288.15f : 1013.25f);
        } else if (kind == 1) {  // near a binade top
            const int e = (int)(U(g) * 40) - 20;
            x = std::ldexp(T(1), e) * (T(1) - T(std::pow(2.0, -1 - 10 * U(g))));
            c = std::ldexp(T(1), e - (int)(U(g) * 30)) * T(U(g));
        } else if (kind == 2) {  // ties: c = (k + 1/2) ulp(x)
            int e;
            x = T(1 + U(g)) * std::ldexp(T(1), (int)(U(g) * 20) - 10);
            (void)std::frexp(x, &e);
            const T u = std::ldexp(T(1), e - (sizeof(T) == 4 ? 24 : 53));
            c = u * (T((int)(U(g) * 1000)) + T(0.5));
        } else if (kind == 3) {  // negative values / increments
            x = T((U(g) - 0.5) * 2000);
            c = T((U(g) - 0.5) * 10);
        } else if (kind == 4) {  // specials
            x = specials[(int)(U(g) * 8)];
            c = U(g) < 0.5 ? specials[(int)(U(g) * 8)] : T(U(g));
        } else if (kind == 5) {  // tiny increments
            x = T(1 + 1000 * U(g));
            c = T(std::pow(10.0, -20 * U(g)));
        } else {  // anything
            x = T(std::ldexp(U(g), (int)(U(g) * 60) - 30));
            c = T(std::ldexp(U(g), (int)(U(g) * 60) - 30));
        }
        const int n = kind == 0 ? N(g) : N(g) % 300;
        const T a = ws::repeat_add(x, c, n), b = loop(x, c, n);
        if (!same(a, b)) {
            if (*bad < 5)
                std::printf("MISMATCH %s x=%.17g c=%.17g n=%d bulk=%.17g loop=%.17g\n", sizeof(T) == 4 ? "f32" : "f64",
                            (double)x, (double)c, n, (double)a, (double)b);
            ++*bad;
        }
        ++done;
    }
    return done;
}

int main() {
    std::mt19937_64 g(12345);
    long bad = 0, n = 0;
    n += check<float>(g, 400000, &bad);
    n += check<double>(g, 400000, &bad);
    std::printf("mismatches %ld cases %ld\n", bad, n);
    return bad != 0;
}
