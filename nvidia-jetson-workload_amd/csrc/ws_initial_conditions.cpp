// Initial conditions, computed on the host in the simulation precision and uploaded once.
//
// Reference: src/weather-sim/cpp/src/initial_conditions.cpp:48-608 (scalar_t = float, or
// double for the fp64 build). Expression types are kept exactly as the reference writes
// them -- e.g. `u_max * std::sin(M_PI * y_norm)` is evaluated in double and then narrowed,
// `std::exp(1.0f - r_norm * r_norm)` in scalar_t, `std::pow(y_norm - 0.5f, 2)` in double --
// so the fields are bit-identical to the reference on the same libm (pinned by
// tests/golden/ref_small_*.npz "ic/*" cases). Parameters round-trip through
// std::to_string / std::stof like ParameterizedInitialCondition::setParameter/getParameter
// (include/weather_sim/initial_conditions.hpp:75-119).
#include "ws_ic.h"

#include <algorithm>
#include <cmath>
#include <random>
#include <string>

namespace ws {
namespace {

// The reference build (g++ -O3) fuses a sin and a cos of the same argument into one libm
// sincos / sincosf call (its .so imports sincos@GLIBC, no cos); glibc's sincos can differ
// from cos by 1 ulp, so the fused call is reproduced explicitly.
inline void ref_sincos(double x, double* s, double* c) { ::sincos(x, s, c); }
inline void ref_sincos(float x, float* s, float* c) { ::sincosf(x, s, c); }

// setParameter(name, scalar_t value) -> std::to_string; getParameter<float> -> std::stof
template <typename T>
float param_roundtrip(double v) {
    return std::stof(std::to_string(static_cast<T>(v)));
}

template <typename T>
struct P {
    const double* p;
    int n;
    float get(int i, float dflt) const { return i < n ? param_roundtrip<T>(p[i]) : dflt; }
};

template <typename T>
void uniform(IcFields<T>& f, const P<T>& a) {
    const T u = a.get(0, 0.0f), v = a.get(1, 0.0f), h = a.get(2, 10.0f), p = a.get(3, 1000.0f),
            t = a.get(4, 300.0f), q = a.get(5, 0.0f);
    for (size_t i = 0; i < f.n(); ++i) {
        f.u[i] = u; f.v[i] = v; f.h[i] = h; f.p[i] = p; f.t[i] = t; f.q[i] = q;
    }
    f.wrote = kU | kV | kH | kP | kT | kQ;
}

template <typename T>
void random_ic(IcFields<T>& f, const P<T>& a) {
    // setParameter("seed", static_cast<int>(seed)) -> std::stoi
    const int seed = a.n > 0 ? static_cast<int>(static_cast<unsigned int>(a.p[0])) : 0;
    const T amplitude = a.get(1, 1.0f);
    std::mt19937 rng(seed);
    std::uniform_real_distribution<T> dist(-amplitude, amplitude);
    for (int y = 0; y < f.y1(); ++y)  // the whole sequence up to the last owned row
        for (int x = 0; x < f.W; ++x) {
            const T u = dist(rng);
            const T v = dist(rng);
            const T h = 10.0f + dist(rng);
            if (y < f.y0) continue;
            const size_t i = f.idx(x, y);
            f.u[i] = u; f.v[i] = v; f.h[i] = h;
        }
    f.wrote = kU | kV | kH;
}

template <typename T>
void zonal_flow(IcFields<T>& f, const P<T>& a) {
    const T u_max = a.get(0, 10.0f), h_mean = a.get(1, 10.0f), beta = a.get(2, 0.1f);
    for (int y = f.y0; y < f.y1(); ++y) {
        const T y_norm = static_cast<T>(y) / (f.H - 1);
        const T u = u_max * std::sin(M_PI * y_norm);
        const T h_base = h_mean;
        for (int x = 0; x < f.W; ++x) {
            const size_t i = f.idx(x, y);
            f.u[i] = u; f.v[i] = 0.0f;
            const T fc = 1.0e-4f + beta * (y_norm - 0.5f);
            const T h = h_base - 0.5f * fc * u * u / 9.81f;
            f.h[i] = h;
        }
    }
    f.wrote = kU | kV | kH;
}

template <typename T>
void vortex(IcFields<T>& f, const P<T>& a) {
    const T x_center = a.get(0, 0.5f), y_center = a.get(1, 0.5f), radius = a.get(2, 0.1f),
            strength = a.get(3, 10.0f), h_mean = a.get(4, 10.0f);
    const T x_center_grid = x_center * (f.W - 1);
    const T y_center_grid = y_center * (f.H - 1);
    const T radius_grid = radius * std::min(f.W, f.H);
    for (int y = f.y0; y < f.y1(); ++y)
        for (int x = 0; x < f.W; ++x) {
            const T dx = x - x_center_grid;
            const T dy = y - y_center_grid;
            const T r = std::sqrt(dx * dx + dy * dy);
            T angular_velocity = 0.0f;
            T h = h_mean;
            if (r > 0.0f && r <= radius_grid) {
                const T r_norm = r / radius_grid;
                angular_velocity = strength * r_norm * std::exp(1.0f - r_norm * r_norm);
                h = h_mean - 0.5f * angular_velocity * angular_velocity / 9.81f;
            }
            const T u = -angular_velocity * dy / std::max<T>(r, 1.0e-6f);
            const T v = angular_velocity * dx / std::max<T>(r, 1.0e-6f);
            const size_t i = f.idx(x, y);
            f.u[i] = u; f.v[i] = v; f.h[i] = h;
        }
    f.wrote = kU | kV | kH;
}

template <typename T>
void jet_stream(IcFields<T>& f, const P<T>& a) {
    const T y_center = a.get(0, 0.5f), width_param = a.get(1, 0.1f), strength = a.get(2, 10.0f),
            h_mean = a.get(3, 10.0f);
    const T y_center_grid = y_center * (f.H - 1);
    const T width_grid = width_param * f.H;
    for (int y = f.y0; y < f.y1(); ++y) {
        const T dy = y - y_center_grid;
        const T u = strength * std::exp(-(dy * dy) / (2.0f * width_grid * width_grid));
        const T dh_dy = -1.0e-4f * u / 9.81f;
        for (int x = 0; x < f.W; ++x) {
            const size_t i = f.idx(x, y);
            f.u[i] = u; f.v[i] = 0.0f;
            const T h = h_mean + dh_dy * dy;
            f.h[i] = h;
        }
    }
    f.wrote = kU | kV | kH;
}

template <typename T>
void breaking_wave(IcFields<T>& f, const P<T>& a) {
    const T amplitude = a.get(0, 1.0f), wavelength = a.get(1, 0.2f), h_mean = a.get(2, 10.0f);
    const T wave_k = 2.0f * M_PI / (wavelength * f.W);
    for (int y = f.y0; y < f.y1(); ++y) {
        const T y_norm = static_cast<T>(y) / (f.H - 1);
        const T u_base = 5.0f * std::sin(M_PI * y_norm);
        for (int x = 0; x < f.W; ++x) {
            const T wave_phase = wave_k * x - 0.1f * y_norm;
            const T wave_amp = amplitude * std::exp(-std::pow(y_norm - 0.5f, 2) / 0.05f);
            T sn, cs;
            ref_sincos(wave_phase, &sn, &cs);
            const T u = u_base + wave_amp * sn;
            const T v = wave_amp * cs;
            const T h = h_mean + wave_amp * cs;
            const size_t i = f.idx(x, y);
            f.u[i] = u; f.v[i] = v; f.h[i] = h;
        }
    }
    f.wrote = kU | kV | kH;
}

template <typename T>
void front(IcFields<T>& f, const P<T>& a) {
    const T y_position = a.get(0, 0.5f), width = a.get(1, 0.05f), temp_difference = a.get(2, 10.0f),
            wind_shear = a.get(3, 5.0f);
    const T y_pos_grid = y_position * (f.H - 1);
    const T width_grid = width * f.H;
    for (int y = f.y0; y < f.y1(); ++y) {
        const T dy = y - y_pos_grid;
        const T t_transition = std::tanh(dy / width_grid);
        const T temperature_val = 288.15f + 0.5f * temp_difference * t_transition;
        const T u = 0.5f * wind_shear * t_transition;
        for (int x = 0; x < f.W; ++x) {
            const size_t i = f.idx(x, y);
            f.u[i] = u; f.v[i] = 0.0f;
            f.t[i] = temperature_val;
            const T p = 1013.25f - 0.1f * temp_difference * t_transition;
            f.p[i] = p;
        }
    }
    f.wrote = kU | kV | kT | kP;
}

template <typename T>
void mountain(IcFields<T>& f, const P<T>& a) {
    const T x_center = a.get(0, 0.3f), y_center = a.get(1, 0.5f), radius = a.get(2, 0.1f),
            mountain_height = a.get(3, 1.0f), u_base = a.get(4, 5.0f);
    const T x_center_grid = x_center * (f.W - 1);
    const T y_center_grid = y_center * (f.H - 1);
    const T radius_grid = radius * std::min(f.W, f.H);
    for (int y = f.y0; y < f.y1(); ++y)
        for (int x = 0; x < f.W; ++x) {
            const T dx = x - x_center_grid;
            const T dy = y - y_center_grid;
            const T r = std::sqrt(dx * dx + dy * dy);
            T mountain_profile = 0.0f;
            if (r <= 2.0f * radius_grid) mountain_profile = mountain_height * std::exp(-(r * r) / (radius_grid * radius_grid));
            const T h = 10.0f + mountain_profile;
            T u = u_base;
            T v = 0.0f;
            if (r <= 3.0f * radius_grid) {
                const T flow_reduction = 0.7f * mountain_profile / mountain_height;
                u *= (1.0f - flow_reduction);
                if (r > 0.0f) v = -0.5f * flow_reduction * u_base * dy / r;
            }
            const size_t i = f.idx(x, y);
            f.u[i] = u; f.v[i] = v; f.h[i] = h;
        }
    f.wrote = kU | kV | kH;
}

// initial_conditions.cpp:537-608
template <typename T>
struct Profile {
    T p[10], t[10], q[10], u[10], v[10];
};

template <typename T>
Profile<T> load_profile(const std::string& name) {
    static const float S[5][10] = {
        {1013.0f, 1011.0f, 1009.0f, 1005.0f, 1000.0f, 995.0f, 990.0f, 985.0f, 980.0f, 975.0f},
        {298.0f, 295.0f, 292.0f, 288.0f, 285.0f, 282.0f, 278.0f, 275.0f, 272.0f, 268.0f},
        {0.8f, 0.75f, 0.7f, 0.65f, 0.6f, 0.55f, 0.5f, 0.45f, 0.4f, 0.35f},
        {2.0f, 4.0f, 6.0f, 8.0f, 10.0f, 12.0f, 10.0f, 8.0f, 6.0f, 4.0f},
        {0.0f, 1.0f, 2.0f, 1.0f, 0.0f, -1.0f, -2.0f, -1.0f, 0.0f, 1.0f}};
    static const float Tr[5][10] = {
        {1010.0f, 1009.0f, 1008.0f, 1007.0f, 1006.0f, 1005.0f, 1004.0f, 1003.0f, 1002.0f, 1001.0f},
        {303.0f, 302.0f, 301.0f, 300.0f, 299.0f, 298.0f, 297.0f, 296.0f, 295.0f, 294.0f},
        {0.9f, 0.89f, 0.88f, 0.87f, 0.86f, 0.85f, 0.84f, 0.83f, 0.82f, 0.81f},
        {-5.0f, -6.0f, -7.0f, -8.0f, -7.0f, -6.0f, -5.0f, -4.0f, -3.0f, -2.0f},
        {-1.0f, -0.5f, 0.0f, 0.5f, 1.0f, 1.0f, 0.5f, 0.0f, -0.5f, -1.0f}};
    static const float Po[5][10] = {
        {1020.0f, 1018.0f, 1016.0f, 1014.0f, 1012.0f, 1010.0f, 1008.0f, 1006.0f, 1004.0f, 1002.0f},
        {260.0f, 258.0f, 256.0f, 254.0f, 252.0f, 250.0f, 248.0f, 246.0f, 244.0f, 242.0f},
        {0.3f, 0.29f, 0.28f, 0.27f, 0.26f, 0.25f, 0.24f, 0.23f, 0.22f, 0.21f},
        {10.0f, 12.0f, 14.0f, 16.0f, 18.0f, 20.0f, 18.0f, 16.0f, 14.0f, 12.0f},
        {0.0f, -1.0f, -2.0f, -3.0f, -4.0f, -3.0f, -2.0f, -1.0f, 0.0f, 1.0f}};
    const float(*src)[10] = name == "tropical" ? Tr : name == "polar" ? Po : S;  // unknown -> standard
    Profile<T> pr;
    for (int i = 0; i < 10; ++i) {
        pr.p[i] = src[0][i]; pr.t[i] = src[1][i]; pr.q[i] = src[2][i]; pr.u[i] = src[3][i]; pr.v[i] = src[4][i];
    }
    return pr;
}

template <typename T>
void atmospheric_profile(IcFields<T>& f, const std::string& profile_name) {
    const Profile<T> pr = load_profile<T>(profile_name);
    const size_t size = 10;
    for (int y = f.y0; y < f.y1(); ++y) {
        const T y_norm = static_cast<T>(y) / (f.H - 1);
        size_t idx = static_cast<size_t>(y_norm * (size - 1));
        idx = std::min(idx, size - 1);
        const T t_base = pr.t[idx], p_base = pr.p[idx], q_base = pr.q[idx], u_base = pr.u[idx], v_base = pr.v[idx];
        for (int x = 0; x < f.W; ++x) {
            const T x_norm = static_cast<T>(x) / (f.W - 1);
            double sn, cs;
            ref_sincos(2.0f * M_PI * x_norm, &sn, &cs);
            const T t_var = 2.0f * sn;
            const T p_var = 2.0f * cs;
            const T q_var = 0.02f * std::sin(4.0f * M_PI * x_norm);
            const size_t i = f.idx(x, y);
            f.t[i] = t_base + t_var;
            f.p[i] = p_base + p_var;
            f.q[i] = q_base + q_var;
            f.u[i] = u_base; f.v[i] = v_base;
        }
    }
    f.wrote = kU | kV | kT | kP | kQ;
}

}  // namespace

template <typename T>
bool compute_initial_condition(const std::string& name, const double* params, int nparams, const std::string& sparam,
                               IcFields<T>& f) {
    const P<T> a{params, params ? nparams : 0};
    if (name == "uniform") uniform(f, a);
    else if (name == "random") random_ic(f, a);
    else if (name == "zonal_flow") zonal_flow(f, a);
    else if (name == "vortex") vortex(f, a);
    else if (name == "jet_stream") jet_stream(f, a);
    else if (name == "breaking_wave") breaking_wave(f, a);
    else if (name == "front") front(f, a);
    else if (name == "mountain") mountain(f, a);
    else if (name == "atmospheric_profile") atmospheric_profile(f, sparam.empty() ? std::string("standard") : sparam);
    // factory aliases (initial_conditions.cpp:654-665)
    else if (name == "standard_atmosphere") atmospheric_profile(f, "standard");
    else if (name == "tropical_atmosphere") atmospheric_profile(f, "tropical");
    else if (name == "polar_atmosphere") atmospheric_profile(f, "polar");
    else return false;
    return true;
}

template bool compute_initial_condition<float>(const std::string&, const double*, int, const std::string&,
                                               IcFields<float>&);
template bool compute_initial_condition<double>(const std::string&, const double*, int, const std::string&,
                                                IcFields<double>&);

}  // namespace ws
