"""NumPy oracle of the physics-mode layered primitive-equation model -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/ and bench.py's cpu_baseline leg, as the checker; the product
(nvidia-jetson-workload_amd/weather_sim/physics.py over libws_hip.so) never imports it.

Why an oracle of our own: SURVEY §8(f)2 / BASELINE config C4 describe a 3-D primitive-
equation model ("3D stencil, vertical columns in LDS"), but the reference has none -- its
PrimitiveEquations model runs the 2-D shallow-water tendencies on every level independently
(src/weather-sim/cpp/src/weather_simulation.cpp:542-560, reproduced bit for bit by
WeatherSimulation). This model's parity is therefore "unpinned" against the reference; it
is pinned to properties of the discrete system (tests/test_layered_pe_oracle.py): exact
mass conservation per layer, rest with level interfaces stays at rest, L = 1 gravity waves
and L = 2 baroclinic waves at their discrete phase speeds.

Model: the hydrostatic primitive equations in isopycnal coordinates -- L stacked layers of
constant density (k = 0 at the top), thickness h_k, velocity (u_k, v_k), flat bottom, doubly
periodic W x H grid. Hydrostatic balance couples the layers through the Montgomery
potential, a vertical scan of every column:
    eta_k = sum_{j >= k} h_j                 (height of layer k's upper interface)
    M_0   = g * eta_0,   M_k = M_{k-1} + g' * eta_k    (g' = reduced gravity of each interface)
and each layer obeys
    du/dt = -u u_x - v u_y - M_x + f v,   dv/dt = -u v_x - v v_y - M_y - f u,
    dh/dt = -(h u)_x - (h v)_y
with centred differences (periodic). Evaluation order (shared with the device kernel so the
fp64 comparison is tight): total = h_0 + h_1 + ... ; eta_k = total - (h_0 + ... + h_{k-1});
every difference is (a[+1] - a[-1]) * (1 / (2 d)).
Integrators: forward Euler, RK2 midpoint, classical RK4.
"""
import numpy as np

EULER, RK2, RK4 = 0, 1, 2


def _r(a, dy, dx):
    """a[..., y + dy, x + dx] with periodic wrap (last two axes)."""
    return np.roll(a, (-dy, -dx), axis=(-2, -1))


def montgomery(h, g, gp):
    """h: (L, H, W) -> M: (L, H, W), in the kernel's evaluation order."""
    total = np.zeros_like(h[0])
    for k in range(h.shape[0]):
        total = total + h[k]
    M = np.empty_like(h)
    prefix = np.zeros_like(h[0])
    for k in range(h.shape[0]):
        eta = total - prefix
        M[k] = g * eta if k == 0 else M[k - 1] + gp * eta
        prefix = prefix + h[k]
    return M


def tendency(u, v, h, dx, dy, g, gp, f):
    ix, iy = 1.0 / (2.0 * dx), 1.0 / (2.0 * dy)
    M = montgomery(h, g, gp)
    ddx = lambda a: (_r(a, 0, 1) - _r(a, 0, -1)) * ix
    ddy = lambda a: (_r(a, 1, 0) - _r(a, -1, 0)) * iy
    u_x, u_y, v_x, v_y = ddx(u), ddy(u), ddx(v), ddy(v)
    du = -u * u_x - v * u_y - ddx(M) + f * v
    dv = -u * v_x - v * v_y - ddy(M) - f * u
    dh = -ddx(h * u) - ddy(h * v)
    return du, dv, dh


def step(state, dt, dx, dy, g, gp, f, method=RK4, dtype=np.float64):
    """One step in `dtype` (float32 reproduces the device's fp32 arithmetic: Python-float
    parameters act as weak scalars, rounded to float32 at each operation as the kernel
    rounds them once)."""
    u, v, h = (a.astype(dtype) for a in state)
    F = lambda a, b, c: tendency(a, b, c, dx, dy, g, gp, f)
    ax = lambda s, c, k: tuple(si + c * ki for si, ki in zip(s, k))
    y = (u, v, h)
    if method == EULER:
        return ax(y, dt, F(*y))
    if method == RK2:
        return ax(y, dt, F(*ax(y, 0.5 * dt, F(*y))))
    k1 = F(*y)
    k2 = F(*ax(y, 0.5 * dt, k1))
    k3 = F(*ax(y, 0.5 * dt, k2))
    k4 = F(*ax(y, dt, k3))
    return tuple(yi + dt / 6.0 * (((a + 2 * b) + 2 * c) + d) for yi, a, b, c, d in zip(y, k1, k2, k3, k4))


def run(state, steps, dt, dx, dy, g, gp, f, method=RK4, dtype=np.float64):
    s = tuple(a.astype(dtype) for a in state)
    for _ in range(steps):
        s = step(s, dt, dx, dy, g, gp, f, method, dtype)
    return s


def rest_state(L, H, W, thickness):
    """u = v = 0, layer thicknesses `thickness[k]` everywhere."""
    h = np.empty((L, H, W))
    for k in range(L):
        h[k] = thickness[k]
    return np.zeros((L, H, W)), np.zeros((L, H, W)), h


def gravity_wave_speed_discrete(c, kx, W, dx):
    """Phase speed of a small-amplitude wave exp(i 2 pi kx x / W) under centred differences:
    omega = c sin(2 pi kx / W) / dx."""
    return c * np.sin(2 * np.pi * kx / W) / dx / (2 * np.pi * kx / (W * dx))
