"""NumPy oracle of the physics-mode barotropic vorticity model -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/ and bench.py's cpu_baseline leg, as the checker; the product
(nvidia-jetson-workload_amd/weather_sim/physics.py over libws_hip.so) never imports it.

Why an oracle of our own: SURVEY §8(f)2 / BASELINE config C3 describe a barotropic
"Jacobian + Laplacian" model, but the reference has none -- its Barotropic model runs the
shallow-water tendencies (src/weather-sim/cpp/src/weather_simulation.cpp:542-560). So this
model has NO reference semantics and its parity is "unpinned" against the reference; it is
pinned instead against analytic properties of the discrete system (tests/test_bvort_oracle.py):
  * a single Fourier mode is an exact solution of the semi-discrete equations (the Arakawa
    Jacobian of a mode with itself vanishes): a Rossby wave with the discrete dispersion
    relation, decaying at the discrete Laplacian's rate;
  * with beta = nu = 0 the Arakawa Jacobian conserves discrete energy and enstrophy;
  * the spectral Poisson solve inverts the 5-point Laplacian to round-off.
The config fields `beta` and `viscosity` (weather_sim.hpp:176-178, accepted but never read
by the reference) are the model's parameters.

Model (doubly periodic W x H grid, spacing dx, dy; x = column, y = row):
    d(zeta)/dt = -J(psi, zeta) - beta * d(psi)/dx + nu * lap(zeta),     lap(psi) = zeta
  J      Arakawa (1966) 9-point Jacobian, (J++ + J+x + Jx+) / 3, each over 4 dx dy
  d/dx   (psi[x+1] - psi[x-1]) / (2 dx)
  lap    5-point: (a[x+1] + a[x-1] - 2a) / dx^2 + (a[y+1] + a[y-1] - 2a) / dy^2
  psi    spectral inverse of the 5-point Laplacian: psi_hat = zeta_hat / lambda(k, l),
         lambda = (2 cos(2 pi k / W) - 2) / dx^2 + (2 cos(2 pi l / H) - 2) / dy^2, psi_hat(0,0) = 0
Integrators: forward Euler, RK2 midpoint, classical RK4 (a new model: none of the
reference's RK4 aliasing, SURVEY §0.3, applies). Velocities u = -d(psi)/dy, v = d(psi)/dx.
"""
import numpy as np

EULER, RK2, RK4 = 0, 1, 2


def _r(a, dy, dx):
    """a[y + dy, x + dx] with periodic wrap."""
    return np.roll(a, (-dy, -dx), axis=(0, 1))


def arakawa_jacobian(psi, zeta, dx, dy):
    p, z = psi, zeta
    pe, pw, pn, ps = _r(p, 0, 1), _r(p, 0, -1), _r(p, 1, 0), _r(p, -1, 0)
    ze, zw, zn, zs = _r(z, 0, 1), _r(z, 0, -1), _r(z, 1, 0), _r(z, -1, 0)
    pne, pnw, pse, psw = _r(p, 1, 1), _r(p, 1, -1), _r(p, -1, 1), _r(p, -1, -1)
    zne, znw, zse, zsw = _r(z, 1, 1), _r(z, 1, -1), _r(z, -1, 1), _r(z, -1, -1)
    jpp = (pe - pw) * (zn - zs) - (pn - ps) * (ze - zw)
    jpx = pe * (zne - zse) - pw * (znw - zsw) - pn * (zne - znw) + ps * (zse - zsw)
    jxp = zn * (pne - pnw) - zs * (pse - psw) - ze * (pne - pse) + zw * (pnw - psw)
    return (jpp + jpx + jxp) / (12.0 * dx * dy)


def laplacian(a, dx, dy):
    return (_r(a, 0, 1) + _r(a, 0, -1) - 2 * a) / (dx * dx) + (_r(a, 1, 0) + _r(a, -1, 0) - 2 * a) / (dy * dy)


def laplacian_eigenvalues(W, H, dx, dy):
    k = np.arange(W // 2 + 1)
    l = np.arange(H)
    lam = ((2 * np.cos(2 * np.pi * k / W) - 2) / (dx * dx))[None, :] + \
          ((2 * np.cos(2 * np.pi * l / H) - 2) / (dy * dy))[:, None]
    return lam


def poisson(zeta, dx, dy):
    H, W = zeta.shape
    lam = laplacian_eigenvalues(W, H, dx, dy)
    inv = np.zeros_like(lam)
    nz = lam != 0
    inv[nz] = 1.0 / lam[nz]
    return np.fft.irfft2(np.fft.rfft2(zeta.astype(np.float64)) * inv, s=(H, W))


def tendency(zeta, dx, dy, beta, nu):
    psi = poisson(zeta, dx, dy)
    k = -arakawa_jacobian(psi, zeta, dx, dy)
    if beta:
        k = k - beta * (_r(psi, 0, 1) - _r(psi, 0, -1)) / (2 * dx)
    if nu:
        k = k + nu * laplacian(zeta, dx, dy)
    return k


def step(zeta, dt, dx, dy, beta=0.0, nu=0.0, method=RK4):
    z = zeta.astype(np.float64)
    f = lambda a: tendency(a, dx, dy, beta, nu)
    if method == EULER:
        return z + dt * f(z)
    if method == RK2:
        return z + dt * f(z + 0.5 * dt * f(z))
    k1 = f(z)
    k2 = f(z + 0.5 * dt * k1)
    k3 = f(z + 0.5 * dt * k2)
    k4 = f(z + dt * k3)
    return z + dt / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)


def run(zeta, steps, dt, dx, dy, beta=0.0, nu=0.0, method=RK4):
    z = zeta.astype(np.float64)
    for _ in range(steps):
        z = step(z, dt, dx, dy, beta, nu, method)
    return z


def velocity(zeta, dx, dy):
    psi = poisson(zeta, dx, dy)
    u = -(_r(psi, 1, 0) - _r(psi, -1, 0)) / (2 * dy)
    v = (_r(psi, 0, 1) - _r(psi, 0, -1)) / (2 * dx)
    return u, v


def energy(zeta, dx, dy):
    """Discrete kinetic energy -1/2 sum(psi * zeta) (conserved by the Arakawa Jacobian)."""
    return -0.5 * float(np.sum(poisson(zeta, dx, dy) * zeta))


def enstrophy(zeta):
    return 0.5 * float(np.sum(zeta.astype(np.float64) ** 2))


def rossby_mode(W, H, dx, dy, kx, ky, amp=1.0, phase=0.0):
    """zeta = amp cos(2 pi (kx x / W + ky y / H) + phase) on cell indices."""
    y, x = np.mgrid[0:H, 0:W]
    return amp * np.cos(2 * np.pi * (kx * x / W + ky * y / H) + phase)


def rossby_exact(W, H, dx, dy, kx, ky, t, beta, nu, amp=1.0):
    """Exact solution of the semi-discrete system for one mode: frequency from the discrete
    d/dx and Laplacian, decay from the discrete Laplacian."""
    lam = (2 * np.cos(2 * np.pi * kx / W) - 2) / dx ** 2 + (2 * np.cos(2 * np.pi * ky / H) - 2) / dy ** 2
    sx = np.sin(2 * np.pi * kx / W) / dx
    # d zeta_hat/dt = (-i beta sx / lam + nu lam) zeta_hat for zeta = Re(zeta_hat e^{i theta}):
    # zeta = amp e^{nu lam t} cos(theta - omega t), omega = beta sx / lam
    omega = beta * sx / lam
    return np.exp(nu * lam * t) * rossby_mode(W, H, dx, dy, kx, ky, amp, phase=-omega * t)
