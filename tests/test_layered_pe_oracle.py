"""CPU: the physics-mode layered primitive-equation oracle (oracle/layered_pe_oracle.py)
pinned against properties of the discrete system -- the model has no reference semantics
(SURVEY §8(f)2), so these are its pins ("parity unpinned" against the reference itself)."""
import numpy as np
import pytest

from oracle import layered_pe_oracle as lp

G, GP = 9.81, 0.05


def wave_state(L, H, W, thick, amps, kx, dx, with_u):
    """Small-amplitude wave exp(i 2 pi kx x / W) in each layer: h_k += amps[k] cos(theta)."""
    u, v, h = lp.rest_state(L, H, W, thick)
    x = np.arange(W)
    th = 2 * np.pi * kx * x / W
    for k in range(L):
        h[k] += amps[k] * np.cos(th)[None, :]
        if with_u is not None:
            u[k] += with_u[k] * np.cos(th)[None, :]
    return u, v, h


def test_rest_with_level_interfaces_stays_at_rest_exactly():
    s = lp.rest_state(4, 12, 16, [100.0, 200.0, 300.0, 400.0])
    out = lp.run(s, 5, 0.5, 1000.0, 1000.0, G, GP, 1e-4, lp.RK4)
    for a, b in zip(out, s):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("method", [lp.EULER, lp.RK2, lp.RK4])
def test_mass_per_layer_conserved(method):
    rng = np.random.default_rng(0)
    L, H, W = 3, 20, 24
    u, v, h = lp.rest_state(L, H, W, [50.0, 80.0, 120.0])
    u += rng.standard_normal((L, H, W)) * 0.1
    v += rng.standard_normal((L, H, W)) * 0.1
    h += rng.standard_normal((L, H, W))
    m0 = h.sum(axis=(1, 2))
    out = lp.run((u, v, h), 20, 5.0, 1000.0, 1200.0, G, GP, 1e-4, method)
    np.testing.assert_allclose(out[2].sum(axis=(1, 2)), m0, rtol=1e-13)


def test_single_layer_gravity_wave_speed():
    W, H, dx, H0, kx, a = 128, 4, 1000.0, 100.0, 2, 1e-3
    c = np.sqrt(G * H0)
    # right-going wave: u = (c / H0) h'
    s = wave_state(1, H, W, [H0], [a], kx, dx, [c / H0 * a])
    dt, n = 5.0, 200
    out = lp.run(s, n, dt, dx, dx, G, GP, 0.0, lp.RK4)
    k = 2 * np.pi * kx / (W * dx)
    omega = c * np.sin(k * dx) / dx
    want = H0 + a * np.cos(2 * np.pi * kx * np.arange(W) / W - omega * n * dt)
    err = np.abs(out[2][0, 0] - want).max() / a
    assert err < 2e-3  # nonlinear O(a / H0) and RK4 error


def test_two_layer_baroclinic_mode_speed():
    W, H, dx, H0, H1, kx, a = 128, 4, 1000.0, 200.0, 300.0, 1, 1e-2
    A = np.array([[G * H0, G * H0], [G * H1, (G + GP) * H1]])
    lam, vec = np.linalg.eig(A)
    i = int(np.argmin(lam))  # the slow (baroclinic) mode
    c, e = np.sqrt(lam[i]), vec[:, i] / np.abs(vec[:, i]).max()
    amps = a * e
    # a right-going mode: u_k = c / H_k * h'_k (from dh/dt = -H du/dx)
    s = wave_state(2, H, W, [H0, H1], amps, kx, dx, [c / H0 * amps[0], c / H1 * amps[1]])
    dt, n = 20.0, 150
    out = lp.run(s, n, dt, dx, dx, G, GP, 0.0, lp.RK4)
    k = 2 * np.pi * kx / (W * dx)
    omega = c * np.sin(k * dx) / dx
    th = 2 * np.pi * kx * np.arange(W) / W - omega * n * dt
    for lay, H_ in ((0, H0), (1, H1)):
        want = H_ + amps[lay] * np.cos(th)
        assert np.abs(out[2][lay, 0] - want).max() < 0.02 * abs(amps).max()


def test_montgomery_single_layer_is_g_h():
    h = np.random.default_rng(1).uniform(1, 2, (1, 5, 6))
    np.testing.assert_array_equal(lp.montgomery(h, G, GP)[0], G * h[0])
