"""CPU: the physics-mode barotropic oracle (oracle/bvort_oracle.py) pinned against analytic
properties of the discrete system -- the model has no reference semantics,
so these are its pins ("parity unpinned" against the reference itself)."""
import numpy as np
import pytest

from oracle import bvort_oracle as bo


@pytest.mark.parametrize("dx,dy", [(1.0, 1.0), (1.0, 1.5), (2.0, 0.5)])
def test_poisson_inverts_the_5_point_laplacian(dx, dy):
    rng = np.random.default_rng(1)
    z = rng.standard_normal((40, 56))
    z -= z.mean()
    psi = bo.poisson(z, dx, dy)
    assert abs(psi.mean()) < 1e-13
    np.testing.assert_allclose(bo.laplacian(psi, dx, dy), z, atol=1e-12)


def test_arakawa_jacobian_antisymmetric_and_self_zero():
    rng = np.random.default_rng(2)
    a, b = rng.standard_normal((2, 32, 48))
    np.testing.assert_allclose(bo.arakawa_jacobian(a, b, 1.0, 1.0), -bo.arakawa_jacobian(b, a, 1.0, 1.0), atol=1e-12)
    assert np.abs(bo.arakawa_jacobian(a, a, 1.0, 1.0)).max() < 1e-12
    # the domain integrals of J, psi J and zeta J vanish (energy / enstrophy conservation)
    J = bo.arakawa_jacobian(a, b, 1.0, 1.0)
    assert abs(J.sum()) < 1e-10 and abs((a * J).sum()) < 1e-10 and abs((b * J).sum()) < 1e-10


@pytest.mark.parametrize("method,tol", [(bo.EULER, 0.1), (bo.RK2, 3e-3), (bo.RK4, 1e-6)])
@pytest.mark.parametrize("nu", [0.0, 0.1])
def test_rossby_wave_matches_discrete_dispersion(method, tol, nu):
    W, H, dx, dy, beta, dt, n = 64, 48, 1.0, 1.5, 0.5, 0.05, 40
    z0 = bo.rossby_mode(W, H, dx, dy, 3, 2, amp=1e-2)
    z = bo.run(z0, n, dt, dx, dy, beta, nu, method)
    ex = bo.rossby_exact(W, H, dx, dy, 3, 2, n * dt, beta, nu, amp=1e-2)
    assert np.linalg.norm(z - ex) / np.linalg.norm(ex) < tol


def test_rk4_converges_at_fourth_order():
    W, H, beta = 32, 32, 1.0
    z0 = bo.rossby_mode(W, H, 1.0, 1.0, 2, 1)
    errs = []
    for dt, n in ((0.2, 10), (0.1, 20)):
        ex = bo.rossby_exact(W, H, 1.0, 1.0, 2, 1, dt * n, beta, 0.0)
        errs.append(np.linalg.norm(bo.run(z0, n, dt, 1.0, 1.0, beta, 0.0, bo.RK4) - ex))
    assert 12 < errs[0] / errs[1] < 20  # 2^4 = 16


def test_energy_and_enstrophy_conserved_without_forcing():
    rng = np.random.default_rng(3)
    z = rng.standard_normal((48, 64))
    z -= z.mean()
    z = bo.run(z, 0, 0.0, 1.0, 1.0)
    E0, Z0 = bo.energy(z, 1.0, 1.0), bo.enstrophy(z)
    z1 = bo.run(z, 50, 0.005, 1.0, 1.0, 0.0, 0.0, bo.RK4)
    assert abs(bo.energy(z1, 1.0, 1.0) - E0) / E0 < 1e-9
    assert abs(bo.enstrophy(z1) - Z0) / Z0 < 1e-9
    assert np.linalg.norm(z1 - z) / np.linalg.norm(z) > 1e-3  # it did move
