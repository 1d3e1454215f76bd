"""GPU: physics-mode barotropic vorticity model (libws_hip.so ws_bvort_*) against its oracle
(oracle/bvort_oracle.py) and against analytic solutions. Tolerances: FFTs round
differently in rocFFT and pocketfft, so agreement is to a relative L2 of 1e-11 (fp64) /
1e-4 (fp32) after the steps below, not bitwise."""
import numpy as np
import pytest

from oracle import bvort_oracle as bo

pytestmark = pytest.mark.gpu


def model(W, H, method=2, fp64=True, dx=1.0, dy=1.0, dt=0.05, beta=0.0, nu=0.0, poisson="auto"):
    import weather_sim as ws
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height = W, H
    c.integration_method = method
    c.double_precision = fp64
    c.dx, c.dy, c.dt, c.beta, c.viscosity = dx, dy, dt, beta, nu
    return ws.BarotropicVorticityModel(c, poisson=poisson)


def smooth_field(W, H, seed=0):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:H, 0:W]
    z = np.zeros((H, W))
    for _ in range(6):
        kx, ky = rng.integers(1, 4, 2)
        z += rng.standard_normal() * np.cos(2 * np.pi * (kx * x / W + ky * y / H) + rng.uniform(0, 6.28))
    return z


def rel(a, b):
    return float(np.linalg.norm(a.astype(np.float64) - b) / np.linalg.norm(b))


@pytest.mark.parametrize("W,H", [(64, 48), (96, 80), (37, 29), (130, 20), (8, 8)])
@pytest.mark.parametrize("method", [0, 1, 2])
def test_matches_oracle_fp64(W, H, method):
    kw = dict(dx=1.0, dy=1.25, dt=0.05, beta=0.3, nu=0.02)
    m = model(W, H, method, True, **kw)
    z0 = smooth_field(W, H, seed=W + H)
    m.set_vorticity(z0)
    m.run(12)
    want = bo.run(z0, 12, kw["dt"], kw["dx"], kw["dy"], kw["beta"], kw["nu"], method)
    assert rel(m.get_vorticity_field(), want) < 1e-11
    assert m.get_current_step() == 12


@pytest.mark.parametrize("method", [0, 1, 2])
def test_matches_oracle_fp32(method):
    W, H = 128, 96
    m = model(W, H, method, False, dt=0.05, beta=0.2, nu=0.01)
    z0 = smooth_field(W, H, seed=5)
    m.set_vorticity(z0)
    m.run(10)
    got = m.get_vorticity_field()
    assert got.dtype == np.float32
    assert rel(got, bo.run(z0, 10, 0.05, 1.0, 1.0, 0.2, 0.01, method)) < 1e-4


def test_streamfunction_and_velocity_match_oracle():
    W, H = 64, 40
    m = model(W, H, dx=1.0, dy=2.0)
    z0 = smooth_field(W, H, seed=9)
    z0 -= z0.mean()
    m.set_vorticity(z0)
    psi = m.get_streamfunction()
    assert rel(psi, bo.poisson(z0, 1.0, 2.0)) < 1e-12
    u, v = m.get_velocity_field()
    ue, ve = bo.velocity(z0, 1.0, 2.0)
    assert rel(u, ue) < 1e-12 and rel(v, ve) < 1e-12


@pytest.mark.parametrize("nu", [0.0, 0.05])
def test_rossby_wave_analytic(nu):
    W, H, dx, dy, beta, dt, n = 128, 64, 1.0, 1.5, 0.5, 0.05, 40
    m = model(W, H, 2, True, dx=dx, dy=dy, dt=dt, beta=beta, nu=nu)
    m.set_vorticity(bo.rossby_mode(W, H, dx, dy, 3, 2, amp=1e-2))
    m.run(n)
    ex = bo.rossby_exact(W, H, dx, dy, 3, 2, n * dt, beta, nu, amp=1e-2)
    got = m.get_vorticity_field()
    assert rel(got, ex) < 1e-5  # RK4 time-stepping error of this dt (the oracle's is the same)
    z = bo.run(bo.rossby_mode(W, H, dx, dy, 3, 2, amp=1e-2), n, dt, dx, dy, beta, nu, bo.RK4)
    assert rel(got, z) < 1e-11


def test_energy_enstrophy_conserved_on_device():
    W, H = 128, 128
    m = model(W, H, 2, True, dt=0.01)
    z0 = smooth_field(W, H, seed=11)
    z0 -= z0.mean()
    m.set_vorticity(z0)
    E0, Z0 = m.energy(), m.enstrophy()
    m.run(100)
    assert abs(m.energy() - E0) / E0 < 1e-9
    assert abs(m.enstrophy() - Z0) / Z0 < 1e-9
    assert rel(m.get_vorticity_field(), z0) > 1e-3


def test_errors():
    import weather_sim as ws
    m = model(32, 24)
    with pytest.raises(RuntimeError):
        m.set_vorticity(np.zeros((24, 31)))
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height = 2, 10
    with pytest.raises(ValueError):
        ws.BarotropicVorticityModel(c)


@pytest.mark.parametrize("W,H", [(64, 32), (256, 128), (16, 512), (4096, 16), (32, 4096), (2048, 2048)])
@pytest.mark.parametrize("fft", ["lds", "hipfft"])
def test_poisson_paths_fp64(W, H, fft, monkeypatch):
    """Power-of-two grids take the three-pass LDS FFT Poisson solve (ws_bvort.hip
    bv_rowfft_fwd / bv_colsolve / bv_rowfft_inv); poisson="hipfft" the library's 2-D plans.
    Both against the oracle's pocketfft solve and three RK4 steps. On the strongly
    anisotropic grids (aspect 256) the Jacobian's derivatives along the long axis amplify
    the FFTs' round-off (either FFT; ~3e-9 relative after three steps), hence 1e-8 there."""
    # the smooth field's streamfunction (and so its velocity) grows with the grid: keep the
    # advective CFL number below ~0.5
    kw = dict(dx=1.0, dy=1.25, dt=0.05 * min(1.0, 64.0 / max(W, H)), beta=0.3, nu=0.02)
    m = model(W, H, 2, True, poisson="auto" if fft == "lds" else "hipfft", **kw)
    z0 = smooth_field(W, H, seed=W + 3 * H)
    z0 -= z0.mean()
    m.set_vorticity(z0)
    assert rel(m.get_streamfunction(), bo.poisson(z0, kw["dx"], kw["dy"])) < 1e-12
    m.run(3)
    want = bo.run(z0, 3, kw["dt"], kw["dx"], kw["dy"], kw["beta"], kw["nu"], 2)
    assert rel(m.get_vorticity_field(), want) < (1e-11 if max(W, H) <= 8 * min(W, H) else 1e-8)


@pytest.mark.parametrize("W,H", [(256, 128), (2048, 2048)])
def test_poisson_lds_fft_fp32(W, H):
    dt = 0.05 * min(1.0, 64.0 / max(W, H))
    m = model(W, H, 2, False, dt=dt, beta=0.2, nu=0.01)
    z0 = smooth_field(W, H, seed=7)
    z0 -= z0.mean()
    m.set_vorticity(z0)
    assert rel(m.get_streamfunction(), bo.poisson(z0, 1.0, 1.0)) < 1e-5
    m.run(5)
    assert rel(m.get_vorticity_field(), bo.run(z0, 5, dt, 1.0, 1.0, 0.2, 0.01, 2)) < 1e-4


def test_bench_size_c3p_vs_oracle():
    """The bench workload itself (config c3p: 2048^2 fp32 RK4, two Rossby modes, dt 0.05,
    beta 1e-3, nu 0.01 -- bench.py bench_bvort) for 2 steps against the fp64 oracle: the
    LDS-FFT Poisson path at its production size, every multi-workgroup seam of the stencil
    tiles and the column pass. fp32 tolerance as above."""
    W = H = 2048
    m = model(W, H, 2, False, dt=0.05, beta=1e-3, nu=0.01)
    z0 = bo.rossby_mode(W, H, 1.0, 1.0, 5, 3, amp=1e-2) + bo.rossby_mode(W, H, 1.0, 1.0, 2, 7, amp=5e-3)
    z0 = z0 + 1e-3 * smooth_field(W, H, seed=11)
    m.set_vorticity(z0)
    m.run(2)
    want = bo.run(z0.astype(np.float32).astype(np.float64), 2, 0.05, 1.0, 1.0, 1e-3, 0.01, 2)
    assert rel(m.get_vorticity_field(), want) < 1e-4
