"""GPU: physics-mode layered primitive-equation model (libws_hip.so ws_lpe_*) against its
oracle (oracle/layered_pe_oracle.py) and against properties of the discrete system. The
kernel evaluates every expression in the oracle's order: fp64 agrees with the fp64 oracle to
a relative L2 of 1e-13, fp32 with the oracle run in float32 to 1e-5."""
import numpy as np
import pytest

from oracle import layered_pe_oracle as lp

pytestmark = pytest.mark.gpu
G, GP = 9.81, 0.05


def model(W, H, L, method=2, fp64=True, dx=1000.0, dy=1000.0, dt=5.0, f=1e-4, gp=GP):
    import weather_sim as ws
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.num_levels = W, H, L
    c.integration_method = method
    c.double_precision = fp64
    c.dx, c.dy, c.dt, c.gravity, c.coriolis_f = dx, dy, dt, G, f
    return ws.LayeredPrimitiveEquationsModel(c, reduced_gravity=gp)


def perturbed(L, H, W, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:H, 0:W]
    u, v, h = lp.rest_state(L, H, W, [100.0 + 40.0 * k for k in range(L)])
    for k in range(L):
        for _ in range(3):
            kx, ky = rng.integers(1, 3, 2)
            ph = rng.uniform(0, 6.28)
            h[k] += rng.uniform(0.2, 1.0) * np.cos(2 * np.pi * (kx * x / W + ky * y / H) + ph)
            u[k] += 0.05 * rng.standard_normal() * np.sin(2 * np.pi * (kx * x / W) + ph)
            v[k] += 0.05 * rng.standard_normal() * np.cos(2 * np.pi * (ky * y / H) + ph)
    return u, v, h


def rel(a, b):
    return float(np.linalg.norm(a.astype(np.float64) - b) / max(np.linalg.norm(b), 1e-300))


@pytest.mark.parametrize("W,H,L", [(64, 48, 4), (37, 29, 3), (70, 20, 1), (40, 40, 32), (33, 9, 11)])
@pytest.mark.parametrize("method", [0, 1, 2])
def test_matches_oracle_fp64(W, H, L, method):
    m = model(W, H, L, method, True, dx=1000.0, dy=1300.0)
    s0 = perturbed(L, H, W, W + L)
    m.set_state(*s0)
    m.run(10)
    want = lp.run(s0, 10, 5.0, 1000.0, 1300.0, G, GP, 1e-4, method)
    for got, w in zip(m.get_state(), want):
        assert rel(got, w) < 1e-13
    assert m.get_current_step() == 10


@pytest.mark.parametrize("W,H,L", [(300, 37, 11), (257, 13, 19), (512, 9, 8)])
@pytest.mark.parametrize("fp64", [True, False])
def test_multi_tile_widths_and_partial_chunks(W, H, L, fp64):
    """Several 128-column tiles in x (the tile-to-tile halo, the periodic wrap across tiles,
    the LDS h-neighbour path at tile seams), widths that are not a multiple of the tile, and
    level counts that leave a partial chunk of WS_LPE_CHUNK (8) levels; RK4, fp64 against the
    fp64 oracle, fp32 against the float32 oracle."""
    m = model(W, H, L, 2, fp64, dx=1000.0, dy=1300.0)
    s0 = perturbed(L, H, W, W * L)
    m.set_state(*s0)
    m.run(6)
    want = lp.run(s0, 6, 5.0, 1000.0, 1300.0, G, GP, 1e-4, 2, dtype=np.float64 if fp64 else np.float32)
    for got, w in zip(m.get_state(), want):
        assert rel(got, w.astype(np.float64)) < (1e-13 if fp64 else 1e-5)


@pytest.mark.parametrize("method", [0, 2])
def test_matches_oracle_fp32(method):
    W, H, L = 96, 64, 8
    m = model(W, H, L, method, False)
    s0 = perturbed(L, H, W, 3)
    m.set_state(*s0)
    m.run(10)
    got = m.get_state()
    assert got[2].dtype == np.float32
    # against the oracle evaluated in float32 (the same operations and rounding points); the
    # fp64 oracle differs by fp32 round-off of M ~ g * 1400 m (~1e-3 m^2/s^2 per level)
    want32 = lp.run(s0, 10, 5.0, 1000.0, 1000.0, G, GP, 1e-4, method, dtype=np.float32)
    for g_, w in zip(got, want32):
        assert rel(g_, w.astype(np.float64)) < 1e-5
    want64 = lp.run(s0, 10, 5.0, 1000.0, 1000.0, G, GP, 1e-4, method)
    assert rel(got[2], want64[2]) < 1e-6


def test_rest_state_stays_at_rest_and_mass_is_conserved():
    W, H, L = 64, 64, 6
    m = model(W, H, L)
    s0 = lp.rest_state(L, H, W, [50.0 * (k + 1) for k in range(L)])
    m.set_state(*s0)
    m.run(20)
    for got, want in zip(m.get_state(), s0):
        assert np.array_equal(got, want)
    m2 = model(W, H, L)
    s1 = perturbed(L, H, W, 5)
    m2.set_state(*s1)
    m0 = s1[2].sum(axis=(1, 2))
    m2.run(50)
    np.testing.assert_allclose(m2.layer_mass(), m0, rtol=1e-13)


def test_two_layer_baroclinic_wave_speed_on_device():
    W, H, dx, H0, H1, kx, a = 128, 8, 1000.0, 200.0, 300.0, 1, 1e-2
    A = np.array([[G * H0, G * H0], [G * H1, (G + GP) * H1]])
    lam, vec = np.linalg.eig(A)
    i = int(np.argmin(lam))
    c, e = np.sqrt(lam[i]), vec[:, i] / np.abs(vec[:, i]).max()
    amps = a * e
    u, v, h = lp.rest_state(2, H, W, [H0, H1])
    th = 2 * np.pi * kx * np.arange(W) / W
    for k, Hk in ((0, H0), (1, H1)):
        h[k] += amps[k] * np.cos(th)[None, :]
        u[k] += c / Hk * amps[k] * np.cos(th)[None, :]
    m = model(W, H, 2, 2, True, dx=dx, dy=dx, dt=20.0, f=0.0)
    m.set_state(u, v, h)
    m.run(150)
    omega = c * np.sin(2 * np.pi * kx / W) / dx
    hh = m.get_field("h")
    for k, Hk in ((0, H0), (1, H1)):
        want = Hk + amps[k] * np.cos(th - omega * 150 * 20.0)
        assert np.abs(hh[k, 0] - want).max() < 0.02 * np.abs(amps).max()


def test_errors():
    import weather_sim as ws
    m = model(16, 16, 2)
    with pytest.raises(RuntimeError):
        m.set_field("h", np.zeros((2, 16, 15)))
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.num_levels = 2, 16, 4
    with pytest.raises(ValueError):
        ws.LayeredPrimitiveEquationsModel(c)


def test_bench_size_c4p_vs_oracle():
    """The bench workload itself (config c4p: 1024^2 x 32 layers fp32 RK4, dx 1 km, dt 5 s,
    f 1e-4, g' 0.02 -- bench.py bench_lpe's initial state) for one step against the float32
    oracle: 8 x 256 tiles, 4 chunks of levels, the production launch. One step keeps the NumPy
    oracle to ~20 s."""
    W = H = 1024
    L = 32
    m = model(W, H, L, 2, False, dx=1000.0, dy=1000.0, dt=5.0, f=1e-4, gp=0.02)
    u, v, h = lp.rest_state(L, H, W, [40.0 + 2.0 * k for k in range(L)])
    x = np.arange(W)[None, :]
    y = np.arange(H)[:, None]
    for k in range(L):
        h[k] += 0.5 * np.cos(2 * np.pi * (3 * x / W + 2 * y / H) + 0.1 * k)
        u[k] += 0.01 * np.sin(2 * np.pi * (x / W + 0.05 * k))
    m.set_state(u, v, h)
    m.run(1)
    want = lp.run((u, v, h), 1, 5.0, 1000.0, 1000.0, G, 0.02, 1e-4, 2, dtype=np.float32)
    for got, w in zip(m.get_state(), want):
        assert rel(got, w.astype(np.float64)) < 1e-5

