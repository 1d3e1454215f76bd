"""GPU: slab decomposition of the physics-mode barotropic vorticity model
(ws_bvort_create_multi / ws_bvort_create_slab) against the single-domain model, bit for bit.

A decomposed model runs the single domain's passes on the same data: each slab's row FFTs
on its own row pairs, a block transpose of the spectrum so that slab q's column pass solves
global columns [q nc, (q + 1) nc) over all rows, the transpose back, the inverse row FFTs, and
the stencil with one halo row of psi and zeta from the ring neighbours. Every value is
computed by the same instructions on the same inputs, so vorticity, streamfunction and
velocities must be identical to the single domain's. Slabs share device 0 here; the RCCL
transport (block all-to-all, periodic halo plan) runs with one rank."""
import numpy as np
import pytest

from test_gpu_bvort import smooth_field

pytestmark = pytest.mark.gpu


def cfg(W, H, method, fp64, **kw):
    import weather_sim as ws
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height = W, H
    c.integration_method = method
    c.double_precision = fp64
    c.dx, c.dy, c.dt = kw.get("dx", 1.0), kw.get("dy", 1.25), kw.get("dt", 0.05)
    c.beta, c.viscosity = kw.get("beta", 0.3), kw.get("nu", 0.02)
    return c


def fields(m):
    u, v = m.get_velocity_field()
    return m.get_vorticity_field(), m.get_streamfunction(), u, v


@pytest.mark.parametrize("W,H,n", [(64, 64, 2), (128, 64, 4), (64, 32, 8), (256, 128, 2), (32, 128, 16)])
@pytest.mark.parametrize("method", [0, 1, 2])
@pytest.mark.parametrize("fp64", [True, False])
def test_slabs_match_single_domain(W, H, n, method, fp64):
    """2 .. 16 slabs (8 slabs of 4 rows at 64 x 32; 16 slabs of one column each of the W / 2 =
    16 spectrum columns at 32 x 128), runs split across calls, a field write between runs."""
    import weather_sim as ws
    whole = ws.BarotropicVorticityModel(cfg(W, H, method, fp64))
    parts = ws.BarotropicVorticityModel(cfg(W, H, method, fp64), devices=[0] * n)
    assert (parts.nslabs, parts.row0, parts.rows) == (n, 0, H)
    z0 = smooth_field(W, H, seed=W + H + n)
    for m in (whole, parts):
        m.set_vorticity(z0)
        m.run(3)
        m.run(2)
    for a, b in zip(fields(whole), fields(parts)):
        assert np.array_equal(a, b)
    z1 = whole.get_vorticity_field()
    z1[H // 3] += 0.5
    for m in (whole, parts):
        m.set_vorticity(z1)
        m.run(2)
    for a, b in zip(fields(whole), fields(parts)):
        assert np.array_equal(a, b)
    assert parts.get_current_step() == whole.get_current_step() == 7
    assert parts.get_current_time() == whole.get_current_time()


def test_c3p_size_eight_slabs():
    """The c3p bench workload's shape (2048^2 fp32 RK4) in 8 slabs on one device: 2 steps,
    bitwise equal to one domain."""
    import weather_sim as ws
    W = H = 2048
    c = cfg(W, H, 2, False, dx=1.0, dy=1.0, dt=0.05, beta=1e-3, nu=1e-4)
    whole = ws.BarotropicVorticityModel(c)
    parts = ws.BarotropicVorticityModel(c, devices=[0] * 8)
    z0 = smooth_field(W, H, seed=11)
    for m in (whole, parts):
        m.set_vorticity(z0)
        m.run(2)
    assert np.array_equal(whole.get_vorticity_field(), parts.get_vorticity_field())
    assert np.array_equal(whole.get_streamfunction(), parts.get_streamfunction())


def test_one_rank_rccl_slab_and_config_devices():
    import weather_sim as ws
    W, H = 64, 64
    c = cfg(W, H, 2, True)
    b = ws.BarotropicVorticityModel(c, slab=(0, 1, ws.new_comm_id()))
    assert (b.nslabs, b.row0, b.rows) == (1, 0, H)
    c2 = cfg(W, H, 2, True)
    c2.devices = [0, 0, 0, 0]
    a = ws.BarotropicVorticityModel(c2)
    assert a.nslabs == 4
    w = ws.BarotropicVorticityModel(cfg(W, H, 2, True))
    z0 = smooth_field(W, H, seed=3)
    for m in (a, b, w):
        m.set_vorticity(z0)
        m.run(4)
    for x in (a, b):
        for p, q in zip(fields(x), fields(w)):
            assert np.array_equal(p, q)


def test_slab_errors():
    import weather_sim as ws
    with pytest.raises(ValueError):  # not a power-of-two grid: no LDS-FFT path to decompose
        ws.BarotropicVorticityModel(cfg(96, 64, 2, True), devices=[0, 0])
    with pytest.raises(ValueError):  # three slabs: not a power of two
        ws.BarotropicVorticityModel(cfg(64, 48, 2, True), devices=[0, 0, 0])
    with pytest.raises(ValueError):  # odd rows per slab
        ws.BarotropicVorticityModel(cfg(64, 16, 2, True), devices=[0] * 16)
    with pytest.raises(ValueError):  # the hipFFT path is not decomposed
        ws.BarotropicVorticityModel(cfg(64, 64, 2, True), poisson="hipfft", devices=[0, 0])
    with pytest.raises(RuntimeError):
        ws.BarotropicVorticityModel(cfg(64, 64, 2, True), devices=[0, 4096])
