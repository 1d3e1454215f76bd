"""GPU: slab decomposition of the physics-mode layered PE model (ws_lpe_create_multi /
ws_lpe_create_slab) against the single-domain model, bit for bit.

The decomposed model runs the same stage kernel on every slab with one halo row per level
refreshed before each RK stage (the one-process transport: a pull kernel reading the ring
neighbours' rows; rows that wrap around the ring come from the last / first slab), so each
cell's arithmetic is the single domain's: the results must be identical, not merely close.
Slabs share device 0 here (a one-GPU box); distinct devices take the same code path with
peer access. The RCCL transport's ring protocol is tests/test_lpe_slab_protocol.py (CPU,
gloo); a 1-rank RCCL slab runs here."""
import numpy as np
import pytest

from test_gpu_layered_pe import model, perturbed

pytestmark = pytest.mark.gpu


def sliced(W, H, L, method, fp64, n, **kw):
    import weather_sim as ws
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.num_levels = W, H, L
    c.integration_method = method
    c.double_precision = fp64
    c.dx, c.dy, c.dt, c.gravity, c.coriolis_f = kw.get("dx", 1000.0), kw.get("dy", 1300.0), 5.0, 9.81, 1e-4
    return ws.LayeredPrimitiveEquationsModel(c, reduced_gravity=kw.get("gp", 0.05), devices=[0] * n)


def same(a, b):
    return all(np.array_equal(x, y) for x, y in zip(a, b))


@pytest.mark.parametrize("W,H,L,n", [(64, 48, 4, 2), (37, 29, 3, 3), (300, 37, 11, 4), (40, 40, 32, 5),
                                     (33, 9, 11, 9), (257, 13, 19, 2)])
@pytest.mark.parametrize("method", [0, 1, 2])
@pytest.mark.parametrize("fp64", [True, False])
def test_slabs_match_single_domain(W, H, L, n, method, fp64):
    """2..9 slabs (9 slabs of one row at H = 9: every halo row is a neighbour's only row),
    tile-partial widths, partial level chunks, runs split across calls and a field write
    between runs (the totals of a freshly written field are summed by the stage again)."""
    whole = model(W, H, L, method, fp64, dx=1000.0, dy=1300.0)
    parts = sliced(W, H, L, method, fp64, n)
    assert (parts.nslabs, parts.row0, parts.rows) == (n, 0, H)
    s0 = perturbed(L, H, W, W + L + n)
    for m in (whole, parts):
        m.set_state(*s0)
        m.run(3)
        m.run(2)
    assert same(whole.get_state(), parts.get_state())
    h = whole.get_field("h")
    h[:, H // 2] += 0.25
    for m in (whole, parts):
        m.set_field("h", h)
        m.run(3)
    assert same(whole.get_state(), parts.get_state())
    assert parts.get_current_step() == whole.get_current_step() == 8
    assert parts.get_current_time() == whole.get_current_time()
    ms, launches = parts.last_run_stats()
    stages = {0: 1, 1: 2, 2: 4}[method]
    assert ms > 0 and launches == 3 * stages * 2 * n  # a stage and a halo pull per slab and stage


def test_c4p_size_eight_slabs():
    """The c4p bench workload (1024^2 x 32 layers fp32 RK4) in 8 slabs on one device against
    one domain: 3 steps, bitwise."""
    W = H = 1024
    L = 32
    import oracle.layered_pe_oracle as lp
    whole = model(W, H, L, 2, False, dx=1000.0, dy=1000.0, gp=0.02)
    parts = sliced(W, H, L, 2, False, 8, dx=1000.0, dy=1000.0, gp=0.02)
    u, v, h = lp.rest_state(L, H, W, [40.0 + 2.0 * k for k in range(L)])
    x = np.arange(W)[None, :]
    y = np.arange(H)[:, None]
    for k in range(L):
        h[k] += 0.5 * np.cos(2 * np.pi * (3 * x / W + 2 * y / H) + 0.1 * k)
        u[k] += 0.01 * np.sin(2 * np.pi * (x / W + 0.05 * k))
        v[k] += 0.01 * np.cos(2 * np.pi * (y / H + 0.03 * k))
    for m in (whole, parts):
        m.set_state(u, v, h)
        m.run(3)
    assert same(whole.get_state(), parts.get_state())


def test_config_devices_and_one_rank_rccl_slab():
    """config.devices with > 1 entry builds the decomposed model; a 1-rank RCCL slab
    (ws_lpe_create_slab: the communicator bootstrap on one GPU) is the single domain."""
    import weather_sim as ws
    W, H, L = 48, 20, 3
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.num_levels = W, H, L
    c.double_precision = True
    c.dx, c.dy, c.dt = 1000.0, 1000.0, 5.0
    c.devices = [0, 0, 0]
    a = ws.LayeredPrimitiveEquationsModel(c)
    assert a.nslabs == 3
    c.devices = None
    b = ws.LayeredPrimitiveEquationsModel(c, slab=(0, 1, ws.new_comm_id()))
    assert (b.nslabs, b.row0, b.rows) == (1, 0, H)
    w = ws.LayeredPrimitiveEquationsModel(c)
    s0 = perturbed(L, H, W, 7)
    for m in (a, b, w):
        m.set_state(*s0)
        m.run(4)
    assert same(a.get_state(), w.get_state())
    assert same(b.get_state(), w.get_state())


def test_slab_errors():
    import weather_sim as ws
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.num_levels = 16, 4, 2
    with pytest.raises(ValueError):
        ws.LayeredPrimitiveEquationsModel(c, devices=[0] * 5)  # more slabs than rows
    with pytest.raises(ValueError):
        ws.LayeredPrimitiveEquationsModel(c, devices=[0, 0], slab=(0, 1, ws.new_comm_id()))
    with pytest.raises(ValueError):
        ws.LayeredPrimitiveEquationsModel(c, slab=(0, 1, b"short"))
    with pytest.raises(ValueError):
        ws.LayeredPrimitiveEquationsModel(c, slab=(1, 1, ws.new_comm_id()))
    with pytest.raises(RuntimeError):
        ws.LayeredPrimitiveEquationsModel(c, devices=[0, 4096])
    m = ws.LayeredPrimitiveEquationsModel(c, devices=[0, 0])
    with pytest.raises(RuntimeError):
        m.set_field("h", np.zeros((2, 2, 16)))  # the whole field, not a slab's rows
