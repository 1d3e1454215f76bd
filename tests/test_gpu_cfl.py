"""CFL number by device max-reduction (ws_hip.h ws_sim_cfl; csrc/ws_reduce.hip) against NumPy.

The reference has no CFL (its dt is fixed), so this north_star extension is checked against
a NumPy evaluation of the same per-cell formula in the simulation's precision:
c = max((|u| + sqrt(g h)) dt / dx, (|v| + sqrt(g h)) dt / dy), max over the grid (per level).
Every operation is one IEEE rounding in both, so the maxima agree to the last bit in fp64 and
within one fp32 rounding of sqrt's implementation in fp32.
"""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

ws = pytest.importorskip("weather_sim")
if not ws.is_cuda_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)


def numpy_cfl(u, v, h, g, dt, dx, dy, dtype):
    u, v, h = (np.asarray(a, dtype) for a in (u, v, h))
    with np.errstate(invalid="ignore"):
        c = np.sqrt(dtype(g) * h)
    cx, cy = dtype(dt) / dtype(dx), dtype(dt) / dtype(dy)
    a = (np.abs(u) + c) * cx
    b = (np.abs(v) + c) * cy
    return np.max(np.maximum(a, b), axis=(-2, -1)).astype(np.float64)


def make(W, H, fp64, L=1, model=0, dx=1.0, dy=1.0, dt=0.01, g=9.81):
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.num_levels, c.model = W, H, L, model
    c.double_precision = fp64
    c.dx, c.dy, c.dt, c.gravity = dx, dy, dt, g
    c.max_time = 1e30
    return ws.WeatherSimulation(c)


@pytest.mark.parametrize("variant", ["f32", "f64"])
def test_cfl_matches_numpy_on_reference_fixtures(variant):
    gold = golden(variant)
    fp64 = variant == "f64"
    dtype = np.float64 if fp64 else np.float32
    n = 0
    for case in gold.cases("step/"):
        cfg = gold.meta[case]["cfg"]
        dx, dy, dt, g = cfg.get("dx", 1.0), cfg.get("dy", 1.0), cfg.get("dt", 0.01), cfg.get("g", 9.81)
        sim = make(cfg["width"], cfg["height"], fp64, dx=dx, dy=dy, dt=dt, g=g)
        sim.initialize()
        s = gold.snap(case, "s50")
        gr = sim.get_current_grid()
        gr.set_velocity_field(s["u"], s["v"])
        gr.set_height_field(s["h"])
        got, ms = sim.get_cfl(with_time=True)
        want = float(numpy_cfl(s["u"], s["v"], s["h"], g, dt, dx, dy, dtype))
        if fp64:
            assert got == want, (case, got, want)
        else:
            assert abs(got - want) <= 2 * np.finfo(np.float32).eps * want, (case, got, want)
        assert ms > 0
        n += 1
    assert n >= 20


@pytest.mark.parametrize("shape", [(4096, 4096), (333, 1025), (7, 5), (1, 1)])
def test_cfl_large_and_ragged(shape):
    """Grid-stride and multi-workgroup paths (>= 1024 partials per level at 4096 rows), ragged
    widths; the maximum placed in a single cell far from the origin."""
    W, H = shape
    sim = make(W, H, True)
    sim.initialize()
    rng = np.random.default_rng(7)
    u = rng.uniform(-1, 1, (H, W))
    v = rng.uniform(-1, 1, (H, W))
    h = rng.uniform(5, 10, (H, W))
    u[H - 1, W - 1] = 55.0  # the global max sits in the very last cell
    g = sim.get_current_grid()
    g.set_velocity_field(u, v)
    g.set_height_field(h)
    assert sim.get_cfl() == float(numpy_cfl(u, v, h, 9.81, 0.01, 1.0, 1.0, np.float64))


def test_cfl_per_level_and_nan():
    """Per-level maxima (PE, 5 levels); a negative depth on one level gives NaN there (and in
    the overall maximum), the other levels keep their values."""
    W, H, L = 130, 70, 5
    sim = make(W, H, True, L=L, model=2, dx=2.0, dy=0.5)
    sim.initialize()
    g = sim.get_current_grid()
    rng = np.random.default_rng(3)
    want = []
    for k in range(L):
        u = rng.uniform(-3, 3, (H, W)) * (k + 1)
        v = rng.uniform(-3, 3, (H, W))
        h = rng.uniform(1, 20, (H, W))
        if k == 3:
            h[10, 20] = -1.0
        g.set_velocity_field(u, v, level=k)
        g.set_height_field(h, level=k)
        want.append(numpy_cfl(u, v, h, 9.81, 0.01, 2.0, 0.5, np.float64))
    top, per = sim.get_cfl(per_level=True)
    assert np.isnan(top) and np.isnan(per[3])
    for k in (0, 1, 2, 4):
        assert per[k] == want[k], (k, per[k], want[k])


def test_cfl_after_steps_and_on_slabs():
    """After a run (the current grid after rotation / two-step launches) and on a slab
    decomposition: the maximum over slabs equals the single domain's."""
    W, H = 300, 96
    one = make(W, H, True)
    one.set_initial_condition(ws.BreakingWaveInitialCondition(1.5, 0.05, 10.0))
    one.initialize()
    one.run(7)
    g = one.get_current_grid()
    u, v = g.get_velocity_field()
    want = float(numpy_cfl(u, v, g.get_height_field(), 9.81, 0.01, 1.0, 1.0, np.float64))
    assert one.get_cfl() == want
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.double_precision, c.max_time = W, H, True, 1e30
    group = ws.SlabGroup(c, 3)
    group.set_initial_condition(ws.BreakingWaveInitialCondition(1.5, 0.05, 10.0))
    group.initialize()
    group.run(7)
    assert max(group.slab(r).get_cfl() for r in range(3)) == want
