"""Fast numerics (ws_hip.h WS_NUMERICS_FAST, ws_fused.h kSpFast*) against the reference.

Fast numerics re-associate the reference's tendencies and integrators for the hardware
(fused multiply-adds, the 1/(2dx) factor folded into the update constants, RK4's final
combination as y + dt/3 ((k2 + k3) + k4)); it is the fp64 default. The north_star tolerance
is <= 1e-10 relative L2 per field against the reference CPU solver on identical initial
conditions; every check below asserts it (TOL), and most land near 1e-15:

* the reference's own fixtures (tests/golden/ref_small_f64.npz, 48 x 32, 50 steps, every
  model / integrator / initial condition with dx == dy) for every fused variant;
* a 4096 x 2048 fp64 RK4 run against the C oracle (pinned bitwise to the reference);
* C2 itself (4096^2 fp64 RK4, jet_stream): the fast run against the exact run of the same
  library, which is the reference bit for bit (test_gpu_parity.py::test_full_size_digests
  pins it to the reference's SHA-256 digests), over 200 steps.
Anisotropic spacing (dx != dy) keeps the exact kernels: bitwise.
"""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

ws = pytest.importorskip("weather_sim")
if not ws.is_cuda_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

TOL = 1e-10  # relative L2 per field (BASELINE.json north_star, fp64)


def rel_l2(got, want):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    n = np.linalg.norm(want)
    return float(np.linalg.norm(got - want) / (n if n > 0 else 1.0))


def make_sim(W, H, model, method, fp64, dx=1.0, dy=1.0, dt=0.01, g=9.81, f=0.0, max_time=1e30):
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height = W, H
    c.model, c.integration_method, c.double_precision = model, method, fp64
    c.dx, c.dy, c.dt, c.gravity, c.coriolis_f, c.max_time = dx, dy, dt, g, f, max_time
    return ws.WeatherSimulation(c)


def fields(sim):
    g = sim.get_current_grid()
    u, v = g.get_velocity_field()
    return {"u": u, "v": v, "h": g.get_height_field()}


def test_default_numerics_by_precision(monkeypatch):
    monkeypatch.delenv("WS_NUMERICS", raising=False)
    assert make_sim(64, 32, 0, 2, True).get_numerics() == "fast"
    assert make_sim(64, 32, 0, 2, False).get_numerics() == "exact"
    monkeypatch.setenv("WS_NUMERICS", "exact")
    assert make_sim(64, 32, 0, 2, True).get_numerics() == "exact"
    s = make_sim(64, 32, 0, 2, True)
    s.set_numerics("fast")
    assert s.get_numerics() == "fast"
    with pytest.raises(KeyError):
        s.set_numerics("approximate")


@pytest.mark.parametrize("kernel,tb", [("dppy", "1"), ("dppy", "2"), ("dppy", "4"), ("x2y", "1"), ("x2y", "2"), ("pc", "2"), ("pc2", "2"),
                                      ("lds", "1")],
                         ids=["dppy", "dppy_tb2", "dppy_tb4", "x2y", "x2y_tb2", "pc_tb2", "pc2_tb2", "lds"])
def test_fast_matches_reference_fixtures(kernel, tb, monkeypatch):
    monkeypatch.setenv("WS_NUMERICS", "fast")
    monkeypatch.setenv("WS_KERNEL", kernel)
    monkeypatch.setenv("WS_TB", tb)
    gold = golden("f64")
    n_iso = n_aniso = 0
    worst = 0.0
    for case in gold.cases("step/"):
        cfg = gold.meta[case]["cfg"]
        sim = make_sim(cfg["width"], cfg["height"], cfg["model"], cfg["method"], True, dx=cfg.get("dx", 1.0),
                       dy=cfg.get("dy", 1.0), dt=cfg.get("dt", 0.01), g=cfg.get("g", 9.81), f=cfg.get("f", 0.0))
        s0 = gold.snap(case, "s0")
        sim.initialize()
        gr = sim.get_current_grid()
        gr.set_velocity_field(s0["u"], s0["v"])
        gr.set_height_field(s0["h"])
        gr.set_pressure_field(s0["p"])
        gr.set_temperature_field(s0["t"])
        gr.set_humidity_field(s0["q"])
        sim.run(gold.meta[case]["s50"]["step"])
        ref = gold.snap(case, "s50")
        got = fields(sim)
        if cfg.get("dx", 1.0) == cfg.get("dy", 1.0):
            for k in ("u", "v", "h"):
                e = rel_l2(got[k], ref[k])
                worst = max(worst, e)
                assert e <= TOL, (case, k, e)
            n_iso += 1
        else:  # anisotropic spacing: the exact kernels run
            for k in ("u", "v", "h"):
                np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{case} {k}")
            n_aniso += 1
    assert n_iso >= 10
    print(f"{kernel}: worst relative L2 over {n_iso} fixture cases = {worst:.3e}")


@pytest.mark.parametrize("tb", ["1", "2", "4"])
@pytest.mark.parametrize("method", [0, 1, 2])
def test_fast_large_grid_vs_oracle(method, tb, monkeypatch):
    """4096 x 2048 fp64 (every strip / segment seam of the production tiling), 3 steps,
    f != 0 (the Coriolis instantiation) against the C oracle."""
    from oracle.ws_oracle import OracleSim

    monkeypatch.setenv("WS_NUMERICS", "fast")
    monkeypatch.setenv("WS_KERNEL", "dppy")
    monkeypatch.setenv("WS_TB", tb)
    W, H, steps = 4096, 2048, 5 if tb == "4" else 3  # (tb 4: a four-step launch where it applies)
    sim = make_sim(W, H, 0, method, True, f=1e-4)
    sim.set_initial_condition(ws.BreakingWaveInitialCondition(1.5, 0.05, 10.0))
    sim.initialize()
    s0 = fields(sim)
    ref = OracleSim(W, H, 0, method, coriolis_f=1e-4, max_time=1e30, precision="f64")
    ref.initialize()
    for k in ("u", "v", "h"):
        ref.set_field(k, s0[k])
    sim.run(steps)
    ref.run(steps)
    got = fields(sim)
    for k in ("u", "v", "h"):
        e = rel_l2(got[k], ref.get_field(k))
        assert e <= TOL, (k, e)
    # vorticity is computed from the (fast) u, v by the exact diagnostics kernel
    assert rel_l2(sim.get_current_grid().get_vorticity_field(), ref.get_field("vort")) <= 1e-8


def test_fast_c2_long_run_vs_exact(monkeypatch):
    """C2 (the bench workload): 4096^2 fp64 RK4 jet_stream, 200 steps, fast vs exact."""
    out = {}
    for mode in ("exact", "fast"):
        monkeypatch.setenv("WS_NUMERICS", mode)
        sim = make_sim(4096, 4096, 0, 2, True)
        sim.set_initial_condition(ws.JetStreamInitialCondition())
        sim.initialize()
        assert sim.run(200) == 200
        out[mode] = fields(sim)
        del sim
    for k in ("u", "v", "h"):
        e = rel_l2(out["fast"][k], out["exact"][k])
        assert e <= TOL, (k, e)
        print(f"C2 200 steps {k}: relative L2 {e:.3e}")
