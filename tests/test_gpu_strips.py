"""Fused-kernel strip edge cases, bitwise vs the CPU oracle: odd widths (x2y's last column
pair straddles x = W-1), widths narrower than one strip, widths that end exactly on a strip
boundary, non-power-of-two spacing (IEEE-divide instantiation), line-aligned strips."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ws = pytest.importorskip("weather_sim")
if not ws.is_cuda_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)


def run_both(W, H, method, fp64, steps, dx=1.0, dy=2.0, f=0.3, align=None):
    from oracle.ws_oracle import OracleSim

    c = ws.SimulationConfig()
    c.grid_width, c.grid_height = W, H
    c.integration_method, c.double_precision = method, fp64
    c.dx, c.dy, c.coriolis_f = dx, dy, f
    sim = ws.WeatherSimulation(c)
    if align is not None:
        sim.pin_variant(align=align)
    sim.set_initial_condition(ws.BreakingWaveInitialCondition(1.5, 0.05, 10.0))
    sim.initialize()
    g = sim.get_current_grid()
    ref = OracleSim(W, H, 0, method, dx=dx, dy=dy, coriolis_f=f, precision="f64" if fp64 else "f32")
    ref.initialize()
    u, v = g.get_velocity_field()
    for k, a in (("u", u), ("v", v), ("h", g.get_height_field())):
        ref.set_field(k, a)
    sim.run(steps)
    ref.run(steps)
    g = sim.get_current_grid()
    u, v = g.get_velocity_field()
    got = {"u": u, "v": v, "h": g.get_height_field(), "vort": g.get_vorticity_field()}
    for k in got:
        np.testing.assert_array_equal(got[k], ref.get_field(k), err_msg=f"W={W} {k}")


@pytest.mark.parametrize("W", [2, 3, 7, 56, 57, 64, 120, 121, 127, 128, 129, 240, 241, 333])
@pytest.mark.parametrize("kernel,tb", [("dppy", "1"), ("dppy", "2"), ("dppy", "4"), ("dppy", "8"), ("x2y", "1"),
                                      ("x2y", "2"), ("x2y", "4"), ("x2y", "8"), ("pc", "2"), ("pc2", "2")],
                         ids=["dppy", "dppy_tb2", "dppy_tb4", "dppy_tb8", "x2y", "x2y_tb2", "x2y_tb4", "x2y_tb8",
                              "pc_tb2", "pc2_tb2"])
@pytest.mark.parametrize("method", [0, 1, 2])
@pytest.mark.parametrize("fp64", [False, True])
def test_strip_widths(W, kernel, tb, method, fp64, monkeypatch):
    monkeypatch.setenv("WS_KERNEL", kernel)
    monkeypatch.setenv("WS_TB", tb)
    monkeypatch.setenv("WS_SEG_ROWS", "7")
    run_both(W, 29, method, fp64, 5)


@pytest.mark.parametrize("kernel,tb", [("dppy", "1"), ("dppy", "2"), ("x2y", "1"), ("x2y", "2"), ("pc", "2"), ("pc2", "2"),
                                      ("lds", "1")],
                         ids=["dppy", "dppy_tb2", "x2y", "x2y_tb2", "pc_tb2", "pc2_tb2", "lds"])
@pytest.mark.parametrize("method", [0, 1, 2])
def test_non_pow2_spacing(kernel, tb, method, monkeypatch):
    monkeypatch.setenv("WS_KERNEL", kernel)
    monkeypatch.setenv("WS_TB", tb)
    run_both(301, 40, method, True, 4, dx=0.75, dy=1.3)


@pytest.mark.parametrize("W", [61, 300, 700])
@pytest.mark.parametrize("kernel,tb", [("dppy", "1"), ("dppy", "2"), ("x2y", "1"), ("x2y", "2"), ("pc", "2"), ("pc2", "2"),
                                      ("lds", "1")],
                         ids=["dppy", "dppy_tb2", "x2y", "x2y_tb2", "pc_tb2", "pc2_tb2", "lds"])
@pytest.mark.parametrize("method", [0, 1, 2])
@pytest.mark.parametrize("fp64", [False, True])
def test_line_aligned_strips(W, kernel, tb, method, fp64, monkeypatch):
    """align=1 (ws_sim_pin_variant): strip output windows cut to whole 128-byte lines
    (asymmetric margins)."""
    monkeypatch.setenv("WS_KERNEL", kernel)
    monkeypatch.setenv("WS_TB", tb)
    monkeypatch.setenv("WS_SEG_ROWS", "9")
    run_both(W, 37, method, fp64, 5, align=True)
