"""HIP path vs the reference, through the C ABI (weather_sim -> libws_hip.so). GPU only.

Small cases compare bit-for-bit (max-ulp 0, fp32 AND fp64) with the reference's own
outputs in tests/golden/ref_small_*.npz: every (model, method, IC, spacing/physics) case
after 1, 10 and 50 steps, all seven fields incl. vorticity; every initial condition; and
the API-behaviour quirks (max_time cap, run_until step count, p/T/q alternation, PE T/P
drift, stale grid handle, set_dt, re-initialize). Full-size cases compare SHA-256 digests
of the reference's outputs (tests/golden/ref_large.json) -- bitwise at BASELINE sizes.
"""
import hashlib

import numpy as np
import pytest

from conftest import golden, large_digests

pytestmark = pytest.mark.gpu

ws = pytest.importorskip("weather_sim")
if not ws.is_cuda_available():  # pragma: no cover - the gpu marker is deselected on CPU
    pytest.skip("no HIP device", allow_module_level=True)

FIELDS = ("u", "v", "h", "p", "t", "q", "vort")


def make_sim(width, height, model, method, fp64, dx=1.0, dy=1.0, dt=0.01, g=9.81, f=0.0, max_time=10.0, levels=1):
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.num_levels = width, height, levels
    c.model, c.integration_method = model, method
    c.dx, c.dy, c.dt, c.gravity, c.coriolis_f, c.max_time = dx, dy, dt, g, f, max_time
    c.double_precision = fp64
    return ws.WeatherSimulation(c)


def state(grid, level=None):
    u, v = grid.get_velocity_field(level)
    return {"u": u, "v": v, "h": grid.get_height_field(level), "p": grid.get_pressure_field(level),
            "t": grid.get_temperature_field(level), "q": grid.get_humidity_field(level),
            "vort": grid.get_vorticity_field(level)}


def assert_bitwise(grid, ref, what, fields=FIELDS):
    got = state(grid)
    for k in fields:
        assert got[k].dtype == ref[k].dtype, (what, k)
        np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{what}: field {k}")


def load(sim, s0):
    sim.initialize()
    g = sim.get_current_grid()
    g.set_velocity_field(s0["u"], s0["v"])
    g.set_height_field(s0["h"])
    g.set_pressure_field(s0["p"])
    g.set_temperature_field(s0["t"])
    g.set_humidity_field(s0["q"])


# (WS_FUSED, WS_KERNEL, WS_TB): every fused variant, dppy also with two steps per launch
# (temporal blocking: run(n) advances pairs of steps per launch), and the per-stage kernels
# (tb 4 / 8: four (eight: Euler) steps per launch where the kernel takes them -- dppy, x2y in
# fp32 -- else the largest it takes)
KERNELS = [("1", "dppy", "1"), ("1", "dppy", "2"), ("1", "dppy", "4"), ("1", "dppy", "8"), ("1", "x2y", "1"),
           ("1", "x2y", "2"), ("1", "x2y", "4"), ("1", "x2y", "8"), ("1", "pc", "2"), ("1", "pc2", "2"),
           ("1", "lds", "1"), ("0", "x2y", "1")]
KERNEL_IDS = ["fused_dppy", "fused_dppy_tb2", "fused_dppy_tb4", "fused_dppy_tb8", "fused_x2y", "fused_x2y_tb2",
              "fused_x2y_tb4", "fused_x2y_tb8", "fused_pc_tb2", "fused_pc2_tb2", "fused_lds", "stage_kernels"]
# (kernel, steps per launch) of the fused variants
FUSED = [("dppy", "1"), ("dppy", "2"), ("dppy", "4"), ("x2y", "1"), ("x2y", "2"), ("x2y", "4"), ("pc", "2"),
         ("pc2", "2"), ("lds", "1")]
FUSED_IDS = ["dppy", "dppy_tb2", "dppy_tb4", "x2y", "x2y_tb2", "x2y_tb4", "pc_tb2", "pc2_tb2", "lds"]


@pytest.mark.parametrize("fused,kernel,tb", KERNELS, ids=KERNEL_IDS)
@pytest.mark.parametrize("variant", ["f32", "f64"])
def test_stepping_bitwise(variant, fused, kernel, tb, monkeypatch):
    monkeypatch.setenv("WS_FUSED", fused)
    monkeypatch.setenv("WS_KERNEL", kernel)
    monkeypatch.setenv("WS_TB", tb)
    gold = golden(variant)
    cases = gold.cases("step/")
    assert len(cases) >= 20
    for case in cases:
        cfg = gold.meta[case]["cfg"]
        sim = make_sim(cfg["width"], cfg["height"], cfg["model"], cfg["method"], variant == "f64",
                       dx=cfg.get("dx", 1.0), dy=cfg.get("dy", 1.0), dt=cfg.get("dt", 0.01), g=cfg.get("g", 9.81),
                       f=cfg.get("f", 0.0))
        load(sim, gold.snap(case, "s0"))
        sim.step()
        for snap, n in (("s1", 0), ("s10", 9), ("s50", 40)):
            if n:
                sim.run(n)
            ref = gold.snap(case, snap)
            assert sim.get_current_step() == ref["step"]
            assert sim.get_current_time() == ref["time"]
            assert_bitwise(sim.get_current_grid(), ref, f"{case} {snap}")


@pytest.mark.parametrize("variant", ["f32", "f64"])
def test_initial_conditions_bitwise(variant):
    gold = golden(variant)
    cases = gold.cases("ic/") + gold.cases("ic37x53/")
    for case in cases:
        name = case.split("/", 1)[1]
        W, H = (48, 32) if case.startswith("ic/") else (37, 53)
        args = {"random": (42, 1.0), "atmospheric_profile_tropical": ("tropical",),
                "atmospheric_profile_polar": ("polar",), "jet_stream_custom": (0.3, 0.07, 13.5, 9.75),
                "vortex_custom": (0.4, 0.6, 0.2, 5.0, 11.0)}.get(name, ())
        base = name.replace("_tropical", "").replace("_polar", "").replace("_custom", "")
        cls = {"uniform": ws.UniformInitialCondition, "random": ws.RandomInitialCondition,
               "zonal_flow": ws.ZonalFlowInitialCondition, "vortex": ws.VortexInitialCondition,
               "jet_stream": ws.JetStreamInitialCondition, "breaking_wave": ws.BreakingWaveInitialCondition,
               "front": ws.FrontInitialCondition, "mountain": ws.MountainInitialCondition,
               "atmospheric_profile": ws.AtmosphericProfileInitialCondition}[base]
        sim = make_sim(W, H, 0, 2, variant == "f64")
        sim.set_initial_condition(cls(*args))
        sim.initialize()
        assert_bitwise(sim.get_current_grid(), gold.snap(case, "s0"), case)


@pytest.mark.parametrize("variant", ["f32", "f64"])
def test_api_behaviour(variant):
    gold = golden(variant)
    fp64 = variant == "f64"
    # run(2000) with max_time = 10 stops at t >= max_time
    sim = make_sim(16, 12, 0, 0, fp64)
    sim.set_initial_condition(ws.JetStreamInitialCondition())
    sim.initialize()
    ref = gold.snap("api/max_time_cap", "end")
    assert sim.run(2000) == ref["step"]
    assert sim.get_current_time() == ref["time"]
    assert_bitwise(sim.get_current_grid(), ref, "max_time_cap")
    # run_until
    sim = make_sim(16, 12, 0, 1, fp64, dt=0.1)
    sim.set_initial_condition(ws.ZonalFlowInitialCondition())
    sim.initialize()
    for snap, t in (("a", 0.5), ("b", 0.55), ("c", 1.25)):
        sim.run_until(t)
        ref = gold.snap("api/run_until", snap)
        assert sim.get_current_step() == ref["step"], snap
        assert sim.get_current_time() == ref["time"]
        assert_bitwise(sim.get_current_grid(), ref, f"run_until {snap}")
    # alternation of p/T/q between the two grids; PE T/P drift
    for model in (0, 2):
        sim = make_sim(16, 12, model, 0, fp64)
        sim.set_initial_condition(ws.UniformInitialCondition(1.0, 0.5, 10.0, 1000.0, 300.0, 0.25))
        sim.initialize()
        for snap in "abc":
            sim.step()
            assert_bitwise(sim.get_current_grid(), gold.snap(f"api/alternation_m{model}", snap), f"alt m{model} {snap}")
    # stale handle
    sim = make_sim(16, 12, 0, 2, fp64)
    sim.set_initial_condition(ws.BreakingWaveInitialCondition())
    sim.initialize()
    sim.step()
    sim.step()
    held = sim.get_current_grid()
    assert_bitwise(held, gold.snap("api/stale_handle", "a"), "stale a")
    sim.step()
    assert_bitwise(held, gold.snap("api/stale_handle", "b"), "stale b")
    assert_bitwise(sim.get_current_grid(), gold.snap("api/stale_handle", "c"), "stale c")
    sim.step()
    assert_bitwise(held, gold.snap("api/stale_handle", "d"), "stale d")
    # set_dt mid-run
    sim = make_sim(16, 12, 0, 2, fp64)
    sim.set_initial_condition(ws.JetStreamInitialCondition())
    sim.initialize()
    for _ in range(3):
        sim.step()
    sim.set_dt(0.02)
    for _ in range(4):
        sim.step()
    ref = gold.snap("api/set_dt", "a")
    assert sim.get_current_time() == ref["time"]
    assert_bitwise(sim.get_current_grid(), ref, "set_dt")
    # re-initialize after stepping
    sim = make_sim(16, 12, 0, 0, fp64)
    sim.set_initial_condition(ws.UniformInitialCondition(1.0, 0.5, 10.0, 1000.0, 300.0, 0.25))
    sim.initialize()
    sim.run(3)
    sim.initialize()
    sim.step()
    assert_bitwise(sim.get_current_grid(), gold.snap("api/reinit", "a"), "reinit a")
    sim.step()
    assert_bitwise(sim.get_current_grid(), gold.snap("api/reinit", "b"), "reinit b")


def test_wrapper_snapshots_and_errors():
    w = ws.WeatherSimulationWrapper(48, 32, integration_method="rk4", output_interval=5)
    w.set_initial_condition("breaking_wave")
    for _ in range(10):
        w.step()
    out = w.get_output_data()
    assert [o["step"] for o in out] == [5, 10]
    ref = golden("f32").snap("step/m0_i2_breaking_wave", "s10")
    np.testing.assert_array_equal(out[1]["u"], ref["u"])
    np.testing.assert_array_equal(out[1]["vorticity"], ref["vort"])
    g = w.get_grid()
    with pytest.raises(RuntimeError):
        g.set_height_field(np.zeros((3, 3), np.float32))
    with pytest.raises(RuntimeError):
        g.set_height_field(np.zeros(48 * 32, np.float32))
    with pytest.raises(ValueError):
        g.set_spacing(0.0, 1.0)
    with pytest.raises(ValueError):
        ws.WeatherGrid(0, 10)
    m = w.get_metrics()
    assert m.num_steps == 10 and m.compute_time_ms > 0


def test_kernel_adapter_step():
    """The KernelAdapter plugin API (gpu_adaptability.hpp:242-329): executeShallowWaterStep on
    two grids == the reference Euler step; the raw-pointer launchers are covered by
    tests/test_gpu_raw_abi.py."""
    gold = golden("f32")
    s0 = gold.snap("step/m0_i0_jet_stream", "s0")
    s1 = gold.snap("step/m0_i0_jet_stream", "s1")
    a = ws.KernelAdapterFactory.get_instance().get_best_adapter()
    assert a.get_name() == "HIPAdapter"
    gin, gout = ws.WeatherGrid(48, 32), ws.WeatherGrid(48, 32)
    gin.set_velocity_field(s0["u"], s0["v"])
    gin.set_height_field(s0["h"])
    ms = a.execute_shallow_water_step(gin, gout, 0.01)
    assert ms >= 0
    u, v = gout.get_velocity_field()
    np.testing.assert_array_equal(u, s1["u"])
    np.testing.assert_array_equal(v, s1["v"])
    np.testing.assert_array_equal(gout.get_height_field(), s1["h"])
    np.testing.assert_array_equal(gout.get_vorticity_field(), s1["vort"])


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("entry,case", [("execute_shallow_water_step", "step/m0_i0_jet_stream"),
                                        ("execute_barotropic_step", "step/m1_i0_breaking_wave"),
                                        ("execute_primitive_equations_step", "step/m2_i0_jet_stream"),
                                        ("execute_gcm_step", "step/m0_i0_jet_stream")])
def test_kernel_adapter_entry_points(entry, case, precision):
    """Every KernelAdapter step entry point (gpu_adaptability.hpp:242-329) against the
    reference's Euler step of that model (its s0 -> s1 fixture), bitwise in both precisions:
    u, v, h and the vorticity diagnostic, and for the primitive-equations entry the T / P
    update with the reference's stale tendencies (+ dt 288.15, + dt 1013.25). The steps run
    the fused one-step kernel; repeated calls reuse the grid's timing events."""
    gold = golden(precision)
    s0, s1 = gold.snap(case, "s0"), gold.snap(case, "s1")
    H, W = s0["u"].shape
    a = ws.KernelAdapterFactory.get_instance().get_best_adapter()
    fp64 = precision == "f64"
    gin, gout = ws.WeatherGrid(W, H, double_precision=fp64), ws.WeatherGrid(W, H, double_precision=fp64)
    gin.set_velocity_field(s0["u"], s0["v"])
    gin.set_height_field(s0["h"])
    gin.set_pressure_field(s0["p"])
    gin.set_temperature_field(s0["t"])
    for _ in range(3):  # the same result every call
        ms = getattr(a, entry)(gin, gout, 0.01)
        assert ms >= 0
        got = state(gout)
        for k in ("u", "v", "h", "vort"):
            np.testing.assert_array_equal(got[k], s1[k], err_msg=f"{entry} {precision} {k}")
        if entry == "execute_primitive_equations_step":
            np.testing.assert_array_equal(got["t"], s1["t"], err_msg="T drift")
            np.testing.assert_array_equal(got["p"], s1["p"], err_msg="P drift")


def _digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _dam_break(W, H, width_cells, dtype):
    x = np.arange(W, dtype=np.float64)
    row = 10.0 + 0.5 * (1.0 - np.tanh((x - W / 2) / width_cells))
    return np.broadcast_to(row, (H, W)).astype(dtype)


@pytest.mark.parametrize("tb", ["1", "2", "4", "x2y4", "pc", "pc2", "chain"])
@pytest.mark.parametrize("name", ["C1_dam_break_256_i0_f32", "C1_dam_break_256_i2_f32", "C2_dam_break_4096_i2_f64",
                                  "C2_dam_break_4096_i0_f64", "C2_jet_stream_4096_i2_f64",
                                  "C3_zonal_flow_2048_baro_f32"])
def test_full_size_digests(name, tb, monkeypatch):
    """Full-size reference digests; tb = 2 pins the two-step launches (dppy) at full size, 4 /
    x2y4 the four-step launches of dppy / x2y (Euler / RK2 cases; two steps for RK4), pc / pc2
    the producer / consumer split of the two-step march (one column / a column pair per lane)."""
    if tb in ("2", "4", "x2y4", "pc", "pc2", "chain"):
        monkeypatch.setenv("WS_KERNEL", tb if tb in ("pc", "pc2") else "x2y" if tb == "x2y4" else "dppy")
        monkeypatch.setenv("WS_TB", "4" if tb in ("4", "x2y4") else "2")
    if tb == "chain":  # the chain schedule, one chain per SIMD
        monkeypatch.setenv("WS_SEG_ROWS", "-2")
    d = large_digests()[name]
    spec = {k: v for k, v in (l.split()[1:3] for l in d["spec"] if l.startswith("cfg "))}
    W, H = int(spec["width"]), int(spec["height"])
    fp64 = d["variant"] == "f64"
    sim = make_sim(W, H, int(spec["model"]), int(spec["method"]), fp64, max_time=float(spec["max_time"]))
    ic = [l for l in d["spec"] if l.startswith("ic ")]
    if ic:
        name_ic = ic[0].split()[1]
        sim.set_initial_condition({"jet_stream": ws.JetStreamInitialCondition,
                                   "zonal_flow": ws.ZonalFlowInitialCondition}[name_ic]())
    sim.initialize()
    if not ic:
        sim.get_current_grid().set_height_field(_dam_break(W, H, 8.0 if W == 256 else 128.0,
                                                           np.float64 if fp64 else np.float32))
    steps = int([l for l in d["spec"] if l.startswith("run ")][0].split()[1])
    assert sim.run(steps) == d["step"]
    g = sim.get_current_grid()
    got = state(g)
    for k, h in d["sha256"].items():
        if _digest(got[k]) != h:
            ref_l2 = d["l2"][k]
            pytest.fail(f"{name}: {k} digest mismatch (|got|={np.linalg.norm(got[k].astype(np.float64))!r} "
                        f"|ref|={ref_l2!r})")


LONG_CASE = "C2_jet_stream_4096_i2_f64_240"


@pytest.mark.parametrize("kernel", [None, "dppy", "pc", "pc2", "dppy-chain"])
def test_long_horizon_benched_workload(kernel, monkeypatch):
    """The benched workload (bench.py c2: 4096^2 fp64 jet_stream RK4) pinned to the reference
    over a long horizon (tests/golden/gen_golden.py --long: 240 steps, 120 two-step launches):
    exact numerics bitwise, and the default fast numerics (what the bench times) within the
    north_star tolerance of 1e-10 relative L2 per field of that exact (= reference) state.
    kernel None = the autotuned choice; else a pinned two-step variant (-chain: on the chain
    schedule, one chain per SIMD)."""
    if kernel:
        monkeypatch.setenv("WS_KERNEL", kernel.replace("-chain", ""))
        monkeypatch.setenv("WS_TB", "2")
        if kernel.endswith("-chain"):
            monkeypatch.setenv("WS_SEG_ROWS", "-2")
    d = large_digests()[LONG_CASE]
    steps = int([l for l in d["spec"] if l.startswith("run ")][0].split()[1])
    runs = {}
    for numerics in ("exact", "fast"):
        sim = make_sim(4096, 4096, 0, 2, True, max_time=1e30)
        sim.set_numerics(numerics)
        sim.set_initial_condition(ws.JetStreamInitialCondition())
        sim.initialize()
        assert sim.run(steps) == d["step"] == steps
        g = sim.get_current_grid()
        u, v = g.get_velocity_field()
        runs[numerics] = {"u": u, "v": v, "h": g.get_height_field(), "vort": g.get_vorticity_field()}
        del sim
    for k, h in d["sha256"].items():
        assert _digest(runs["exact"][k]) == h, f"{LONG_CASE}: exact {k} differs from the reference"
    for k in ("u", "v", "h"):
        ex, fa = runs["exact"][k], runs["fast"][k]
        rel = float(np.linalg.norm(fa - ex) / np.linalg.norm(ex))
        assert rel <= 1e-10, f"{LONG_CASE}: fast {k} relative L2 {rel:.3e} > 1e-10"


@pytest.mark.parametrize("kernel,tb", [(None, "0"), ("dppy", "2"), ("x2y", "2"), ("pc", "2"), ("pc2", "2")])
def test_pe_levels_match_reference_per_level(kernel, tb, monkeypatch):
    """C4: PE 1024^2 x 32 levels, level k = jet_stream(strength 10(1+k/32)); each level
    must equal a standalone reference run of that level (bitwise) -- the T / P update on
    the second stream, with the autotuned kernel and with two steps per launch (every
    two-step variant, two T / P updates per launch)."""
    if kernel:
        monkeypatch.setenv("WS_KERNEL", kernel)
        monkeypatch.setenv("WS_TB", tb)
    digests = large_digests()
    L = 32
    sim = make_sim(1024, 1024, 2, 2, False, max_time=1e30, levels=L)
    sim.initialize()
    g = sim.get_current_grid()
    for k in range(L):
        ws.JetStreamInitialCondition(0.5, 0.1, 10.0 * (1.0 + k / 32.0), 10.0).initialize(g, level=k)
    sim.run(10)
    g = sim.get_current_grid()
    for k in (0, 7, 31):
        d = digests[f"C4_pe_1024_level{k}_f32"]
        got = state(g, level=k)
        for f, h in d["sha256"].items():
            assert _digest(got[f]) == h, (k, f)


@pytest.mark.parametrize("kernel,tb", FUSED, ids=FUSED_IDS)
@pytest.mark.parametrize("seg_rows", ["0", "5", "33", "-2", "-4"])
@pytest.mark.parametrize("method", [0, 1, 2])
@pytest.mark.parametrize("fp64", [False, True])
def test_fused_tiling_vs_oracle(fp64, method, seg_rows, kernel, tb, monkeypatch):
    """Strip (x) and segment (y) seams of the fused kernel: 700 x 77 grid spans three
    256-lane strips and (with WS_SEG_ROWS) many ragged segments; bitwise vs the oracle.
    seg_rows -2 / -4: the chain schedule (1 / 3 chains per SIMD, chains of
    cost-balanced lengths, y-clamped chains shorter)."""
    from oracle.ws_oracle import OracleSim

    monkeypatch.setenv("WS_SEG_ROWS", seg_rows)
    monkeypatch.setenv("WS_KERNEL", kernel)
    monkeypatch.setenv("WS_TB", tb)
    W, H = 700, 77
    sim = make_sim(W, H, 0, method, fp64, dx=1.0, dy=2.0, f=0.3)
    sim.set_initial_condition(ws.BreakingWaveInitialCondition(1.5, 0.05, 10.0))
    sim.initialize()
    g = sim.get_current_grid()
    ref = OracleSim(W, H, 0, method, dx=1.0, dy=2.0, coriolis_f=0.3, precision="f64" if fp64 else "f32")
    ref.initialize()
    u, v = g.get_velocity_field()
    for k, a in (("u", u), ("v", v), ("h", g.get_height_field())):
        ref.set_field(k, a)
    sim.run(6)
    ref.run(6)
    g = sim.get_current_grid()
    got = state(g)
    for k in ("u", "v", "h", "vort"):
        np.testing.assert_array_equal(got[k], ref.get_field(k), err_msg=k)


_LARGE_REF = {}


@pytest.mark.parametrize("kernel,tb", FUSED, ids=FUSED_IDS)
@pytest.mark.parametrize("case", ["rk4_f64", "rk2_f32"])
def test_every_variant_large_grid_vs_oracle(case, kernel, tb, monkeypatch):
    """Every variant pinned at a grid large enough that late-dispatched workgroups run
    beside finished ones (4096 x 2048, segments of 64 rows): a 16-byte store data hazard
    corrupted fused_x2y here and never at the small tiling sizes; bitwise vs the oracle."""
    from oracle.ws_oracle import OracleSim

    method, fp64 = (2, True) if case == "rk4_f64" else (1, False)
    monkeypatch.setenv("WS_SEG_ROWS", "64")
    monkeypatch.setenv("WS_KERNEL", kernel)
    monkeypatch.setenv("WS_TB", tb)
    W, H, steps = 4096, 2048, 2
    sim = make_sim(W, H, 0, method, fp64, dx=1.0, dy=1.0, f=1e-4, max_time=1e30)
    sim.set_initial_condition(ws.BreakingWaveInitialCondition(1.5, 0.05, 10.0))
    sim.initialize()
    if case not in _LARGE_REF:
        g = sim.get_current_grid()
        ref = OracleSim(W, H, 0, method, coriolis_f=1e-4, max_time=1e30, precision="f64" if fp64 else "f32")
        ref.initialize()
        u, v = g.get_velocity_field()
        for k, a in (("u", u), ("v", v), ("h", g.get_height_field())):
            ref.set_field(k, a)
        ref.run(steps)
        _LARGE_REF[case] = {k: ref.get_field(k) for k in ("u", "v", "h")}
    sim.run(steps)
    got = state(sim.get_current_grid())
    for k in ("u", "v", "h"):
        bad = np.argwhere(got[k] != _LARGE_REF[case][k])
        assert len(bad) == 0, f"{kernel} {case} {k}: {len(bad)} cells differ, first {bad[:4].tolist()}"


def test_fused_non_pow2_spacing_vs_oracle():
    """dx = 0.75: 2dx is not a power of two -> the IEEE-divide instantiation."""
    from oracle.ws_oracle import OracleSim

    W, H = 300, 40
    sim = make_sim(W, H, 0, 2, False, dx=0.75, dy=1.3)
    sim.set_initial_condition(ws.VortexInitialCondition(0.5, 0.5, 0.3, 3.0, 10.0))
    sim.initialize()
    g = sim.get_current_grid()
    ref = OracleSim(W, H, 0, 2, dx=0.75, dy=1.3)
    ref.initialize()
    u, v = g.get_velocity_field()
    for k, a in (("u", u), ("v", v), ("h", g.get_height_field())):
        ref.set_field(k, a)
    sim.run(4)
    ref.run(4)
    got = state(sim.get_current_grid())
    for k in ("u", "v", "h", "vort"):
        np.testing.assert_array_equal(got[k], ref.get_field(k), err_msg=k)


@pytest.mark.parametrize("kernel,seg_rows,tb", [("dppy", "6", "1"), ("dppy", "0", "1"), ("dppy", "6", "2"),
                                                 ("dppy", "0", "2"), ("x2y", "6", "1"), ("x2y", "0", "1"),
                                                 ("x2y", "6", "2"), ("dppy", "0", "4"), ("x2y", "6", "4"),
                                                 ("pc", "6", "2"), ("pc", "0", "2"), ("pc2", "6", "2"),
                                                 ("lds", "6", "1"), ("lds", "0", "1")])
@pytest.mark.parametrize("nslabs", [2, 3, 5])
@pytest.mark.parametrize("method", [0, 1, 2])
@pytest.mark.parametrize("fp64", [False, True])
def test_slab_group_matches_single_domain(fp64, method, nslabs, kernel, seg_rows, tb, monkeypatch):
    """y-slab decomposition (interior segments, halo exchange, edge segments) == one domain,
    bit-for-bit, for uneven slab heights and several segment sizes (dppy also with two steps
    per launch inside the deep-halo blocks)."""
    monkeypatch.setenv("WS_KERNEL", kernel)
    monkeypatch.setenv("WS_SEG_ROWS", seg_rows)
    monkeypatch.setenv("WS_TB", tb)
    W, H, steps = 300, 83, 7

    def cfg():
        c = ws.SimulationConfig()
        c.grid_width, c.grid_height = W, H
        c.integration_method, c.double_precision = method, fp64
        c.dx, c.dy, c.coriolis_f = 1.0, 2.0, 0.25
        return c

    ic = ws.BreakingWaveInitialCondition(1.5, 0.05, 10.0)
    one = ws.WeatherSimulation(cfg())
    one.set_initial_condition(ic)
    one.initialize()
    group = ws.SlabGroup(cfg(), nslabs)
    group.set_initial_condition(ic)
    group.initialize()
    for name in ("u", "v", "h"):  # the IC evaluated per slab in global coordinates
        np.testing.assert_array_equal(group.gather(name), one.get_current_grid()._get(name), err_msg=f"ic {name}")
    assert group.run(steps) == steps
    one.run(steps)
    g1 = one.get_current_grid()
    for name in ("u", "v", "h", "vorticity", "divergence"):
        np.testing.assert_array_equal(group.gather(name), g1._get(name), err_msg=name)
    assert group.slab(nslabs - 1).get_current_time() == one.get_current_time()


def test_slab_group_levels_and_pe():
    """PE (T/P drift) with 3 levels over 4 slabs == one domain."""
    W, H, L = 130, 40, 3

    def cfg():
        c = ws.SimulationConfig()
        c.grid_width, c.grid_height, c.num_levels = W, H, L
        c.model, c.integration_method = ws.SimulationModel.PrimitiveEquations, ws.IntegrationMethod.RungeKutta4
        return c

    one = ws.WeatherSimulation(cfg())
    one.set_initial_condition(ws.FrontInitialCondition())
    one.initialize()
    group = ws.SlabGroup(cfg(), 4)
    group.set_initial_condition(ws.FrontInitialCondition())
    group.initialize()
    group.run(5)
    one.run(5)
    for name in ("u", "v", "h", "t", "p", "q"):
        np.testing.assert_array_equal(group.gather(name), one.get_current_grid()._get(name), err_msg=name)


@pytest.mark.parametrize("kernel,fp64,method,pin,want", [("x2y", False, 1, 4, 4), ("dppy", False, 0, 4, 4),
                                                         ("dppy", True, 1, 4, 4), ("x2y", True, 1, 4, 2),
                                                         ("dppy", False, 2, 4, 2), ("pc", False, 1, 4, 2),
                                                         ("x2y", False, 0, 8, 8), ("dppy", True, 0, 8, 8),
                                                         ("dppy", True, 1, 8, 4)])
def test_four_step_launches(kernel, fp64, method, pin, want, monkeypatch):
    """WS_TB=4 / 8: four steps per launch where the kernel takes them (Euler / RK2 on dppy, x2y
    in fp32), eight for Euler, else the largest it takes; run(n) splits n greedily into 8-, 4-,
    2- and 1-step launches, and the result is bit-for-bit the one-step run (ws_schedule.cpp
    launch_of)."""
    monkeypatch.setenv("WS_KERNEL", kernel)
    monkeypatch.setenv("WS_TB", str(pin))
    sim = make_sim(300, 83, 0, method, fp64)
    sim.set_initial_condition(ws.JetStreamInitialCondition())
    sim.initialize()
    assert sim.run(11) == 11
    assert sim.steps_per_launch() == want
    _, launches = sim.last_run_stats()
    expect, left = 0, 11
    for k in (8, 4, 2, 1):
        if k <= want:
            expect += left // k
            left %= k
    assert launches == expect
    monkeypatch.setenv("WS_KERNEL", "dppy")
    monkeypatch.setenv("WS_TB", "1")
    ref = make_sim(300, 83, 0, method, fp64)
    ref.set_initial_condition(ws.JetStreamInitialCondition())
    ref.initialize()
    ref.run(11)
    got, exp = state(sim.get_current_grid()), state(ref.get_current_grid())
    for k in ("u", "v", "h", "vort"):
        np.testing.assert_array_equal(got[k], exp[k], err_msg=k)


@pytest.mark.parametrize("tb", ["1", "2", "4"])
@pytest.mark.parametrize("fail_after", [1, 2])
def test_pe_drift_on_a_failed_run(fail_after, tb, monkeypatch):
    """A run that fails after some launches (ws_sim_inject_failure) leaves a consistent state:
    T / P carry exactly the drift of the steps the completed launches took (== that many
    step() calls, bit for bit), and nothing pending lands later -- neither on a following run
    nor on fields reset by initialize()."""
    monkeypatch.setenv("WS_KERNEL", "x2y")
    monkeypatch.setenv("WS_TB", tb)
    sims = []
    for _ in range(3):
        sim = make_sim(200, 72, 2, 1, False, levels=3, max_time=1e30)
        sim.set_initial_condition(ws.JetStreamInitialCondition())
        sim.initialize()
        sims.append(sim)
    a, b, c = sims
    assert a.run(2) == 2
    ws._native.check(ws._native.lib.ws_sim_inject_failure(a._h, fail_after))
    with pytest.raises(ws._native.WsDeviceError, match="injected"):
        a.run(11)
    k = a.get_current_step()
    assert 2 < k < 13
    for _ in range(k):
        b.step()
    assert b.get_current_time() == a.get_current_time()
    ga, gb = a.get_current_grid(), b.get_current_grid()
    for get in ("get_temperature_field", "get_pressure_field", "get_height_field", "get_velocity_field"):
        np.testing.assert_array_equal(getattr(ga, get)(), getattr(gb, get)(), err_msg=get)
    # a later run continues from there exactly
    assert a.run(5) == 5
    for _ in range(5):
        b.step()
    for get in ("get_temperature_field", "get_pressure_field", "get_height_field"):
        np.testing.assert_array_equal(getattr(a.get_current_grid(), get)(), getattr(b.get_current_grid(), get)(),
                                      err_msg=get)
    # a failed run followed by initialize(): no drift of the failed run reaches the reset fields
    ws._native.check(ws._native.lib.ws_sim_inject_failure(a._h, fail_after))
    with pytest.raises(ws._native.WsDeviceError):
        a.run(9)
    a.initialize()
    assert a.run(4) == c.run(4) == 4
    for get in ("get_temperature_field", "get_pressure_field", "get_height_field"):
        np.testing.assert_array_equal(getattr(a.get_current_grid(), get)(), getattr(c.get_current_grid(), get)(),
                                      err_msg=get)


@pytest.mark.parametrize("tb", ["1", "2", "4"])
@pytest.mark.parametrize("k", [1, 3, 7, 12])
def test_pe_drift_once_per_run(k, tb, monkeypatch):
    """PE T / P: run(k) applies the k steps' drift in one pass at its end (ws_schedule.cpp
    tp_flush); the current grid's T and P equal k single step() calls bit for bit, with one-,
    two- and four-step launches (fp32, RK2: the four-step kernel)."""
    monkeypatch.setenv("WS_KERNEL", "x2y")
    monkeypatch.setenv("WS_TB", tb)
    sims = []
    for _ in range(2):
        sim = make_sim(200, 72, 2, 1, False, levels=3)
        sim.set_initial_condition(ws.JetStreamInitialCondition())
        sim.initialize()
        sims.append(sim)
    assert sims[0].run(k) == k
    for _ in range(k):
        sims[1].step()
    a, b = sims[0].get_current_grid(), sims[1].get_current_grid()
    for get in ("get_temperature_field", "get_pressure_field", "get_height_field"):
        np.testing.assert_array_equal(getattr(a, get)(), getattr(b, get)(), err_msg=get)


def test_cpu_backend_runs_hip_with_one_warning(monkeypatch):
    """ComputeBackend.CPU (the reference's own tests request it) runs the HIP path:
    same bits as the CUDA backend, and one RuntimeWarning per process saying so (D8)."""
    from weather_sim import weather_simulation as wsm
    monkeypatch.setattr(wsm, "_CPU_WARNED", [])
    out = []
    for backend in (ws.ComputeBackend.CUDA, ws.ComputeBackend.CPU, ws.ComputeBackend.CPU):
        c = ws.SimulationConfig()
        c.grid_width, c.grid_height = 64, 48
        c.compute_backend = backend
        import warnings
        with warnings.catch_warnings(record=True) as rec:
            warnings.simplefilter("always")
            sim = ws.WeatherSimulation(c)
        out.append(sum(issubclass(w.category, RuntimeWarning) and "CPU" in str(w.message) for w in rec))
        sim.set_initial_condition(ws.VortexInitialCondition())
        sim.initialize()
        sim.run(7)
        out.append(sim.get_current_grid().get_height_field())
    assert out[0] == 0 and out[2] == 1 and out[4] == 0
    assert np.array_equal(out[1], out[3]) and np.array_equal(out[1], out[5])
