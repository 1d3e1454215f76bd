"""Pin the CPU oracle (oracle/ws_oracle.c) to the reference's own outputs.

Every stepping case in tests/golden/ref_small_{f32,f64}.npz was produced by the reference
solver (weather_simulation.cpp) itself; the oracle must reproduce each one bit-for-bit
(max-ulp 0) in both precisions before it may be trusted as the checker for the HIP path.
"""
import numpy as np
import pytest

from conftest import golden
from oracle.ws_oracle import OracleSim, tendency

FIELDS = ("u", "v", "h", "p", "t", "q", "vort")


def _mk(gold, cfg):
    kw = dict(dx=cfg.get("dx", 1.0), dy=cfg.get("dy", 1.0), dt=cfg.get("dt", 0.01), gravity=cfg.get("g", 9.81),
              coriolis_f=cfg.get("f", 0.0))
    return OracleSim(cfg["width"], cfg["height"], cfg["model"], cfg["method"], precision=gold.variant, **kw)


def _load_state(sim, s0):
    sim.initialize()
    for k in ("u", "v", "h", "p", "t", "q"):
        sim.set_field(k, s0[k])
    sim.calculate_diagnostics()


def _assert_bitwise(sim, ref, case, snap):
    for k in FIELDS:
        got = sim.get_field(k)
        np.testing.assert_array_equal(got, ref[k], err_msg=f"{case} {snap} field {k}")
    assert sim.step_count == ref["step"]
    assert sim.time == ref["time"]


@pytest.mark.parametrize("variant", ["f32", "f64"])
def test_oracle_stepping_matches_reference(variant):
    gold = golden(variant)
    cases = gold.cases("step/")
    assert len(cases) >= 20
    for case in cases:
        cfg = gold.meta[case]["cfg"]
        sim = _mk(gold, cfg)
        _load_state(sim, gold.snap(case, "s0"))
        sim.step()
        _assert_bitwise(sim, gold.snap(case, "s1"), case, "s1")
        sim.run(9)
        _assert_bitwise(sim, gold.snap(case, "s10"), case, "s10")
        sim.run(40)
        _assert_bitwise(sim, gold.snap(case, "s50"), case, "s50")


@pytest.mark.parametrize("variant", ["f32", "f64"])
def test_oracle_api_behaviour(variant):
    gold = golden(variant)
    dt = np.float32 if variant == "f32" else np.float64
    # run(2000) stops at t >= max_time (10.0): 1000 steps, t = 10.000134 in fp32
    ref = gold.snap("api/max_time_cap", "end")
    s = OracleSim(16, 12, 0, 0, precision=variant)
    s.initialize()
    assert s.run(2000) == ref["step"] == (1000 if variant == "f32" else 1001)  # fp64 sum(0.01) < 10 at 1000
    assert dt(s.time) == dt(ref["time"])
    # run_until(0.5) at dt=0.1 -> int(0.5/0.1)+1 = 6 steps; (0.55) -> 0; (1.25) -> int(0.65/0.1)+1
    ref_a = gold.snap("api/run_until", "a")
    s = OracleSim(16, 12, 0, 1, dt=0.1, precision=variant)
    s.initialize()
    assert s.run_until(0.5) == ref_a["step"] == 6
    assert dt(s.time) == dt(ref_a["time"])
    assert s.run_until(0.55) == gold.snap("api/run_until", "b")["step"] - 6
    s.run_until(1.25)
    assert s.step_count == gold.snap("api/run_until", "c")["step"]
    assert dt(s.time) == dt(gold.snap("api/run_until", "c")["time"])


@pytest.mark.parametrize("variant", ["f32", "f64"])
def test_oracle_alternation_and_pe_drift(variant):
    gold = golden(variant)
    for model in (0, 2):
        case = f"api/alternation_m{model}"
        sim = OracleSim(16, 12, model, 0, precision=variant)
        sim.initialize()
        # the IC (uniform 1, .5, 10, 1000, 300, .25) as it stood before step 1
        H, W = 12, 16
        c = np.ones((H, W), sim.dtype)
        for k, val in (("u", 1.0), ("v", 0.5), ("h", 10.0), ("p", 1000.0), ("t", 300.0), ("q", 0.25)):
            sim.set_field(k, c * sim.dtype(np.float32(val)))
        for snap in "abc":
            sim.step()
            ref = gold.snap(case, snap)
            for k in FIELDS:
                np.testing.assert_array_equal(sim.get_field(k), ref[k], err_msg=f"{case} {snap} {k}")


def test_oracle_tendency_uniform_is_zero():
    # reference gtest Step (weather_simulation_test.cpp:107-122) expects motion on a
    # uniform field; the centred difference of a constant is exactly 0
    u = np.ones((8, 8), np.float32)
    du, dv, dh = tendency(u, u * 0, u * 10)
    assert not du.any() and not dv.any() and not dh.any()
