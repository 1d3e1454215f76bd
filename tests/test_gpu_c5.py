"""C5 (BASELINE configs[4]): Shallow Water 16384 x 16384 fp64 RK4 at full size, pinned
bit-for-bit to the reference.

Fixtures (tests/golden/gen_c5_bands.py): the reference solver evaluates each initial
condition on the full 16384^2 grid and runs halo-extended row bands -- exact on the compared
rows by the stencil's dependency cone (4 rows per RK4 step, clamp-to-self edges,
weather_simulation.cpp:510-513) -- and stores SHA-256 digests of u, v, h and the vorticity on
64 compared rows per band. ref_c5_bands50.json: C5's benchmark length, 50 steps (200-row cone
margins), bands at the global top and bottom and at EVERY seam of the 8-way split (rows
2048 k +- 32, k = 1..7); ref_c5_bands.json (round 2): 4 steps, top / bottom / rows 2048 and
8192.

Here the whole grid runs on one GPU (~34 GB of fields: 64-bit element offsets, buffer
segments far past 2^31 bytes from the field base), with one-step and two-step launches, and
as the 8-slab decomposition C5 names (the RCCL path's halo plan with device-copy
transport); each must reproduce every band digest. Fast numerics (the fp64 default) must
stay within the north_star tolerance of the exact run on the full grid.
"""
import gc
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

ws = pytest.importorskip("weather_sim")
if not ws.is_cuda_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

TOL = 1e-10  # relative L2 per field, fp64 (BASELINE.json north_star)


def _fixtures(name="ref_c5_bands50.json"):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def _cfg(fx):
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height = fx["width"], fx["height"]
    c.integration_method = ws.IntegrationMethod.RungeKutta4
    c.double_precision = True
    c.max_time = 1e30
    return c


def _ic(name):
    return {"jet_stream": lambda: ws.JetStreamInitialCondition(),
            "random": lambda: ws.RandomInitialCondition(42, 1.0)}[name]()


def _check_bands(fx, ic, fields):
    checked = 0
    for case, ref in fx["cases"].items():
        if not case.startswith(ic + "/"):
            continue
        y0, y1 = ref["rows"]
        for f, want in ref["sha256"].items():
            got = np.ascontiguousarray(fields[f][y0:y1])
            if hashlib.sha256(got.tobytes()).hexdigest() != want:
                pytest.fail(f"C5 {case} {f}: digest mismatch (|got| = {np.linalg.norm(got)!r}, "
                            f"|ref| = {ref['l2'][f]!r})")
            checked += 1
    assert checked == 4 * sum(c.startswith(ic + "/") for c in fx["cases"]) > 0, checked


def _fields(grid):
    u, v = grid.get_velocity_field()
    return {"u": u, "v": v, "h": grid.get_height_field(), "vort": grid.get_vorticity_field()}


@pytest.mark.parametrize("ic,kernel,tb,fixture", [("jet_stream", None, None, "ref_c5_bands50.json"),
                                                  ("jet_stream", None, None, "ref_c5_bands.json"),
                                                  ("random", "dppy", "1", "ref_c5_bands50.json"),
                                                  ("random", "dppy", "2", "ref_c5_bands50.json"),
                                                  ("random", "x2y", "2", "ref_c5_bands50.json"),
                                                  ("random", "pc", "2", "ref_c5_bands50.json"),
                                                  ("random", "pc2", "2", "ref_c5_bands50.json")])
def test_c5_single_gpu_matches_reference_bands(ic, kernel, tb, fixture, monkeypatch):
    if tb:
        monkeypatch.setenv("WS_KERNEL", kernel)
        monkeypatch.setenv("WS_TB", tb)
    fx = _fixtures(fixture)
    sim = ws.WeatherSimulation(_cfg(fx))
    sim.set_initial_condition(_ic(ic))
    sim.initialize()
    assert sim.run(fx["steps"]) == fx["steps"]
    _check_bands(fx, ic, _fields(sim.get_current_grid()))
    del sim
    gc.collect()


@pytest.mark.parametrize("overlap", ["off", "on"])
def test_c5_eight_slabs_match_reference_bands(overlap):
    """C5's decomposition: 8 y-slabs of 2048 rows (deep-halo blocks, the library's exchange
    plan, stream-ordered and overlapped), the global initial state scattered into them, 50
    steps against the reference's bands at every seam."""
    fx = _fixtures()
    one = ws.WeatherSimulation(_cfg(fx))
    one.set_initial_condition(_ic("random"))
    one.initialize()
    g = one.get_current_grid()
    init = {name: g._get(name) for name in ("u", "v", "h")}
    del one, g
    gc.collect()
    group = ws.SlabGroup(_cfg(fx), 8)
    group.set_slab_schedule(6, overlap)
    group.initialize()
    for name, a in init.items():
        group.scatter(name, a)
    del init
    assert group.run(fx["steps"]) == fx["steps"]
    got = {"u": group.gather("u"), "v": group.gather("v"), "h": group.gather("h"), "vort": group.gather("vorticity")}
    del group
    gc.collect()
    _check_bands(fx, "random", got)


@pytest.mark.parametrize("ic", ["jet_stream", "random"])
def test_c5_fast_numerics_within_tolerance(ic, monkeypatch):
    """The fp64 default (fast numerics) against the exact run, which the band digests pin to
    the reference: relative L2 per field over the full 16384^2 grid."""
    fx = _fixtures()
    out = {}
    for mode in ("exact", "fast"):
        monkeypatch.setenv("WS_NUMERICS", mode)
        sim = ws.WeatherSimulation(_cfg(fx))
        sim.set_initial_condition(_ic(ic))
        sim.initialize()
        sim.run(fx["steps"])
        out[mode] = _fields(sim.get_current_grid())
        del sim
        gc.collect()
    for f in ("u", "v", "h"):
        want = out["exact"][f]
        n = np.linalg.norm(want)
        e = float(np.linalg.norm(out["fast"][f] - want) / (n if n > 0 else 1.0))
        assert e <= TOL, (ic, f, e)
