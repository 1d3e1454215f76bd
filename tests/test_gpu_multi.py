"""The one-process multi-GPU simulation (ws_hip.h ws_multi_*, weather_sim.MultiGPUSimulation):
one simulation object over a device list, the drop-in API unchanged.

On the one-GPU box two transports are reachable: devices=[0] runs the RCCL rank path on a
worker thread of the library (a 1-rank communicator: the thread pool, communicator creation
and every collective call of a rank), and devices=[0]*N runs N slabs on device 0 through a
slab group (device-copy halos). Both must be bit-for-bit equal to one domain, and the
C2 case equal to the reference's digest (tests/golden/ref_slab_digests.json)."""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ws = pytest.importorskip("weather_sim")
if not ws.is_cuda_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(W=160, H=96, L=1, method=2, fp64=True, model=0, devices=None):
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.num_levels = W, H, L
    c.model = model
    c.integration_method = method
    c.double_precision = fp64
    c.max_time = 1e30
    c.devices = devices
    return c


def _fields(sim):
    g = sim.get_current_grid()
    u, v = g.get_velocity_field()
    return {"u": u, "v": v, "h": g.get_height_field(), "p": g.get_pressure_field(), "t": g.get_temperature_field(),
            "vort": g.get_vorticity_field()}


def _same(a, b):
    for k in a:
        assert a[k].shape == b[k].shape, k
        assert np.array_equal(a[k], b[k]), f"{k}: {np.count_nonzero(a[k] != b[k])} cells differ"


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0], [0] * 8])
@pytest.mark.parametrize("method,fp64", [(2, True), (2, False), (1, True), (0, False)])
def test_multi_equals_one_domain(devices, method, fp64):
    ic = ws.JetStreamInitialCondition()
    one = ws.WeatherSimulation(_cfg(method=method, fp64=fp64))
    one.set_initial_condition(ic)
    one.initialize()
    multi = ws.MultiGPUSimulation(_cfg(method=method, fp64=fp64), devices=devices)
    assert multi.nslabs == len(devices)
    assert multi.shared_device == (len(devices) > 1)
    multi.set_initial_condition(ic)
    multi.initialize()
    _same(_fields(multi), _fields(one))
    assert multi.run(13) == one.run(13) == 13
    _same(_fields(multi), _fields(one))
    multi.step()
    one.step()
    assert multi.get_current_step() == one.get_current_step() == 14
    assert multi.get_current_time() == one.get_current_time()
    _same(_fields(multi), _fields(one))
    assert multi.get_cfl() == one.get_cfl()


def test_config_devices_dispatch_and_wrapper():
    """WeatherSimulation(config) with config.devices of more than one device is the multi
    simulation; the high-level wrapper takes devices=[...] and its snapshots match."""
    sim = ws.WeatherSimulation(_cfg(devices=[0, 0]))
    assert isinstance(sim, ws.MultiGPUSimulation) and sim.nslabs == 2
    assert type(ws.WeatherSimulation(_cfg(devices=[0]))) is ws.WeatherSimulation  # one device: plain
    a = ws.WeatherSimulationWrapper(width=64, height=48, integration_method="rk4", output_interval=5, devices=[0, 0, 0])
    b = ws.WeatherSimulationWrapper(width=64, height=48, integration_method="rk4", output_interval=5)
    assert isinstance(a.simulation, ws.MultiGPUSimulation)
    for w in (a, b):
        w.set_initial_condition("vortex")
        for _ in range(10):  # step() stores a snapshot every output_interval steps (run() does not)
            w.step()
    assert len(a.get_output_data()) == len(b.get_output_data()) == 2
    for x, y in zip(a.get_output_data(), b.get_output_data()):
        for k in x:
            if isinstance(x[k], np.ndarray):
                assert np.array_equal(x[k], y[k]), k
            else:
                assert x[k] == y[k], k


@pytest.mark.parametrize("devices", [[0], [0, 0, 0, 0]])
def test_multi_run_until_and_fields(devices):
    one = ws.WeatherSimulation(_cfg(W=96, H=64, fp64=False))
    multi = ws.MultiGPUSimulation(_cfg(W=96, H=64, fp64=False), devices=devices)
    rng = np.random.default_rng(5)
    h = (10 + rng.random((64, 96))).astype(np.float32)
    u = rng.standard_normal((64, 96)).astype(np.float32)
    for s in (one, multi):
        s.initialize()
        g = s.get_current_grid()
        g.set_height_field(h)
        g.set_velocity_field(u, -u)
        s.set_dt(0.005)
    assert multi.run_until(0.0625) == one.run_until(0.0625)
    assert multi.get_current_time() == one.get_current_time()
    _same(_fields(multi), _fields(one))
    g = multi.get_current_grid()
    assert (g.get_width(), g.get_height()) == (96, 64)
    with pytest.raises(RuntimeError):
        g.set_height_field(np.zeros((63, 96), np.float32))


def test_multi_pe_levels_random_ic():
    """Multi-level PE (the packed exchange) with the random IC (global RNG order per slab)."""
    cfg = dict(W=72, H=80, L=4, model=2, method=2, fp64=False)
    one = ws.WeatherSimulation(_cfg(**cfg))
    multi = ws.MultiGPUSimulation(_cfg(**cfg), devices=[0, 0, 0])
    for s in (one, multi):
        s.set_initial_condition(ws.RandomInitialCondition(seed=7, amplitude=0.5))
        s.initialize()
    _same(_fields(multi), _fields(one))
    assert multi.run(9) == one.run(9) == 9
    _same(_fields(multi), _fields(one))


@pytest.mark.parametrize("devices", [[0], [0] * 4, [0] * 8])
def test_multi_c2_matches_reference_digest(devices):
    """C2 (4096^2 fp64 jet_stream RK4), 13 steps, exact numerics: the assembled global fields
    hash to the reference's whole-grid digests."""
    with open(os.path.join(ROOT, "tests", "golden", "ref_slab_digests.json")) as f:
        gold = json.load(f)
    W, H = gold["grid"]
    multi = ws.MultiGPUSimulation(_cfg(W=W, H=H), devices=devices)
    multi.set_initial_condition(ws.JetStreamInitialCondition())
    multi.initialize()
    assert multi.run(gold["steps"]) == gold["steps"]
    f = _fields(multi)
    want = gold["slabs"]["1"][0]["sha256"]
    for k in gold["fields"]:
        assert hashlib.sha256(np.ascontiguousarray(f[k]).tobytes()).hexdigest() == want[k], k


def test_multi_errors():
    with pytest.raises(ValueError):
        ws.MultiGPUSimulation(_cfg(), devices=[])
    with pytest.raises(ws._native.WsDeviceError):
        ws.MultiGPUSimulation(_cfg(), devices=[0, 10**6])
    with pytest.raises(ValueError):  # fewer than 4 rows per slab
        ws.MultiGPUSimulation(_cfg(H=12), devices=[0, 0, 0, 0])
    n = ws._native.device_count()
    if n >= 2:  # pragma: no cover - multi-GPU boxes only
        with pytest.raises(ValueError):  # mixed: neither all distinct nor all equal
            ws.MultiGPUSimulation(_cfg(), devices=[0, 0, 1])
