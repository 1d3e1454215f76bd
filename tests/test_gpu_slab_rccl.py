"""The RCCL slab path (ws_sim_create_slab) on one GPU: a 1-rank communicator goes through
the same bootstrap, step_begin/step_end, end-of-run halo refresh and collectives as an
N-rank job (the exchanges are no-ops), and must equal the plain single-domain simulation
bit-for-bit. The N-rank seam logic itself is covered by test_slab_group_* (same kernels,
same segment split, device-copy transport) and by tests/test_slab_protocol.py (gloo).
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ws = pytest.importorskip("weather_sim")
if not ws.is_cuda_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from weather_sim import _native  # noqa: E402


def _uid():
    buf = (ctypes.c_uint8 * _native.COMM_ID_BYTES)()
    _native.check(_native.lib.ws_comm_get_unique_id(buf))
    return bytes(buf)


@pytest.mark.parametrize("method", [0, 1, 2])
@pytest.mark.parametrize("fp64", [False, True])
def test_one_rank_rccl_slab_matches_single_domain(method, fp64):
    def cfg():
        c = ws.SimulationConfig()
        c.grid_width, c.grid_height = 200, 61
        c.integration_method, c.double_precision = method, fp64
        c.dx, c.dy, c.coriolis_f = 1.0, 2.0, 0.25
        return c

    ic = ws.VortexInitialCondition()
    one = ws.WeatherSimulation(cfg())
    one.set_initial_condition(ic)
    one.initialize()
    slab = ws.WeatherSimulation(cfg(), _slab=(0, 1, _uid()))
    assert (slab.row0, slab.rows) == (0, 61)
    slab.set_initial_condition(ic)
    slab.initialize()
    one.run(9)
    slab.run(9)
    for name in ("u", "v", "h", "vorticity", "divergence"):
        np.testing.assert_array_equal(slab.get_current_grid()._get(name), one.get_current_grid()._get(name),
                                      err_msg=name)
    assert slab.comm_allreduce_max(3.5) == 3.5
    slab.comm_barrier()


def test_public_slab_simulation_api():
    """The public form of a rank (weather_sim.SlabSimulation + new_comm_id; no bench.py
    helpers, no private kwargs): one rank of one, equal to one domain."""
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.integration_method = 128, 40, 2
    one = ws.WeatherSimulation(c)
    slab = ws.SlabSimulation(c, 0, 1, ws.new_comm_id())
    assert (slab.rank, slab.nranks, slab.row0, slab.rows) == (0, 1, 0, 40)
    for s in (one, slab):
        s.set_initial_condition(ws.JetStreamInitialCondition())
        s.initialize()
        assert s.run(6) == 6
    np.testing.assert_array_equal(slab.get_current_grid().get_height_field(), one.get_current_grid().get_height_field())
    with pytest.raises(ValueError):
        ws.SlabSimulation(c, 0, 1, b"short")


@pytest.mark.parametrize("block", ["1", "2", "3"])
@pytest.mark.parametrize("kernel", ["dppy", "x2y", "lds"])
@pytest.mark.parametrize("method", [0, 1, 2])
def test_slab_blocks_are_bitwise(block, kernel, method, monkeypatch):
    """Slabs advance `block` steps per halo exchange (block x NST halo rows, steps computed
    on rows extended into the halo): 4 slabs == one domain bit-for-bit for every block
    size, kernel and integrator, over a run that ends mid-block."""
    monkeypatch.setenv("WS_KERNEL", kernel)

    def cfg():
        c = ws.SimulationConfig()
        c.grid_width, c.grid_height = 150, 61
        c.integration_method, c.double_precision = method, True
        c.dx, c.dy, c.coriolis_f = 1.0, 2.0, 0.25
        return c

    ic = ws.BreakingWaveInitialCondition(1.5, 0.05, 10.0)
    one = ws.WeatherSimulation(cfg())
    one.set_initial_condition(ic)
    one.initialize()
    group = ws.SlabGroup(cfg(), 4)
    group.set_slab_schedule(int(block), "off")
    group.set_initial_condition(ic)
    group.initialize()
    for n in (7, 2):  # 7 = two blocks of 3 + one step; a second run starts a new block
        assert group.run(n) == n
        one.run(n)
    g1 = one.get_current_grid()
    for name in ("u", "v", "h", "vorticity", "divergence"):
        np.testing.assert_array_equal(group.gather(name), g1._get(name), err_msg=name)
