"""The reference per-slab digests bench.py's self-check compares against
(tests/golden/ref_slab_digests.json: C2 jet_stream, SWE 4096^2 fp64 RK4, 13 steps), checked
on the GPU: the slab group (one process, device-copy transport; the same per-rank schedule as
the RCCL path) at 2 / 4 / 8 slabs, stream-ordered and overlapped, every slab's owned rows
bit-for-bit; and bench.self_check itself on one domain (exact == reference, fast numerics
within 1e-10 relative L2)."""
import json
import os

import pytest

pytestmark = pytest.mark.gpu

ws = pytest.importorskip("weather_sim")
if not ws.is_cuda_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

import bench  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
with open(os.path.join(ROOT, "tests", "golden", "ref_slab_digests.json")) as f:
    GOLD = json.load(f)


def _cfg():
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height = GOLD["grid"]
    c.integration_method = ws.IntegrationMethod.RungeKutta4
    c.double_precision = True
    c.max_time = 1e30
    return c


@pytest.mark.parametrize("overlap", ["0", "1"])
@pytest.mark.parametrize("nslabs", [2, 4, 8])
def test_group_slabs_match_reference_digests(nslabs, overlap, monkeypatch):
    monkeypatch.setenv("WS_SLAB_OVERLAP", overlap)
    group = ws.SlabGroup(_cfg(), nslabs)
    group.set_initial_condition(ws.JetStreamInitialCondition())
    group.initialize()
    assert group.slab(0).slab_schedule() == (6, overlap == "1")
    assert group.run(GOLD["steps"]) == GOLD["steps"]
    for r in range(nslabs):
        s = group.slab(r)
        fields = bench.slab_fields(s)
        want = GOLD["slabs"][str(nslabs)][r]
        assert (s.row0, fields["u"].shape[0]) == (want["row0"], want["rows"])
        assert bench.slab_sha256(fields) == want["sha256"], f"slab {r}"


def test_bench_self_check_one_domain(monkeypatch):
    monkeypatch.delenv("WS_NUMERICS", raising=False)  # the bench's default: fast for fp64
    sim = ws.WeatherSimulation(_cfg())
    assert sim.get_numerics() == "fast"
    verdict, detail = bench.self_check(sim, ws.JetStreamInitialCondition(), None, 0, 1, GOLD)
    assert verdict == "ok", detail
    assert detail["exact"] == "bitwise == reference"
    assert max(detail["fast_rel_l2"].values()) <= 1e-10
    assert 0 < max(detail["fast_rel_l2"].values())  # fast numerics really ran
    assert sim.get_numerics() == "fast"


def test_fresh_overlap_groups_repeatable(monkeypatch):
    """Regression: the overlap grids of a slab are allocated at the first overlapped run; their
    zeroing once ran as a legacy-stream hipMemset, unordered with the (non-blocking) slab
    streams, and raced with the first edge-band launches (seam 0/1 wrong in ~1 of 4 fresh
    4-slab groups). Fresh groups, run at once, several times."""
    monkeypatch.setenv("WS_SLAB_OVERLAP", "1")
    for _ in range(4):
        group = ws.SlabGroup(_cfg(), 4)
        group.set_initial_condition(ws.JetStreamInitialCondition())
        group.initialize()
        assert group.run(GOLD["steps"]) == GOLD["steps"]
        for r in range(4):
            assert bench.slab_sha256(bench.slab_fields(group.slab(r))) == GOLD["slabs"]["4"][r]["sha256"], f"slab {r}"
        del group
