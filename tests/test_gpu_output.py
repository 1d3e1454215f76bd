"""Output managers on a real simulation (GPU): CSVOutputManager writes at the reference's
output steps (weather_simulation.cpp:84-88) and its files hold exactly the grid's fields;
the protobuf result of a multi-level run carries every level."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ws = pytest.importorskip("weather_sim")
if not ws.is_cuda_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)


@pytest.mark.parametrize("fp64", [False, True])
def test_csv_output_manager(tmp_path, fp64):
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.output_interval, c.double_precision = 40, 24, 7, fp64
    sim = ws.WeatherSimulation(c)
    sim.set_initial_condition(ws.JetStreamInitialCondition())
    oc = ws.OutputConfig()
    oc.output_dir, oc.prefix = str(tmp_path), "run"
    om = ws.CSVOutputManager(oc)
    sim.set_output_manager(om)
    sim.initialize()
    assert sim.run(20) == 20
    assert [p.rsplit("/", 1)[1] for p in om.written] == ["run_000007.csv", "run_000014.csv"]
    sim.run(1)  # step 21: another output
    meta, back = ws.read_csv(om.written[-1])
    assert meta["step"] == "21"
    g = sim.get_current_grid()
    dtype = np.float64 if fp64 else np.float32
    for col in ("u", "v", "h", "p", "t", "q", "vorticity", "divergence"):
        np.testing.assert_array_equal(back[col][0].astype(dtype), g._get(col), err_msg=col)
    om.finalize(sim)
    assert (tmp_path / "run_index.txt").read_text().split() == ["run_000007.csv", "run_000014.csv", "run_000021.csv"]


def test_protobuf_result_levels():
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.num_levels = 16, 12, 3
    c.model = ws.SimulationModel.PrimitiveEquations
    sim = ws.WeatherSimulation(c)
    sim.set_initial_condition(ws.FrontInitialCondition())
    sim.initialize()
    sim.run(5)
    snap = ws.Snapshot.of(sim)
    r = ws.weather_sim_result(snap, run_id="pe")
    assert [s.z_level for s in r.atmospheric_slices] == [0, 1, 2]
    t2 = sim.get_current_grid().get_temperature_field(2)
    assert r.atmospheric_slices[2].cells[5 * 16 + 9].temperature == float(t2[5, 9])
