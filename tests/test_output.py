"""Output formats on synthetic snapshots (CPU): CSV round trip is exact in
fp32 and fp64; the protobuf messages of src/proto/weather.proto serialize, parse back and
carry the fields the mapping in weather_sim/output.py documents."""
import numpy as np
import pytest

from weather_sim import output


def snap(dtype, L=2, H=5, W=7):
    rng = np.random.default_rng(3)
    f = {k: rng.standard_normal((L, H, W)).astype(dtype) * s
         for k, s in (("u", 3), ("v", 2), ("h", 10), ("p", 1000), ("t", 280), ("q", 0.01),
                      ("vorticity", 0.1), ("divergence", 0.1))}
    return output.Snapshot(width=W, height=H, levels=L, dtype=np.dtype(dtype).type, time=1.25, step=125,
                           dx=2.0, dy=0.5, dt=0.01, max_time=10.0, fields=f, total_time_ms=12.5)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("compress", [False, True])
def test_csv_round_trip_is_exact(tmp_path, dtype, compress):
    s = snap(dtype)
    cols = output.csv_columns(["velocity", "height", "pressure", "temperature", "humidity", "vorticity",
                               "divergence"])
    path = output.write_csv(s, str(tmp_path / "x.csv"), cols, compress)
    meta, back = output.read_csv(path)
    assert meta["step"] == "125" and int(meta["levels"]) == 2
    for c in cols:
        np.testing.assert_array_equal(back[c].astype(dtype), s.fields[c], err_msg=c)


def test_csv_columns_follow_output_config():
    assert output.csv_columns(["velocity", "height"]) == ["u", "v", "h"]
    assert output.csv_columns(["height", "vorticity", "divergence"], include_diagnostics=False) == ["h"]
    with pytest.raises(ValueError):
        output.csv_columns(["wind"])


def test_weather_sim_result_protobuf():
    s = snap(np.float64)
    r = output.weather_sim_result(s, run_id="r1")
    P = output.proto_classes()
    back = P["WeatherSimResult"]()
    back.ParseFromString(r.SerializeToString())
    assert back.base_result.workload_type == "weather_sim" and back.base_result.config.run_id == "r1"
    assert back.config.grid_size_x == 7 and back.config.grid_size_y == 5 and back.config.grid_size_z == 2
    assert back.config.domain_size_x == 14.0 and back.config.domain_size_y == 2.5
    assert back.simulation_time == 1.25 and len(back.atmospheric_slices) == 2
    sl = back.atmospheric_slices[1]
    assert (sl.z_level, sl.width, sl.height, len(sl.cells)) == (1, 7, 5, 35)
    c = sl.cells[2 * 7 + 3]  # y = 2, x = 3
    assert c.temperature == s.fields["t"][1, 2, 3] and c.wind_velocity_y == s.fields["v"][1, 2, 3]
    assert back.max_temperature == s.fields["t"].max()
    assert back.max_wind_speed == pytest.approx(np.hypot(s.fields["u"], s.fields["v"]).max())
    ops = back.base_result.metrics.operations_per_second
    assert ops == pytest.approx(7 * 5 * 2 * 125 / 12.5e-3)


def test_weather_sim_update_protobuf_and_stride():
    s = snap(np.float32, L=1, H=8, W=8)
    u = output.weather_sim_update(s, run_id="r2", output_stride=2)
    P = output.proto_classes()
    back = P["WeatherSimUpdate"]()
    back.ParseFromString(u.SerializeToString())
    assert back.percent_complete == pytest.approx(12.5)
    assert (back.current_slice.width, back.current_slice.height) == (4, 4)
    assert back.current_slice.cells[5].pressure == np.float64(s.fields["p"][0, 2, 2])
