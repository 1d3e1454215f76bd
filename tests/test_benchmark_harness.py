"""benchmark_suite.py-compatible weather harness: CLI flags, result dict
and file naming on CPU; one real run on the GPU."""
import json

import pytest

from weather_sim import benchmark


def test_flags_match_reference_suite():
    a = benchmark.parser().parse_args(["--weather", "--weather-grid", "64", "--weather-steps", "5",
                                       "--weather-model", "barotropic", "--device", "0", "--output", "r"])
    assert (a.weather, a.weather_grid, a.weather_steps, a.weather_model, a.device, a.output) == \
        (True, 64, 5, "barotropic", 0, "r")
    d = benchmark.parser().parse_args([])
    assert (d.weather_grid, d.weather_steps, d.weather_model, d.output) == (512, 1000, "shallow_water", "results")
    with pytest.raises(SystemExit):
        benchmark.parser().parse_args(["--weather-model", "gcm"])


def test_nothing_selected_returns_2():
    assert benchmark.main([]) == 2


def test_result_dict_round_trip(tmp_path):
    r = benchmark.BenchmarkResult("weather_sim", "dev", {"name": "dev"}, 1.5, {"host": 1.0, "device": 2.0},
                                  throughput=10.0, additional_metrics={"grid_size": 8})
    path = benchmark.save_result(r, str(tmp_path))
    assert path.name.startswith("weather_sim_") and path.suffix == ".json"
    d = json.loads(path.read_text())
    assert set(d) == {"workload_name", "device_name", "device_capabilities", "execution_time", "memory_usage",
                      "gpu_utilization", "energy_consumption", "throughput", "additional_metrics",
                      "cost_metrics", "timestamp"}
    back = benchmark.BenchmarkResult.from_dict(d)
    assert back.to_dict() == d


@pytest.mark.gpu
def test_harness_runs_on_gpu(tmp_path):
    ws = pytest.importorskip("weather_sim")
    if not ws.is_cuda_available():  # pragma: no cover
        pytest.skip("no HIP device")
    assert benchmark.main(["--weather", "--weather-grid", "256", "--weather-steps", "20",
                           "--output", str(tmp_path)]) == 0
    (f,) = list(tmp_path.glob("weather_sim_*.json"))
    d = json.loads(f.read_text())
    m = d["additional_metrics"]
    assert m["grid_size"] == 256 and m["num_steps"] == 20 and m["grid_points_per_second"] > 0
    assert d["device_capabilities"]["compute_capability"].startswith("gfx")
