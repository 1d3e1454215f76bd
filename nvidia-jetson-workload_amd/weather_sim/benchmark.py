"""Weather-sim leg of the reference's benchmark suite, runnable.

The reference harness (``benchmark/benchmark_suite.py``) drives the weather workload with
``WeatherSimulationBenchmark.run(grid_size, num_steps, dt, model)`` (:524-597) and the CLI
flags ``--weather --weather-grid --weather-steps --weather-model --device --output``
(:1237-1264), and saves a ``BenchmarkResult`` dict as ``<output>/weather_sim_<timestamp>.json``
(:36-91, :1167-1181). As written it cannot run (it calls ``WeatherSimulation()`` without a
config and ``initialize(grid_size=...)``/``step(dt)``, which the package does not have,
SURVEY §3(E)). This module keeps its names, flags, result fields and file naming and runs
the MI355X path: the same square grid, model and step count, ``dt`` as given, timed around
``run(num_steps)`` after a short warm-up (which also runs the kernel autotuner).

  python -m weather_sim.benchmark --weather --weather-grid 4096 --weather-steps 100 \\
         --weather-model shallow_water [--weather-precision fp64] [--device 0] [--output results]
"""
import argparse
import ctypes
import json
import os
import sys
import time
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, Optional

MODELS = {"shallow_water": 0, "barotropic": 1, "primitive": 2}


class BenchmarkResult:
    """Container for benchmark results (benchmark_suite.py:36-91, same fields)."""

    def __init__(self, workload_name: str, device_name: str, device_capabilities: Dict[str, Any],
                 execution_time: float, memory_usage: Dict[str, float], gpu_utilization: Optional[float] = None,
                 energy_consumption: Optional[float] = None, throughput: Optional[float] = None,
                 additional_metrics: Optional[Dict[str, Any]] = None,
                 cost_metrics: Optional[Dict[str, Any]] = None):
        self.workload_name = workload_name
        self.device_name = device_name
        self.device_capabilities = device_capabilities
        self.execution_time = execution_time
        self.memory_usage = memory_usage
        self.gpu_utilization = gpu_utilization
        self.energy_consumption = energy_consumption
        self.throughput = throughput
        self.additional_metrics = additional_metrics or {}
        self.cost_metrics = cost_metrics or {}
        self.timestamp = datetime.now().isoformat()

    def to_dict(self) -> Dict[str, Any]:
        return {
            "workload_name": self.workload_name, "device_name": self.device_name,
            "device_capabilities": self.device_capabilities, "execution_time": self.execution_time,
            "memory_usage": self.memory_usage, "gpu_utilization": self.gpu_utilization,
            "energy_consumption": self.energy_consumption, "throughput": self.throughput,
            "additional_metrics": self.additional_metrics, "cost_metrics": self.cost_metrics,
            "timestamp": self.timestamp,
        }

    @classmethod
    def from_dict(cls, data: Dict[str, Any]) -> "BenchmarkResult":
        r = cls(data["workload_name"], data["device_name"], data["device_capabilities"], data["execution_time"],
                data["memory_usage"], data.get("gpu_utilization"), data.get("energy_consumption"),
                data.get("throughput"), data.get("additional_metrics"), data.get("cost_metrics"))
        r.timestamp = data.get("timestamp", r.timestamp)
        return r


def _device_capabilities(device_id: int) -> Dict[str, Any]:
    """benchmark_suite.py:263-279's dict, from the HIP device."""
    from . import _native
    info = _native.ws_device_info_t()
    _native.check(_native.lib.ws_device_info(device_id, ctypes.byref(info)))
    return {"name": info.device_name.decode(), "compute_capability": info.arch.decode(),
            "total_memory": info.global_memory / (1024 ** 2), "clock_rate": info.clock_rate_khz / 1000,
            "num_multiprocessors": info.multiprocessors}


def _memory_usage(device_id: int) -> Dict[str, float]:
    """benchmark_suite.py:298-313: host RSS and device memory in use, MB."""
    from . import _native
    host = 0.0
    try:
        import psutil
        host = psutil.Process(os.getpid()).memory_info().rss / (1024 * 1024)
    except ImportError:
        pass
    free, total = ctypes.c_int64(), ctypes.c_int64()
    _native.check(_native.lib.ws_device_memory(device_id, ctypes.byref(free), ctypes.byref(total)))
    return {"host": host, "device": (total.value - free.value) / (1024 * 1024)}


class WeatherSimulationBenchmark:
    """WeatherSimulationBenchmark (benchmark_suite.py:524-597) on the MI355X path."""

    def __init__(self, device_id: int = 0):
        self.name = "weather_sim"
        self.device_id = device_id
        self.device_capabilities = _device_capabilities(device_id)
        self.device_name = self.device_capabilities["name"]

    def run(self, grid_size: int = 512, num_steps: int = 1000, dt: float = 0.01, model: str = "shallow_water",
            integration_method: str = "rk4", double_precision: bool = False, warmup_steps: int = 10,
            **kwargs) -> BenchmarkResult:
        from . import weather_simulation as wsm
        if model not in MODELS:
            raise ValueError(f"model must be one of {sorted(MODELS)}")
        cfg = wsm.SimulationConfig()
        cfg.grid_width = cfg.grid_height = int(grid_size)
        cfg.model = MODELS[model]
        cfg.integration_method = {"euler": 0, "rk2": 1, "rk4": 2}[integration_method]
        cfg.dt = dt
        cfg.double_precision = bool(double_precision)
        cfg.device_id = self.device_id
        cfg.max_time = 1e30  # run exactly num_steps (the reference loop calls step() num_steps times)
        sim = wsm.WeatherSimulation(cfg)
        sim.set_initial_condition(wsm.JetStreamInitialCondition())
        memory_before = _memory_usage(self.device_id)
        sim.initialize()
        if warmup_steps > 0:
            sim.run(warmup_steps)
        start = time.time()
        sim.run(num_steps)
        execution_time = time.time() - start
        memory_after = _memory_usage(self.device_id)
        throughput = num_steps / execution_time
        kernel, seg_rows, out_cols = sim.fused_variant()
        return BenchmarkResult(
            workload_name=self.name, device_name=self.device_name, device_capabilities=self.device_capabilities,
            execution_time=execution_time,
            memory_usage={"host": memory_after["host"] - memory_before["host"],
                          "device": memory_after["device"] - memory_before["device"]},
            gpu_utilization=None, throughput=throughput,
            additional_metrics={"grid_size": grid_size, "num_steps": num_steps,
                                "grid_points_per_second": grid_size ** 2 * throughput, "model": model,
                                "integration_method": integration_method,
                                "precision": "fp64" if double_precision else "fp32", "warmup_steps": warmup_steps,
                                "kernel": kernel, "seg_rows": seg_rows, "strip_out_cols": out_cols})


def save_result(result: BenchmarkResult, output_dir: str) -> Path:
    """benchmark_suite.py:1167-1181: <output_dir>/<workload>_<YYYYmmdd_HHMMSS>.json."""
    out = Path(output_dir)
    out.mkdir(parents=True, exist_ok=True)
    path = out / f"{result.workload_name}_{datetime.now().strftime('%Y%m%d_%H%M%S')}.json"
    with open(path, "w") as f:
        json.dump(result.to_dict(), f, indent=2)
    return path


def parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Weather Simulation benchmark (benchmark_suite.py flags)")
    p.add_argument("--device", type=int, default=0, help="GPU device ID to use")
    p.add_argument("--output", type=str, default="results", help="Directory to store results")
    p.add_argument("--weather", action="store_true", help="Run Weather Simulation benchmark")
    p.add_argument("--all", action="store_true", help="Run all benchmarks (here: the weather one)")
    p.add_argument("--weather-grid", type=int, default=512, help="Grid size for Weather Simulation")
    p.add_argument("--weather-steps", type=int, default=1000, help="Number of steps for Weather Simulation")
    p.add_argument("--weather-model", type=str, default="shallow_water", choices=sorted(MODELS),
                   help="Model for Weather Simulation")
    p.add_argument("--weather-method", type=str, default="rk4", choices=["euler", "rk2", "rk4"])
    p.add_argument("--weather-precision", type=str, default="fp32", choices=["fp32", "fp64"])
    p.add_argument("--weather-dt", type=float, default=0.01)
    return p


def main(argv=None) -> int:
    args = parser().parse_args(argv)
    if not (args.weather or args.all):
        print("nothing to run: pass --weather (or --all)", file=sys.stderr)
        return 2
    bench = WeatherSimulationBenchmark(args.device)
    result = bench.run(grid_size=args.weather_grid, num_steps=args.weather_steps, dt=args.weather_dt,
                       model=args.weather_model, integration_method=args.weather_method,
                       double_precision=args.weather_precision == "fp64")
    path = save_result(result, args.output)
    m = result.additional_metrics
    print(f"weather_sim: {m['grid_points_per_second'] / 1e9:.2f} G grid-points/s "
          f"({result.throughput:.1f} steps/s, {result.execution_time:.3f} s) -> {path}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
