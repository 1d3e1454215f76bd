"""CPU checks of the C-ABI boundary and the host-side API (no GPU compute).

* libws_hip.so loads and exports every entry point include/ws_hip.h declares, and the
  ctypes signature table covers exactly that set.
* ws_config_t / ws_metrics_t / ws_device_info_t layouts match the C header (compiled probe).
* Without a HIP device the product fails loudly (no CPU fallback).
* Host-side API surface mirrors the reference module's names and defaults.
"""
import ctypes
import os
import re
import subprocess
import textwrap

import numpy as np
import pytest

from conftest import ROOT

import weather_sim as ws
from weather_sim import _native

HEADER = os.path.join(ROOT, "include", "ws_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^(?:int|void|const char\*)\s+(ws_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 40
    lib = ctypes.CDLL(_native.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), f"{n} declared in ws_hip.h but not exported"
    assert sorted(_native.SIGNATURES) == names, "ctypes signature table != header declarations"
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True).stdout
    exported = sorted(set(re.findall(r" T (ws_\w+)", out)))
    assert exported == names, "library exports undeclared ws_* symbols"


def test_struct_layouts_match_header(tmp_path):
    probe = tmp_path / "probe.c"
    probe.write_text(textwrap.dedent("""
        #include <stdio.h>
        #include <stddef.h>
        #include "ws_hip.h"
        int main(void) {
            printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(ws_config_t), offsetof(ws_config_t, max_time),
                   offsetof(ws_config_t, random_seed), sizeof(ws_metrics_t), sizeof(ws_device_info_t),
                   offsetof(ws_device_info_t, global_memory));
            return 0;
        }"""))
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-I", os.path.dirname(HEADER), str(probe), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    want = [ctypes.sizeof(_native.ws_config_t), _native.ws_config_t.max_time.offset,
            _native.ws_config_t.random_seed.offset, ctypes.sizeof(_native.ws_metrics_t),
            ctypes.sizeof(_native.ws_device_info_t), _native.ws_device_info_t.global_memory.offset]
    assert got == want


def test_config_default_matches_reference_defaults():
    c = _native.ws_config_t()
    _native.lib.ws_config_default(ctypes.byref(c))
    py = ws.SimulationConfig()
    for name, _ in _native.ws_config_t._fields_:
        if name == "random_seed":
            continue
        assert getattr(c, name) == pytest.approx(float(getattr(py, name))), name
    # weather_sim.hpp:155-191
    assert (py.grid_width, py.grid_height, py.num_levels) == (256, 256, 1)
    assert (py.dx, py.dy, py.dt, py.gravity, py.coriolis_f, py.max_time) == (1.0, 1.0, 0.01, 9.81, 0.0, 10.0)
    assert py.integration_method == ws.IntegrationMethod.RungeKutta4
    assert py.compute_backend == ws.ComputeBackend.CUDA and py.output_interval == 10


def test_abi_version_and_availability():
    assert _native.lib.ws_abi_version() == 2
    assert isinstance(_native.is_available(), bool)


@pytest.mark.skipif(_native.is_available(), reason="checks the no-device behaviour")
def test_no_device_fails_loudly():
    with pytest.raises(_native.WsDeviceError):
        ws.WeatherGrid(16, 16)
    with pytest.raises(_native.WsDeviceError):
        ws.WeatherSimulation(ws.SimulationConfig())
    with pytest.raises(_native.WsDeviceError):
        ws.WeatherSimulationWrapper(16, 16)
    with pytest.raises(_native.WsDeviceError):
        ws.BarotropicVorticityModel(ws.SimulationConfig())
    with pytest.raises(_native.WsDeviceError):
        ws.LayeredPrimitiveEquationsModel(ws.SimulationConfig())
    assert ws.is_cuda_available() is False


def test_physics_models_validate_before_touching_the_device():
    c = ws.SimulationConfig()
    c.grid_width = 2
    with pytest.raises(ValueError):
        ws.BarotropicVorticityModel(c)
    with pytest.raises(ValueError):
        ws.LayeredPrimitiveEquationsModel(c)
    c = ws.SimulationConfig()
    c.dx = 0.0
    with pytest.raises(ValueError):
        ws.BarotropicVorticityModel(c)
    with pytest.raises(TypeError):
        ws.BarotropicVorticityModel({"grid_width": 64})


def test_cpu_backend_runs_the_hip_path():
    """ComputeBackend.CPU (backend="cpu"): the reference runs it through its CPU solver
    (weather_simulation.cpp:562-591) and its own tests request it; this build has only the HIP
    path, which every backend takes -- so CPU is accepted like the GPU-class backends (here,
    without a device, every one fails for want of a device, never with NotImplementedError).
    The one-time warning is checked on the GPU (tests/test_gpu_parity.py)."""
    c = ws.SimulationConfig()
    c.compute_backend = ws.ComputeBackend.CPU
    if not _native.is_available():
        with pytest.raises(_native.WsDeviceError):
            ws.WeatherSimulation(c)
        for b in ("cpu", "cuda", "hybrid", "adaptive"):
            with pytest.raises(_native.WsDeviceError):
                ws.WeatherSimulationWrapper(16, 16, backend=b)


def test_slab_partition_is_balanced_and_covers_rows():
    for H in (7, 256, 4096, 16384):
        for n in (1, 2, 3, 4, 8):
            if H < n:
                continue
            rows = []
            for r in range(n):
                r0, nr = ctypes.c_int32(), ctypes.c_int32()
                _native.check(_native.lib.ws_slab_partition(H, r, n, ctypes.byref(r0), ctypes.byref(nr)))
                rows.append((r0.value, nr.value))
            assert rows[0][0] == 0 and sum(nr for _, nr in rows) == H
            assert all(rows[i][0] + rows[i][1] == rows[i + 1][0] for i in range(n - 1))
            assert max(nr for _, nr in rows) - min(nr for _, nr in rows) <= 1
    with pytest.raises(ValueError):
        _native.check(_native.lib.ws_slab_partition(2, 0, 4, ctypes.byref(ctypes.c_int32()),
                                                    ctypes.byref(ctypes.c_int32())))


def test_api_surface_mirrors_reference():
    # names imported by the reference's weather_simulation.py (:16-26) and its __init__
    for name in ("WeatherGrid", "WeatherSimulation", "SimulationConfig", "InitialConditionFactory",
                 "AdaptiveKernelManager", "PerformanceMetrics", "OutputConfig", "SimulationModel",
                 "IntegrationMethod", "GridType", "BoundaryCondition", "ComputeBackend", "DeviceType", "OutputFormat",
                 "UniformInitialCondition", "RandomInitialCondition", "ZonalFlowInitialCondition",
                 "VortexInitialCondition", "JetStreamInitialCondition", "BreakingWaveInitialCondition",
                 "FrontInitialCondition", "MountainInitialCondition", "AtmosphericProfileInitialCondition",
                 "register_all_initial_conditions", "WeatherSimulationWrapper", "create_initial_condition",
                 "get_available_initial_conditions", "is_cuda_available", "get_device_info"):
        assert hasattr(ws, name), name
    assert ws.get_available_initial_conditions() == sorted(
        ["uniform", "random", "zonal_flow", "vortex", "jet_stream", "breaking_wave", "front", "mountain",
         "standard_atmosphere", "tropical_atmosphere", "polar_atmosphere"])
    assert ws.create_initial_condition("jet_stream", strength=12.0).get_name() == "jet_stream"
    assert ws.create_initial_condition("polar_atmosphere").get_name() == "atmospheric_profile"
    assert ws.create_initial_condition("no_such_ic") is None
    assert [m.value for m in ws.IntegrationMethod] == [0, 1, 2, 3, 4]
    info = ws.get_device_info()
    assert "cuda_available" in info and "device_name" in info


def test_environment_switches_are_few_and_documented():
    """The library reads at most 8 WS_* environment variables, each listed in ws_hip.h (the
    rest of the configuration is ABI arguments: ws_sim_pin_variant, ws_sim_set_slab_schedule,
    ws_sim_create_slab_emulated, ws_bvort_create_poisson)."""
    import glob
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    names = set()
    for f in glob.glob(os.path.join(root, "nvidia-jetson-workload_amd", "csrc", "*")):
        if f.endswith((".cpp", ".hip", ".h")):
            names |= set(re.findall(r'(?:getenv|env_str|env_int)\("(WS_[A-Z0-9_]+)"', open(f).read()))
    header = open(os.path.join(root, "include", "ws_hip.h")).read()
    assert 0 < len(names) <= 8, sorted(names)
    for n in names:
        assert f" *   {n}=" in header, n


def test_kernel_variant_ids_match_header():
    """The Python variant names (pin_variant / fused_variant) use the header's WS_KERNEL_* ids,
    and the library's WS_KERNEL switch accepts every one of them (ws_runtime.cpp)."""
    hdr = open(os.path.join(ROOT, "include", "ws_hip.h")).read()
    ids = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"#define WS_KERNEL_([A-Z0-9]+) (\d+)", hdr)}
    assert ids == ws.WeatherSimulation._KERNELS
    src = open(os.path.join(ROOT, "nvidia-jetson-workload_amd", "csrc", "ws_runtime.cpp")).read()
    for name in ids:
        assert f'{{"{name}", ' in src, name


def test_single_device_list_names_the_device():
    """config.devices with one entry is the device of a one-GPU run (it used to be
    ignored, the run going to device_id 0); a device_id that disagrees with it is an error."""
    c = ws.SimulationConfig()
    assert c._to_c().device_id == 0
    c.devices = [2]
    assert c._to_c().device_id == 2
    c.device_id = 2
    assert c._to_c().device_id == 2
    c.device_id = 1
    with pytest.raises(ValueError):
        c._to_c()
    c.devices = [0, 1]  # several: the multi-GPU path, device_id untouched
    assert c._to_c().device_id == 1
