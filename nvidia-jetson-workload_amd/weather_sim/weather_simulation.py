"""Weather Simulation Python API -- MI355X-native drop-in for the reference module.

Mirrors /root/reference/src/weather-sim/python/weather_simulation.py (the high-level
wrapper and helpers) and the names that module imports from the pybind module
`pyweather_sim` (src/weather-sim/cpp/src/python_bindings.cpp:116-372): same class names,
method names, argument meanings, defaults and error types. Underneath, every grid lives in
MI355X HBM and every step runs as hand-written HIP kernels through libws_hip.so (the C ABI
in include/ws_hip.h). There is no CPU compute path and no mock fallback.

Deliberate deviations from the reference (documented in DESIGN.md):
  * ComputeBackend CUDA / Hybrid / AdaptiveHybrid run the HIP path (the reference runs
    every backend through its CPU solver; its CUDA branch was an empty placeholder,
    weather_simulation.cpp:492-500, 562-591). ComputeBackend.CPU (backend="cpu") runs the
    HIP path too, with a one-time RuntimeWarning saying so: this build has no CPU solver, and
    the HIP results are the CPU solver's bits.
  * SimulationConfig.double_precision is honoured (fp64 grids); fp32 is the default and
    matches the reference bit-for-bit.
  * num_levels > 1 stores [L, H, W] fields of independent 2-D levels (the reference
    ignores num_levels, weather_grid.cpp:36-48); getters then return (L, H, W) arrays.
  * PerformanceMetrics times are device milliseconds, not integer-truncated host ms.
  * Vorticity / divergence are computed lazily (when read), with identical values.
"""
import ctypes
import os
import random
import time
import warnings
from enum import IntEnum
from typing import Dict, List, Optional, Union

import numpy as np

from . import _native
from ._native import FIELD, WS_F32, WS_F64, check, lib

VERBOSE = os.environ.get("WS_QUIET", "0") in ("", "0")


def _say(msg):
    if VERBOSE:
        print(msg)


# ---------------------------------------------------------------------------------
# Enumerations (weather_sim.hpp:30-76, python_bindings.cpp:120-171)
# ---------------------------------------------------------------------------------
class SimulationModel(IntEnum):
    ShallowWater = 0
    Barotropic = 1
    PrimitiveEquations = 2
    General = 3


class IntegrationMethod(IntEnum):
    ExplicitEuler = 0
    RungeKutta2 = 1
    RungeKutta4 = 2
    AdamsBashforth = 3
    SemiImplicit = 4


class GridType(IntEnum):
    Cartesian = 0
    Staggered = 1
    Icosahedral = 2
    SphericalHarmonic = 3


class BoundaryCondition(IntEnum):
    Periodic = 0
    Reflective = 1
    Outflow = 2
    Custom = 3


class ComputeBackend(IntEnum):
    CUDA = 0  # kept as the GPU value for API compatibility: the HIP device
    CPU = 1
    Hybrid = 2
    AdaptiveHybrid = 3


class DeviceType(IntEnum):
    Unknown = 0
    CPU = 1
    JetsonOrinNX = 2
    T4 = 3
    HighEndGPU = 4
    OtherGPU = 5


class OutputFormat(IntEnum):
    CSV = 0
    NetCDF = 1
    VTK = 2
    PNG = 3
    Custom = 4


# ---------------------------------------------------------------------------------
# Structures
# ---------------------------------------------------------------------------------
class SimulationConfig:
    """SimulationConfig (weather_sim.hpp:155-191) with the C++ defaults."""

    def __init__(self):
        self.model = SimulationModel.ShallowWater
        self.grid_type = GridType.Staggered
        self.integration_method = IntegrationMethod.RungeKutta4
        self.boundary_condition = BoundaryCondition.Periodic
        self.grid_width = 256
        self.grid_height = 256
        self.num_levels = 1
        self.dx = 1.0
        self.dy = 1.0
        self.dt = 0.01
        self.gravity = 9.81
        self.coriolis_f = 0.0
        self.beta = 0.0
        self.viscosity = 0.0
        self.diffusivity = 0.0
        self.compute_backend = ComputeBackend.CUDA
        self.double_precision = False
        self.device_id = 0
        self.num_threads = 0
        self.max_time = 10.0
        self.max_steps = 1000
        self.output_interval = 10
        self.output_path = "./output"
        self.random_seed = random.SystemRandom().getrandbits(32)  # std::random_device{}()
        # extension: HIP device ids of a one-process multi-GPU run -- more than
        # one makes WeatherSimulation(config) a MultiGPUSimulation (one y-slab per device)
        self.devices = None

    def _to_c(self):
        c = _native.ws_config_t()
        for name, _ in _native.ws_config_t._fields_:
            setattr(c, name, type(getattr(c, name))(getattr(self, name)))
        c.device_id = self._single_device()
        return c

    def _single_device(self):
        """devices=[d] (one entry) names the device of a one-GPU run: it is device_id, and a
        device_id other than the default 0 that disagrees with it is an error (a single entry
        used to be ignored silently)."""
        devs = list(self.devices or ())
        if len(devs) != 1:
            return int(self.device_id)
        d = int(devs[0])
        if int(self.device_id) not in (0, d):
            raise ValueError(f"devices={devs} disagrees with device_id={self.device_id}")
        return d

    @classmethod
    def _from_c(cls, c, output_path="./output"):
        self = cls()
        for name, _ in _native.ws_config_t._fields_:
            setattr(self, name, getattr(c, name))
        self.model = SimulationModel(self.model)
        self.integration_method = IntegrationMethod(self.integration_method)
        self.grid_type = GridType(self.grid_type)
        self.boundary_condition = BoundaryCondition(self.boundary_condition)
        self.compute_backend = ComputeBackend(self.compute_backend)
        self.double_precision = bool(self.double_precision)
        self.output_path = output_path
        return self

    def __repr__(self):
        return f"SimulationConfig({self.grid_width}x{self.grid_height}x{self.num_levels}, model={self.model!r}, " \
               f"method={self.integration_method!r}, dt={self.dt}, fp64={self.double_precision})"


class PerformanceMetrics:
    """PerformanceMetrics (weather_sim.hpp:196-223)."""

    def __init__(self):
        self.total_time_ms = 0.0
        self.compute_time_ms = 0.0
        self.memory_transfer_time_ms = 0.0
        self.io_time_ms = 0.0
        self.num_steps = 0

    def reset(self):
        self.__init__()

    def print(self):
        t = self.total_time_ms or float("nan")
        print("Performance Metrics:")
        print(f"  Total time: {self.total_time_ms} ms")
        print(f"  Compute time: {self.compute_time_ms} ms ({self.compute_time_ms / t * 100.0}%)")
        print(f"  Memory transfer time: {self.memory_transfer_time_ms} ms ({self.memory_transfer_time_ms / t * 100.0}%)")
        print(f"  I/O time: {self.io_time_ms} ms ({self.io_time_ms / t * 100.0}%)")
        print(f"  Steps: {self.num_steps}")
        print(f"  Time per step: {self.total_time_ms / self.num_steps if self.num_steps else float('nan')} ms")


class OutputConfig:
    """OutputConfig (output_manager.hpp:35-47); the CSV writer is output.CSVOutputManager."""

    def __init__(self):
        self.output_dir = "./output"
        self.prefix = "weather_sim"
        self.format = OutputFormat.CSV
        self.output_interval = 10
        self.compress = False
        self.include_diagnostics = True
        self.fields = ["velocity", "height", "pressure", "temperature", "humidity", "vorticity", "divergence"]


class DeviceCapabilities:
    """DeviceCapabilities (gpu_adaptability.hpp:35-88) for the HIP device."""

    def __init__(self, info=None):
        self.device_type = DeviceType.Unknown
        self.device_name = "Unknown"
        self.arch = ""
        self.compute_capability_major = 0
        self.compute_capability_minor = 0
        self.cuda_cores = 0
        self.multiprocessors = 0
        self.global_memory = 0
        self.shared_memory_per_block = 0
        self.max_threads_per_block = 0
        self.max_threads_per_multiprocessor = 0
        self.clock_rate_khz = 0
        self.memory_clock_rate_khz = 0
        self.memory_bus_width = 0
        self.compute_power_ratio = 0.0
        if info is not None:
            for name, _ in _native.ws_device_info_t._fields_:
                v = getattr(info, name)
                setattr(self, name, v.decode() if isinstance(v, bytes) else v)
            self.device_type = DeviceType.HighEndGPU
            self.compute_power_ratio = 1.0

    def get_summary(self):
        return (f"Device: {self.device_name} ({self.arch}), CUs: {self.multiprocessors}, "
                f"Memory: {self.global_memory / 2**30:.1f} GiB, wavefront 64")


# ---------------------------------------------------------------------------------
# WeatherGrid (weather_sim.hpp:254-412; python_bindings.cpp:240-284)
# ---------------------------------------------------------------------------------
class WeatherGrid:
    """A device-resident grid. `WeatherGrid(width, height, num_levels=1)` or
    `WeatherGrid(config)`; extension keywords: double_precision, device_id."""

    def __init__(self, width, height=None, num_levels=1, *, double_precision=False, device_id=0, _handle=None,
                 _owner=None):
        self._owner = _owner  # keeps the owning simulation alive
        if _handle is not None:
            self._h = ctypes.c_void_p(_handle)
            self._owned = False
        else:
            dx = dy = None
            if isinstance(width, SimulationConfig):
                cfg = width
                width, height, num_levels = cfg.grid_width, cfg.grid_height, cfg.num_levels
                double_precision, device_id = cfg.double_precision, cfg.device_id
                dx, dy = cfg.dx, cfg.dy
            if height is None:
                raise TypeError("WeatherGrid(width, height, num_levels=1) or WeatherGrid(config)")
            h = ctypes.c_void_p()
            check(lib.ws_grid_create(int(width), int(height), int(num_levels), WS_F64 if double_precision else WS_F32,
                                     int(device_id), ctypes.byref(h)))
            self._h = h
            self._owned = True
            if dx is not None:
                check(lib.ws_grid_set_spacing(self._h, float(dx), float(dy)))
        w, hh, l, dt = (ctypes.c_int32() for _ in range(4))
        check(lib.ws_grid_get_dims(self._h, ctypes.byref(w), ctypes.byref(hh), ctypes.byref(l), ctypes.byref(dt)))
        self._W, self._H, self._L = w.value, hh.value, l.value
        self._dtype = np.float64 if dt.value == WS_F64 else np.float32
        self._ws_dtype = dt.value

    def __del__(self):
        if getattr(self, "_owned", False) and self._h:
            lib.ws_grid_destroy(self._h)
            self._h = None

    # -- dimensions / spacing
    def reset(self):
        check(lib.ws_grid_reset(self._h))

    def get_width(self):
        return self._W

    def get_height(self):
        return self._H

    def get_num_levels(self):
        return self._L

    def get_dx(self):
        dx, dy = ctypes.c_double(), ctypes.c_double()
        check(lib.ws_grid_get_spacing(self._h, ctypes.byref(dx), ctypes.byref(dy)))
        return dx.value

    def get_dy(self):
        dx, dy = ctypes.c_double(), ctypes.c_double()
        check(lib.ws_grid_get_spacing(self._h, ctypes.byref(dx), ctypes.byref(dy)))
        return dy.value

    def set_spacing(self, dx, dy):
        check(lib.ws_grid_set_spacing(self._h, float(dx), float(dy)))

    def calculate_diagnostics(self):
        check(lib.ws_grid_calculate_diagnostics(self._h))

    @property
    def dtype(self):
        return self._dtype

    # -- field copies (python_bindings.cpp:22-114)
    def _get(self, name, level=None):
        lvl = -1 if level is None else int(level)
        shape = (self._H, self._W) if (self._L == 1 or lvl >= 0) else (self._L, self._H, self._W)
        if self._L == 1 and lvl == -1:
            lvl = 0
        out = np.empty(shape, self._dtype)
        check(lib.ws_grid_get_field(self._h, FIELD[name], lvl, out.ctypes.data, self._H, self._W, self._ws_dtype))
        return out

    def _set(self, name, arr, level=None):
        a = np.asarray(arr)
        if level is not None:
            lvl = int(level)
            want_ndim = 2
        elif self._L > 1 and a.ndim == 3:
            lvl, want_ndim = -1, 3
        else:
            lvl, want_ndim = (-1 if self._L > 1 else 0), 2
        if a.ndim != want_ndim:
            raise RuntimeError(f"Number of dimensions must be {want_ndim}")
        if a.shape[-2:] != (self._H, self._W) or (want_ndim == 3 and a.shape[0] != self._L):
            raise RuntimeError("Array dimensions must match field dimensions")
        if want_ndim == 2 and lvl == -1:  # one (H, W) array for every level
            a = np.broadcast_to(a, (self._L, self._H, self._W))
        a = np.ascontiguousarray(a, dtype=self._dtype)
        check(lib.ws_grid_set_field(self._h, FIELD[name], lvl, a.ctypes.data, self._H, self._W, self._ws_dtype))

    def get_velocity_field(self, level=None):
        return self._get("u", level), self._get("v", level)

    def get_height_field(self, level=None):
        return self._get("h", level)

    def get_pressure_field(self, level=None):
        return self._get("p", level)

    def get_temperature_field(self, level=None):
        return self._get("t", level)

    def get_humidity_field(self, level=None):
        return self._get("q", level)

    def get_vorticity_field(self, level=None):
        return self._get("vorticity", level)

    def get_divergence_field(self, level=None):
        """Extension: the reference computes divergence but binds no getter."""
        return self._get("divergence", level)

    def set_velocity_field(self, u, v, level=None):
        # reference checks both arrays before writing (python_bindings.cpp:92-104)
        for a in (u, v):
            a = np.asarray(a)
            if a.ndim not in (2, 3):
                raise RuntimeError("Number of dimensions must be 2")
            if a.shape[-2:] != (self._H, self._W):
                raise RuntimeError("Array dimensions must match field dimensions")
        self._set("u", u, level)
        self._set("v", v, level)

    def set_height_field(self, h, level=None):
        self._set("h", h, level)

    def set_pressure_field(self, p, level=None):
        self._set("p", p, level)

    def set_temperature_field(self, t, level=None):
        self._set("t", t, level)

    def set_humidity_field(self, q, level=None):
        self._set("q", q, level)

    def device_field(self, name):
        """Extension: (device pointer, row pitch, level stride) of a field, for zero-copy interop."""
        p, pitch, ls = ctypes.c_void_p(), ctypes.c_int64(), ctypes.c_int64()
        check(lib.ws_grid_device_field(self._h, FIELD[name], ctypes.byref(p), ctypes.byref(pitch), ctypes.byref(ls)))
        return p.value, pitch.value, ls.value


# ---------------------------------------------------------------------------------
# Initial conditions (initial_conditions.hpp / initial_conditions.cpp:48-666)
# ---------------------------------------------------------------------------------
class InitialCondition:
    _ws_name = None

    def __init__(self, *params, sparam=""):
        self._params = [float(p) for p in params]
        self._sparam = sparam

    def initialize(self, grid: WeatherGrid, level: Optional[int] = None):
        arr = (ctypes.c_double * max(1, len(self._params)))(*self._params)
        # a multi-GPU grid (SlabbedGrid): every slab in global coordinates, its own rows
        for g in getattr(grid, "slab_grids", None) or [grid]:
            check(lib.ws_grid_apply_initial_condition(g._h, self._ws_name.encode(), arr, len(self._params),
                                                      self._sparam.encode(), -1 if level is None else int(level)))

    def get_name(self):
        return self._ws_name


class UniformInitialCondition(InitialCondition):
    _ws_name = "uniform"

    def __init__(self, u=0.0, v=0.0, h=10.0, p=1000.0, t=300.0, q=0.0):
        super().__init__(u, v, h, p, t, q)


class RandomInitialCondition(InitialCondition):
    _ws_name = "random"

    def __init__(self, seed=0, amplitude=1.0):
        super().__init__(int(seed) & 0xFFFFFFFF, amplitude)


class ZonalFlowInitialCondition(InitialCondition):
    _ws_name = "zonal_flow"

    def __init__(self, u_max=10.0, h_mean=10.0, beta=0.1):
        super().__init__(u_max, h_mean, beta)


class VortexInitialCondition(InitialCondition):
    _ws_name = "vortex"

    def __init__(self, x_center=0.5, y_center=0.5, radius=0.1, strength=10.0, h_mean=10.0):
        super().__init__(x_center, y_center, radius, strength, h_mean)


class JetStreamInitialCondition(InitialCondition):
    _ws_name = "jet_stream"

    def __init__(self, y_center=0.5, width=0.1, strength=10.0, h_mean=10.0):
        super().__init__(y_center, width, strength, h_mean)


class BreakingWaveInitialCondition(InitialCondition):
    _ws_name = "breaking_wave"

    def __init__(self, amplitude=1.0, wavelength=0.2, h_mean=10.0):
        super().__init__(amplitude, wavelength, h_mean)


class FrontInitialCondition(InitialCondition):
    _ws_name = "front"

    def __init__(self, y_position=0.5, width=0.05, temp_difference=10.0, wind_shear=5.0):
        super().__init__(y_position, width, temp_difference, wind_shear)


class MountainInitialCondition(InitialCondition):
    _ws_name = "mountain"

    def __init__(self, x_center=0.3, y_center=0.5, radius=0.1, height=1.0, u_base=5.0):
        super().__init__(x_center, y_center, radius, height, u_base)


class AtmosphericProfileInitialCondition(InitialCondition):
    _ws_name = "atmospheric_profile"

    def __init__(self, profile_name="standard"):
        super().__init__(sparam=profile_name)


class InitialConditionFactory:
    """Singleton registry (initial_conditions.cpp:16-45)."""
    _instance = None

    def __init__(self):
        self._creators = {}

    @classmethod
    def get_instance(cls):
        if cls._instance is None:
            cls._instance = cls()
        return cls._instance

    def register_initial_condition(self, name, creator):
        self._creators[name] = creator

    def create_initial_condition(self, name):
        c = self._creators.get(name)
        return c() if c else None

    def get_available_initial_conditions(self):
        return sorted(self._creators)  # std::map iteration order


def register_all_initial_conditions():
    """initial_conditions.cpp:611-666"""
    f = InitialConditionFactory.get_instance()
    f.register_initial_condition("uniform", UniformInitialCondition)
    f.register_initial_condition("random", RandomInitialCondition)
    f.register_initial_condition("zonal_flow", ZonalFlowInitialCondition)
    f.register_initial_condition("vortex", VortexInitialCondition)
    f.register_initial_condition("jet_stream", JetStreamInitialCondition)
    f.register_initial_condition("breaking_wave", BreakingWaveInitialCondition)
    f.register_initial_condition("front", FrontInitialCondition)
    f.register_initial_condition("mountain", MountainInitialCondition)
    f.register_initial_condition("standard_atmosphere", lambda: AtmosphericProfileInitialCondition("standard"))
    f.register_initial_condition("tropical_atmosphere", lambda: AtmosphericProfileInitialCondition("tropical"))
    f.register_initial_condition("polar_atmosphere", lambda: AtmosphericProfileInitialCondition("polar"))


# ---------------------------------------------------------------------------------
# Output manager interface (weather_sim.hpp:549-570)
# ---------------------------------------------------------------------------------
class OutputManager:
    def initialize(self, simulation):
        pass

    def write_output(self, simulation):
        pass

    def finalize(self, simulation):
        pass


# ---------------------------------------------------------------------------------
# WeatherSimulation (weather_sim.hpp:417-544; weather_simulation.cpp)
# ---------------------------------------------------------------------------------
_BACKEND_NAMES = {0: "HIP GPU (MI355X)", 1: "HIP GPU (MI355X; CPU requested)", 2: "HIP GPU (MI355X; hybrid requested)",
                  3: "HIP GPU (MI355X; adaptive hybrid requested)"}


_CPU_WARNED = []


def _warn_cpu_backend(config):
    """ComputeBackend.CPU runs the HIP kernels (no CPU solver in this build): say so, once."""
    if int(config.compute_backend) == int(ComputeBackend.CPU) and not _CPU_WARNED:
        _CPU_WARNED.append(True)
        warnings.warn("ComputeBackend.CPU requested: libws_hip has no CPU solver, the HIP kernels run on the GPU "
                      "instead (results bit-identical to the reference CPU solver in fp32 / exact fp64)",
                      RuntimeWarning, stacklevel=3)


class WeatherSimulation:
    def __new__(cls, config=None, *args, **kw):
        # config.devices with more than one device: the one-process multi-GPU simulation
        if (cls is WeatherSimulation and not args and not kw and config is not None
                and len(getattr(config, "devices", None) or ()) > 1):
            return super().__new__(MultiGPUSimulation)
        return super().__new__(cls)

    def __init__(self, config: SimulationConfig, _slab=None, _handle=None, _owner=None):
        self._config_py = config
        self._owner = _owner
        self._ic = None
        self._om = None
        if _handle is not None:  # a slab owned by a SlabGroup
            self._h = ctypes.c_void_p(_handle)
            self._owned = False
            self.row0, self.rows = _slab
            return
        self._owned = True
        c = config._to_c()
        h = ctypes.c_void_p()
        self.row0, self.rows = 0, config.grid_height
        if _slab is None:
            check(lib.ws_sim_create(ctypes.byref(c), ctypes.byref(h)))
        else:
            # (rank, nranks, uid): one rank's slab over RCCL; (rank, nranks, None, xfer_us): the
            # communicator-less measurement slab (ws_hip.h ws_sim_create_slab_emulated)
            rank, nranks, uid = _slab[:3]
            r0, nr = ctypes.c_int32(), ctypes.c_int32()
            if uid is None:
                xfer_us = float(_slab[3]) if len(_slab) > 3 else 0.0
                check(lib.ws_sim_create_slab_emulated(ctypes.byref(c), int(rank), int(nranks), xfer_us,
                                                      ctypes.byref(h), ctypes.byref(r0), ctypes.byref(nr)))
            else:
                idbuf = (ctypes.c_uint8 * _native.COMM_ID_BYTES).from_buffer_copy(uid)
                check(lib.ws_sim_create_slab(ctypes.byref(c), int(rank), int(nranks), idbuf, ctypes.byref(h),
                                             ctypes.byref(r0), ctypes.byref(nr)))
            self.row0, self.rows = r0.value, nr.value
        self._h = h
        _warn_cpu_backend(config)
        _say(f"Using compute backend: {_BACKEND_NAMES.get(int(config.compute_backend), 'HIP GPU (MI355X)')}")

    def __del__(self):
        if getattr(self, "_owned", False) and getattr(self, "_h", None):
            lib.ws_sim_destroy(self._h)
            self._h = None

    def set_initial_condition(self, initial_condition):
        self._ic = initial_condition

    def set_output_manager(self, output_manager):
        self._om = output_manager

    def initialize(self):
        check(lib.ws_sim_initialize(self._h))
        if self._ic is not None:
            self._ic.initialize(self.get_current_grid())
        if self._om is not None:
            self._om.initialize(self)

    def step(self):
        check(lib.ws_sim_step(self._h))

    def _run_native(self, n):
        taken = ctypes.c_int32()
        check(lib.ws_sim_run(self._h, int(n), ctypes.byref(taken)))
        return taken.value

    def run(self, num_steps):
        """weather_simulation.cpp:68-103 (stops after the step at which t >= max_time)."""
        if num_steps <= 0:
            return 0
        t0 = time.perf_counter()
        if self._om is None:
            taken = self._run_native(num_steps)
        else:  # writeOutput every output_interval steps (:84-88): run in chunks ending there
            taken = 0
            interval = self._config_py.output_interval
            while taken < num_steps:
                chunk = num_steps - taken
                if interval > 0:
                    chunk = min(chunk, interval - self.get_current_step() % interval)
                k = self._run_native(chunk)
                taken += k
                if k > 0 and interval > 0 and self.get_current_step() % interval == 0:
                    self._om.write_output(self)
                if k < chunk or self.get_current_time() >= self._max_time():
                    break
        ms = (time.perf_counter() - t0) * 1000.0
        _say(f"Completed {num_steps} steps in {ms:.0f} ms ({ms / num_steps} ms/step)")
        return taken

    def _max_time(self):
        return float(np.float64(self._config_py.max_time) if self._config_py.double_precision
                     else np.float32(self._config_py.max_time))

    def run_until(self, max_time):
        """weather_simulation.cpp:105-115: run(int((T - t) / dt) + 1)."""
        if self._om is not None:
            dtype = np.float64 if self._config_py.double_precision else np.float32
            T, t, dt = dtype(max_time), dtype(self.get_current_time()), dtype(self.get_dt())
            if T <= t:
                return 0
            return self.run(int((T - t) / dt) + 1)
        taken = ctypes.c_int32()
        check(lib.ws_sim_run_until(self._h, float(max_time), ctypes.byref(taken)))
        return taken.value

    def get_current_time(self):
        t = ctypes.c_double()
        check(lib.ws_sim_get_time(self._h, ctypes.byref(t)))
        return t.value

    def get_current_step(self):
        s = ctypes.c_int32()
        check(lib.ws_sim_get_step(self._h, ctypes.byref(s)))
        return s.value

    def get_dt(self):
        d = ctypes.c_double()
        check(lib.ws_sim_get_dt(self._h, ctypes.byref(d)))
        return d.value

    def set_dt(self, dt):
        check(lib.ws_sim_set_dt(self._h, float(dt)))

    def get_config(self):
        c = _native.ws_config_t()
        check(lib.ws_sim_get_config(self._h, ctypes.byref(c)))
        return SimulationConfig._from_c(c, self._config_py.output_path)

    def get_current_grid(self):
        g = ctypes.c_void_p()
        check(lib.ws_sim_grid(self._h, 0, ctypes.byref(g)))
        return WeatherGrid(None, _handle=g.value, _owner=self)

    def get_performance_metrics(self):
        m = _native.ws_metrics_t()
        check(lib.ws_sim_get_metrics(self._h, ctypes.byref(m)))
        out = PerformanceMetrics()
        for name, _ in _native.ws_metrics_t._fields_:
            setattr(out, name, getattr(m, name))
        return out

    def reset_performance_metrics(self):
        check(lib.ws_sim_reset_metrics(self._h))

    # -- extensions
    def synchronize(self):
        check(lib.ws_sim_synchronize(self._h))

    def last_run_stats(self):
        """(device ms, kernel launches) of the last run()/run_until()/step()."""
        ms, n = ctypes.c_double(), ctypes.c_int64()
        check(lib.ws_sim_last_run_stats(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def set_kernel_timing(self, enable=True, reserve=0):
        """Per-launch device timing; `reserve` launches get their events created now."""
        check(lib.ws_sim_set_kernel_timing(self._h, max(2, int(reserve)) if enable and reserve else int(bool(enable))))

    def kernel_timing(self):
        """{stage kind: (launches, total device ms, algorithmic bytes per launch)}"""
        out = {}
        for k in range(8):
            n, ms, b = ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
            check(lib.ws_sim_kernel_timing(self._h, k, ctypes.byref(n), ctypes.byref(ms), ctypes.byref(b)))
            if n.value:
                out[k] = (n.value, ms.value, b.value)
        return out

    def fused_variant(self):
        """(kernel name, rows per segment, output columns per strip) of the fused step kernel
        in use (chosen at the first run)."""
        k, seg, cols = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        check(lib.ws_sim_fused_variant(self._h, ctypes.byref(k), ctypes.byref(seg), ctypes.byref(cols)))
        names = {v: "fused_" + n for n, v in self._KERNELS.items()}
        return names.get(k.value, "stage_kernels"), seg.value, cols.value

    def get_cfl(self, per_level=False, with_time=False):
        """Extension: the CFL number max((|u| + sqrt(g h)) dt / dx, (|v| + sqrt(g h)) dt / dy)
        of the current state by a device reduction (ws_hip.h ws_sim_cfl; on a multi-GPU slab a
        collective over all ranks). per_level=True: (max, per-level array); with_time=True
        also returns the reduction's device milliseconds."""
        c, ms = ctypes.c_double(), ctypes.c_double()
        L = int(self._config_py.num_levels)
        arr = np.empty(max(1, L), np.float64)
        check(lib.ws_sim_cfl(self._h, ctypes.byref(c), arr.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), arr.size,
                             ctypes.byref(ms)))
        out = (c.value, arr) if per_level else c.value
        return (out, ms.value) if with_time else out

    def kernel_occupancy(self):
        """Extension: waves per SIMD a launch of the fused step kernel in use holds (ws_hip.h
        ws_sim_kernel_occupancy; 0 for the per-stage kernels)."""
        n = ctypes.c_int32()
        check(lib.ws_sim_kernel_occupancy(self._h, ctypes.byref(n)))
        return n.value

    def steps_per_launch(self):
        """Extension: time steps one fused launch advances inside run() (1, or 2 / 4 with
        temporal blocking; ws_hip.h ws_sim_steps_per_launch)."""
        n = ctypes.c_int32()
        check(lib.ws_sim_steps_per_launch(self._h, ctypes.byref(n)))
        return n.value

    def slab_schedule(self):
        """Extension: (steps per halo exchange, overlap schedule on) of a slab (ws_hip.h
        ws_sim_slab_schedule; (1, False) for a whole domain)."""
        b, o = ctypes.c_int32(), ctypes.c_int32()
        check(lib.ws_sim_slab_schedule(self._h, ctypes.byref(b), ctypes.byref(o)))
        return b.value, bool(o.value)

    _OVERLAP = {"off": 0, "on": 1, "auto": 2, False: 0, True: 1}
    _KERNELS = {"lds": 0, "dppy": 4, "x2y": 5, "pc": 6, "pc2": 7}

    def set_slab_schedule(self, block=0, overlap="auto"):
        """Extension: steps per halo exchange (block > 0; 0 keeps it) and the overlap schedule
        ("off" / "on" / "auto": chosen from a measured exchange; ws_hip.h
        ws_sim_set_slab_schedule). Every rank of a decomposition must pass the same values."""
        check(lib.ws_sim_set_slab_schedule(self._h, int(block), self._OVERLAP[overlap]))

    def slab_exchange_us(self):
        """Extension: the halo exchange time the auto schedule measured (-1: not measured)."""
        us = ctypes.c_double()
        check(lib.ws_sim_slab_exchange_us(self._h, ctypes.byref(us)))
        return us.value

    def slab_trial_ms(self):
        """Extension: the auto schedule's trial (ms per block period stream-ordered,
        overlapped; max over ranks; (-1, -1) until a trial ran). The overlap is kept iff
        overlapped < stream-ordered x (1 - OVERLAP_MARGIN) (ws_hip.h ws_sim_slab_trial_ms)."""
        ms = (ctypes.c_double * 2)()
        check(lib.ws_sim_slab_trial_ms(self._h, ms))
        return ms[0], ms[1]

    OVERLAP_MARGIN = 0.02  # ws_hip.h WS_OVERLAP_MARGIN

    def pin_variant(self, kernel=None, steps_per_launch=None, seg_rows=None, align=None):
        """Extension: fix (parts of) the fused-kernel variant the autotuner would choose
        (ws_hip.h ws_sim_pin_variant); None leaves a part to the autotuner."""
        check(lib.ws_sim_pin_variant(self._h, -1 if kernel is None else self._KERNELS[kernel],
                                     -1 if steps_per_launch is None else int(steps_per_launch),
                                     -1 if seg_rows is None else int(seg_rows),
                                     -1 if align is None else int(bool(align))))

    def set_numerics(self, mode):
        """Extension: "exact" (bit-for-bit with the reference) or "fast" (FMA re-association,
        the fp64 default; ws_hip.h WS_NUMERICS_*) for the fused step kernels."""
        check(lib.ws_sim_set_numerics(self._h, _native.NUMERICS[mode]))

    def get_numerics(self):
        m = ctypes.c_int32()
        check(lib.ws_sim_get_numerics(self._h, ctypes.byref(m)))
        return {v: k for k, v in _native.NUMERICS.items()}[m.value]

    def comm_allreduce_max(self, value):
        out = ctypes.c_double()
        check(lib.ws_sim_comm_allreduce_max(self._h, float(value), ctypes.byref(out)))
        return out.value

    def comm_barrier(self):
        check(lib.ws_sim_comm_barrier(self._h))


class SlabGroup:
    """Extension: the y-slab decomposition of one global grid inside one process on one
    device (halo rows by device copies, same step schedule as the multi-GPU RCCL path).
    `slab(r)` is a WeatherSimulation view of rank r's rows [row0, row0 + rows)."""

    def __init__(self, config: SimulationConfig, nslabs: int):
        self._config_py = config
        c = config._to_c()
        h = ctypes.c_void_p()
        check(lib.ws_group_create(ctypes.byref(c), int(nslabs), ctypes.byref(h)))
        self._h = h
        self.nslabs = int(nslabs)
        self._slabs = []
        for r in range(self.nslabs):
            s, r0, nr = ctypes.c_void_p(), ctypes.c_int32(), ctypes.c_int32()
            check(lib.ws_group_slab(self._h, r, ctypes.byref(s), ctypes.byref(r0), ctypes.byref(nr)))
            self._slabs.append(WeatherSimulation(config, _slab=(r0.value, nr.value), _handle=s.value, _owner=self))
        self._ic = None

    def __del__(self):
        if getattr(self, "_h", None):
            self._slabs = []
            lib.ws_group_destroy(self._h)
            self._h = None

    def slab(self, rank):
        return self._slabs[rank]

    def set_slab_schedule(self, block=0, overlap="auto"):
        """Every slab's block and overlap schedule (WeatherSimulation.set_slab_schedule)."""
        for s in self._slabs:
            s.set_slab_schedule(block, overlap)

    def pin_variant(self, **kw):
        for s in self._slabs:
            s.pin_variant(**kw)

    def set_initial_condition(self, ic):
        self._ic = ic

    def initialize(self):
        for s in self._slabs:
            check(lib.ws_sim_initialize(s._h))
            if self._ic is not None:
                self._ic.initialize(s.get_current_grid())  # global coordinates, own rows

    def run(self, num_steps):
        taken = ctypes.c_int32()
        check(lib.ws_group_run(self._h, int(num_steps), ctypes.byref(taken)))
        return taken.value

    def gather(self, name):
        """The global (H, W) (or (L, H, W)) field assembled from the slabs."""
        parts = [s.get_current_grid()._get(name) for s in self._slabs]
        return np.concatenate(parts, axis=-2)

    def scatter(self, name, arr):
        """Set a global field from a (H, W) / (L, H, W) array."""
        a = np.asarray(arr)
        for s in self._slabs:
            s.get_current_grid()._set(name, a[..., s.row0:s.row0 + s.rows, :])


def new_comm_id() -> bytes:
    """Extension: a fresh RCCL communicator id (ws_hip.h ws_comm_get_unique_id, 128 bytes) for a
    decomposition over processes: create it on ONE rank and hand the same bytes to every rank
    (any channel: torch.distributed, MPI, a file), then build each rank's SlabSimulation."""
    buf = (ctypes.c_uint8 * _native.COMM_ID_BYTES)()
    check(lib.ws_comm_get_unique_id(buf))
    return bytes(buf)


class SlabSimulation(WeatherSimulation):
    """Extension: rank `rank` of `nranks` processes, one GPU each
    (config.device_id), owning rows [row0, row0 + rows) of the global grid config describes;
    halo rows move over RCCL inside run() (ws_hip.h ws_sim_create_slab). Every collective call
    (run, step, run_until, get_cfl, initialize's IC) must be made by every rank alike. Fields
    read or written through its grid are its own rows; results equal one domain bit for bit.
    (One process driving several GPUs: MultiGPUSimulation / config.devices.)"""

    def __init__(self, config: SimulationConfig, rank: int, nranks: int, comm_id: bytes):
        if comm_id is None or len(comm_id) != _native.COMM_ID_BYTES:
            raise ValueError(f"comm_id must be the {_native.COMM_ID_BYTES} bytes of new_comm_id() from one rank")
        super().__init__(config, _slab=(int(rank), int(nranks), bytes(comm_id)))
        self.rank, self.nranks = int(rank), int(nranks)


class SlabbedGrid(WeatherGrid):
    """Extension: the global view of one grid slot of a y-slab decomposition (a
    MultiGPUSimulation's current grid). Field reads assemble the (H, W) / (L, H, W) array
    from the slabs' owned rows, writes scatter it; `slab_grids` are the per-slab grids."""

    def __init__(self, grids, owner):
        self._owner = owner
        self._owned = False
        self._h = None
        self.slab_grids = list(grids)
        g0 = self.slab_grids[0]
        self._W, self._L, self._dtype, self._ws_dtype = g0._W, g0._L, g0._dtype, g0._ws_dtype
        self._rows, r0 = [], 0
        for g in self.slab_grids:
            self._rows.append((r0, g._H))
            r0 += g._H
        self._H = r0

    def reset(self):
        for g in self.slab_grids:
            g.reset()

    def get_dx(self):
        return self.slab_grids[0].get_dx()

    def get_dy(self):
        return self.slab_grids[0].get_dy()

    def set_spacing(self, dx, dy):
        for g in self.slab_grids:
            g.set_spacing(dx, dy)

    def calculate_diagnostics(self):
        for g in self.slab_grids:
            g.calculate_diagnostics()

    def _get(self, name, level=None):
        return np.concatenate([g._get(name, level) for g in self.slab_grids], axis=-2)

    def _set(self, name, arr, level=None):
        a = np.asarray(arr)
        if a.ndim not in (2, 3):
            raise RuntimeError("Number of dimensions must be 2")
        if a.shape[-2:] != (self._H, self._W):
            raise RuntimeError("Array dimensions must match field dimensions")
        for g, (r0, n) in zip(self.slab_grids, self._rows):
            g._set(name, a[..., r0:r0 + n, :], level)
        if name in ("u", "v") and self._owner is not None:
            self._owner._diag_halo()  # seam diagnostics read the neighbours' new rows

    def device_field(self, name):
        raise NotImplementedError("a multi-GPU grid has one device field per slab: use slab_grids[r].device_field")


class MultiGPUSimulation(WeatherSimulation):
    """Extension: ONE simulation object over several GPUs of one process --
    `WeatherSimulation(config)` with `config.devices = [0, 1, ...]`, or
    `MultiGPUSimulation(config, devices=[...])`. The global grid is y-slab decomposed, slab r
    on devices[r]; distinct devices exchange halo rows over RCCL (xGMI), each slab driven by a
    host thread of the library (ws_hip.h ws_multi_*), all-equal devices share one GPU through
    device copies. The API is the single-domain one: run / step / run_until, the current
    grid's fields as global arrays, bitwise identical to one domain (and the reference)."""

    def __init__(self, config: SimulationConfig, devices=None):
        self._config_py = config
        self._owner = None
        self._ic = None
        self._om = None
        self._owned = False  # the slabs belong to the multi simulation (ws_multi_destroy)
        devices = [int(d) for d in (config.devices if devices is None else devices)]
        if not devices:
            raise ValueError("MultiGPUSimulation needs at least one device")
        arr = (ctypes.c_int32 * len(devices))(*devices)
        h = ctypes.c_void_p()
        check(lib.ws_multi_create(ctypes.byref(config._to_c()), arr, len(devices), ctypes.byref(h)))
        self._m = h
        self.devices = devices
        n, shared = ctypes.c_int32(), ctypes.c_int32()
        check(lib.ws_multi_size(self._m, ctypes.byref(n), ctypes.byref(shared)))
        self.shared_device = bool(shared.value)
        self._slabs = []
        for r in range(n.value):
            s, r0, nr = ctypes.c_void_p(), ctypes.c_int32(), ctypes.c_int32()
            check(lib.ws_multi_slab(self._m, r, ctypes.byref(s), ctypes.byref(r0), ctypes.byref(nr)))
            self._slabs.append(WeatherSimulation(config, _slab=(r0.value, nr.value), _handle=s.value, _owner=self))
        self._h = self._slabs[0]._h  # per-slab state every slab shares (time, step, dt, variant) is read here
        self.row0, self.rows = 0, config.grid_height
        _warn_cpu_backend(config)
        _say(f"Using compute backend: HIP GPU (MI355X) x {len(devices)} "
             f"({'one device, device-copy halos' if self.shared_device else 'RCCL halos'})")

    def __del__(self):
        if getattr(self, "_m", None):
            self._slabs = []
            lib.ws_multi_destroy(self._m)
            self._m = None

    @property
    def nslabs(self):
        return len(self._slabs)

    def slab(self, rank):
        """Rank `rank`'s slab (a WeatherSimulation view of rows [row0, row0 + rows))."""
        return self._slabs[rank]

    def initialize(self):
        for s in self._slabs:
            check(lib.ws_sim_initialize(s._h))
        if self._ic is not None:
            self._ic.initialize(self.get_current_grid())
        self._diag_halo()
        if self._om is not None:
            self._om.initialize(self)

    def _diag_halo(self):
        check(lib.ws_multi_exchange_diag_halo(self._m))

    def step(self):
        check(lib.ws_multi_step(self._m))

    def _run_native(self, n):
        taken = ctypes.c_int32()
        check(lib.ws_multi_run(self._m, int(n), ctypes.byref(taken)))
        return taken.value

    def run_until(self, max_time):
        if self._om is not None:
            return super().run_until(max_time)
        taken = ctypes.c_int32()
        check(lib.ws_multi_run_until(self._m, float(max_time), ctypes.byref(taken)))
        return taken.value

    def set_dt(self, dt):
        for s in self._slabs:
            s.set_dt(dt)

    def get_current_grid(self):
        return SlabbedGrid([s.get_current_grid() for s in self._slabs], self)

    def reset_performance_metrics(self):
        for s in self._slabs:
            s.reset_performance_metrics()

    def synchronize(self):
        check(lib.ws_multi_synchronize(self._m))

    def set_kernel_timing(self, enable=True, reserve=0):
        for s in self._slabs:
            s.set_kernel_timing(enable, reserve)

    def get_cfl(self, per_level=False, with_time=False):
        c, ms = ctypes.c_double(), ctypes.c_double()
        arr = np.empty(max(1, int(self._config_py.num_levels)), np.float64)
        check(lib.ws_multi_cfl(self._m, ctypes.byref(c), arr.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), arr.size,
                               ctypes.byref(ms)))
        out = (c.value, arr) if per_level else c.value
        return (out, ms.value) if with_time else out

    def set_slab_schedule(self, block=0, overlap="auto"):
        for s in self._slabs:
            s.set_slab_schedule(block, overlap)

    def pin_variant(self, **kw):
        for s in self._slabs:
            s.pin_variant(**kw)

    def set_numerics(self, mode):
        for s in self._slabs:
            s.set_numerics(mode)

    def comm_allreduce_max(self, value):
        return float(value)  # one process holds every rank

    def comm_barrier(self):
        self.synchronize()


# ---------------------------------------------------------------------------------
# KernelAdapter plugin API (gpu_adaptability.hpp:242-379)
# ---------------------------------------------------------------------------------
class KernelAdapter:
    def initialize(self, device_id=0):
        raise NotImplementedError

    def is_compatible(self):
        raise NotImplementedError

    def get_name(self):
        raise NotImplementedError

    def get_priority(self):
        raise NotImplementedError


class HIPKernelAdapter(KernelAdapter):
    """The MI355X adapter: one forward-Euler step in -> out per call (the semantics of the
    reference's fused shallowWaterStepKernel_*). Returns device milliseconds; -1.0 when
    not initialized (HybridExecutionManager::executeHybridStep convention)."""

    def __init__(self, gravity=9.81, coriolis_f=0.0):
        self.gravity, self.coriolis_f = gravity, coriolis_f
        self._ready = False

    def initialize(self, device_id=0):
        self._ready = _native.is_available() and 0 <= device_id < _native.device_count()
        return self._ready

    def is_compatible(self):
        return _native.is_available()

    def get_name(self):
        return "HIPAdapter"

    def get_priority(self):
        return 100

    def _exec(self, fn, in_grid, out_grid, dt):
        if not self._ready:
            return -1.0
        ms = ctypes.c_double()
        check(fn(in_grid._h, out_grid._h, float(dt), float(self.gravity), float(self.coriolis_f), ctypes.byref(ms)))
        return ms.value

    def execute_shallow_water_step(self, in_grid, out_grid, dt):
        return self._exec(lib.ws_adapter_execute_shallow_water_step, in_grid, out_grid, dt)

    def execute_barotropic_step(self, in_grid, out_grid, dt):
        return self._exec(lib.ws_adapter_execute_barotropic_step, in_grid, out_grid, dt)

    def execute_primitive_equations_step(self, in_grid, out_grid, dt):
        return self._exec(lib.ws_adapter_execute_primitive_equations_step, in_grid, out_grid, dt)

    def execute_gcm_step(self, in_grid, out_grid, dt):
        return self._exec(lib.ws_adapter_execute_gcm_step, in_grid, out_grid, dt)

    def calculate_diagnostics(self, grid):
        if not self._ready:
            return -1.0
        ms = ctypes.c_double()
        check(lib.ws_adapter_calculate_diagnostics(grid._h, ctypes.byref(ms)))
        return ms.value


class KernelAdapterFactory:
    """gpu_adaptability.cpp:544-592"""
    _instance = None

    def __init__(self):
        self._adapters = []

    @classmethod
    def get_instance(cls):
        if cls._instance is None:
            cls._instance = cls()
            cls._instance.register_adapter(HIPKernelAdapter())
        return cls._instance

    def register_adapter(self, adapter):
        self._adapters.append(adapter)

    def get_best_adapter(self, device_id=0):
        best = None
        for a in self._adapters:
            if a.is_compatible() and (best is None or a.get_priority() > best.get_priority()):
                best = a
        if best is not None:
            best.initialize(device_id)
        return best

    def get_adapter(self, name, device_id=0):
        for a in self._adapters:
            if a.get_name() == name:
                a.initialize(device_id)
                return a
        return None

    def get_available_adapters(self):
        return [a.get_name() for a in self._adapters]


class AdaptiveKernelManager:
    """AdaptiveKernelManager (gpu_adaptability.hpp:128-237) reduced to what the Python API
    uses: device detection and capabilities. There is one device kind, so workload ratios
    are 1.0 (all on the GPU) and the optimal backend is the GPU."""
    _instance = None

    def __init__(self):
        self._caps = DeviceCapabilities()
        self._init = False

    @classmethod
    def get_instance(cls):
        if cls._instance is None:
            cls._instance = cls()
        return cls._instance

    def initialize(self, device_id=0):
        if _native.is_available():
            info = _native.ws_device_info_t()
            check(lib.ws_device_info(int(device_id), ctypes.byref(info)))
            self._caps = DeviceCapabilities(info)
        else:
            self._caps = DeviceCapabilities()
            self._caps.device_type = DeviceType.CPU
        self._init = True
        return True

    def is_cuda_available(self):
        return _native.is_available()

    def get_device_capabilities(self):
        if not self._init:
            self.initialize()
        return self._caps

    def get_gpu_workload_ratio(self, *args, **kwargs):
        return 1.0 if self.is_cuda_available() else 0.0

    def determine_optimal_backend(self, *args, **kwargs):
        return ComputeBackend.CUDA


# ---------------------------------------------------------------------------------
# High-level wrapper and helpers (the reference's weather_simulation.py:194-520)
#
# Table-driven: the string-argument maps, the initial-condition parameter lists and the
# snapshot / device-info layouts are data; the behaviour (defaults, silent fallback for an
# unknown name, snapshot every output_interval steps, None + a message on a bad IC) is the
# reference's, pinned by tests/test_gpu_parity.py::test_wrapper_snapshots_and_errors and
# tests/test_output.py.
# ---------------------------------------------------------------------------------

# wrapper string arguments -> enum values; an unknown string takes the default, silently
# (reference :235-269)
_ENUM_ARGS = {
    "model": ({"shallow_water": SimulationModel.ShallowWater, "barotropic": SimulationModel.Barotropic,
               "primitive": SimulationModel.PrimitiveEquations, "general": SimulationModel.General},
              SimulationModel.ShallowWater),
    "integration_method": ({"euler": IntegrationMethod.ExplicitEuler, "rk2": IntegrationMethod.RungeKutta2,
                            "rk4": IntegrationMethod.RungeKutta4, "adams_bashforth": IntegrationMethod.AdamsBashforth,
                            "semi_implicit": IntegrationMethod.SemiImplicit},
                           IntegrationMethod.RungeKutta4),
    "compute_backend": ({"cuda": ComputeBackend.CUDA, "hip": ComputeBackend.CUDA, "cpu": ComputeBackend.CPU,
                         "hybrid": ComputeBackend.Hybrid, "adaptive": ComputeBackend.AdaptiveHybrid},
                        ComputeBackend.AdaptiveHybrid),
}


def _enum_arg(field, value):
    names, default = _ENUM_ARGS[field]
    return names.get(value.lower(), default) if isinstance(value, str) else value


# initial condition name -> (class, constructor parameters as (keyword, default)) --
# the keywords and defaults create_initial_condition accepts (reference :376-470)
_IC_TABLE = {
    "uniform": (UniformInitialCondition, (("u", 0.0), ("v", 0.0), ("h", 10.0), ("p", 1000.0), ("t", 300.0),
                                          ("q", 0.0))),
    "random": (RandomInitialCondition, (("seed", 0), ("amplitude", 1.0))),
    "zonal_flow": (ZonalFlowInitialCondition, (("u_max", 10.0), ("h_mean", 10.0), ("beta", 0.1))),
    "vortex": (VortexInitialCondition, (("x_center", 0.5), ("y_center", 0.5), ("radius", 0.1), ("strength", 10.0),
                                        ("h_mean", 10.0))),
    "jet_stream": (JetStreamInitialCondition, (("y_center", 0.5), ("width", 0.1), ("strength", 10.0),
                                               ("h_mean", 10.0))),
    "breaking_wave": (BreakingWaveInitialCondition, (("amplitude", 1.0), ("wavelength", 0.2), ("h_mean", 10.0))),
    "front": (FrontInitialCondition, (("y_position", 0.5), ("width", 0.05), ("temp_difference", 10.0),
                                      ("wind_shear", 5.0))),
    "mountain": (MountainInitialCondition, (("x_center", 0.3), ("y_center", 0.5), ("radius", 0.1), ("height", 1.0),
                                            ("u_base", 5.0))),
    "atmospheric_profile": (AtmosphericProfileInitialCondition, (("profile_name", "standard"),)),
}

# the wrapper's snapshot dict: key -> how to read it from (simulation, current grid)
_SNAPSHOT = (
    ("time", lambda sim, g: sim.get_current_time()),
    ("step", lambda sim, g: sim.get_current_step()),
    ("u", lambda sim, g: g.get_velocity_field()[0].copy()),
    ("v", lambda sim, g: g.get_velocity_field()[1].copy()),
    ("height", lambda sim, g: g.get_height_field().copy()),
    ("vorticity", lambda sim, g: g.get_vorticity_field().copy()),
)


class WeatherSimulationWrapper:
    """High-level wrapper: string arguments, lazy initialisation and periodic snapshots
    around one WeatherSimulation (same constructor signature and defaults as the reference,
    plus double_precision / num_levels, and devices=[...] for one simulation over several GPUs)."""

    def __init__(self, width: int = 256, height: int = 256, model: Union[str, int] = "shallow_water", dt: float = 0.01,
                 integration_method: Union[str, int] = "rk4", backend: Union[str, int] = "adaptive",
                 device_id: int = 0, threads: int = 0, output_interval: int = 10, output_path: str = "./output",
                 double_precision: bool = False, num_levels: int = 1, devices: Optional[List[int]] = None):
        cfg = SimulationConfig()
        for field, value in (("grid_width", width), ("grid_height", height), ("dt", dt),
                             ("output_interval", output_interval), ("output_path", output_path),
                             ("device_id", device_id), ("num_threads", threads),
                             ("double_precision", double_precision), ("num_levels", num_levels),
                             ("model", _enum_arg("model", model)),
                             ("integration_method", _enum_arg("integration_method", integration_method)),
                             ("compute_backend", _enum_arg("compute_backend", backend))):
            setattr(cfg, field, value)
        cfg.devices = list(devices) if devices else None  # extension: > 1 device = MultiGPUSimulation
        self.config = cfg
        self.simulation = WeatherSimulation(cfg)
        self.initialized = False
        self.output_data = []

    def set_initial_condition(self, condition_name: str, **kwargs):
        ic = create_initial_condition(condition_name, **kwargs)
        if ic:
            self.simulation.set_initial_condition(ic)

    def initialize(self):
        self.simulation.initialize()
        self.initialized = True

    def _ready(self):
        if not self.initialized:
            self.initialize()

    def step(self):
        self._ready()
        self.simulation.step()
        every = self.config.output_interval
        if every > 0 and self.simulation.get_current_step() % every == 0:
            self._store_output()

    def _timed(self, advance, describe):
        self._ready()
        t0 = time.time()
        advance()
        ms = (time.time() - t0) * 1000
        _say(describe(ms))

    def run(self, steps: int):
        self._timed(lambda: self.simulation.run(steps),
                    lambda ms: f"Completed {steps} steps in {ms:.2f} ms ({ms / steps:.2f} ms/step)")

    def run_until(self, max_time: float):
        # the per-step figure divides by the simulation's total step count, as the reference does
        self._timed(lambda: self.simulation.run_until(max_time),
                    lambda ms: f"Reached time {max_time} in {ms:.2f} ms "
                               f"({ms / self.simulation.get_current_step():.2f} ms/step)")

    def get_grid(self):
        return self.simulation.get_current_grid()

    def get_metrics(self):
        return self.simulation.get_performance_metrics()

    def get_output_data(self):
        return self.output_data

    def _store_output(self):
        grid = self.simulation.get_current_grid()
        self.output_data.append({key: read(self.simulation, grid) for key, read in _SNAPSHOT})


def create_initial_condition(name: str, **kwargs) -> Optional[object]:
    """An initial condition by name with keyword parameters (defaults: _IC_TABLE); other
    names go to the factory. On failure: a message and None, as the reference."""
    try:
        if name not in _IC_TABLE:
            return InitialConditionFactory.get_instance().create_initial_condition(name)
        cls, params = _IC_TABLE[name]
        return cls(*(kwargs.get(key, default) for key, default in params))
    except Exception as e:
        print(f"Error creating initial condition '{name}': {e}")
        return None


def get_available_initial_conditions() -> List[str]:
    try:
        return InitialConditionFactory.get_instance().get_available_initial_conditions()
    except Exception:
        return list(_IC_TABLE)


def is_cuda_available() -> bool:
    """True when the HIP device (MI355X) is usable (the reference's name is kept)."""
    try:
        return AdaptiveKernelManager.get_instance().is_cuda_available()
    except Exception:
        return False


_DEVICE_TYPE_NAMES = {DeviceType.Unknown: "Unknown", DeviceType.CPU: "CPU", DeviceType.JetsonOrinNX: "Jetson Orin NX",
                      DeviceType.T4: "NVIDIA T4", DeviceType.HighEndGPU: "High-End GPU",
                      DeviceType.OtherGPU: "Other GPU"}
# get_device_info's keys: key -> how to read it from (capabilities, manager)
_DEVICE_INFO = (
    ("device_type", lambda c, m: _DEVICE_TYPE_NAMES.get(c.device_type, "Unknown")),
    ("device_name", lambda c, m: c.device_name),
    ("compute_capability", lambda c, m: f"{c.compute_capability_major}.{c.compute_capability_minor}"),
    ("cuda_cores", lambda c, m: c.cuda_cores),
    ("multiprocessors", lambda c, m: c.multiprocessors),
    ("global_memory_mb", lambda c, m: c.global_memory / (1024 * 1024)),
    ("compute_power_ratio", lambda c, m: c.compute_power_ratio),
    ("cuda_available", lambda c, m: m.is_cuda_available()),
    ("arch", lambda c, m: c.arch),
)


def get_device_info() -> Dict:
    try:
        manager = AdaptiveKernelManager.get_instance()
        manager.initialize()
        caps = manager.get_device_capabilities()
        return {key: read(caps, manager) for key, read in _DEVICE_INFO}
    except Exception as e:
        return {"device_type": "Unknown", "device_name": "Unknown", "error": str(e), "cuda_available": False}


register_all_initial_conditions()
