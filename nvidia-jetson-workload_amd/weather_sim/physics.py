"""Physics-mode barotropic vorticity model over libws_hip.so.

BASELINE config C3 describes a barotropic "Jacobian + Laplacian" model. The reference has
none: its `SimulationModel.Barotropic` runs the shallow-water tendencies
(src/weather-sim/cpp/src/weather_simulation.cpp:542-560), which `WeatherSimulation`
reproduces bit for bit. This class is the physical model that description names -- a new
model, defined by oracle/bvort_oracle.py and checked against it and against analytic
solutions (tests/test_bvort_oracle.py, tests/test_gpu_bvort.py):

    d(zeta)/dt = -J(psi, zeta) - beta * d(psi)/dx + nu * lap(zeta),    lap(psi) = zeta

on a doubly periodic grid: Arakawa 9-point Jacobian, 5-point Laplacian, spectral Poisson
inverse (hipFFT), Euler / RK2 midpoint / classical RK4. It takes the reference's
`SimulationConfig` and reads the fields the reference accepts but never uses: `beta` and
`viscosity` (weather_sim.hpp:176-178).

    cfg = SimulationConfig(); cfg.grid_width = cfg.grid_height = 2048
    cfg.beta, cfg.viscosity, cfg.dt = 1e-3, 1e-4, 0.05
    m = BarotropicVorticityModel(cfg)
    m.set_vorticity(zeta0); m.run(100); u, v = m.get_velocity_field()
"""
import ctypes

import numpy as np

from ._native import WS_F32, WS_F64, check, lib

_FIELDS = {"vorticity": 0, "streamfunction": 1, "u": 2, "v": 3}


class BarotropicVorticityModel:
    """One barotropic vorticity model on the device (no CPU path: fails without a GPU)."""

    _POISSON = {"auto": 0, "hipfft": 1}

    def __init__(self, config, poisson="auto", devices=None, slab=None):
        """poisson: "auto" (LDS-resident FFT passes on power-of-two grids up to 4096, hipFFT
        otherwise) or "hipfft" (hipFFT's 2-D plans always; ws_hip.h ws_bvort_create_poisson).

        Slab decomposition (power-of-two grids; bitwise equal to one domain): `devices=[...]`
        (or `config.devices` with more than one entry) -- one model over len(devices) slabs in
        this process, whole fields in and out; `slab=(rank, nranks, comm_id)` -- one rank of a
        process-per-GPU decomposition over RCCL, fields of the rank's rows [row0, row0 + rows).
        """
        from ._native import COMM_ID_BYTES
        from .weather_simulation import SimulationConfig
        if not isinstance(config, SimulationConfig):
            raise TypeError("BarotropicVorticityModel expects a SimulationConfig")
        if poisson not in self._POISSON:
            raise ValueError(f"poisson must be one of {sorted(self._POISSON)}")
        if devices is None and slab is None and len(getattr(config, "devices", None) or ()) > 1:
            devices = config.devices
        if devices is not None and slab is not None:
            raise ValueError("devices= and slab= are exclusive")
        self._cfg = config
        raw = config._to_c()
        h = ctypes.c_void_p()
        mode = self._POISSON[poisson]
        if slab is not None:
            rank, nranks, comm_id = slab
            if comm_id is None or len(comm_id) != COMM_ID_BYTES:
                raise ValueError(f"comm_id must be {COMM_ID_BYTES} bytes (weather_sim.new_comm_id())")
            idb = (ctypes.c_uint8 * COMM_ID_BYTES)(*comm_id)
            r0, nr = ctypes.c_int32(), ctypes.c_int32()
            check(lib.ws_bvort_create_slab(ctypes.byref(raw), mode, int(rank), int(nranks), idb, ctypes.byref(h),
                                           ctypes.byref(r0), ctypes.byref(nr)))
        elif devices is not None:
            devs = [int(d) for d in devices]
            if not devs:
                raise ValueError("devices must name at least one device")
            arr = (ctypes.c_int32 * len(devs))(*devs)
            check(lib.ws_bvort_create_multi(ctypes.byref(raw), mode, arr, len(devs), ctypes.byref(h)))
        else:
            check(lib.ws_bvort_create_poisson(ctypes.byref(raw), mode, ctypes.byref(h)))
        self._h = h
        ns, r0, nr = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        check(lib.ws_bvort_layout(self._h, ctypes.byref(ns), ctypes.byref(r0), ctypes.byref(nr)))
        self.nslabs, self.row0, self.rows = ns.value, r0.value, nr.value
        # a process's slab holds its own rows only
        self.width, self.height = int(config.grid_width), self.rows
        self.global_height = int(config.grid_height)
        self.dtype = np.float64 if config.double_precision else np.float32

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.ws_bvort_destroy(h)
            self._h = None

    # -- state ---------------------------------------------------------------------
    def set_vorticity(self, zeta):
        a = np.ascontiguousarray(zeta)
        if a.ndim != 2:
            raise RuntimeError("vorticity must be a 2-D (height, width) array")
        if a.dtype not in (np.float32, np.float64):
            a = a.astype(np.float64)
        code = WS_F64 if a.dtype == np.float64 else WS_F32
        check(lib.ws_bvort_set_vorticity(self._h, a.ctypes.data_as(ctypes.c_void_p), a.shape[0], a.shape[1], code))

    def _get(self, which):
        out = np.empty((self.height, self.width), dtype=self.dtype)
        code = WS_F64 if self.dtype == np.float64 else WS_F32
        check(lib.ws_bvort_get_field(self._h, _FIELDS[which], out.ctypes.data_as(ctypes.c_void_p), self.height,
                                     self.width, code))
        return out

    def get_vorticity_field(self):
        return self._get("vorticity")

    def get_streamfunction(self):
        return self._get("streamfunction")

    def get_velocity_field(self):
        """(u, v) = (-d(psi)/dy, d(psi)/dx), centred differences."""
        return self._get("u"), self._get("v")

    # -- stepping ------------------------------------------------------------------
    def step(self):
        self.run(1)

    def run(self, num_steps):
        check(lib.ws_bvort_run(self._h, int(num_steps)))
        return int(num_steps)

    def _state(self):
        t, s, ms, n = ctypes.c_double(), ctypes.c_int32(), ctypes.c_double(), ctypes.c_int64()
        check(lib.ws_bvort_get_state(self._h, ctypes.byref(t), ctypes.byref(s), ctypes.byref(ms), ctypes.byref(n)))
        return t.value, s.value, ms.value, n.value

    def get_current_time(self):
        return self._state()[0]

    def get_current_step(self):
        return self._state()[1]

    def last_run_stats(self):
        """(device ms of the last run(), kernel + FFT launches it made)"""
        _, _, ms, n = self._state()
        return ms, n

    # -- diagnostics (host reductions of fields already copied out) -----------------
    def energy(self):
        """Discrete kinetic energy -1/2 sum(psi * zeta): conserved by the Arakawa Jacobian."""
        return -0.5 * float(np.sum(self.get_streamfunction().astype(np.float64) *
                                   self.get_vorticity_field().astype(np.float64)))

    def enstrophy(self):
        return 0.5 * float(np.sum(self.get_vorticity_field().astype(np.float64) ** 2))


_LPE_FIELDS = {"u": 0, "v": 1, "h": 2}


class LayeredPrimitiveEquationsModel:
    """Physics-mode primitive equations: `config.num_levels` stacked
    constant-density layers (k = 0 on top) over a flat bottom, doubly periodic, coupled by
    hydrostatic balance through the Montgomery potential

        M_0 = g * eta_0,  M_k = M_{k-1} + g' * eta_k     (eta_k = sum_{j >= k} h_j)
        du/dt = -u u_x - v u_y - M_x + f v,  dv/dt = -u v_x - v v_y - M_y - f u,
        dh/dt = -(h u)_x - (h v)_y

    -- the "3D stencil, vertical columns" model BASELINE's C4 describes, which the reference
    never implemented (its PrimitiveEquations model steps each level with the SWE tendencies,
    weather_simulation.cpp:542-560; `WeatherSimulation` reproduces that bit for bit). Defined
    by oracle/layered_pe_oracle.py; g = config.gravity, f = config.coriolis_f,
    g' = `reduced_gravity`. Fields are (levels, height, width) arrays; h is layer thickness.

    Slab decomposition (y-slabs around the periodic ring, one halo row per level refreshed
    before every RK stage; bitwise identical to one domain):
      * `devices=[d0, d1, ...]` (or `config.devices` with more than one entry): one model over
        len(devices) slabs in this process, slab r on devices[r] (repeats share a device);
        the API is unchanged -- fields are the whole (levels, height, width) arrays;
      * `slab=(rank, nranks, comm_id)`: one rank of a process-per-GPU decomposition over RCCL
        (`comm_id` from weather_sim.new_comm_id() on one rank, the same bytes everywhere);
        fields are the rank's rows, (levels, rows, width), rows [row0, row0 + rows); run() is
        collective.
    """

    def __init__(self, config, reduced_gravity=0.05, devices=None, slab=None):
        from ._native import COMM_ID_BYTES
        from .weather_simulation import SimulationConfig
        if not isinstance(config, SimulationConfig):
            raise TypeError("LayeredPrimitiveEquationsModel expects a SimulationConfig")
        raw = config._to_c()
        h = ctypes.c_void_p()
        if devices is None and slab is None and len(getattr(config, "devices", None) or ()) > 1:
            devices = config.devices
        if devices is not None and slab is not None:
            raise ValueError("devices= and slab= are exclusive")
        if slab is not None:
            rank, nranks, comm_id = slab
            if comm_id is None or len(comm_id) != COMM_ID_BYTES:
                raise ValueError(f"comm_id must be {COMM_ID_BYTES} bytes (weather_sim.new_comm_id())")
            idb = (ctypes.c_uint8 * COMM_ID_BYTES)(*comm_id)
            r0, nr = ctypes.c_int32(), ctypes.c_int32()
            check(lib.ws_lpe_create_slab(ctypes.byref(raw), float(reduced_gravity), int(rank), int(nranks), idb,
                                         ctypes.byref(h), ctypes.byref(r0), ctypes.byref(nr)))
        elif devices is not None:
            devs = [int(d) for d in devices]
            if not devs:
                raise ValueError("devices must name at least one device")
            arr = (ctypes.c_int32 * len(devs))(*devs)
            check(lib.ws_lpe_create_multi(ctypes.byref(raw), float(reduced_gravity), arr, len(devs),
                                          ctypes.byref(h)))
        else:
            check(lib.ws_lpe_create(ctypes.byref(raw), float(reduced_gravity), ctypes.byref(h)))
        self._h = h
        ns, r0, nr = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        check(lib.ws_lpe_layout(self._h, ctypes.byref(ns), ctypes.byref(r0), ctypes.byref(nr)))
        self.nslabs, self.row0, self.rows = ns.value, r0.value, nr.value
        self.levels = int(config.num_levels)
        # a process's slab holds its own rows only
        self.width, self.height = int(config.grid_width), self.rows
        self.global_height = int(config.grid_height)
        self.dtype = np.float64 if config.double_precision else np.float32
        self.reduced_gravity = float(reduced_gravity)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.ws_lpe_destroy(h)
            self._h = None

    def _shape(self):
        return (self.levels, self.height, self.width)

    def set_field(self, name, arr):
        a = np.ascontiguousarray(np.asarray(arr, dtype=self.dtype))
        if a.shape != self._shape():
            raise RuntimeError(f"{name}: expected shape {self._shape()}, got {a.shape}")
        code = WS_F64 if self.dtype == np.float64 else WS_F32
        check(lib.ws_lpe_set_field(self._h, _LPE_FIELDS[name], a.ctypes.data_as(ctypes.c_void_p), *a.shape, code))

    def get_field(self, name):
        out = np.empty(self._shape(), dtype=self.dtype)
        code = WS_F64 if self.dtype == np.float64 else WS_F32
        check(lib.ws_lpe_get_field(self._h, _LPE_FIELDS[name], out.ctypes.data_as(ctypes.c_void_p), *out.shape, code))
        return out

    def set_state(self, u, v, h):
        for name, a in (("u", u), ("v", v), ("h", h)):
            self.set_field(name, a)

    def get_state(self):
        return self.get_field("u"), self.get_field("v"), self.get_field("h")

    def step(self):
        self.run(1)

    def run(self, num_steps):
        check(lib.ws_lpe_run(self._h, int(num_steps)))
        return int(num_steps)

    def _st(self):
        t, s, ms, n = ctypes.c_double(), ctypes.c_int32(), ctypes.c_double(), ctypes.c_int64()
        check(lib.ws_lpe_get_state(self._h, ctypes.byref(t), ctypes.byref(s), ctypes.byref(ms), ctypes.byref(n)))
        return t.value, s.value, ms.value, n.value

    def get_current_time(self):
        return self._st()[0]

    def get_current_step(self):
        return self._st()[1]

    def last_run_stats(self):
        """(device ms of the last run(), kernel launches it made)"""
        _, _, ms, n = self._st()
        return ms, n

    def layer_mass(self):
        """sum of h over each layer (conserved exactly by the flux-form continuity equation)"""
        return self.get_field("h").astype(np.float64).sum(axis=(1, 2))
