"""ctypes front-end of the CPU oracle (oracle/ws_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker; the product package (nvidia-jetson-workload_amd/weather_sim) never imports it.
The restatement follows /root/reference/src/weather-sim/cpp/src/weather_simulation.cpp
(see ws_oracle_impl.h for the file:line map) and is pinned bitwise against the reference's
own outputs in tests/golden/ (tests/test_oracle.py).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

FIELD_IDS = {"u": 0, "v": 1, "h": 2, "p": 3, "t": 4, "q": 5, "vort": 6, "div": 7}


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        for sfx in ("f32", "f64"):
            f = getattr(lib, f"ws_oracle_{sfx}_create")
            f.restype = ctypes.c_void_p
            f.argtypes = [ctypes.c_int] * 4 + [ctypes.c_double] * 6
            for name, res, args in (
                ("destroy", None, [ctypes.c_void_p]),
                ("initialize", None, [ctypes.c_void_p]),
                ("set_field", None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
                ("get_field", None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
                ("calc_diagnostics", None, [ctypes.c_void_p]),
                ("get_time", ctypes.c_double, [ctypes.c_void_p]),
                ("get_step", ctypes.c_int, [ctypes.c_void_p]),
                ("set_dt", None, [ctypes.c_void_p, ctypes.c_double]),
                ("step", None, [ctypes.c_void_p]),
                ("run", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
                ("run_until", ctypes.c_int, [ctypes.c_void_p, ctypes.c_double]),
                ("tendency", None, [ctypes.c_void_p] * 6 + [ctypes.c_int] * 2 + [
                    ctypes.c_float if sfx == "f32" else ctypes.c_double] * 4),
            ):
                fn = getattr(lib, f"ws_oracle_{sfx}_{name}")
                fn.restype = res
                fn.argtypes = args
        _lib = lib
    return _lib


class OracleSim:
    """Reference-equivalent CPU simulation (2-D, one level)."""

    def __init__(self, width, height, model=0, method=2, dx=1.0, dy=1.0, dt=0.01, gravity=9.81,
                 coriolis_f=0.0, max_time=10.0, precision="f32"):
        self.lib = _load()
        self.sfx = precision
        self.dtype = np.float32 if precision == "f32" else np.float64
        self.W, self.H = width, height
        self._p = getattr(self.lib, f"ws_oracle_{self.sfx}_create")(
            width, height, model, method, dx, dy, dt, gravity, coriolis_f, max_time)
        if not self._p:
            raise ValueError("Grid dimensions must be positive")

    def _f(self, name):
        return getattr(self.lib, f"ws_oracle_{self.sfx}_{name}")

    def __del__(self):
        if getattr(self, "_p", None):
            self._f("destroy")(self._p)
            self._p = None

    def initialize(self):
        self._f("initialize")(self._p)

    def set_field(self, name, arr):
        a = np.ascontiguousarray(arr, dtype=self.dtype)
        assert a.shape == (self.H, self.W)
        self._f("set_field")(self._p, FIELD_IDS[name], a.ctypes.data)

    def get_field(self, name):
        a = np.empty((self.H, self.W), self.dtype)
        self._f("get_field")(self._p, FIELD_IDS[name], a.ctypes.data)
        return a

    def calculate_diagnostics(self):
        self._f("calc_diagnostics")(self._p)

    def step(self):
        self._f("step")(self._p)

    def run(self, n):
        return self._f("run")(self._p, n)

    def run_until(self, t):
        return self._f("run_until")(self._p, t)

    def set_dt(self, dt):
        self._f("set_dt")(self._p, dt)

    @property
    def time(self):
        return self._f("get_time")(self._p)

    @property
    def step_count(self):
        return self._f("get_step")(self._p)


def tendency(u, v, h, dx=1.0, dy=1.0, gravity=9.81, coriolis_f=0.0):
    """One SWE tendency evaluation (weather_simulation.cpp:473-540)."""
    lib = _load()
    dt = u.dtype
    sfx = "f32" if dt == np.float32 else "f64"
    H, W = u.shape
    out = [np.empty_like(u) for _ in range(3)]
    ins = [np.ascontiguousarray(a, dtype=dt) for a in (u, v, h)]
    getattr(lib, f"ws_oracle_{sfx}_tendency")(*(a.ctypes.data for a in ins), *(o.ctypes.data for o in out),
                                             W, H, dx, dy, gravity, coriolis_f)
    return out
