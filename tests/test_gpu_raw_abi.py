"""The kernel-level ABI on caller-owned device memory: ws_launch_shallow_water_kernel and
ws_launch_diagnostics_kernels, the replacements of the reference's raw-pointer launchers
launchShallowWaterKernel (/root/reference/src/weather-sim/cpp/src/kernels/
shallow_water_kernels.cu:704-719: one Euler step from d_u, d_v, d_h into d_*_out) and
launchDiagnosticsKernels (:830-840: vorticity / divergence).

The device buffers belong to the caller: hipMalloc'd here through the HIP runtime the
library itself is linked against (one runtime per process), with row pitch != width and NaN
padding, the way a caller with padded rows would hold them; the library only launches. Results are
checked bit-for-bit against the reference's own Euler step (tests/golden, "s1" of every
Euler case, vorticity included) and against the oracle's divergence, fp32 and fp64, with
non-default spacing / Coriolis where the fixture has them.
"""
import ctypes

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

ws = pytest.importorskip("weather_sim")
if not ws.is_cuda_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from weather_sim import _native  # noqa: E402


class Hip:
    """The HIP runtime libws_hip.so is linked against (ROCm's, /opt/rocm/lib; PyTorch may
    have loaded its own bundled copy into the process too), through ctypes."""

    def __init__(self):
        paths = {l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l}
        path = next(p for p in sorted(paths) if "site-packages" not in p and "dist-packages" not in p)
        self.lib = ctypes.CDLL(path)
        self.bufs = []

    def check(self, rc):
        assert rc == 0, f"HIP error {rc}"

    def alloc(self, nbytes):
        p = ctypes.c_void_p()
        self.check(self.lib.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes)))
        self.bufs.append(p)
        return p

    def upload(self, a, pitch):
        """A (H, pitch) device buffer holding a in its first W columns; padding = NaN, so a
        launcher that read past the row width would poison the result."""
        H, W = a.shape
        host = np.full((H, pitch), np.nan, a.dtype)
        host[:, :W] = a
        p = self.alloc(host.nbytes)
        self.check(self.lib.hipMemcpy(p, host.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(host.nbytes), 1))
        return p

    def nan_buffer(self, H, pitch, dtype):
        return self.upload(np.full((H, 0), np.nan, dtype), pitch)

    def download(self, p, H, pitch, dtype):
        host = np.empty((H, pitch), dtype)
        self.check(self.lib.hipDeviceSynchronize())
        self.check(self.lib.hipMemcpy(host.ctypes.data_as(ctypes.c_void_p), p, ctypes.c_size_t(host.nbytes), 2))
        return host

    def free(self):
        for p in self.bufs:
            self.lib.hipFree(p)
        self.bufs = []


@pytest.mark.parametrize("pad", [0, 13, 64])
@pytest.mark.parametrize("variant", ["f32", "f64"])
def test_raw_shallow_water_and_diagnostics_launchers(variant, pad):
    from oracle.ws_oracle import OracleSim

    gold = golden(variant)
    fp64 = variant == "f64"
    dt_np = np.float64 if fp64 else np.float32
    dtype = _native.WS_F64 if fp64 else _native.WS_F32
    cases = [c for c in gold.cases("step/") if gold.meta[c]["cfg"]["model"] == 0 and gold.meta[c]["cfg"]["method"] == 0]
    assert len(cases) >= 5
    hip = Hip()
    try:
        for case in cases:
            cfg = gold.meta[case]["cfg"]
            W, H = cfg["width"], cfg["height"]
            dx, dy, f = cfg.get("dx", 1.0), cfg.get("dy", 1.0), cfg.get("f", 0.0)
            dt, g = cfg.get("dt", 0.01), cfg.get("g", 9.81)
            pitch = W + pad
            s0, s1 = gold.snap(case, "s0"), gold.snap(case, "s1")
            ins = [hip.upload(s0[k], pitch) for k in ("u", "v", "h")]
            outs = [hip.nan_buffer(H, pitch, dt_np) for _ in range(3)]
            _native.check(_native.lib.ws_launch_shallow_water_kernel(*ins, *outs, W, H, pitch, dt, g, dx, dy, f, dtype,
                                                                     None))
            for name, p in zip(("u", "v", "h"), outs):
                got = hip.download(p, H, pitch, dt_np)
                np.testing.assert_array_equal(got[:, :W], s1[name], err_msg=f"{case} {name}")
                # the launcher writes the W columns only: the caller's padding is untouched
                assert np.isnan(got[:, W:]).all(), f"{case} {name}: padding written"
            vort, div = hip.nan_buffer(H, pitch, dt_np), hip.nan_buffer(H, pitch, dt_np)
            _native.check(_native.lib.ws_launch_diagnostics_kernels(outs[0], outs[1], vort, div, W, H, pitch, dx, dy,
                                                                    dtype, None))
            np.testing.assert_array_equal(hip.download(vort, H, pitch, dt_np)[:, :W], s1["vort"],
                                          err_msg=f"{case} vorticity")
            ref = OracleSim(W, H, 0, 0, dx=dx, dy=dy, dt=dt, gravity=g, coriolis_f=f, precision=variant)
            ref.initialize()
            ref.set_field("u", s1["u"])
            ref.set_field("v", s1["v"])
            ref.calculate_diagnostics()
            np.testing.assert_array_equal(hip.download(div, H, pitch, dt_np)[:, :W], ref.get_field("div"),
                                          err_msg=f"{case} divergence")
            hip.free()
    finally:
        hip.free()


def test_raw_launcher_argument_errors():
    z = ctypes.c_void_p(0)
    p = ctypes.c_void_p(16)
    with pytest.raises(ValueError):  # null pointers
        _native.check(_native.lib.ws_launch_shallow_water_kernel(z, p, p, p, p, p, 8, 8, 8, 0.01, 9.81, 1.0, 1.0, 0.0,
                                                                 _native.WS_F32, None))
    with pytest.raises(ValueError):  # pitch < width
        _native.check(_native.lib.ws_launch_shallow_water_kernel(p, p, p, p, p, p, 8, 8, 7, 0.01, 9.81, 1.0, 1.0, 0.0,
                                                                 _native.WS_F32, None))
    with pytest.raises(ValueError):  # non-positive spacing (weather_grid.cpp:29-31)
        _native.check(_native.lib.ws_launch_diagnostics_kernels(p, p, p, p, 8, 8, 8, 0.0, 1.0, _native.WS_F64, None))
    with pytest.raises(ValueError):  # bad dtype
        _native.check(_native.lib.ws_launch_diagnostics_kernels(p, p, p, p, 8, 8, 8, 1.0, 1.0, 7, None))
