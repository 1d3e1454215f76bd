"""ctypes binding of libws_hip.so (the C ABI in include/ws_hip.h).

The library is loaded from the package tree (nvidia-jetson-workload_amd/lib/libws_hip.so,
built by `make -C nvidia-jetson-workload_amd/csrc` / __graft_entry__.build()). There is no
fallback: if the library is missing, importing weather_sim raises ImportError; if there is
no HIP device, creating a grid or simulation raises RuntimeError. (The reference silently
degrades to a mock whose step() only advances time, weather_simulation.py:30-189; this
build refuses to.)

ctypes releases the GIL for the duration of every call, so a long run() does not block
other Python threads (the reference's pybind run() holds it).
"""
import ctypes
import os

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("WS_HIP_LIB", os.path.join(_PKG_ROOT, "lib", "libws_hip.so"))

WS_OK, WS_ERR_INVALID, WS_ERR_DEVICE, WS_ERR_SHAPE, WS_ERR_UNSUPPORTED, WS_ERR_COMM = range(6)
WS_F32, WS_F64 = 0, 1
FIELD = {"u": 0, "v": 1, "h": 2, "p": 3, "t": 4, "q": 5, "vorticity": 6, "divergence": 7}
COMM_ID_BYTES = 128
NUMERICS = {"exact": 0, "fast": 1}


class ws_config_t(ctypes.Structure):
    _fields_ = [
        ("model", ctypes.c_int32), ("grid_type", ctypes.c_int32), ("integration_method", ctypes.c_int32),
        ("boundary_condition", ctypes.c_int32), ("grid_width", ctypes.c_int32), ("grid_height", ctypes.c_int32),
        ("num_levels", ctypes.c_int32), ("dx", ctypes.c_double), ("dy", ctypes.c_double), ("dt", ctypes.c_double),
        ("gravity", ctypes.c_double), ("coriolis_f", ctypes.c_double), ("beta", ctypes.c_double),
        ("viscosity", ctypes.c_double), ("diffusivity", ctypes.c_double), ("compute_backend", ctypes.c_int32),
        ("double_precision", ctypes.c_int32), ("device_id", ctypes.c_int32), ("num_threads", ctypes.c_int32),
        ("max_time", ctypes.c_double), ("max_steps", ctypes.c_int32), ("output_interval", ctypes.c_int32),
        ("random_seed", ctypes.c_uint32),
    ]


class ws_xfer_t(ctypes.Structure):
    _fields_ = [("peer", ctypes.c_int32), ("kind", ctypes.c_int32), ("field", ctypes.c_int32),
                ("level", ctypes.c_int32), ("offset", ctypes.c_int64), ("bytes", ctypes.c_int64),
                ("msg_offset", ctypes.c_int64)]


class ws_metrics_t(ctypes.Structure):
    _fields_ = [("total_time_ms", ctypes.c_double), ("compute_time_ms", ctypes.c_double),
                ("memory_transfer_time_ms", ctypes.c_double), ("io_time_ms", ctypes.c_double),
                ("num_steps", ctypes.c_int32)]


class ws_device_info_t(ctypes.Structure):
    _fields_ = [
        ("device_name", ctypes.c_char * 256), ("arch", ctypes.c_char * 64),
        ("compute_capability_major", ctypes.c_int32), ("compute_capability_minor", ctypes.c_int32),
        ("multiprocessors", ctypes.c_int32), ("cuda_cores", ctypes.c_int32), ("global_memory", ctypes.c_int64),
        ("shared_memory_per_block", ctypes.c_int32), ("max_threads_per_block", ctypes.c_int32),
        ("max_threads_per_multiprocessor", ctypes.c_int32), ("clock_rate_khz", ctypes.c_int32),
        ("memory_clock_rate_khz", ctypes.c_int32), ("memory_bus_width", ctypes.c_int32),
        ("wavefront_size", ctypes.c_int32),
    ]


_P = ctypes.c_void_p
_I = ctypes.c_int32
_D = ctypes.c_double
_PI = ctypes.POINTER(ctypes.c_int32)
_PD = ctypes.POINTER(ctypes.c_double)
_PL = ctypes.POINTER(ctypes.c_int64)
_PP = ctypes.POINTER(ctypes.c_void_p)

# name -> argtypes (all return int status unless listed in _RESTYPES)
SIGNATURES = {
    "ws_last_error": [],
    "ws_abi_version": [],
    "ws_is_available": [_PI],
    "ws_device_count": [_PI],
    "ws_device_info": [_I, ctypes.POINTER(ws_device_info_t)],
    "ws_device_memory": [_I, _PL, _PL],
    "ws_config_default": [ctypes.POINTER(ws_config_t)],
    "ws_grid_create": [_I, _I, _I, _I, _I, _PP],
    "ws_grid_destroy": [_P],
    "ws_grid_reset": [_P],
    "ws_grid_get_dims": [_P, _PI, _PI, _PI, _PI],
    "ws_grid_set_spacing": [_P, _D, _D],
    "ws_grid_get_spacing": [_P, _PD, _PD],
    "ws_grid_set_field": [_P, _I, _I, _P, _I, _I, _I],
    "ws_grid_get_field": [_P, _I, _I, _P, _I, _I, _I],
    "ws_grid_device_field": [_P, _I, _PP, _PL, _PL],
    "ws_grid_calculate_diagnostics": [_P],
    "ws_grid_apply_initial_condition": [_P, ctypes.c_char_p, _PD, _I, ctypes.c_char_p, _I],
    "ws_sim_create": [ctypes.POINTER(ws_config_t), _PP],
    "ws_sim_destroy": [_P],
    "ws_sim_grid": [_P, _I, _PP],
    "ws_sim_initialize": [_P],
    "ws_sim_step": [_P],
    "ws_sim_run": [_P, _I, _PI],
    "ws_sim_run_until": [_P, _D, _PI],
    "ws_sim_get_time": [_P, _PD],
    "ws_sim_get_step": [_P, _PI],
    "ws_sim_get_dt": [_P, _PD],
    "ws_sim_set_dt": [_P, _D],
    "ws_sim_get_config": [_P, ctypes.POINTER(ws_config_t)],
    "ws_sim_get_metrics": [_P, ctypes.POINTER(ws_metrics_t)],
    "ws_sim_reset_metrics": [_P],
    "ws_sim_synchronize": [_P],
    "ws_sim_last_run_stats": [_P, _PD, _PL],
    "ws_sim_inject_failure": [_P, _I],
    "ws_adapter_execute_shallow_water_step": [_P, _P, _D, _D, _D, _PD],
    "ws_adapter_execute_barotropic_step": [_P, _P, _D, _D, _D, _PD],
    "ws_adapter_execute_primitive_equations_step": [_P, _P, _D, _D, _D, _PD],
    "ws_adapter_execute_gcm_step": [_P, _P, _D, _D, _D, _PD],
    "ws_adapter_calculate_diagnostics": [_P, _PD],
    "ws_launch_shallow_water_kernel": [_P, _P, _P, _P, _P, _P, _I, _I, ctypes.c_int64, _D, _D, _D, _D, _D, _I, _P],
    "ws_launch_diagnostics_kernels": [_P, _P, _P, _P, _I, _I, ctypes.c_int64, _D, _D, _I, _P],
    "ws_comm_get_unique_id": [ctypes.POINTER(ctypes.c_uint8)],
    "ws_sim_create_slab": [ctypes.POINTER(ws_config_t), _I, _I, ctypes.POINTER(ctypes.c_uint8), _PP, _PI, _PI],
    "ws_sim_create_slab_emulated": [ctypes.POINTER(ws_config_t), _I, _I, _D, _PP, _PI, _PI],
    "ws_sim_set_slab_schedule": [_P, _I, _I],
    "ws_sim_slab_exchange_us": [_P, _PD],
    "ws_sim_slab_trial_ms": [_P, _PD],
    "ws_sim_pin_variant": [_P, _I, _I, _I, _I],
    "ws_slab_partition": [_I, _I, _I, _PI, _PI],
    "ws_sim_comm_allreduce_max": [_P, _D, _PD],
    "ws_sim_comm_barrier": [_P],
    "ws_group_create": [ctypes.POINTER(ws_config_t), _I, _PP],
    "ws_group_destroy": [_P],
    "ws_group_slab": [_P, _I, _PP, _PI, _PI],
    "ws_group_run": [_P, _I, _PI],
    "ws_multi_create": [ctypes.POINTER(ws_config_t), _PI, _I, _PP],
    "ws_multi_destroy": [_P],
    "ws_multi_size": [_P, _PI, _PI],
    "ws_multi_slab": [_P, _I, _PP, _PI, _PI],
    "ws_multi_step": [_P],
    "ws_multi_run": [_P, _I, _PI],
    "ws_multi_run_until": [_P, _D, _PI],
    "ws_multi_cfl": [_P, _PD, _PD, _I, _PD],
    "ws_multi_synchronize": [_P],
    "ws_multi_exchange_diag_halo": [_P],
    "ws_sim_set_kernel_timing": [_P, _I],
    "ws_sim_kernel_timing": [_P, _I, _PL, _PD, _PD],
    "ws_sim_fused_variant": [_P, _PI, _PI, _PI],
    "ws_sim_steps_per_launch": [_P, _PI],
    "ws_sim_slab_schedule": [_P, _PI, _PI],
    "ws_sim_cfl": [_P, _PD, _PD, _I, _PD],
    "ws_sim_kernel_occupancy": [_P, _PI],
    "ws_sim_set_numerics": [_P, _I],
    "ws_sim_get_numerics": [_P, _PI],
    "ws_slab_exchange_plan": [_I, _I, _I, _I, _I, _I, _I, _I, ctypes.POINTER(ws_xfer_t), _I, _PI, _PL, _PL],
    "ws_bvort_create": [ctypes.POINTER(ws_config_t), _PP],
    "ws_bvort_create_poisson": [ctypes.POINTER(ws_config_t), _I, _PP],
    "ws_bvort_destroy": [_P],
    "ws_bvort_set_vorticity": [_P, _P, _I, _I, _I],
    "ws_bvort_get_field": [_P, _I, _P, _I, _I, _I],
    "ws_bvort_run": [_P, _I],
    "ws_bvort_get_state": [_P, _PD, _PI, _PD, _PL],
    "ws_bvort_create_multi": [ctypes.POINTER(ws_config_t), _I, _PI, _I, _PP],
    "ws_bvort_create_slab": [ctypes.POINTER(ws_config_t), _I, _I, _I, ctypes.POINTER(ctypes.c_uint8), _PP, _PI, _PI],
    "ws_bvort_layout": [_P, _PI, _PI, _PI],
    "ws_lpe_create": [ctypes.POINTER(ws_config_t), _D, _PP],
    "ws_lpe_destroy": [_P],
    "ws_lpe_set_field": [_P, _I, _P, _I, _I, _I, _I],
    "ws_lpe_get_field": [_P, _I, _P, _I, _I, _I, _I],
    "ws_lpe_run": [_P, _I],
    "ws_lpe_get_state": [_P, _PD, _PI, _PD, _PL],
    "ws_lpe_create_multi": [ctypes.POINTER(ws_config_t), _D, _PI, _I, _PP],
    "ws_lpe_create_slab": [ctypes.POINTER(ws_config_t), _D, _I, _I, ctypes.POINTER(ctypes.c_uint8), _PP, _PI, _PI],
    "ws_lpe_layout": [_P, _PI, _PI, _PI],
    "ws_lpe_exchange_plan": [_I, _I, _I, _I, _I, _I, ctypes.POINTER(ws_xfer_t), _I, _PI, _PL],
}
_RESTYPES = {"ws_last_error": ctypes.c_char_p, "ws_config_default": None}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"weather_sim: native library {LIB_PATH} not found; build it with "
            "`make -C nvidia-jetson-workload_amd/csrc` (or __graft_entry__.build()). "
            "There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    return lib


lib = _load()


class WsDeviceError(RuntimeError):
    pass


def check(status):
    """Map a C-ABI status to the reference's Python exception types."""
    if status == WS_OK:
        return
    msg = (lib.ws_last_error() or b"").decode(errors="replace")
    if status == WS_ERR_INVALID:
        raise ValueError(msg)
    if status == WS_ERR_SHAPE:
        raise RuntimeError(msg)  # pybind maps the setters' std::runtime_error to RuntimeError
    if status == WS_ERR_DEVICE:
        raise WsDeviceError(msg)
    if status == WS_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)  # a RuntimeError subclass: e.g. ComputeBackend.CPU (no CPU path)
    raise RuntimeError(f"ws_hip error {status}: {msg}")


def device_count():
    n = ctypes.c_int32(0)
    check(lib.ws_device_count(ctypes.byref(n)))
    return n.value


def is_available():
    a = ctypes.c_int32(0)
    check(lib.ws_is_available(ctypes.byref(a)))
    return bool(a.value)


def exchange_plan(width, rows, levels, fp64, rank, nranks, nfields, depth):
    """The library's halo exchange plan (ws_slab_exchange_plan): (list of ws_xfer_t,
    pitch, level_stride) for one slab of the decomposition."""
    n, pitch, lstride = ctypes.c_int32(0), ctypes.c_int64(0), ctypes.c_int64(0)
    dt = WS_F64 if fp64 else WS_F32
    check(lib.ws_slab_exchange_plan(width, rows, levels, dt, rank, nranks, nfields, depth, None, 0,
                                    ctypes.byref(n), ctypes.byref(pitch), ctypes.byref(lstride)))
    buf = (ws_xfer_t * max(1, n.value))()
    check(lib.ws_slab_exchange_plan(width, rows, levels, dt, rank, nranks, nfields, depth, buf, n.value,
                                    ctypes.byref(n), None, None))
    return list(buf[:n.value]), pitch.value, lstride.value


def lpe_exchange_plan(width, rows, levels, fp64, rank, nranks):
    """The layered model's periodic halo plan (ws_lpe_exchange_plan): (list of ws_xfer_t,
    level_stride) for one slab of the ring (pitch = width, one halo row)."""
    n, lstride = ctypes.c_int32(0), ctypes.c_int64(0)
    dt = WS_F64 if fp64 else WS_F32
    check(lib.ws_lpe_exchange_plan(width, rows, levels, dt, rank, nranks, None, 0, ctypes.byref(n),
                                   ctypes.byref(lstride)))
    buf = (ws_xfer_t * max(1, n.value))()
    check(lib.ws_lpe_exchange_plan(width, rows, levels, dt, rank, nranks, buf, n.value, ctypes.byref(n), None))
    return list(buf[:n.value]), lstride.value
