"""Output formats on the far side of run().

* ``Snapshot`` -- host copy of a simulation's state (all levels, fields, time, step,
  metrics). Everything below encodes a Snapshot, so the formats are testable without a GPU.
* ``CSVOutputManager`` -- the ``OutputManager`` the reference declares
  (``cpp/include/weather_sim/output_manager.hpp:52-97``, ``OutputConfig`` :35-47) but never
  implements: one CSV file per output step, ``<output_dir>/<prefix>_<step:06d>.csv`` (``.gz``
  with ``compress``), a header line then one row per cell ``level,y,x,<fields>``, values
  printed with enough digits to read back bit-exactly (9 significant digits fp32, 17 fp64).
  ``OutputConfig.fields`` selects columns ("velocity" -> u, v; "height" -> h; "pressure" ->
  p; "temperature" -> t; "humidity" -> q; "vorticity"; "divergence"); diagnostics only with
  ``include_diagnostics``.
* ``weather_sim_result`` / ``weather_sim_update`` -- the protobuf messages of
  ``src/proto/weather.proto:11-117`` (with ``common.proto``'s ``WorkloadConfig``,
  ``WorkloadResult``, ``PerformanceMetrics``), built from descriptors declared here (no
  protoc in the image; field names and numbers follow the .proto files). A 2-D level maps
  to an ``AtmosphericSlice`` (z_level = level); per cell: temperature <- T, pressure <- p,
  humidity <- q, wind_velocity_x/y <- u/v; the reference model has no vertical wind,
  precipitation or clouds, so those fields stay 0 and the severe-weather flags false.
"""
import gzip
import os
import socket
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

FIELD_COLUMNS = {
    "velocity": ("u", "v"), "height": ("h",), "pressure": ("p",), "temperature": ("t",),
    "humidity": ("q",), "vorticity": ("vorticity",), "divergence": ("divergence",),
}
DIAGNOSTICS = ("vorticity", "divergence")


@dataclass
class Snapshot:
    """Host copy of a simulation state; fields[name] has shape (levels, height, width)."""
    width: int
    height: int
    levels: int
    dtype: type
    time: float
    step: int
    dx: float = 1.0
    dy: float = 1.0
    dt: float = 0.01
    max_time: float = 10.0
    fields: Dict[str, np.ndarray] = field(default_factory=dict)
    total_time_ms: float = 0.0

    @classmethod
    def of(cls, sim, names=("u", "v", "h", "p", "t", "q", "vorticity", "divergence")):
        """Copy the current state of a WeatherSimulation (every level) to the host."""
        g = sim.get_current_grid()
        cfg = sim.get_config()
        levels = max(1, int(getattr(cfg, "num_levels", 1)))
        arrays = {}
        for n in names:
            arrays[n] = np.stack([g._get(n, level=l) for l in range(levels)])
        first = arrays[names[0]]
        m = sim.get_performance_metrics()
        return cls(width=first.shape[2], height=first.shape[1], levels=levels, dtype=first.dtype.type,
                   time=float(sim.get_current_time()), step=int(sim.get_current_step()), dx=float(cfg.dx),
                   dy=float(cfg.dy), dt=float(sim.get_dt()), max_time=float(cfg.max_time), fields=arrays,
                   total_time_ms=float(m.total_time_ms))


# ---------------------------------------------------------------------------------------
# CSV
# ---------------------------------------------------------------------------------------
def csv_columns(fields: List[str], include_diagnostics: bool = True) -> List[str]:
    cols = []
    for f in fields:
        if f not in FIELD_COLUMNS:
            raise ValueError(f"unknown output field {f!r}; known: {sorted(FIELD_COLUMNS)}")
        if f in DIAGNOSTICS and not include_diagnostics:
            continue
        cols.extend(c for c in FIELD_COLUMNS[f] if c not in cols)
    return cols


def write_csv(snap: Snapshot, path: str, columns: List[str], compress: bool = False) -> str:
    """Write one snapshot as CSV (header + level,y,x,<columns> rows). Returns the path."""
    digits = 17 if np.dtype(snap.dtype).itemsize == 8 else 9
    L, H, W = snap.levels, snap.height, snap.width
    lv, yy, xx = np.meshgrid(np.arange(L), np.arange(H), np.arange(W), indexing="ij")
    idx = np.stack([lv.ravel(), yy.ravel(), xx.ravel()], axis=1)
    vals = np.stack([snap.fields[c].astype(np.float64).ravel() for c in columns], axis=1)
    header = (f"# weather_sim step={snap.step} time={snap.time!r} width={W} height={H} levels={L}\n"
              + ",".join(["level", "y", "x"] + columns) + "\n")
    rows = [",".join(map(str, i)) + "," + ",".join(f"{v:.{digits}g}" for v in r) for i, r in zip(idx, vals)]
    body = header + "\n".join(rows) + ("\n" if rows else "")
    if compress:
        path = path + ".gz"
        with gzip.open(path, "wt") as f:
            f.write(body)
    else:
        with open(path, "w") as f:
            f.write(body)
    return path


def read_csv(path: str):
    """Read a file written by write_csv: (meta dict, {column: (levels, height, width) array})."""
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rt") as f:
        meta_line = f.readline().strip()
        cols = f.readline().strip().split(",")
        data = np.loadtxt(f, delimiter=",", ndmin=2)
    meta = dict(kv.split("=", 1) for kv in meta_line.split()[2:])
    L, H, W = int(meta["levels"]), int(meta["height"]), int(meta["width"])
    out = {}
    for j, c in enumerate(cols[3:], start=3):
        a = np.zeros((L, H, W))
        a[data[:, 0].astype(int), data[:, 1].astype(int), data[:, 2].astype(int)] = data[:, j]
        out[c] = a
    return meta, out


class CSVOutputManager:
    """OutputManager (output_manager.hpp:52-97) writing CSV snapshots every output step.

    Attach with ``WeatherSimulation.set_output_manager``; ``run()`` then calls
    ``write_output`` every ``SimulationConfig.output_interval`` steps (weather_simulation.cpp:
    86-90). ``written`` lists the files in order."""

    def __init__(self, config=None):
        from .weather_simulation import OutputConfig
        self.config = config or OutputConfig()
        self.written: List[str] = []
        self._columns = csv_columns(list(self.config.fields), self.config.include_diagnostics)

    def get_config(self):
        return self.config

    def set_config(self, config):
        self.config = config
        self._columns = csv_columns(list(config.fields), config.include_diagnostics)

    def initialize(self, simulation):
        os.makedirs(self.config.output_dir, exist_ok=True)
        self.written = []

    def write_output(self, simulation):
        snap = Snapshot.of(simulation, names=tuple(self._columns))
        path = os.path.join(self.config.output_dir, f"{self.config.prefix}_{snap.step:06d}.csv")
        self.written.append(write_csv(snap, path, self._columns, self.config.compress))

    def finalize(self, simulation):
        with open(os.path.join(self.config.output_dir, f"{self.config.prefix}_index.txt"), "w") as f:
            f.write("\n".join(os.path.basename(p) for p in self.written) + "\n")


# ---------------------------------------------------------------------------------------
# Protobuf (src/proto/common.proto, src/proto/weather.proto)
# ---------------------------------------------------------------------------------------
_CLASSES = None


def _proto_classes():
    """Message classes for the reference schema, from descriptors built here."""
    global _CLASSES
    if _CLASSES is not None:
        return _CLASSES
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    F = descriptor_pb2.FieldDescriptorProto
    T = {"double": F.TYPE_DOUBLE, "int32": F.TYPE_INT32, "int64": F.TYPE_INT64, "bool": F.TYPE_BOOL,
         "string": F.TYPE_STRING}

    def msg(fd, name, fields, maps=()):
        m = fd.message_type.add(name=name)
        for fname, num, ftype, *rest in fields:
            repeated = bool(rest and rest[0] == "repeated")
            f = m.field.add(name=fname, number=num,
                            label=F.LABEL_REPEATED if repeated else F.LABEL_OPTIONAL)
            if ftype in T:
                f.type = T[ftype]
            elif ftype.startswith("enum:"):
                f.type, f.type_name = F.TYPE_ENUM, ftype[5:]
            else:
                f.type, f.type_name = F.TYPE_MESSAGE, ftype
        for fname, num, ktype, vtype in maps:  # map<k, v> = repeated nested XEntry {key=1; value=2}
            entry = "".join(p.capitalize() for p in fname.split("_")) + "Entry"
            e = m.nested_type.add(name=entry)
            e.options.map_entry = True
            e.field.add(name="key", number=1, label=F.LABEL_OPTIONAL, type=T[ktype])
            e.field.add(name="value", number=2, label=F.LABEL_OPTIONAL, type=T[vtype])
            m.field.add(name=fname, number=num, label=F.LABEL_REPEATED, type=F.TYPE_MESSAGE,
                        type_name=f".{fd.package}.{name}.{entry}")
        return m

    pool = descriptor_pool.DescriptorPool()
    common = descriptor_pb2.FileDescriptorProto(name="common.proto", package="nvidia.jetson.workload",
                                                syntax="proto3")
    msg(common, "PerformanceMetrics", [  # common.proto:9-36
        ("total_time_ms", 1, "double"), ("gpu_memory_mb", 2, "double"), ("cpu_memory_mb", 3, "double"),
        ("gpu_utilization", 4, "double"), ("cpu_utilization", 5, "double"),
        ("power_consumption_watts", 6, "double"), ("temperature_celsius", 7, "double"),
        ("operations_per_second", 8, "double")], maps=[("time_breakdown_ms", 9, "string", "double")])
    msg(common, "WorkloadConfig", [  # common.proto:39-63
        ("run_id", 1, "string"), ("workload_name", 2, "string"), ("version", 3, "string"),
        ("timestamp", 4, "int64"), ("node_name", 5, "string"), ("collect_metrics", 6, "bool"),
        ("generate_visualization", 7, "bool")], maps=[("parameters", 8, "string", "string")])
    st = common.enum_type.add(name="Status")  # common.proto:66-71
    for i, n in enumerate(("SUCCESS", "ERROR", "IN_PROGRESS", "CANCELLED")):
        st.value.add(name=n, number=i)
    msg(common, "WorkloadResult", [  # common.proto:74-89
        ("config", 1, ".nvidia.jetson.workload.WorkloadConfig"),
        ("metrics", 2, ".nvidia.jetson.workload.PerformanceMetrics"),
        ("status", 3, "enum:.nvidia.jetson.workload.Status"), ("error_message", 4, "string"),
        ("workload_type", 5, "string")])
    pool.Add(common)

    w = descriptor_pb2.FileDescriptorProto(name="weather.proto", package="nvidia.jetson.workload.weather",
                                           syntax="proto3", dependency=["common.proto"])
    msg(w, "WeatherSimConfig", [  # weather.proto:11-53
        ("base_config", 1, ".nvidia.jetson.workload.WorkloadConfig"), ("grid_size_x", 2, "int32"),
        ("grid_size_y", 3, "int32"), ("grid_size_z", 4, "int32"), ("domain_size_x", 5, "double"),
        ("domain_size_y", 6, "double"), ("domain_size_z", 7, "double"), ("time_step", 8, "double"),
        ("total_simulation_time", 9, "double"), ("initial_temperature", 10, "double"),
        ("pressure", 11, "double"), ("humidity", 12, "double"), ("initial_wind_speed_x", 13, "double"),
        ("initial_wind_speed_y", 14, "double"), ("initial_wind_speed_z", 15, "double"),
        ("terrain_complexity", 16, "double"), ("simulate_precipitation", 17, "bool"),
        ("include_solar_radiation", 18, "bool"), ("output_resolution_x", 19, "int32"),
        ("output_resolution_y", 20, "int32"), ("output_resolution_z", 21, "int32")])
    msg(w, "AtmosphericCell", [  # weather.proto:56-65
        ("temperature", 1, "double"), ("pressure", 2, "double"), ("humidity", 3, "double"),
        ("wind_velocity_x", 4, "double"), ("wind_velocity_y", 5, "double"), ("wind_velocity_z", 6, "double"),
        ("precipitation_rate", 7, "double"), ("cloud_density", 8, "double")])
    msg(w, "AtmosphericSlice", [  # weather.proto:68-73
        ("z_level", 1, "int32"), ("cells", 2, ".nvidia.jetson.workload.weather.AtmosphericCell", "repeated"),
        ("width", 3, "int32"), ("height", 4, "int32")])
    msg(w, "WeatherSimResult", [  # weather.proto:76-100
        ("base_result", 1, ".nvidia.jetson.workload.WorkloadResult"),
        ("config", 2, ".nvidia.jetson.workload.weather.WeatherSimConfig"), ("simulation_time", 3, "double"),
        ("atmospheric_slices", 4, ".nvidia.jetson.workload.weather.AtmosphericSlice", "repeated"),
        ("max_temperature", 5, "double"), ("min_temperature", 6, "double"), ("max_wind_speed", 7, "double"),
        ("total_precipitation", 8, "double"), ("storm_detected", 9, "bool"),
        ("high_wind_warning", 10, "bool"), ("flooding_risk", 11, "bool")])
    msg(w, "WeatherSimUpdate", [  # weather.proto:103-117
        ("run_id", 1, "string"), ("current_time", 2, "double"), ("percent_complete", 3, "double"),
        ("current_slice", 4, ".nvidia.jetson.workload.weather.AtmosphericSlice"),
        ("current_metrics", 5, ".nvidia.jetson.workload.PerformanceMetrics")])
    pool.Add(w)

    names = ["nvidia.jetson.workload.PerformanceMetrics", "nvidia.jetson.workload.WorkloadConfig",
             "nvidia.jetson.workload.WorkloadResult", "nvidia.jetson.workload.weather.WeatherSimConfig",
             "nvidia.jetson.workload.weather.AtmosphericCell", "nvidia.jetson.workload.weather.AtmosphericSlice",
             "nvidia.jetson.workload.weather.WeatherSimResult", "nvidia.jetson.workload.weather.WeatherSimUpdate"]
    _CLASSES = {n.split(".")[-1]: message_factory.GetMessageClass(pool.FindMessageTypeByName(n)) for n in names}
    return _CLASSES


def proto_classes():
    """{message name: class} for PerformanceMetrics, WorkloadConfig, WorkloadResult,
    WeatherSimConfig, AtmosphericCell, AtmosphericSlice, WeatherSimResult, WeatherSimUpdate."""
    return dict(_proto_classes())


def _fill_slice(sl, snap: Snapshot, level: int, stride: int = 1):
    sl.z_level = level
    sub = {k: snap.fields[k][level, ::stride, ::stride].astype(np.float64) for k in ("t", "p", "q", "u", "v")}
    sl.height, sl.width = sub["t"].shape
    for t, p, q, u, v in zip(sub["t"].ravel(), sub["p"].ravel(), sub["q"].ravel(), sub["u"].ravel(),
                             sub["v"].ravel()):
        c = sl.cells.add()
        c.temperature, c.pressure, c.humidity = float(t), float(p), float(q)
        c.wind_velocity_x, c.wind_velocity_y = float(u), float(v)


def _metrics(P, snap: Snapshot):
    m = P["PerformanceMetrics"]()
    m.total_time_ms = snap.total_time_ms
    if snap.total_time_ms > 0:
        m.operations_per_second = snap.width * snap.height * snap.levels * snap.step / (snap.total_time_ms * 1e-3)
    return m


def weather_sim_result(snap: Snapshot, run_id: str = "", levels: Optional[List[int]] = None,
                       output_stride: int = 1):
    """WeatherSimResult (weather.proto:76-100) for a snapshot; every level by default,
    cells sub-sampled by output_stride (the config's output_resolution_*)."""
    P = _proto_classes()
    r = P["WeatherSimResult"]()
    b = r.base_result
    b.config.run_id = run_id
    b.config.workload_name = "weather_sim"
    b.config.version = "mi355x"
    b.config.timestamp = int(time.time())
    b.config.node_name = socket.gethostname()
    b.metrics.CopyFrom(_metrics(P, snap))
    b.status = 0  # SUCCESS
    b.workload_type = "weather_sim"
    c = r.config
    c.base_config.CopyFrom(b.config)
    c.grid_size_x, c.grid_size_y, c.grid_size_z = snap.width, snap.height, snap.levels
    c.domain_size_x, c.domain_size_y = snap.width * snap.dx, snap.height * snap.dy
    c.time_step, c.total_simulation_time = snap.dt, snap.max_time
    c.output_resolution_x = (snap.width + output_stride - 1) // output_stride
    c.output_resolution_y = (snap.height + output_stride - 1) // output_stride
    c.output_resolution_z = snap.levels
    r.simulation_time = snap.time
    for l in (range(snap.levels) if levels is None else levels):
        _fill_slice(r.atmospheric_slices.add(), snap, l, output_stride)
    t = snap.fields["t"]
    r.max_temperature, r.min_temperature = float(t.max()), float(t.min())
    r.max_wind_speed = float(np.sqrt(snap.fields["u"].astype(np.float64) ** 2
                                     + snap.fields["v"].astype(np.float64) ** 2).max())
    return r


def weather_sim_update(snap: Snapshot, run_id: str = "", total_time: Optional[float] = None, level: int = 0,
                       output_stride: int = 1):
    """WeatherSimUpdate (weather.proto:103-117): progress + one slice + metrics."""
    P = _proto_classes()
    u = P["WeatherSimUpdate"]()
    u.run_id = run_id
    u.current_time = snap.time
    T = snap.max_time if total_time is None else total_time
    u.percent_complete = min(100.0, 100.0 * snap.time / T) if T > 0 else 0.0
    _fill_slice(u.current_slice, snap, level, output_stride)
    u.current_metrics.CopyFrom(_metrics(P, snap))
    return u
