#!/usr/bin/env python3
"""Per-wave timeline of one fused two-step launch (measurement aid, not product).

Loads a diagnostic build of the library (tools/variant.sh stamps "-DWS_WAVE_STAMPS"), whose
fp64 dppy / x2y two-step kernel records per workgroup: start / end (100 MHz real-time counter,
shader clock), HW_ID (wave slot, SIMD, CU, SE), XCC id and work item. For each pinned variant
it runs C2 (or --config) warm, then one launch, and prints: waves, dispatch spread (first to
last start), wave lifetimes, the launch span, and how many waves each SIMD held over the launch
(the time-weighted occupancy histogram per SIMD) -- the evidence for what limits a launch
that is neither DRAM- nor VALU-bound.
  WS_HIP_LIB=.../libws_hip_stamps.so python tools/wave_timeline.py --pins dppy:2:48:0,dppy:2:184:0
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nvidia-jetson-workload_amd"))
sys.path.insert(0, ROOT)
os.environ.setdefault("WS_QUIET", "1")

import bench  # noqa: E402
import weather_sim as ws  # noqa: E402
from weather_sim import _native  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--method", default="rk4")
ap.add_argument("--pins", default="dppy:2:48:0,dppy:2:88:0,dppy:2:184:0")
ap.add_argument("--json", default="")
args = ap.parse_args()
conf = bench.CONFIGS[args.config]
lib = ctypes.CDLL(_native.LIB_PATH)
lib.ws_diag_wave_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
lib.ws_diag_wave_stamps_reset.argtypes = []
WORDS, MAXW = 8, 1 << 16

out = {}
for pin in args.pins.split(","):
    k, tb, seg, al = pin.split(":")
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.num_levels = conf["W"], conf["H"], conf["L"]
    c.model, c.integration_method = conf["model"], bench.METHODS[args.method]
    c.double_precision = conf["fp64"]
    c.max_time = 1e30
    sim = ws.WeatherSimulation(c)
    sim.pin_variant(kernel=k, steps_per_launch=int(tb), seg_rows=int(seg), align=int(al))
    sim.set_initial_condition(ws.JetStreamInitialCondition())
    sim.initialize()
    sim.run(600)  # clocks up
    sim.synchronize()
    _native.check(lib.ws_diag_wave_stamps_reset())
    sim.run(int(tb))  # the launch recorded (one launch of steps_per_launch steps)
    sim.synchronize()
    buf = np.zeros(MAXW * WORDS, dtype=np.uint64)
    _native.check(lib.ws_diag_wave_stamps(buf.ctypes.data, buf.nbytes))
    rec = buf.reshape(MAXW, WORDS)
    rec = rec[rec[:, 1] > 0]
    r0, r1 = rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64)
    hw, xcc = rec[:, 4].astype(np.int64), rec[:, 5].astype(np.int64)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    sid = (((xcc & 15) * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd  # a global SIMD key
    t0 = r0 - r0.min()
    t1 = r1 - r0.min()
    span = int(t1.max())
    life = t1 - t0
    us = lambda ticks: ticks / 100.0  # 100 MHz real-time counter
    unit = (rec[:, 6] >> np.uint64(32)).astype(np.int64)
    y0_ = (rec[:, 7] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    y1_ = (rec[:, 7] >> np.uint64(32)).astype(np.int64)
    rows_ = y1_ - y0_
    q4 = np.minimum(3, (y0_ + y1_) // 2 * 4 // conf["H"])
    edge = (unit == unit.min()) | (unit == unit.max())
    keys, inv = np.unique(sid, return_inverse=True)
    # time-weighted number of resident waves per SIMD
    grid = np.linspace(0, span, 400)
    occ = np.zeros((len(keys), len(grid)), dtype=np.int32)
    for i in range(len(rec)):
        occ[inv[i]] += (grid >= t0[i]) & (grid < t1[i])
    hist = {int(n): float((occ == n).mean()) for n in range(int(occ.max()) + 1)}
    per_simd_end = np.zeros(len(keys))
    np.maximum.at(per_simd_end, inv, t1)
    res = dict(pin=pin, waves=int(len(rec)), simds_used=int(len(keys)), launch_us=us(span),
               dispatch_spread_us=us(int(t0.max())), start_pct=[us(float(np.percentile(t0, p))) for p in (10, 50, 90)],
               life_us=[us(float(np.percentile(life, p))) for p in (0, 10, 50, 90, 100)],
               mean_life_frac=float(life.mean() / span),
               simd_end_us=[us(float(np.percentile(per_simd_end, p))) for p in (0, 10, 50, 90, 100)],
               occupancy_hist=hist, waves_per_simd_max=int(occ.max()),
               clock_ghz=float(np.median((rec[:, 3] - rec[:, 2]) / np.maximum(r1 - r0, 1)) / 10.0),
               # speed spread of the marches: microseconds per output row of each workgroup
               us_per_row=[us(float(np.percentile(life / np.maximum(rows_, 1), p))) for p in (0, 10, 50, 90, 100)],
               rows=[int(np.percentile(rows_, p)) for p in (0, 50, 100)],
               # per XCD: median us per row, and of the x-clamped strips (first / last)
               xcc_us_per_row=[round(us(float(np.median((life / np.maximum(rows_, 1))[(xcc & 15) == x]))), 3)
                               if np.any((xcc & 15) == x) else None for x in range(8)],
               by_row_quarter_us_per_row=[round(us(float(np.median((life / np.maximum(rows_, 1))[q4 == q]))), 3)
                                          if np.any(q4 == q) else None for q in range(4)],
               edge_strip_us_per_row=round(us(float(np.median((life / np.maximum(rows_, 1))[edge]))), 3)
               if np.any(edge) else None,
               xcc_end_us=[us(int(t1[(xcc & 15) == x].max())) if np.any((xcc & 15) == x) else None for x in range(8)],
               waves_per_simd_at_start=[int(n) for n in np.bincount(np.bincount(inv[t0 < 200]), minlength=4)[:4]])
    out[pin] = res
    print(json.dumps(res), flush=True)
    del sim
if args.json:
    with open(args.json, "w") as f:
        json.dump(out, f, indent=1)
