#!/usr/bin/env python3
"""ms per step of pinned fused-kernel variants on one bench configuration, in ONE process
(measurement aid, not product): each pin gets its own simulation, a warm-up, then the best of
three timed run()s of --steps steps (device-synchronous wall time, like bench.py's region).
Pins are kernel:steps_per_launch:seg_rows:align (seg_rows <= -2: the chain schedule with
-seg-1 rounds; "auto" = the autotuner's choice).
  python tools/pin_timing.py --config c2 --pins auto,dppy:2:56:0,dppy:2:-2:0,pc:2:-2:0
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nvidia-jetson-workload_amd"))
sys.path.insert(0, ROOT)
os.environ.setdefault("WS_QUIET", "1")

import bench  # noqa: E402
import weather_sim as ws  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--method", default="rk4")
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--warmup", type=int, default=600)
ap.add_argument("--pins", default="auto")
args = ap.parse_args()
conf = bench.CONFIGS[args.config]
ic = {"jet_stream": ws.JetStreamInitialCondition, "zonal_flow": ws.ZonalFlowInitialCondition}.get(conf["ic"])

for pin in args.pins.split(","):
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.num_levels = conf["W"], conf["H"], conf["L"]
    c.model, c.integration_method = conf["model"], bench.METHODS[args.method]
    c.double_precision = conf["fp64"]
    c.max_time = 1e30
    sim = ws.WeatherSimulation(c)
    if pin != "auto":
        k, tb, seg, al = pin.split(":")
        sim.pin_variant(kernel=k, steps_per_launch=int(tb), seg_rows=int(seg), align=int(al))
    if ic is not None:
        sim.set_initial_condition(ic())
    sim.initialize()
    sim.run(args.warmup)
    best = None
    for _ in range(3):
        sim.synchronize()
        t0 = time.perf_counter()
        sim.run(args.steps)
        sim.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        best = dt if best is None else min(best, dt)
    variant, seg_rows, out_cols = sim.fused_variant()
    cells = conf["W"] * conf["H"] * conf["L"]
    print(f"{args.config} {args.method} pin={pin:16s} -> {variant} tb={sim.steps_per_launch()} seg={seg_rows} "
          f"cols={out_cols}: {best * 1e3:.4f} ms/step {cells / best / 1e9:.1f} Gcell/s", flush=True)
    del sim
