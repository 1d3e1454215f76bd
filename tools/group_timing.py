#!/usr/bin/env python3
"""Per-rank step time of the y-slab schedule, emulated on ONE GPU (measurement aid).

A SlabGroup of N slabs runs the exact multi-rank schedule (block x NST halo rows copied on
the device at each block start, steps on rows extended into the halo) for all N slabs on
one stream; the wall time per step / N approximates one rank's step on an N-GPU node
without the RCCL transfer. Prints one line per N.
  python tools/group_timing.py [--config c2] [--steps 100]
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
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--slabs", default="1,2,4,8")
args = ap.parse_args()
conf = bench.CONFIGS[args.config]
for n in [int(x) for x in args.slabs.split(",")]:
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height, c.num_levels = conf["W"], conf["H"], conf["L"]
    c.model, c.integration_method, c.double_precision = conf["model"], bench.METHODS[args.method], conf["fp64"]
    c.max_time = 1e30
    sim = ws.SlabGroup(c, n) if n > 1 else ws.WeatherSimulation(c)
    sim.set_initial_condition(ws.JetStreamInitialCondition())
    sim.initialize()
    sim.run(300)  # warm clocks (and autotune for the single domain)
    t0 = time.perf_counter()
    sim.run(args.steps)
    if n == 1:
        sim.synchronize() if hasattr(sim, "synchronize") else None
    dt = (time.perf_counter() - t0) / args.steps
    print(f"slabs={n}: {dt * 1e3:.4f} ms/step total, {dt / n * 1e3:.4f} ms/step per slab "
          f"-> ideal-overlap speedup bound {conf['W'] * conf['H'] * conf['L'] / (dt / n) / 1e9:.1f} Gcell/s/GPU-rank",
          flush=True)
    del sim
