#!/usr/bin/env python3
"""One rank's step time in an N-rank y-slab decomposition, on ONE GPU (measurement aid).

Creates rank r's slab of the global grid WITHOUT a communicator (ws_sim_create_slab_emulated):
its run() executes the rank's exact compute schedule -- deep-halo blocks, stream-ordered or
overlapped (set_slab_schedule) -- with a device-side wait of the given microseconds in place
of each RCCL transfer (around the pack / unpack kernels for the packed transport). Results are
not a simulation (the halo holds the slab's own rows); the time per step is what an
N-GPU rank would spend if the transfer took that long.
  python tools/rank_timing.py [--config c2] [--ranks 2,4,8] [--xfer-us 0,30,60]
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
ap.add_argument("--steps", type=int, default=120)
ap.add_argument("--ranks", default="2,4,8")
ap.add_argument("--xfer-us", default="0,30,60", help="per exchange of a 6-step block; scaled by block / 6 "
                "plus --xfer-lat-us for other block sizes")
ap.add_argument("--xfer-lat-us", type=float, default=10.0)
ap.add_argument("--blocks", default="6")
ap.add_argument("--variants", default="off,on", help="overlap schedules: off, on, auto")
args = ap.parse_args()
conf = bench.CONFIGS[args.config]

for n in [int(x) for x in args.ranks.split(",")]:
    rank = n // 2 if n > 2 else 0  # a middle rank (both neighbours) when there is one
    for us6 in [float(x) for x in args.xfer_us.split(",")]:
        for blk in args.blocks.split(","):
            us = 0.0 if us6 == 0 else args.xfer_lat_us + (us6 - args.xfer_lat_us) * int(blk) / 6
            line = []
            for var in args.variants.split(","):
                c = ws.SimulationConfig()
                c.grid_width, c.grid_height, c.num_levels = conf["W"], conf["H"], conf["L"]
                c.model, c.integration_method = conf["model"], bench.METHODS[args.method]
                c.double_precision = conf["fp64"]
                c.max_time = 1e30
                sim = ws.WeatherSimulation(c, _slab=(rank, n, None, us))
                sim.set_slab_schedule(int(blk), var)
                sim.set_initial_condition(ws.JetStreamInitialCondition())
                sim.initialize()
                sim.run(300)  # autotune (+ the auto schedule's measurement) + warm clocks
                block, on = sim.slab_schedule()
                best = None
                for _ in range(3):
                    t0 = time.perf_counter()
                    sim.run(args.steps)
                    dt = (time.perf_counter() - t0) / args.steps
                    best = dt if best is None else min(best, dt)
                kern, seg, _ = sim.fused_variant()
                line.append(f"overlap={int(on)} {best * 1e3:.4f} [{kern} tb={sim.steps_per_launch()} seg={seg}]")
                del sim
            print(f"ranks={n} rank={rank} block={block} xfer={us:.0f}us/exchange ms/step: " + ", ".join(line),
                  flush=True)
