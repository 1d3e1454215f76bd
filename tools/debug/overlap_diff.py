"""Where does the overlap schedule of a slab group differ from one domain? Prints, per case
and slab, the differing rows (slab coordinates) of u / v / h after `steps` steps.

  python tools/debug/overlap_diff.py            (a built-in case list)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nvidia-jetson-workload_amd"))
os.environ.setdefault("WS_QUIET", "1")
os.environ["WS_NUMERICS"] = "exact"
import weather_sim as ws  # noqa: E402


def cfg(W, H):
    c = ws.SimulationConfig()
    c.grid_width, c.grid_height = W, H
    c.integration_method = ws.IntegrationMethod.RungeKutta4
    c.double_precision = True
    c.max_time = 1e30
    return c


def case(W, H, nslabs, steps, env):
    for k in ("WS_SLAB_OVERLAP", "WS_TB", "WS_SEG_ROWS", "WS_KERNEL", "WS_SLAB_BLOCK", "WS_DBG_OVL"):
        os.environ.pop(k, None)
    os.environ.update(env)
    one = ws.WeatherSimulation(cfg(W, H))
    one.set_initial_condition(ws.JetStreamInitialCondition())
    one.initialize()
    one.run(steps)
    g1 = one.get_current_grid()
    ref = {"u": g1.get_velocity_field()[0], "v": g1.get_velocity_field()[1], "h": g1.get_height_field()}
    grp = ws.SlabGroup(cfg(W, H), nslabs)
    grp.set_initial_condition(ws.JetStreamInitialCondition())
    grp.initialize()
    grp.run(steps)
    out = []
    for r in range(nslabs):
        s = grp.slab(r)
        g = s.get_current_grid()
        got = {"u": g.get_velocity_field()[0], "v": g.get_velocity_field()[1], "h": g.get_height_field()}
        for k in ("u", "v", "h"):
            d = got[k] != ref[k][s.row0:s.row0 + s.rows]
            if d.any():
                rows = np.nonzero(d.any(axis=1))[0]
                cols = np.nonzero(d.any(axis=0))[0]
                out.append(f"slab {r} {k}: {d.sum()} cells, rows {rows.min()}..{rows.max()} ({len(rows)}), "
                           f"cols {cols.min()}..{cols.max()} ({len(cols)})")
    sched = grp.slab(0).slab_schedule()
    print(f"{W}x{H} /{nslabs} steps {steps} {env} sched {sched} variant {grp.slab(0).fused_variant()} "
          f"tb {grp.slab(0).steps_per_launch()}: {'OK' if not out else 'DIFF'}", flush=True)
    for line in out[:12]:
        print("   ", line, flush=True)
    del grp, one


if __name__ == "__main__":
    cases = []
    for mode in ("0", "0", "2", "0"):
        for rep in range(4):
            cases.append((4096, 4096, 4, 13, {"WS_SLAB_OVERLAP": "1", "WS_DBG_OVL": mode}))
    for c in cases:
        case(*c)
