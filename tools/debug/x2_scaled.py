"""Debug aid: one small step per fused variant vs the oracle, printing where cells differ."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "nvidia-jetson-workload_amd"), ROOT]
os.environ.setdefault("WS_QUIET", "1")
import weather_sim as ws
from oracle.ws_oracle import OracleSim
from weather_sim import _native
lib = _native.lib
W, H = int(os.environ.get("W", 48)), int(os.environ.get("H", 32))
method = int(os.environ.get("M", 0))
cfg = ws.SimulationConfig()
cfg.grid_width, cfg.grid_height = W, H
cfg.integration_method = method
sim = ws.WeatherSimulation(cfg)
sim.set_initial_condition(ws.BreakingWaveInitialCondition())
sim.initialize()
g = sim.get_current_grid(); u0, v0 = g.get_velocity_field(); h0 = g.get_height_field()
ref = OracleSim(W, H, 0, method, precision="f32"); ref.initialize()
for n, a in (("u", u0), ("v", v0), ("h", h0)): ref.set_field(n, a)
sim.run(1); ref.run(1)
g = sim.get_current_grid(); u, v = g.get_velocity_field()
print(os.environ.get("WS_KERNEL"), os.environ.get("WS_SCALED"), sim.fused_variant())
for n, got in (("u", u), ("v", v), ("h", g.get_height_field())):
    want = ref.get_field(n)
    bad = np.argwhere(got != want)
    print(n, "bad", len(bad), "rows", sorted(set(bad[:, 0]))[:10] if len(bad) else "", "cols", sorted(set(bad[:, 1]))[:20] if len(bad) else "")
    if len(bad):
        y, x = bad[0]; print("  first", y, x, got[y, x], want[y, x], "ratio", (got[y,x]-u0[y,x] if n=='u' else 0))
