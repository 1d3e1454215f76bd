import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "nvidia-jetson-workload_amd"))
os.environ["WS_QUIET"] = "1"
import numpy as np
import weather_sim as ws

def run(kernel, fp64, method, W, H, seg=None):
    os.environ["WS_KERNEL"] = kernel
    if seg: os.environ["WS_SEG_ROWS"] = str(seg)
    else: os.environ.pop("WS_SEG_ROWS", None)
    c = ws.SimulationConfig(); c.grid_width, c.grid_height = W, H
    c.integration_method, c.double_precision = method, fp64
    s = ws.WeatherSimulation(c); s.set_initial_condition(ws.BreakingWaveInitialCondition()); s.initialize()
    s.run(1)
    return s.get_current_grid()._get("u")

for fp64 in (False, True):
    for method in (0, 2):
        for (W, H, seg) in ((48, 32, None), (300, 70, 9)):
            a = run("dpp", fp64, method, W, H, seg); b = run("dppdma", fp64, method, W, H, seg)
            bad = np.argwhere(a != b)
            print(f"fp64={fp64} m={method} {W}x{H} seg={seg}: {len(bad)} bad", bad[:12].tolist(), flush=True)
