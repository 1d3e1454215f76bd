"""Debug aid: one fused variant vs the C oracle on a dam-break grid, printing where cells differ."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "nvidia-jetson-workload_amd"), ROOT, os.path.join(ROOT, "tests")]
os.environ.setdefault("WS_QUIET", "1")
import weather_sim as ws
from oracle.ws_oracle import OracleSim
from test_gpu_parity import _dam_break, make_sim, state

for spec in os.environ.get("CASES", "512x512:5 4096x256:5 256x4096:5").split():
    wh, steps = spec.split(":")
    W, H = map(int, wh.split("x"))
    steps = int(steps)
    for seg in os.environ.get("SEGS", "0 40 96").split():
        os.environ["WS_KERNEL"] = os.environ.get("KERN", "x2y")
        if seg != "0":
            os.environ["WS_SEG_ROWS"] = seg
        else:
            os.environ.pop("WS_SEG_ROWS", None)
        sim = make_sim(W, H, 0, 2, True, max_time=1e30)
        sim.initialize()
        h0 = _dam_break(W, H, 128.0 if W >= 1024 else 8.0, np.float64)
        sim.get_current_grid().set_height_field(h0)
        ref = OracleSim(W, H, 0, 2, max_time=1e30, precision="f64")
        ref.initialize()
        ref.set_field("h", h0)
        sim.run(steps)
        ref.run(steps)
        got = state(sim.get_current_grid())
        msg = []
        for k in ("u", "v", "h"):
            want = ref.get_field(k)
            bad = np.argwhere(got[k] != want)
            if len(bad):
                msg.append(f"{k}:{len(bad)} rows {sorted(set(bad[:,0].tolist()))[:6]} cols {sorted(set(bad[:,1].tolist()))[:8]}")
        print(W, H, seg, sim.fused_variant(), "ok" if not msg else " ; ".join(msg), flush=True)
        del sim
