"""Debug aid: the C2 dam-break RK4 fp64 full-size digest with every fused variant pinned
(and the autotuned choice), to find a variant that breaks bit-exactness at full size."""
import hashlib, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "nvidia-jetson-workload_amd"), ROOT, os.path.join(ROOT, "tests")]
os.environ.setdefault("WS_QUIET", "1")
import weather_sim as ws
from test_gpu_parity import _dam_break, _digest, make_sim, state
from conftest import large_digests

name = sys.argv[1] if len(sys.argv) > 1 else "C2_dam_break_4096_i2_f64"
d = large_digests()[name]
spec = {k: v for k, v in (l.split()[1:3] for l in d["spec"] if l.startswith("cfg "))}
W, H = int(spec["width"]), int(spec["height"])
steps = int([l for l in d["spec"] if l.startswith("run ")][0].split()[1])
for kern in os.environ.get("KERNELS", "auto dpp dppdma dppy x2 x2y lds").split():
    for seg in os.environ.get("SEGS", "0").split():
        if kern == "auto":
            os.environ.pop("WS_KERNEL", None)
        else:
            os.environ["WS_KERNEL"] = kern
        if seg != "0":
            os.environ["WS_SEG_ROWS"] = seg
        else:
            os.environ.pop("WS_SEG_ROWS", None)
        sim = make_sim(W, H, int(spec["model"]), int(spec["method"]), True, max_time=float(spec["max_time"]))
        sim.initialize()
        sim.get_current_grid().set_height_field(_dam_break(W, H, 128.0, np.float64))
        sim.run(steps)
        got = state(sim.get_current_grid())
        bad = [k for k, h in d["sha256"].items() if _digest(got[k]) != h]
        print(kern, seg, sim.fused_variant(), "BAD" if bad else "ok", bad, flush=True)
        del sim
