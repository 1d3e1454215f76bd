#!/usr/bin/env python3
"""C5 fixtures (SWE 16384 x 16384 fp64) from the REFERENCE solver, as row bands (run only in
the survey container; writes tests/golden/ref_c5_bands.json).

A full 16384^2 reference simulation needs ~82 GiB of host memory, more than
this container has, but the stencil's dependency cone makes bands exact: with the
reference's clamp-to-self boundary (weather_simulation.cpp:510-513) an RK4 step moves
information 4 rows (one per stage), so after S steps a band simulation of rows
[y0 - 4S, y1 + 4S) -- whose artificial top / bottom edges are clamped -- holds the exact
global state on [y0, y1) (on the global top / bottom edge the band needs no margin there).
Per IC, the reference evaluates the initial condition ONCE on a full 16384^2 WeatherGrid
(global coordinates; the grid alone fits: 8 fields x 2 GiB) and cuts the bands out
(ref_driver `icband`); each band runs S steps in a 16384-wide simulation, and the compared
rows' SHA-256 digests and L2 norms are stored (the GPU test compares its own full-grid run,
tests/test_gpu_c5.py).

Bands: the global top, the seam between slabs 0 and 1 of an 8-way split (row 2048), the
middle (seam of slabs 3 / 4, row 8192), the global bottom. ICs: jet_stream (the bench
workload) and random (seed 42: every cell differs, so x- and y-tiling seams are all live).

  python gen_c5_bands.py             -> ref_c5_bands.json   (4 steps, the four bands above)
  python gen_c5_bands.py --steps 50  -> ref_c5_bands50.json (C5's benchmark length, SURVEY
                                        §8(d): 200-row cone margins, a band at EVERY seam of
                                        the 8-way split, 2048 k +- 32 rows, k = 1..7)
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import REF, read_snap, run_spec  # noqa: E402

W = H = 16384
K = 64               # compared rows per band
ICS = {"jet_stream": [], "random": ["42", "1.0"]}


def bands(steps):
    """Compared rows [y0, y0 + K) per band."""
    if steps == 4:
        return {"top": 0, "seam2048": 2048 - K // 2, "mid8192": 8192 - K // 2, "bottom": H - K}
    out = {"top": 0}
    out.update({f"seam{2048 * k}": 2048 * k - K // 2 for k in range(1, 8)})
    out["bottom"] = H - K
    return out


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    args = ap.parse_args()
    STEPS = args.steps
    MARGIN = 4 * STEPS   # RK4: 4 rows of cone per step
    BANDS = bands(STEPS)
    name_out = "ref_c5_bands.json" if STEPS == 4 else f"ref_c5_bands{STEPS}.json"
    out = {"width": W, "height": H, "steps": STEPS, "method": 2, "variant": "f64", "compared_rows": K, "cases": {}}
    with tempfile.TemporaryDirectory(prefix="ws_c5_", dir="/tmp") as tmp:
        for ic, params in ICS.items():
            # simulated band per compared band: the cone margin where the band edge is not global
            sim_rows = {}
            for name, y0 in BANDS.items():
                lo = max(0, y0 - MARGIN)
                hi = min(H, y0 + K + MARGIN)
                sim_rows[name] = (lo, hi)
            spec = ",".join(f"{lo}:{hi - lo}" for lo, hi in sim_rows.values())
            run_spec("f64", ["cfg width 16", "cfg height 16", "create",
                             f"icband {ic} {W} {H} {spec} {tmp}/b " + " ".join(params)], tmp)
            for name, y0 in BANDS.items():
                lo, hi = sim_rows[name]
                lines = [f"cfg width {W}", f"cfg height {hi - lo}", "cfg model 0", "cfg method 2",
                         "cfg max_time 1e30", "create", "initialize"]
                lines += [f"setfield {f} {tmp}/b_{lo}_{f}.bin" for f in ("u", "v", "h", "p", "t", "q")]
                lines += [f"run {STEPS}", f"snap {tmp}/S.bin"]
                run_spec("f64", lines, tmp)
                s = read_snap(f"{tmp}/S.bin")
                assert s["step"] == STEPS
                r0 = y0 - lo
                case = {"rows": [y0, y0 + K], "sim_rows": [lo, hi], "time": s["time"],
                        "sha256": {}, "l2": {}}
                for f in ("u", "v", "h", "vort"):
                    a = s[f][r0:r0 + K]
                    case["sha256"][f] = digest(a)
                    case["l2"][f] = float(np.linalg.norm(a.astype(np.float64)))
                out["cases"][f"{ic}/{name}"] = case
                print(ic, name, case["rows"], case["l2"], flush=True)
    with open(os.path.join(HERE, name_out), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
