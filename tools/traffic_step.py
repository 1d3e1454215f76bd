#!/usr/bin/env python3
"""HBM traffic per time step of a multi-kernel step (physics-mode c3p / c4p) from rocprofv3
--pmc passes: the sum over every dispatch of the kernels whose name contains one of the
substrings of (2 x FETCH_SIZE + WRITE_SIZE) bytes (gfx950 FETCH_SIZE halving, see
tools/traffic.py), divided by the time steps the profiled run took.

  tools/traffic_step.py PMC_DIR STEPS OUT_JSON SUBSTRING [SUBSTRING ...]
"""
import csv
import glob
import json
import os
import sys

root, steps, out, subs = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4:]
tot = {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0}
per_kernel = {}
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "")
            c = row["Counter_Name"]
            if c in tot and any(s in name for s in subs):
                v = float(row["Counter_Value"]) * 1024 * (2 if c == "FETCH_SIZE" else 1)
                tot[c] += v
                short = next(s for s in subs if s in name)
                per_kernel[short] = per_kernel.get(short, 0.0) + v
res = {"step": (tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) / steps, "steps_profiled": steps,
       "per_kernel_bytes_per_step": {k: v / steps for k, v in per_kernel.items()},
       "correction": "bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024); gfx950 FETCH_SIZE halving"}
with open(out, "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res))
