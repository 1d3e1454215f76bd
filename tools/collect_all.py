"""Collect tools/measure_all.sh's bench lines (gpurun_out/all/<cfg>_<method>.json) into one
profiles/ summary: python3 tools/collect_all.py gpurun_out/all profiles/r02_all_configs.json"""
import glob
import json
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
out = {"note": "one MI355X, tools/measure_all.sh (300 warm-up + 200 timed steps, autotuned); achieved / frac = "
               "algorithmic bytes per launch (y_n read + y_(n+k) written once, 6 words per cell; bench.py "
               "byte_model; the physics modes: their own words-per-cell models, DESIGN.md sections 10-11) / mean "
               "launch time; one_step_equivalent_gbs = 6 words per cell-update x cell-updates per launch / launch "
               "time; dram_frac = PMC HBM bytes; valu_frac = PMC VALU issue cycles on SIMD-32 "
               "(profiles/traffic_<cfg>_<method>.json)",
       "configs": {}}
for f in sorted(glob.glob(os.path.join(src, "*.json"))):
    d = json.load(open(f))
    r = d["roofline"]
    out["configs"][os.path.basename(f)[:-5]] = {
        "value": d["value"], "ms_per_step": d["ms_per_step"], "kernel": r.get("kernel"),
        "seg_rows": r.get("seg_rows"), "strip_out_cols": r.get("strip_out_cols"),
        "steps_per_launch": r.get("steps_per_launch"), "mean_launch_ms": r.get("mean_launch_ms"),
        "achieved_gbs": r.get("achieved"), "frac": r.get("frac"), "bytes_per_launch": r.get("bytes_per_launch"),
        "one_step_equivalent_gbs": r.get("one_step_equivalent_gbs"), "dram_frac": r.get("dram_frac"),
        "valu_frac": r.get("valu_frac"), "binding": r.get("binding"),
        "cfl": (d.get("cfl") or {}).get("value")}
json.dump(out, open(dst, "w"), indent=1)
print(len(out["configs"]), "configs ->", dst)
