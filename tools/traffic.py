#!/usr/bin/env python3
"""HBM traffic per launch of the fused step kernel from rocprofv3 --pmc passes.

  tools/traffic.py PMC_DIR KERNEL_SUBSTRING OUT_JSON

FETCH_SIZE / WRITE_SIZE are KiB per dispatch. On gfx950 FETCH_SIZE reports half the bytes
of wide coalesced streaming reads (MI355X_MICROARCH.md, HBM section): it is doubled here.
WRITE_SIZE is taken as is. Counters include Infinity-Cache hits (same section)."""
import csv
import glob
import json
import os
import sys

root, sub, out = sys.argv[1], sys.argv[2], sys.argv[3]
F64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")
vals = {"FETCH_SIZE": [], "WRITE_SIZE": [], "SQ_INSTS_VALU": [], "SQ_INSTS_LDS": [], "SQ_LDS_BANK_CONFLICT": [],
        "GRBM_GUI_ACTIVE": [], "SQ_INSTS_VALU_INT32": [], "SQ_INSTS_VALU_FMA_F32": [], "SQ_INSTS_VALU_ADD_F32": [],
        **{k: [] for k in F64}}
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            if sub in row.get("Kernel_Name", "") and row["Counter_Name"] in vals:
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
res = {"kind0": 2 * fetch * 1024 + write * 1024, "fetch_size_kib_reported": fetch, "write_size_kib": write,
       "dispatches": [len(vals["FETCH_SIZE"]), len(vals["WRITE_SIZE"])], "kernel": sub,
       "correction": "bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024); gfx950 FETCH_SIZE halving"}
mean = lambda k: sum(vals[k]) / len(vals[k]) if vals[k] else None  # noqa: E731
res["valu_insts"] = mean("SQ_INSTS_VALU")
res["lds_insts"] = mean("SQ_INSTS_LDS")
res["lds_bank_conflict_cycles"] = mean("SQ_LDS_BANK_CONFLICT")
res["grbm_gui_active"] = mean("GRBM_GUI_ACTIVE")
res["dispatches"] += [len(vals["SQ_INSTS_VALU"])]
# the fp64 share of the VALU instructions (per-type counters; the rest are 32-bit: DPP lane moves,
# integer and fp32 ops)
if all(vals[k] for k in F64) and res["valu_insts"]:
    res["valu_f64_insts"] = sum(mean(k) for k in F64)
    res["valu_f64_frac"] = res["valu_f64_insts"] / res["valu_insts"]
    res["valu_int32_insts"] = mean("SQ_INSTS_VALU_INT32")
with open(out, "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res))
