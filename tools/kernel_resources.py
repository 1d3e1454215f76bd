#!/usr/bin/env python3
"""Per-kernel resources from a rocprofv3 --kernel-trace CSV (the code object's VGPR / AGPR /
SGPR counts, LDS and scratch per workgroup as the dispatches report them), with the dispatch
count and mean duration, and the waves per SIMD the VGPR count allows (512 per SIMD lane,
granule 8; MI355X_MICROARCH.md occupancy table).

On gfx950 this ROCm's trace reports VGPR_Count in units of two registers: the C2 RK4 two-step
kernel the compiler reports at 223 VGPRs (-Rpass-analysis=kernel-resource-usage, occupancy 2)
shows as 112, the 128-VGPR pc kernel as 64. The column `vgpr` below is 2 x the trace's value
(`vgpr_trace` keeps it); the waves per SIMD follow from `vgpr`.

  python tools/kernel_resources.py gpurun_out/.../run_kernel_trace.csv [name-substring]
"""
import csv
import sys
from collections import defaultdict


def waves_per_simd(vgpr, agpr):
    regs = ((vgpr + 7) // 8) * 8 + ((agpr + 7) // 8) * 8
    return min(8, 512 // max(regs, 8))


def summarize(path, pattern=""):
    rows = defaultdict(lambda: {"n": 0, "ns": 0})
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if pattern and pattern not in name:
            continue
        key = (name, int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"]), int(r["SGPR_Count"]), int(r["LDS_Block_Size"]),
               int(r["Scratch_Size"]), int(r["Workgroup_Size_X"]))
        rows[key]["n"] += 1
        rows[key]["ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = []
    for (name, v, a, s, lds, scr, wg), t in sorted(rows.items(), key=lambda kv: -kv[1]["ns"]):
        out.append({"kernel": name, "vgpr": 2 * v, "vgpr_trace": v, "agpr": a, "sgpr": s, "lds_bytes": lds, "scratch_bytes": scr,
                    "workgroup": wg, "waves_per_simd_by_vgpr": waves_per_simd(2 * v, a), "dispatches": t["n"],
                    "mean_us": t["ns"] / t["n"] / 1e3})
    return out


if __name__ == "__main__":
    for r in summarize(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""):
        print(f"{r['dispatches']:6d} x {r['mean_us']:9.2f} us  VGPR {r['vgpr']:3d} (trace {r['vgpr_trace']:3d}) AGPR {r['agpr']:3d} SGPR {r['sgpr']:3d} "
              f"LDS {r['lds_bytes']:6d} B scratch {r['scratch_bytes']:4d} B  WG {r['workgroup']:4d}  "
              f"waves/SIMD (VGPR) {r['waves_per_simd_by_vgpr']}  {r['kernel'][:110]}")
