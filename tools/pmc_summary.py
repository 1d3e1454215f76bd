#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV passes: per kernel, mean counter value per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "?")
            key = (row.get("Dispatch_Id"), row.get("Counter_Name"))
            vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in sorted(vals.items(), key=lambda kv: -len(kv[1])):
    short = k.replace("(anonymous namespace)::", "").split("(")[0][-90:]
    print(short)
    for c, v in sorted(cs.items()):
        print(f"    {c:24s} mean/dispatch {sum(v) / len(v):16.1f}  (n={len(v)})")
