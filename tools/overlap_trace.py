#!/usr/bin/env python3
"""Concurrency of the slab overlap schedule from a rocprofv3 kernel trace (measurement aid).

  rocprofv3 --kernel-trace -d OUT -o run --output-format csv -- python3 tools/rank_timing.py ...
  python3 tools/overlap_trace.py OUT/.../run_kernel_trace.csv

Per HIP stream (or queue when the trace has no stream id): kernels and busy time of the
stencil and halo kernels in the last `--tail` seconds of the trace (the timed runs), and
the time during which kernels of two streams ran at once (the edge bands / exchange beside
the interior).
"""
import argparse
import csv
import glob
import re
import sys

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--tail", type=float, default=0.02, help="seconds at the end of the trace to analyse")
args = ap.parse_args()
path = args.trace if not args.trace.endswith("/") else (glob.glob(args.trace + "**/*kernel_trace.csv", recursive=True) or [""])[0]
rows = list(csv.DictReader(open(path)))
if not rows:
    sys.exit("empty trace")
skey = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
ev = []
for r in rows:
    name = r.get("Kernel_Name", "")
    if not any(k in name for k in ("fused", "halo", "delay")):
        continue
    m = re.search(r"(\w+)(<[^()]*>)?\(", name.replace("(anonymous namespace)", ""))
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[skey], m.group(1) if m else name[:40]))
end = max(e[1] for e in ev)
ev = [e for e in ev if e[0] >= end - args.tail * 1e9]
start = min(e[0] for e in ev)
streams = sorted({e[2] for e in ev})
print(f"window {(end - start) / 1e6:.3f} ms, {len(ev)} kernels, streams ({skey}) {streams}")
for s in streams:
    es = [e for e in ev if e[2] == s]
    busy = sum(e[1] - e[0] for e in es)
    names = sorted({e[3] for e in es})
    print(f"  stream {s}: {len(es)} kernels, busy {busy / 1e6:.3f} ms ({busy / (end - start):.0%}), {names}")
# time with kernels of >= 2 streams running at once
pts = sorted([(e[0], 1, e[2]) for e in ev] + [(e[1], -1, e[2]) for e in ev])
active = {}
both = 0
last = pts[0][0]
for t, d, s in pts:
    if sum(1 for v in active.values() if v > 0) >= 2:
        both += t - last
    active[s] = active.get(s, 0) + d
    last = t
print(f"two streams busy at once: {both / 1e6:.3f} ms ({both / (end - start):.0%} of the window)")
