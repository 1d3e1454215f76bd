#!/usr/bin/env python3
"""Per-slab digests of a REFERENCE run, for bench.py's parity self-check (every N) (run only in the
survey container, where oracle/_ref is built from /root/reference sources).

The reference binary (oracle/_ref/ws_ref_f64, driven as in gen_golden.py) runs the C2 shape
-- SWE 4096 x 4096 fp64, jet_stream, RK4 -- for STEPS steps on the whole grid; the final u,
v, h and vorticity are cut into the y-slabs of ws_slab_partition (rank r of N owns rows
[H r / N, H (r + 1) / N), ws_comm.h slab_rows) for N in {1, 2, 4, 8} (1 = the whole grid), and the SHA-256 of each
slab's owned rows (C order, float64) is stored. STEPS = 13 covers two full 6-step slab
blocks and a partial one, so two block-boundary exchanges (and, with the overlap schedule,
the exchanges on the edge stream) are inside the checked run.

Output: tests/golden/ref_slab_digests.json (data only).
"""
import hashlib
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import RK4, SWE, cfg_lines, ic_line, read_snap, run_spec  # noqa: E402

W = H = 4096
STEPS = 13
NRANKS = (1, 2, 4, 8)
FIELDS = ("u", "v", "h", "vort")
CASE = f"C2_jet_stream_4096_i2_f64_{STEPS}"


def slab_rows(height, rank, nranks):
    """Balanced split (ws_comm.h slab_rows; pinned against the library by tests/test_abi.py)."""
    r0 = height * rank // nranks
    r1 = height * (rank + 1) // nranks
    return r0, r1 - r0


def main():
    with tempfile.TemporaryDirectory(prefix="ws_slab_", dir="/tmp") as tmp:
        lines = cfg_lines(W, H, SWE, RK4, max_time=1e30) + ["create", ic_line("jet_stream"), "initialize",
                                                           f"run {STEPS}", f"snap {tmp}/L.bin"]
        run_spec("f64", lines, tmp)
        s = read_snap(f"{tmp}/L.bin")
    assert s["step"] == STEPS
    out = {"case": CASE, "grid": [W, H], "steps": STEPS, "time": s["time"], "ic": "jet_stream", "method": "rk4",
           "precision": "f64", "numerics": "exact", "fields": list(FIELDS),
           "spec": [l for l in lines if not l.startswith("snap")], "slabs": {}}
    for n in NRANKS:
        per = []
        for r in range(n):
            r0, rows = slab_rows(H, r, n)
            per.append({"row0": r0, "rows": rows,
                        "sha256": {f: hashlib.sha256(s[f][r0:r0 + rows].tobytes()).hexdigest() for f in FIELDS}})
        out["slabs"][str(n)] = per
    with open(os.path.join(HERE, "ref_slab_digests.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", CASE, "time", s["time"])


if __name__ == "__main__":
    main()
