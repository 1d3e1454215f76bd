"""bench.py's parity self-check (run before the timed region at every N): each rank hashes
its owned rows of the golden case and compares them with the reference's per-slab digests
(tests/golden/ref_slab_digests.json, made by tests/golden/gen_slab_digests.py from the
reference binary), and the default fast numerics are held to the north_star 1e-10 relative
L2 over the whole grid (sums over ranks). Every rank must reach the same verdict.

On CPU: gloo world 2 and 3, the library's own slab partition (ws_slab_partition), the CPU
oracle standing in for the GPU slabs (whole-grid run, each rank keeps its rows), and the
same check function bench.py calls; corrupted and out-of-tolerance ranks must fail the job
on every rank."""
import hashlib
import json
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, STEPS = 64, 41, 13


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _partition(height, rank, world):
    import ctypes

    from weather_sim import _native
    r0, nr = ctypes.c_int32(), ctypes.c_int32()
    _native.check(_native.lib.ws_slab_partition(height, rank, world, ctypes.byref(r0), ctypes.byref(nr)))
    return r0.value, nr.value


def _oracle_run():
    from oracle.ws_oracle import OracleSim
    y, x = np.mgrid[0:H, 0:W]
    sim = OracleSim(W, H, 0, 2, 1.0, 1.0, 0.01, 9.81, 0.0, 1e30, "f64")
    sim.initialize()
    sim.set_field("u", np.sin(0.3 * x + 0.1 * y))
    sim.set_field("v", np.cos(0.2 * x - 0.4 * y))
    sim.set_field("h", 10.0 + np.sin(0.05 * x * y))
    sim.run(STEPS)
    return {k: sim.get_field(k) for k in ("u", "v", "h", "vort")}


def _golden(full, worlds):
    g = {"case": "cpu_oracle_64x41", "steps": STEPS, "fields": ["u", "v", "h", "vort"], "slabs": {}}
    for n in worlds:
        per = []
        for r in range(n):
            r0, rows = _partition(H, r, n)
            per.append({"row0": r0, "rows": rows,
                        "sha256": {k: hashlib.sha256(full[k][r0:r0 + rows].tobytes()).hexdigest() for k in full}})
        g["slabs"][str(n)] = per
    return g


def _worker(rank, world, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        full = _oracle_run()
        golden = _golden(full, (world,))
        r0, rows = _partition(H, rank, world)
        mine = {k: a[r0:r0 + rows].copy() for k, a in full.items()}
        out = {}
        # 1. correct slabs, fast numerics a rounding away: ok on every rank
        fast = {k: a * (1 + 1e-15) for k, a in mine.items()}
        out["ok"] = bench.check_slab_parity(dist, rank, world, r0, rows, mine, fast, golden)
        # 2. one cell of the last rank off by one ulp: every rank fails
        bad = {k: a.copy() for k, a in mine.items()}
        if rank == world - 1:
            bad["h"][rows // 2, 3] = np.nextafter(bad["h"][rows // 2, 3], np.inf)
        out["ulp"] = bench.check_slab_parity(dist, rank, world, r0, rows, bad, None, golden)
        # 3. fast numerics outside the tolerance on rank 0 only: every rank fails
        off = {k: a.copy() for k, a in mine.items()}
        if rank == 0:
            off["u"] = off["u"] * (1 + 1e-7)
        out["tol"] = bench.check_slab_parity(dist, rank, world, r0, rows, mine, off, golden)
        # 4. rows of the wrong partition: fails
        out["rows"] = bench.check_slab_parity(dist, rank, world, r0 + 1, rows, mine, None, golden)
        # 5. a world size with no reference digests: fails
        g2 = dict(golden, slabs={})
        out["missing"] = bench.check_slab_parity(dist, rank, world, r0, rows, mine, None, g2)
        results[rank] = {k: v[0] for k, v in out.items()}
        results[f"detail{rank}"] = out["ok"][1]
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_self_check_verdicts_over_gloo(world):
    with mp.Manager() as m:
        results = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), results), nprocs=world, join=True)
        res = dict(results)
    for r in range(world):
        assert res[r] == {"ok": "ok", "ulp": "fail", "tol": "fail", "rows": "fail", "missing": "fail"}, res[r]
    d = res["detail0"]
    assert d["exact"] == "bitwise == reference" and all(v <= 1e-10 for v in d["fast_rel_l2"].values())


def test_single_process_self_check():
    """World 1 (no process group): the same function, whole grid."""
    import bench
    full = _oracle_run()
    golden = _golden(full, (1,))
    v, d = bench.check_slab_parity(None, 0, 1, 0, H, full, full, golden)
    assert v == "ok" and d["fast_rel_l2"] == {"u": 0.0, "v": 0.0, "h": 0.0}
    bad = dict(full, vort=full["vort"] + 1e-300)
    assert bench.check_slab_parity(None, 0, 1, 0, H, bad, None, golden)[0] == "ok"  # 1e-300 is below an ulp
    bad = dict(full, vort=full["vort"] * (1 + 2e-16) + 1e-12)
    assert bench.check_slab_parity(None, 0, 1, 0, H, bad, None, golden)[0] == "fail"


def test_reference_slab_digests_fixture():
    """The committed reference digests: the golden case the bench runs, split exactly as the
    library partitions 4096 rows over 1 / 2 / 4 / 8 ranks."""
    with open(os.path.join(ROOT, "tests", "golden", "ref_slab_digests.json")) as f:
        g = json.load(f)
    assert g["grid"] == [4096, 4096] and g["steps"] == 13 and g["method"] == "rk4" and g["precision"] == "f64"
    assert set(g["slabs"]) == {"1", "2", "4", "8"}
    for n, per in g["slabs"].items():
        n = int(n)
        assert len(per) == n
        for r, e in enumerate(per):
            assert (e["row0"], e["rows"]) == _partition(4096, r, n)
            assert set(e["sha256"]) == {"u", "v", "h", "vort"}
    # the whole-grid entry differs from every slab's (distinct data)
    assert len({e["sha256"]["h"] for per in g["slabs"].values() for e in per}) == 1 + 2 + 4 + 8


def _ramp_worker(rank, world, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import time

        import bench
        bench.RAMP_S = 0.15
        chunks = []

        def chunk():
            # ranks run at different speeds: each alone would stop after a different count
            time.sleep(0.004 * (rank + 1))
            chunks.append(1)
            return 20
        steps = bench.clock_ramp(chunk, dist, True)
        results[rank] = (steps, len(chunks))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_clock_ramp_is_collective(world):
    """every ramp chunk of a slab decomposition is a collective run(), so the ramp's
    stop decision must be the same on every rank (a rank stopping one chunk early would leave
    the others blocked in RCCL)."""
    with mp.Manager() as m:
        results = m.dict()
        mp.spawn(_ramp_worker, args=(world, _free_port(), results), nprocs=world, join=True)
        res = dict(results)
    assert len({res[r] for r in range(world)}) == 1, res
    assert res[0][0] == 20 * res[0][1] and res[0][1] >= 1
