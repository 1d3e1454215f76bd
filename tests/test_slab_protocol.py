"""Multi-rank slab decomposition on CPU (gloo, world_size 2 and 3) -- the N>1 path's logic.

libws_hip.so's y-slab decomposition rests on three claims that do not need
a GPU to check:
  1. ws_slab_partition's balanced rows cover the grid (rank r owns [row0, row0 + rows));
  2. a step of an n-stage integrator needs exactly n halo rows from each neighbour (the
     fused kernel's dependency cone), so `block` steps need block x n rows: a slab that
     receives block x n rows advances `block` steps before the next exchange (clamped only
     at the global top/bottom edges); the end-of-run vorticity/divergence needs one fresh
     row of u, v;
  3. bench.py's bootstrap (rank 0's RCCL unique id broadcast over gloo) and its
     max-over-ranks job time.
Here each rank holds its slab, swaps block x n halo rows with its neighbours over gloo
send/recv (the RCCL exchange's message pattern: top rows to rank-1, bottom rows to rank+1),
steps the CPU oracle `block` steps on the halo-extended slab, keeps its own rows, and
compares them bit-for-bit with the oracle run on the whole grid. The GPU side of the same decomposition is tested
in tests/test_gpu_parity.py::test_slab_group_* and tests/test_gpu_slab_rccl.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W, H = 53, 37
NST = {0: 1, 1: 2, 2: 4}  # Euler, RK2, RK4 stages == halo depth


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _initial(prec):
    y, x = np.mgrid[0:H, 0:W]
    u = np.sin(0.3 * x + 0.1 * y).astype(prec)
    v = np.cos(0.2 * x - 0.4 * y).astype(prec)
    h = (10.0 + np.sin(0.05 * x * y)).astype(prec)
    return u, v, h


def _oracle_step(fields, method, prec, steps=1):
    from oracle.ws_oracle import OracleSim
    u, v, h = fields
    sim = OracleSim(u.shape[1], u.shape[0], 0, method, 1.0, 2.0, 0.01, 9.81, 0.25, 1e30, prec)
    sim.initialize()
    for k, a in zip("uvh", (u, v, h)):
        sim.set_field(k, a)
    sim.calculate_diagnostics()
    sim.run(steps)
    return [sim.get_field(k) for k in ("u", "v", "h", "vort", "div")]


def _swap_halo(arrs, depth, rank, world):
    """Top `depth` rows <-> rank-1's bottom rows; bottom rows <-> rank+1's top rows."""
    top = [np.empty((0, W), a.dtype) for a in arrs]
    bot = [np.empty((0, W), a.dtype) for a in arrs]
    reqs, bufs = [], []
    for i, a in enumerate(arrs):
        if rank > 0:
            reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(a[:depth])), rank - 1))
            t = torch.empty((depth, W), dtype=torch.from_numpy(a[:1]).dtype)
            reqs.append(dist.irecv(t, rank - 1))
            bufs.append(("top", i, t))
        if rank < world - 1:
            reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(a[-depth:])), rank + 1))
            t = torch.empty((depth, W), dtype=torch.from_numpy(a[:1]).dtype)
            reqs.append(dist.irecv(t, rank + 1))
            bufs.append(("bot", i, t))
    for r in reqs:
        r.wait()
    for side, i, t in bufs:
        (top if side == "top" else bot)[i] = t.numpy()
    return top, bot


def _worker(rank, world, port, method, fp64, steps, block):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import ctypes

        from weather_sim import _native
        import bench

        # 3. bootstrap + timing reduction exactly as bench.py runs them
        uid = bench.bootstrap_uid(dist, rank, lambda: bytes(range(128)))
        assert uid == bytes(range(128))
        assert bench.max_over_ranks(dist, 1.0 + rank) == float(world)

        # 1. partition
        r0, nr = ctypes.c_int32(), ctypes.c_int32()
        _native.check(_native.lib.ws_slab_partition(H, rank, world, ctypes.byref(r0), ctypes.byref(nr)))
        row0, rows = r0.value, nr.value

        prec = "f64" if fp64 else "f32"
        full = _initial(np.float64 if fp64 else np.float32)
        own = [a[row0:row0 + rows].copy() for a in full]
        # 2. per block: swap block x NST halo rows, step the extended slab `block` times,
        # keep the owned rows
        done = 0
        while done < steps:
            nb = min(block, steps - done)
            top, bot = _swap_halo(own, nb * NST[method], rank, world)
            ext = [np.concatenate([t, a, b]) for t, a, b in zip(top, own, bot)]
            out = _oracle_step(ext, method, prec, steps=nb)
            lo = top[0].shape[0]
            own = [o[lo:lo + rows] for o in out[:3]]
            done += nb
        top, bot = _swap_halo(own[:2], 1, rank, world)  # end-of-run u, v refresh for diagnostics
        ext = [np.concatenate([t, a, b]) for t, a, b in zip(top, own[:2], bot)]
        ext.append(np.concatenate([np.zeros_like(top[0]), own[2], np.zeros_like(bot[0])]))
        diag = _oracle_step(ext, method, prec, steps=0)
        lo = top[0].shape[0]

        ref = _oracle_step(full, method, prec, steps=steps)
        for name, got, want in zip(("u", "v", "h"), own, ref[:3]):
            np.testing.assert_array_equal(got, want[row0:row0 + rows], err_msg=f"rank {rank} {name}")
        for name, k in (("vorticity", 3), ("divergence", 4)):
            np.testing.assert_array_equal(diag[k][lo:lo + rows], ref[k][row0:row0 + rows],
                                          err_msg=f"rank {rank} {name}")
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,block", [(2, 1), (3, 1), (2, 3), (3, 2)])
@pytest.mark.parametrize("method", [0, 1, 2])
@pytest.mark.parametrize("fp64", [False, True])
def test_slab_protocol_matches_single_domain(world, block, method, fp64):
    mp.spawn(_worker, args=(world, _free_port(), method, fp64, 5, block), nprocs=world, join=True)


def test_halo_depth_is_necessary():
    """With one row fewer than the stage count the seam rows differ: the depth is tight.
    (fp64: the 4th-stage error is ~dt^3 relative, below fp32's ulp.)"""
    prec, method = "f64", 2
    full = _initial(np.float64)
    ref = _oracle_step(full, method, prec)
    split = H // 2
    d = NST[method] - 1
    ext = [a[:split + d] for a in full]
    got = _oracle_step(ext, method, prec)
    assert not np.array_equal(got[0][:split], ref[0][:split])
