"""Slab decomposition of the physics-mode layered PE model on CPU (gloo, world 2 / 3): the
periodic ring's halo protocol, driven by the library's own plan (ws_lpe_exchange_plan).

ws_lpe_create_slab (a process per GPU, RCCL) decomposes the doubly periodic grid into y-slabs
around a RING: slab 0's upper neighbour is the last slab, and with two ranks both neighbours
are the same peer. Each rank keeps its slab in the library's layout (levels of rows + 2 rows,
one halo row above and below, unpadded rows) and, before every RK stage, executes the plan
exactly as SlabComm::exchange does with periodic=True (ws_comm.cpp): the plan lists side 0
(upper neighbour) first, then side 1; per side one packed message (msg_offset order); the
sends are posted side 0 then side 1 and the receives side 1 then side 0, so a pair's k-th
send meets the peer's k-th receive -- which is what makes the two-rank ring (same peer on
both sides) deliver my top row into the peer's bottom halo. The oracle's tendency then runs
on the halo-extended slab, stage by stage, and the owned rows must equal the whole-domain
oracle bit for bit (any wrong offset, side, order or wrap in the plan fails it). The GPU side
(the same stage schedule; the one-process pull transport and the 1-rank RCCL slab) is
tests/test_gpu_lpe_slabs.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import layered_pe_oracle as lp

DT, DX, DY, G, GP, F = 5.0, 1000.0, 1300.0, 9.81, 0.05, 1e-4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _initial(L, H, W, dtype):
    y, x = np.mgrid[0:H, 0:W]
    u, v, h = lp.rest_state(L, H, W, [100.0 + 40.0 * k for k in range(L)])
    for k in range(L):
        h[k] += 0.8 * np.cos(2 * np.pi * (x / W + 2 * y / H) + 0.3 * k)
        u[k] += 0.05 * np.sin(2 * np.pi * (2 * x / W + y / H) + k)
        v[k] += 0.04 * np.cos(2 * np.pi * (3 * y / H) - k)
    return tuple(a.astype(dtype) for a in (u, v, h))


def rk_step(y, tend, method):
    """One step of lp.step's integrators with the tendency supplied (the same expressions)."""
    ax = lambda s, c, k: tuple(si + c * ki for si, ki in zip(s, k))
    if method == lp.EULER:
        return ax(y, DT, tend(*y))
    if method == lp.RK2:
        return ax(y, DT, tend(*ax(y, 0.5 * DT, tend(*y))))
    k1 = tend(*y)
    k2 = tend(*ax(y, 0.5 * DT, k1))
    k3 = tend(*ax(y, 0.5 * DT, k2))
    k4 = tend(*ax(y, DT, k3))
    return tuple(yi + DT / 6.0 * (((a + 2 * b) + 2 * c) + d) for yi, a, b, c, d in zip(y, k1, k2, k3, k4))


def split_sides(plan, L):
    """The plan lists side 0 (upper neighbour) then side 1 (lower), 2 x 3L segments each."""
    assert len(plan) == 2 * 2 * 3 * L
    return plan[:6 * L], plan[6 * L:]


def execute_periodic(ext, plan, L):
    """ext: the three (L, rows + 2, W) arrays; one exchange as SlabComm::exchange(periodic)."""
    es = ext[0].dtype.itemsize
    W = ext[0].shape[2]
    row0 = W * es  # byte offset of row 0 of level 0 (one halo row above)
    raw = [a.reshape(-1).view(np.uint8) for a in ext]
    sides = split_sides(plan, L)
    peer = [s[0].peer for s in sides]
    send, recv = [], []
    for s in sides:
        segs = [x for x in s if x.kind == 0]
        assert len({x.peer for x in s}) == 1
        msg = np.zeros(sum(x.bytes for x in segs), np.uint8)
        for x in segs:
            o = row0 + x.offset
            assert 0 <= o and o + x.bytes <= raw[x.field].size
            msg[x.msg_offset:x.msg_offset + x.bytes] = raw[x.field][o:o + x.bytes]
        send.append(torch.from_numpy(msg))
        recv.append(torch.zeros(msg.size, dtype=torch.uint8))
    reqs = [dist.isend(send[0], peer[0]), dist.isend(send[1], peer[1]),
            dist.irecv(recv[1], peer[1]), dist.irecv(recv[0], peer[0])]
    for r in reqs:
        r.wait()
    for side, s in enumerate(sides):
        m = recv[side].numpy()
        for x in s:
            if x.kind == 1:
                o = row0 + x.offset
                assert 0 <= o and o + x.bytes <= raw[x.field].size
                raw[x.field][o:o + x.bytes] = m[x.msg_offset:x.msg_offset + x.bytes]


def _worker(rank, world, port, W, H, L, method, fp64, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import ctypes

        from weather_sim import _native
        r0, nr = ctypes.c_int32(), ctypes.c_int32()
        _native.check(_native.lib.ws_slab_partition(H, rank, world, ctypes.byref(r0), ctypes.byref(nr)))
        row0, rows = r0.value, nr.value
        dtype = np.float64 if fp64 else np.float32
        full = _initial(L, H, W, dtype)
        plan, lstride = _native.lpe_exchange_plan(W, rows, L, fp64, rank, world)
        assert lstride == (rows + 2) * W

        def tend(u, v, h):
            ext = [np.zeros((L, rows + 2, W), dtype) for _ in range(3)]
            for e, a in zip(ext, (u, v, h)):
                e[:, 1:rows + 1] = a
            execute_periodic(ext, plan, L)
            return tuple(k[:, 1:rows + 1] for k in lp.tendency(*ext, DX, DY, G, GP, F))

        y = tuple(a[:, row0:row0 + rows].copy() for a in full)
        ref = full
        whole = lambda u, v, h: lp.tendency(u, v, h, DX, DY, G, GP, F)
        for _ in range(steps):
            y = rk_step(y, tend, method)
            nxt = rk_step(ref, whole, method)
            # the stage-by-stage restatement is the oracle's step, bit for bit
            for a, b in zip(nxt, lp.step(ref, DT, DX, DY, G, GP, F, method, dtype)):
                np.testing.assert_array_equal(a, b)
            ref = nxt
        for name, a, b in zip("uvh", y, ref):
            np.testing.assert_array_equal(a, b[:, row0:row0 + rows], err_msg=f"rank {rank} {name}")
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("method", [0, 1, 2])
@pytest.mark.parametrize("fp64", [False, True])
def test_lpe_ring_matches_single_domain(world, method, fp64):
    mp.spawn(_worker, args=(world, _free_port(), 23, 17, 3, method, fp64, 3), nprocs=world, join=True)


def test_lpe_ring_one_row_slabs():
    """Three ranks of one row each (H = 3): every halo row is a neighbour's only row."""
    mp.spawn(_worker, args=(3, _free_port(), 9, 3, 2, 2, True, 2), nprocs=3, join=True)


def test_lpe_exchange_plan_layout():
    """Both sides present on every rank of a ring (peers wrap), side 0 listed first; sends
    read the slab's first / last row, receives write rows -1 / rows; one packed message per
    side (field-major, then level)."""
    from weather_sim import _native
    for fp64, W, rows, L in ((True, 23, 6, 3), (False, 1024, 128, 32), (False, 9, 1, 2)):
        es = 8 if fp64 else 4
        row = W * es
        for rank, world, peers in ((0, 3, (2, 1)), (2, 3, (1, 0)), (1, 2, (0, 0)), (1, 4, (0, 2))):
            plan, lstride = _native.lpe_exchange_plan(W, rows, L, fp64, rank, world)
            assert lstride == (rows + 2) * W
            for side, segs in enumerate(split_sides(plan, L)):
                assert {x.peer for x in segs} == {peers[side]}
                for kind, r in ((0, 0 if side == 0 else rows - 1), (1, -1 if side == 0 else rows)):
                    seg = [x for x in segs if x.kind == kind]
                    assert [(x.field, x.level) for x in seg] == [(f, l) for f in range(3) for l in range(L)]
                    for i, x in enumerate(seg):
                        assert x.msg_offset == i * row and x.bytes == row
                        assert x.offset == x.level * lstride * es + r * row
        assert _native.lpe_exchange_plan(W, rows, L, fp64, 0, 1)[0] == []
    with pytest.raises(ValueError):
        _native.lpe_exchange_plan(8, 4, 1, True, 2, 2)
