"""Multi-rank slab decomposition on CPU (gloo, world_size 2 and 3) -- the N>1 path's logic,
driven by the library's own halo exchange plan.

libws_hip.so's y-slab decomposition rests on claims that do not need a GPU:
  1. ws_slab_partition's balanced rows cover the grid (rank r owns [row0, row0 + rows));
  2. the exchange plan (ws_slab_exchange_plan: per neighbour ONE packed message, the byte
     offsets of every (field, level) send / receive segment in the slab-grid layout) moves
     exactly the rows the neighbours need: a step of an n-stage integrator needs n halo rows
     from each neighbour (the fused kernel's dependency cone), so a block of `block` steps
     needs block x n rows (the library always exchanges block x n rows at a block start,
     ws_runtime.cpp step path); the end-of-run vorticity / divergence needs one fresh row of
     u, v (a 2-field, depth-1 plan);
  3. bench.py's bootstrap (rank 0's RCCL unique id broadcast over gloo) and its
     max-over-ranks job time.
Each rank keeps its slab in the library's device layout (kHalo halo rows above and below
every level, rows padded to `pitch` elements) as host byte buffers, and executes the plan
the library returns exactly as the RCCL transport does (ws_comm.cpp SlabComm::exchange:
pack the send segments into one message per neighbour, send / receive, unpack the receive
segments) -- over gloo instead of RCCL. It then steps the CPU oracle on the halo-extended
slab, keeps its own rows, and compares them bit-for-bit with the oracle run on the whole
grid: a wrong offset, length, order or depth in the plan fails the comparison. SWE (one
level) and the Primitive-Equations model with 32 levels (RK4 -> RK2 per the reference) are
covered. The GPU side of the same plan runs in tests/test_gpu_parity.py::test_slab_group_*
(device-copy transport) and tests/test_gpu_slab_rccl.py.
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


def _nst(model, method):
    """Stages per step: the reference runs RK4 as RK2 for the non-SWE models."""
    return NST[1 if (method == 2 and model != 0) else method]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _initial(prec, L=1):
    y, x = np.mgrid[0:H, 0:W]
    out = []
    for k in range(L):
        u = np.sin(0.3 * x + 0.1 * y + 0.2 * k).astype(prec)
        v = np.cos(0.2 * x - 0.4 * y - 0.1 * k).astype(prec)
        h = (10.0 + np.sin(0.05 * x * y) + 0.01 * k).astype(prec)
        out.append((u, v, h))
    return [np.stack([lv[i] for lv in out]) for i in range(3)]  # (L, H, W) each


def _oracle_step(fields, model, method, prec, steps=1):
    """fields: (u, v, h) of one level, (rows, W) each."""
    from oracle.ws_oracle import OracleSim
    u, v, h = fields
    sim = OracleSim(u.shape[1], u.shape[0], model, method, 1.0, 2.0, 0.01, 9.81, 0.25, 1e30, prec)
    sim.initialize()
    for k, a in zip("uvh", (u, v, h)):
        sim.set_field(k, a)
    sim.calculate_diagnostics()
    sim.run(steps)
    return [sim.get_field(k) for k in ("u", "v", "h", "vort", "div")]


class SlabBuffers:
    """Host copy of one rank's slab fields in the library's device layout: field i is a byte
    buffer of L x (rows + 2 halo) x pitch elements; plan offsets count from row 0 of level 0."""

    def __init__(self, nfields, L, rows, pitch, lstride, dtype):
        self.L, self.rows, self.pitch, self.lstride, self.dtype = L, rows, pitch, lstride, np.dtype(dtype)
        self.halo = (lstride // pitch - rows) // 2
        self.buf = [np.zeros(L * lstride, self.dtype) for _ in range(nfields)]
        self.row0_bytes = self.halo * pitch * self.dtype.itemsize

    def rows_view(self, f, level, y0, y1):
        """Rows [y0, y1) (slab coordinates, may be negative) of field f, level `level`."""
        a = self.buf[f][level * self.lstride:(level + 1) * self.lstride].reshape(-1, self.pitch)
        return a[self.halo + y0:self.halo + y1, :W]

    def bytes_of(self, f):
        return self.buf[f].view(np.uint8)


K_DIRECT_SEGS = 4  # ws_halo.h kDirectSegs


def execute_plan(slab, plan):
    """Run one exchange of the library's plan over gloo, as SlabComm::exchange does over RCCL:
    with at most kDirectSegs segments per neighbour (SWE), one send / receive per segment
    straight from / into the field rows, posted in plan order; else pack the send segments
    into one message per peer (msg_offset order), send / receive, unpack into the receive
    segments."""
    peers = sorted({x.peer for x in plan})
    if all(sum(1 for x in plan if x.peer == p and x.kind == 0) <= K_DIRECT_SEGS for p in peers):
        reqs, landing = [], []
        for x in plan:
            buf = slab.bytes_of(x.field)
            o = slab.row0_bytes + x.offset
            assert 0 <= o and o + x.bytes <= buf.size
            if x.kind == 0:
                reqs.append(dist.isend(torch.from_numpy(buf[o:o + x.bytes].copy()), x.peer))
            else:
                t = torch.zeros(x.bytes, dtype=torch.uint8)
                reqs.append(dist.irecv(t, x.peer))
                landing.append((buf, o, t))
        for r in reqs:
            r.wait()
        for buf, o, t in landing:
            buf[o:o + t.numel()] = t.numpy()
        return
    msg_len = {p: max(x.msg_offset + x.bytes for x in plan if x.peer == p and x.kind == 0) for p in peers}
    for p in peers:  # the receive message has the send message's shape
        assert msg_len[p] == max(x.msg_offset + x.bytes for x in plan if x.peer == p and x.kind == 1)
    send = {p: np.zeros(msg_len[p], np.uint8) for p in peers}
    recv = {p: torch.zeros(msg_len[p], dtype=torch.uint8) for p in peers}
    for x in plan:
        if x.kind == 0:
            src = slab.bytes_of(x.field)
            o = slab.row0_bytes + x.offset
            assert 0 <= o and o + x.bytes <= src.size
            send[x.peer][x.msg_offset:x.msg_offset + x.bytes] = src[o:o + x.bytes]
    reqs = []
    for p in peers:
        reqs.append(dist.isend(torch.from_numpy(send[p]), p))
        reqs.append(dist.irecv(recv[p], p))
    for r in reqs:
        r.wait()
    for x in plan:
        if x.kind == 1:
            dst = slab.bytes_of(x.field)
            o = slab.row0_bytes + x.offset
            assert 0 <= o and o + x.bytes <= dst.size
            dst[o:o + x.bytes] = recv[x.peer].numpy()[x.msg_offset:x.msg_offset + x.bytes]


def _worker(rank, world, port, model, method, fp64, L, steps, block):
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
        dtype = np.float64 if fp64 else np.float32
        full = _initial(dtype, L)
        nst = _nst(model, method)
        depth = block * nst
        plan, pitch, lstride = _native.exchange_plan(W, rows, L, fp64, rank, world, 3, depth)
        # one message per neighbour, field-major then level, covering depth rows each
        assert len(plan) == 2 * 3 * L * ((rank > 0) + (rank < world - 1))
        assert all(x.bytes == depth * pitch * np.dtype(dtype).itemsize for x in plan)
        slab = SlabBuffers(3, L, rows, pitch, lstride, dtype)
        for f in range(3):
            for k in range(L):
                slab.rows_view(f, k, 0, rows)[:] = full[f][k, row0:row0 + rows]
        ext_top = depth if rank > 0 else 0
        ext_bot = depth if rank < world - 1 else 0
        # 2. per block: the library's exchange (block x NST rows), step the extended slab
        # `nb` steps per level, keep the owned rows
        done = 0
        while done < steps:
            nb = min(block, steps - done)
            execute_plan(slab, plan)
            for k in range(L):
                ext = [slab.rows_view(f, k, -ext_top, rows + ext_bot).copy() for f in range(3)]
                out = _oracle_step(ext, model, method, prec, steps=nb)
                for f in range(3):
                    slab.rows_view(f, k, 0, rows)[:] = out[f][ext_top:ext_top + rows]
            done += nb
        # end-of-run u, v refresh for the diagnostics: the library's 2-field, depth-1 plan
        dplan, _, _ = _native.exchange_plan(W, rows, L, fp64, rank, world, 2, 1)
        execute_plan(slab, dplan)
        t1, b1 = int(rank > 0), int(rank < world - 1)
        for k in range(L):
            ref = _oracle_step([a[k] for a in full], model, method, prec, steps=steps)
            for f, name in enumerate("uvh"):
                np.testing.assert_array_equal(slab.rows_view(f, k, 0, rows), ref[f][row0:row0 + rows],
                                              err_msg=f"rank {rank} level {k} {name}")
            ext = [slab.rows_view(f, k, -t1, rows + b1).copy() for f in range(2)]
            ext.append(np.zeros_like(ext[0]))
            diag = _oracle_step(ext, model, method, prec, steps=0)
            for name, i in (("vorticity", 3), ("divergence", 4)):
                np.testing.assert_array_equal(diag[i][t1:t1 + rows], ref[i][row0:row0 + rows],
                                              err_msg=f"rank {rank} level {k} {name}")
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,block", [(2, 1), (3, 1), (2, 3), (3, 2)])
@pytest.mark.parametrize("method", [0, 1, 2])
@pytest.mark.parametrize("fp64", [False, True])
def test_slab_protocol_matches_single_domain(world, block, method, fp64):
    mp.spawn(_worker, args=(world, _free_port(), 0, method, fp64, 1, 5, block), nprocs=world, join=True)


@pytest.mark.parametrize("world,block", [(2, 2), (3, 3)])
def test_slab_protocol_pe_32_levels(world, block):
    """C4's shape of exchange: the PE model (RK4 -> RK2), 32 levels in one packed message."""
    mp.spawn(_worker, args=(world, _free_port(), 2, 2, False, 32, 4, block), nprocs=world, join=True)


def test_exchange_plan_layout():
    """The plan's segments: per neighbour the send and receive lists have one segment per
    (field, level) in field-major order, packed back to back; sends read owned rows,
    receives write the halo rows (never an owned row)."""
    from weather_sim import _native
    for fp64, L, rows, depth in ((True, 1, 512, 12), (False, 32, 128, 4), (True, 3, 5, 5)):
        es = 8 if fp64 else 4
        plan, pitch, lstride = _native.exchange_plan(4000, rows, L, fp64, 1, 3, 3, depth)
        row = pitch * es
        halo2 = lstride // pitch - rows  # halo rows above + below
        assert pitch % 64 == 0 and pitch >= 4000 and lstride % pitch == 0 and halo2 % 2 == 0 and halo2 // 2 >= depth
        for peer, send_row, recv_row in ((0, 0, -depth), (2, rows - depth, rows)):
            for kind, r0 in ((0, send_row), (1, recv_row)):
                seg = [x for x in plan if x.peer == peer and x.kind == kind]
                assert [(x.field, x.level) for x in seg] == [(f, l) for f in range(3) for l in range(L)]
                for i, x in enumerate(seg):
                    assert x.msg_offset == i * depth * row and x.bytes == depth * row
                    assert x.offset == x.level * lstride * es + r0 * row
        # edge ranks have one neighbour only
        assert {x.peer for x in _native.exchange_plan(64, rows, L, fp64, 0, 3, 3, depth)[0]} == {1}
        assert {x.peer for x in _native.exchange_plan(64, rows, L, fp64, 2, 3, 3, depth)[0]} == {1}
        assert _native.exchange_plan(64, rows, L, fp64, 0, 1, 3, depth)[0] == []
    _, pitch, lstride = _native.exchange_plan(64, 64, 1, True, 0, 2, 3, 1)
    halo = (lstride // pitch - 64) // 2
    _native.exchange_plan(64, 64, 1, True, 0, 2, 3, halo)  # the whole halo
    with pytest.raises(ValueError):
        _native.exchange_plan(64, 64, 1, True, 0, 2, 3, halo + 1)  # deeper than the halo rows


def test_halo_depth_is_necessary():
    """With one row fewer than the stage count the seam rows differ: the depth is tight.
    (fp64: the 4th-stage error is ~dt^3 relative, below fp32's ulp.)"""
    prec, method = "f64", 2
    full = _initial(np.float64)
    full = [a[0] for a in full]
    ref = _oracle_step(full, 0, method, prec)
    split = H // 2
    d = NST[method] - 1
    ext = [a[:split + d] for a in full]
    got = _oracle_step(ext, 0, method, prec)
    assert not np.array_equal(got[0][:split], ref[0][:split])
