"""Slab decomposition of the physics-mode vorticity model's Poisson solve on CPU (gloo, world
2 / 4): the block-transpose protocol of ws_bvort_create_slab, restated in NumPy.

The library's decomposed solve (csrc/ws_bvort.hip): each rank owns rows
[row0, row0 + rows) (ws_slab_partition) and transforms them along x; the half spectrum's real
bins A(0), A(W/2) are packed into column 0 as A(0) + i A(W/2), so there are W/2 columns, and
a rank's spectrum rows are stored block-major -- block q = the nc = W / (2 n) columns rank q
solves. SlabComm::alltoall sends block q to rank q and receives every rank's block of its own
columns into the column block [H][nc] (rows in rank order); the column pass transforms along
y, scales by 1 / lambda(k, l) with the GLOBAL column k = rank nc + c (column 0's packed pair
recombined as Z'(l) = (s0 + sN) / 2 Z(l) + (s0 - sN) / 2 conj Z(-l)), transforms back; the
transpose back and the inverse row pass give psi on the rank's rows. Each rank runs that
bookkeeping here over gloo (one send / receive per peer and direction, as the RCCL transport
posts them) and its rows of psi must equal the whole-grid spectral solve (the oracle) to
round-off: a wrong block offset, peer, row order, global column or packed-bin formula fails.
The device kernels of the same flow are compared bitwise with the single domain in
tests/test_gpu_bvort_slabs.py.
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import bvort_oracle as bo

DX, DY = 1.0, 1.25


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _field(W, H):
    y, x = np.mgrid[0:H, 0:W]
    rng = np.random.default_rng(7)
    z = np.zeros((H, W))
    for _ in range(5):
        kx, ky = rng.integers(0, W // 2), rng.integers(0, H // 2)
        z += rng.standard_normal() * np.cos(2 * np.pi * (kx * x / W + ky * y / H) + rng.uniform(0, 6.28))
    return z


def alltoall(send, recv_shape, world, rank):
    """send[q]: this rank's block for rank q (complex); returns recv[p] (the block from p), one
    isend / irecv per peer as SlabComm::alltoall posts them (its own block: a copy)."""
    recv = [None] * world
    bufs, reqs = {}, []
    for q in range(world):
        if q == rank:
            recv[q] = send[q].copy()
            continue
        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(send[q]).view(np.float64)), q))
        bufs[q] = torch.zeros(int(np.prod(recv_shape[q])) * 2, dtype=torch.float64)
        reqs.append(dist.irecv(bufs[q], q))
    for r in reqs:
        r.wait()
    for q, b in bufs.items():
        recv[q] = b.numpy().view(np.complex128).reshape(recv_shape[q])
    return recv


def _worker(rank, world, port, W, H):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from weather_sim import _native
        r0, nr = ctypes.c_int32(), ctypes.c_int32()
        _native.check(_native.lib.ws_slab_partition(H, rank, world, ctypes.byref(r0), ctypes.byref(nr)))
        row0, rows = r0.value, nr.value
        assert rows == H // world and rows % 2 == 0  # equal slabs of whole row pairs
        nk = W // 2
        nc = nk // world
        zeta = _field(W, H)

        # row pass on the own rows, real bins packed into column 0
        R = np.fft.rfft(zeta[row0:row0 + rows], axis=1)
        P = R[:, :nk].copy()
        P[:, 0] = R[:, 0].real + 1j * R[:, nk].real
        # block-major spectrum rows: block q = columns [q nc, (q + 1) nc)
        send = [P[:, q * nc:(q + 1) * nc] for q in range(world)]
        got = alltoall(send, [(rows, nc)] * world, world, rank)
        cols = np.concatenate(got, axis=0)  # [H][nc], rows in rank order (row0_p = p rows)
        assert cols.shape == (H, nc)

        # column pass on global columns [rank nc, (rank + 1) nc)
        lam = bo.laplacian_eigenvalues(W, H, DX, DY)  # [H][W/2 + 1]
        F = np.fft.fft(cols, axis=0)
        l = np.arange(H)
        for c in range(nc):
            k = rank * nc + c
            if k == 0:
                s0 = np.where(l == 0, 0.0, 1.0 / np.where(l == 0, 1.0, lam[:, 0]))
                sN = 1.0 / lam[:, nk]
                Zm = F[(-l) % H, c]
                F[:, c] = (s0 + sN) / 2 * F[:, c] + (s0 - sN) / 2 * np.conj(Zm)
            else:
                F[:, c] = F[:, c] / lam[:, k]
        cols = np.fft.ifft(F, axis=0)

        # transpose back: rows [row0_p, row0_p + rows) of the column block go to rank p
        back = alltoall([cols[p * rows:(p + 1) * rows] for p in range(world)], [(rows, nc)] * world, world, rank)
        P2 = np.concatenate(back, axis=1)  # [rows][W/2], block q = columns of rank q
        R2 = np.zeros((rows, nk + 1), dtype=np.complex128)
        R2[:, 1:nk] = P2[:, 1:]
        R2[:, 0] = P2[:, 0].real
        R2[:, nk] = P2[:, 0].imag
        psi = np.fft.irfft(R2, n=W, axis=1)

        want = bo.poisson(zeta, DX, DY)[row0:row0 + rows]
        err = np.linalg.norm(psi - want) / np.linalg.norm(want)
        assert err < 1e-12, (rank, err)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H", [(2, 32, 16), (4, 64, 32), (4, 16, 64), (8, 16, 16)])
def test_bvort_block_transposes_match_the_whole_grid_solve(world, W, H):
    """8 ranks at 16 x 16: one spectrum column and two rows per rank."""
    mp.spawn(_worker, args=(world, _free_port(), W, H), nprocs=world, join=True)
