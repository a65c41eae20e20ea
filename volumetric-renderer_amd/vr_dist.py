"""Image-space (sort-first) sharding of one frame across ranks, one process per GPU.

Row-block-cyclic layout: the frame's rows are cut into blocks of `row_block`
rows; block b belongs to rank b % N.  Each rank ray-marches only its blocks (vr_render_device
with rank/nranks) into a dense shard of vr_shard_rows() rows, the shards are gathered to rank 0
with ONE collective per frame (torch.distributed.gather -> RCCL over xGMI with the "nccl"
backend, gloo on CPU), and rank 0 de-interleaves them (vr_assemble_rows, a permutation kernel).
The volume is replicated per GPU; there is no other exchange on the data path.

The numpy functions restate the kernels' index maps for CPU tests.
"""
from __future__ import annotations

import numpy as np


def shard_rows(height: int, row_block: int, nranks: int) -> int:
    blocks = (height + row_block - 1) // row_block
    return ((blocks + nranks - 1) // nranks) * row_block


def shard_global_rows(height: int, row_block: int, rank: int, nranks: int) -> np.ndarray:
    """Global row of every local shard row (-1 for padding rows past the frame)."""
    sr = shard_rows(height, row_block, nranks)
    ly = np.arange(sr)
    blk = ly // row_block
    gy = (blk * nranks + rank) * row_block + ly % row_block
    return np.where(gy < height, gy, -1)


def assemble_numpy(gathered: np.ndarray, height: int, row_block: int, nranks: int) -> np.ndarray:
    """gathered: (nranks, shard_rows, W, ...) rank-major -> (height, W, ...) (vr_assemble_rows)."""
    y = np.arange(height)
    blk = y // row_block
    rank = blk % nranks
    ly = (blk // nranks) * row_block + y % row_block
    return gathered[rank, ly]


def gather_to_root(local, gathered_views, rank: int, dist, async_op: bool = False):
    """One gather per frame of every rank's shard into rank 0's rank-major buffer views."""
    return dist.gather(local, gathered_views if rank == 0 else None, dst=0, async_op=async_op)


class FramePipeline:
    """Per-frame render -> gather -> assemble with the gather of frame k overlapped with the
    render of frame k+1 (double-buffered shards and gather buffers).

    `render(buf)` enqueues this rank's shard of the next frame into `buf`; `assemble(gbuf)`
    (rank 0) enqueues the de-interleave of a gathered rank-major buffer.  With overlap, the
    gather is issued async_op=True and only waited for (work.wait(): a stream wait for
    NCCL/RCCL, a host wait for gloo) one frame later, right before that frame is assembled
    and before its shard buffer is rendered into again.  overlap=False is the serial form.
    """

    def __init__(self, shards, gather_bufs, rank, world, dist, render, assemble, overlap=True,
                 host_staging=False):
        self.shards = shards            # list of 1 or 2 local shard tensors
        self.gather_bufs = gather_bufs  # rank 0: list of (world, rows, W) tensors, else None
        self.rank, self.world, self.dist = rank, world, dist
        self.render, self.assemble = render, assemble
        # host_staging: device shards gathered through host copies (gloo rehearsal of the
        # multi-GPU path on one device); always serial
        self.host_staging = host_staging
        self.overlap = overlap and world > 1 and len(shards) > 1 and not host_staging
        self.k = 0
        self.pending = None

    def _views(self, i):
        if self.rank != 0:
            return None
        g = self.gather_bufs[i]
        return [g[r] for r in range(self.world)]

    def _finish(self, work, i):
        work.wait()
        if self.rank == 0:
            self.assemble(self.gather_bufs[i])

    def step(self):
        i = self.k % len(self.shards)
        self.k += 1
        buf = self.shards[i]
        self.render(buf)
        if self.world == 1:
            return
        gi = i % len(self.gather_bufs) if self.rank == 0 else 0
        if self.host_staging:
            host = buf.cpu()
            hviews = None
            if self.rank == 0:
                hg = self.gather_bufs[gi].cpu()
                hviews = [hg[r] for r in range(self.world)]
            gather_to_root(host, hviews, self.rank, self.dist)
            if self.rank == 0:
                self.gather_bufs[gi].copy_(hg)
                self.assemble(self.gather_bufs[gi])
            return
        work = gather_to_root(buf, self._views(gi), self.rank, self.dist, async_op=True)
        if not self.overlap:
            self._finish(work, gi)
            return
        if self.pending is not None:
            self._finish(*self.pending)
        self.pending = (work, gi)

    def drain(self):
        if self.pending is not None:
            self._finish(*self.pending)
            self.pending = None
