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


def _blocks(nb: int, r: int, nranks: int, share) -> int:
    """Blocks rank r owns among nb (vr_internal.h share_blocks)."""
    w0, w = share
    P = w0 + (nranks - 1) * w
    q, o = divmod(nb, P)
    wr, off = (w0, 0) if r == 0 else (w, w0 + (r - 1) * w)
    return q * wr + (min(o - off, wr) if o > off else 0)


def shard_rows(height: int, row_block: int, nranks: int, share=(1, 1)) -> int:
    """Rows of every rank's shard (the largest share; vr_shard_rows / vr_shard_rows_ctx)."""
    nb = (height + row_block - 1) // row_block
    return max(_blocks(nb, r, nranks, share) for r in range(min(nranks, 2))) * row_block


def global_block(lb, rank: int, nranks: int, share=(1, 1)):
    """Global block of rank's local block(s) lb (vr_internal.h share_global_block): per period of
    w0 + (n - 1) w blocks rank 0 takes the first w0, rank r > 0 the w after w0 + (r - 1) w."""
    w0, w = share
    P = w0 + (nranks - 1) * w
    wr, off = (w0, 0) if rank == 0 else (w, w0 + (rank - 1) * w)
    return (lb // wr) * P + off + lb % wr


def shard_global_rows(height: int, row_block: int, rank: int, nranks: int, share=(1, 1)) -> np.ndarray:
    """Global row of every local shard row (-1 for padding rows past the frame)."""
    sr = shard_rows(height, row_block, nranks, share)
    ly = np.arange(sr)
    blk = ly // row_block
    gy = global_block(blk, rank, nranks, share) * row_block + ly % row_block
    return np.where(gy < height, gy, -1)


def assemble_numpy(gathered: np.ndarray, height: int, row_block: int, nranks: int,
                   share=(1, 1)) -> np.ndarray:
    """gathered: (nranks, shard_rows, W, ...) rank-major -> (height, W, ...) (vr_assemble_rows)."""
    w0, w = share
    P = w0 + (nranks - 1) * w
    y = np.arange(height)
    blk = y // row_block
    q, o = blk // P, blk % P
    first = o < w0
    rank = np.where(first, 0, 1 + (o - w0) // w)
    lb = np.where(first, q * w0 + o, q * w + (o - w0) % w)
    ly = lb * row_block + y % row_block
    return gathered[rank, ly]


def gather_to_root(local, gathered_views, rank: int, dist, async_op: bool = False):
    """One gather per frame of every rank's shard into rank 0's rank-major buffer views."""
    return dist.gather(local, gathered_views if rank == 0 else None, dst=0, async_op=async_op)


class Slot:
    """One frame in flight: this rank's shard buffer, rank 0's rank-major gather buffer and
    assembled frame, and the stream the frame's work is enqueued on (None on CPU)."""

    def __init__(self, shard, gbuf=None, frame=None, stream=None):
        self.shard, self.gbuf, self.frame, self.stream = shard, gbuf, frame, stream
        self.work = None  # the gather of the frame last rendered in this slot


class FramePipeline:
    """Per-frame render -> gather -> assemble with F = len(slots) frames in flight.

    Frame i uses slot i mod F: `render(slot)` enqueues this rank's shard of the frame into
    slot.shard on slot.stream, the gather to rank 0 is issued from that stream
    (async_op=True; RCCL orders it after the render), and `assemble(slot)` (rank 0)
    de-interleaves slot.gbuf into slot.frame.  The gather is only waited for (work.wait():
    a stream wait for NCCL/RCCL, a host wait for gloo) when the slot comes round again, F
    frames later, right before its assembly and before its buffers are rendered into again.
    So with F >= 2 frame k+1..k+F-1 render while frame k's gather is on the wire, and the
    frames' kernels overlap on the device (the reference keeps MAX_FRAMES_IN_FLIGHT = 2,
    vulkan_context.h:17).  F = 1 is the serial form: each gather is waited for and its
    frame assembled before the next render.
    """

    def __init__(self, slots, rank, world, dist, render, assemble, host_staging=False):
        self.slots = list(slots)
        self.rank, self.world, self.dist = rank, world, dist
        self.render, self.assemble = render, assemble
        # host_staging: device shards gathered through host copies (gloo rehearsal of the
        # multi-GPU path on ranks sharing one device); always serial
        self.host_staging = host_staging
        self.k = 0
        self.order = []  # slots with a gather outstanding, oldest first

    @property
    def last(self):
        """The slot of the most recently issued frame."""
        return self.slots[(self.k - 1) % len(self.slots)]

    def _ctx(self, slot):
        import contextlib
        if slot.stream is None:
            return contextlib.nullcontext()
        import torch
        return torch.cuda.stream(slot.stream)

    def _views(self, slot):
        if self.rank != 0:
            return None
        return [slot.gbuf[r] for r in range(self.world)]

    def _finish(self, slot):
        # called with slot.stream current: the wait orders this stream after the gather
        slot.work.wait()
        slot.work = None
        self.order.remove(slot)
        if self.rank == 0:
            self.assemble(slot)

    def step(self):
        slot = self.slots[self.k % len(self.slots)]
        self.k += 1
        with self._ctx(slot):
            if slot.work is not None:
                self._finish(slot)
            self.render(slot)
            if self.world == 1:
                return
            if self.host_staging:
                host = slot.shard.cpu()
                hviews = None
                if self.rank == 0:
                    hg = slot.gbuf.cpu()
                    hviews = [hg[r] for r in range(self.world)]
                gather_to_root(host, hviews, self.rank, self.dist)
                if self.rank == 0:
                    slot.gbuf.copy_(hg)
                    self.assemble(slot)
                return
            slot.work = gather_to_root(slot.shard, self._views(slot), self.rank, self.dist,
                                       async_op=True)
            self.order.append(slot)
            if len(self.slots) == 1:
                self._finish(slot)

    def drain(self):
        while self.order:
            slot = self.order[0]
            with self._ctx(slot):
                self._finish(slot)
