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


def gather_to_root(local, gathered_views, rank: int, dist) -> None:
    """One gather per frame of every rank's shard into rank 0's rank-major buffer views."""
    dist.gather(local, gathered_views if rank == 0 else None, dst=0)
