"""CPU, world_size 2 (and 3) with the gloo backend: the multi-GPU frame path end to end —
row-block shards rendered per rank (by the CPU oracle, standing in for the device kernel),
one gather to rank 0 (the same vr_dist.gather_to_root the benchmark uses over RCCL), and the
de-interleave — reassembles the single-process frame bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import vr_dist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene(W, H):
    import pyoracle
    import synth
    import vr_amd
    vol = synth.gaussians_numpy((16, 14, 12), seed=3)
    cam = synth.camera("rotA").to_vr_camera()
    p = vr_amd.default_params(shading=1)
    return pyoracle.Scene.from_params(vol, float(vol.min()), float(vol.max()), synth.tf_color(),
                                      cam, W, H, p)


def _worker(rank, world, port, W, H, rb, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for sub in ("volumetric-renderer_amd", "oracle", "tools"):
        sys.path.insert(0, os.path.join(root, sub))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = _scene(W, H)
        rows = vr_dist.shard_global_rows(H, rb, rank, world)
        img, st = sc.render_rows(rows[rows >= 0], nthreads=2)
        shard = np.zeros((len(rows), W, 4), np.float32)
        shard[rows >= 0] = img[rows[rows >= 0]]
        local = torch.from_numpy(shard)
        views = None
        if rank == 0:
            buf = torch.empty((world,) + tuple(local.shape), dtype=local.dtype)
            views = [buf[r] for r in range(world)]
        vr_dist.gather_to_root(local, views, rank, dist)
        samples = torch.tensor([st["samples"]], dtype=torch.int64)
        dist.all_reduce(samples)
        if rank == 0:
            frame = vr_dist.assemble_numpy(buf.numpy(), H, rb, world)
            q.put((frame, int(samples.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,rb", [(2, 16), (2, 4), (3, 8)])
def test_gloo_sharded_frame_matches_single_process(world, rb):
    W, H = 40, 45
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, rb, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame, samples = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full, st = _scene(W, H).render()
    assert np.array_equal(frame, full)
    assert samples == st["samples"]


def test_shard_layout_is_a_partition():
    for H, rb, n in ((1080, 16, 8), (53, 1, 5), (7, 16, 3), (2048, 16, 4)):
        seen = np.concatenate([vr_dist.shard_global_rows(H, rb, r, n) for r in range(n)])
        seen = seen[seen >= 0]
        assert np.array_equal(np.sort(seen), np.arange(H))
        g = np.stack([np.where(vr_dist.shard_global_rows(H, rb, r, n)[:, None] >= 0,
                               vr_dist.shard_global_rows(H, rb, r, n)[:, None], -1) for r in range(n)])
        assert np.array_equal(vr_dist.assemble_numpy(g, H, rb, n)[:, 0], np.arange(H))
