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


def _scene(W, H, k=0):
    import pyoracle
    import synth
    import vr_amd
    vol = synth.gaussians_numpy((16, 14, 12), seed=3)
    cam = vr_amd.make_camera(radius=2.0, rotate=(100.0 + 37.0 * k, 60.0 - 11.0 * k)).to_vr_camera()
    p = vr_amd.default_params(shading=1)
    return pyoracle.Scene.from_params(vol, float(vol.min()), float(vol.max()), synth.tf_color(),
                                      cam, W, H, p)


def _worker(rank, world, port, W, H, rb, inflight, nframes, q, share=(1, 1)):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for sub in ("volumetric-renderer_amd", "oracle", "tools"):
        sys.path.insert(0, os.path.join(root, sub))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = vr_dist.shard_global_rows(H, rb, rank, world, share)
        sr = len(rows)
        slots = [vr_dist.Slot(torch.zeros((sr, W, 4), dtype=torch.float32),
                              torch.zeros((world, sr, W, 4), dtype=torch.float32) if rank == 0 else None)
                 for _ in range(inflight)]
        frames, state = [], {"k": 0, "samples": 0}

        def render(slot):
            buf = slot.shard
            img, st = _scene(W, H, state["k"]).render_rows(rows[rows >= 0], nthreads=2)
            shard = np.zeros((sr, W, 4), np.float32)
            shard[rows >= 0] = img[rows[rows >= 0]]
            buf.copy_(torch.from_numpy(shard))
            state["samples"] += st["samples"]
            state["k"] += 1

        def assemble(slot):
            frames.append(vr_dist.assemble_numpy(slot.gbuf.numpy().copy(), H, rb, world, share))

        pipe = vr_dist.FramePipeline(slots, rank, world, dist, render, assemble)
        for _ in range(nframes):
            pipe.step()
        pipe.drain()
        samples = torch.tensor([state["samples"]], dtype=torch.int64)
        dist.all_reduce(samples)
        if rank == 0:
            q.put((frames, int(samples.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,rb,inflight,nframes,share",
                         [(2, 16, 2, 3, (1, 1)), (2, 4, 1, 3, (1, 1)), (3, 8, 3, 5, (1, 1)),
                          (2, 8, 3, 2, (1, 1)), (3, 4, 2, 3, (1, 2)), (2, 4, 2, 2, (3, 2))])
def test_gloo_sharded_frames_match_single_process(world, rb, inflight, nframes, share):
    """N ranks, several frames through vr_dist.FramePipeline (the benchmark's frame loop):
    every assembled frame equals the single-process oracle frame bit for bit, in order,
    serial (1 frame in flight) and with 2-3 frames in flight (gathers waited for only when
    their slot comes round again; fewer frames than slots too), and with weighted row shares
    (vr_set_row_share: the first rank w0 blocks per w of every other rank)."""
    W, H = 40, 45
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, rb, inflight, nframes, q, share))
             for r in range(world)]
    for p in procs:
        p.start()
    frames, samples = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(frames) == nframes
    total = 0
    for k in range(nframes):
        full, st = _scene(W, H, k).render()
        assert np.array_equal(frames[k], full), k
        total += st["samples"]
    assert samples == total


def test_shard_layout_is_a_partition():
    for H, rb, n in ((1080, 16, 8), (53, 1, 5), (7, 16, 3), (2048, 16, 4)):
        seen = np.concatenate([vr_dist.shard_global_rows(H, rb, r, n) for r in range(n)])
        seen = seen[seen >= 0]
        assert np.array_equal(np.sort(seen), np.arange(H))
        g = np.stack([np.where(vr_dist.shard_global_rows(H, rb, r, n)[:, None] >= 0,
                               vr_dist.shard_global_rows(H, rb, r, n)[:, None], -1) for r in range(n)])
        assert np.array_equal(vr_dist.assemble_numpy(g, H, rb, n)[:, 0], np.arange(H))
