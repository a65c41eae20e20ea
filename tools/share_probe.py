"""Render-only time of one rank's share of a frame on one GPU (measurement tool, not product).

At N GPUs each rank renders the 8-row blocks b = rank (mod N) of the frame, then gathers.  This
renders rank r's share alone on device 0 (vr_render_device with nranks = N, no gather), with
F frames in flight on F streams, and prints ms per frame: the per-device render time an N-GPU
frame cannot beat, so the strong-scaling ceiling of the render part is t(1) / t(N).

    python tools/share_probe.py [--config c3] [--frames 200] [--out file.json]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "volumetric-renderer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402  (configs and the pass setup)
import synth  # noqa: E402
import vr_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=60)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--inflight", default="1,3,6")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    W, H, rb = cfg["W"], cfg["H"], 8
    rp = bench.setup_pass(cfg, 0)
    cam = synth.camera(cfg["cam"]).to_vr_camera()
    rows = []
    for world in [int(x) for x in a.worlds.split(",")]:
        for ranks in sorted({0, world // 2, world - 1}):
            for fif in [int(x) for x in a.inflight.split(",")]:
                p = vr_amd.default_params(shading=cfg["shading"], ert_eps=cfg["ert"],
                                          frames_in_flight=fif)
                sr = vr_amd.shard_rows(H, rb, world)
                bufs = [torch.empty((sr, W), dtype=torch.int32, device="cuda") for _ in range(fif)]
                streams = [torch.cuda.Stream() for _ in range(fif)]

                def frame(i):
                    rp.render_device(cam, p, bufs[i % fif].data_ptr(), vr_amd.OUT_RGBA8, rb,
                                     ranks, world, streams[i % fif].cuda_stream)

                for i in range(a.warmup):
                    frame(i)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(a.frames):
                    frame(i)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / a.frames * 1e3
                work = rp.count_work(cam, p, rb, ranks, world)
                rows.append(dict(world=world, rank=ranks, frames_in_flight=fif,
                                 ms_per_frame=round(ms, 4), samples=work["samples"],
                                 gsamples_per_s=round(work["samples"] / ms * 1e-6, 1)))
                print(json.dumps(rows[-1]), flush=True)
    if a.out:
        json.dump(dict(config=a.config, rows=rows), open(a.out, "w"), indent=1)
    rp.close()


if __name__ == "__main__":
    main()
