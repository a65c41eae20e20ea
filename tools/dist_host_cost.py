"""Host cost of one multi-GPU frame's enqueue (measurement tool, not product).

At N = 8 a rank's share of a C3 frame renders in ~0.06 ms (tools/share_probe.py), so the
host thread that enqueues render -> ncclGather -> assemble must keep up with that.  This
times the library's frame path (vr_dist_render, one rank, RCCL communicator of one) on a frame
small enough that the device never holds the host back, against bare vr_render_device
enqueues of the same frame: the difference is what the frame schedule and the gather cost the
host per frame.

    python tools/dist_host_cost.py [--frames 3000] [--out file.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("", "volumetric-renderer_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, sub))

import synth  # noqa: E402
import vr_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=3000)
    ap.add_argument("--size", default="128x72")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    W, H = (int(v) for v in a.size.split("x"))
    rp = vr_amd.OffscreenPass(W, H, device=0)
    rp.generate_volume((256, 256, 256), seed=2024)
    # the reference's startup TF (one opaque white texel): every ray ends at its first sample,
    # so the kernels take microseconds and the host's enqueue cost is what is timed
    rp.transfer_function_changed(np.array([0xFFFFFFFF], dtype=np.uint32))
    cam = synth.camera("fill").to_vr_camera()
    rows = {}
    for fif in (1, 3):
        p = vr_amd.default_params(shading=1, ert_eps=1e-5, frames_in_flight=fif)
        # bare renders: one stream per frame in flight
        sr = vr_amd.shard_rows(H, 8, 1)
        bufs = [torch.empty((sr, W), dtype=torch.int32, device="cuda") for _ in range(fif)]
        streams = [torch.cuda.Stream() for _ in range(fif)]
        for i in range(200):
            rp.render_device(cam, p, bufs[i % fif].data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1,
                             streams[i % fif].cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.frames):
            rp.render_device(cam, p, bufs[i % fif].data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1,
                             streams[i % fif].cuda_stream)
        torch.cuda.synchronize()
        bare = (time.perf_counter() - t0) / a.frames * 1e6
        # the library's frame path: render -> ncclGather -> assemble, frames in flight
        d = vr_amd.DistFrames(rp, vr_amd.dist_unique_id(), 1, 0, 8, fif)
        frame = torch.empty((H, W), dtype=torch.int32, device="cuda")
        for _ in range(200):
            d.render(cam, p, frame.data_ptr())
        d.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.frames):
            d.render(cam, p, frame.data_ptr())
        d.synchronize()
        torch.cuda.synchronize()
        dist = (time.perf_counter() - t0) / a.frames * 1e6
        d.close()
        rows[f"frames_in_flight_{fif}"] = dict(bare_render_us=round(bare, 2),
                                               dist_frame_us=round(dist, 2))
        print(json.dumps({fif: rows[f"frames_in_flight_{fif}"]}), flush=True)
    out = dict(viewport=f"{W}x{H}", volume="256^3 f32", tf="one opaque texel (rays end at their first sample)",
               shading=1, frames=a.frames, rows=rows)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)
    rp.close()


if __name__ == "__main__":
    main()
