"""Host cost of one vr_render_device call (enqueue only): a tiny frame whose GPU work is
negligible, K calls back to back on one stream, wall time per call; and the same for the
C3 volume at 1080p rank shares (row_block 8, rank 0 of N) with 3 streams.
  python tools/host_enqueue.py [--calls 2000]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("volumetric-renderer_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, sub))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import synth  # noqa: E402
import vr_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    a = ap.parse_args()
    out = {}
    for (W, H, n, shading) in ((64, 64, 64, 0), (64, 64, 64, 1), (1920, 1080, 512, 1)):
        rp = vr_amd.OffscreenPass(W, H)
        rp.generate_volume((n,) * 3, np.float32, seed=2024)
        rp.transfer_function_changed(synth.tf2())
        cam = synth.camera("fill").to_vr_camera()
        p = vr_amd.default_params(shading=shading, ert_eps=1e-5 if shading else 0.0,
                                  frames_in_flight=3)
        nr = 8 if W > 64 else 1
        sr = vr_amd.shard_rows(H, 8, nr)
        streams = [torch.cuda.Stream() for _ in range(3)]
        bufs = [torch.empty((sr, W), dtype=torch.int32, device="cuda") for _ in streams]
        for i in range(30):
            rp.render_device(cam, p, bufs[i % 3].data_ptr(), vr_amd.OUT_RGBA8, 8, 0, nr,
                             streams[i % 3].cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.calls):
            rp.render_device(cam, p, bufs[i % 3].data_ptr(), vr_amd.OUT_RGBA8, 8, 0, nr,
                             streams[i % 3].cuda_stream)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[f"{W}x{H} n={n} shading={shading} ranks={nr}"] = dict(
            enqueue_us=round((t1 - t0) / a.calls * 1e6, 2), wall_us=round((t2 - t0) / a.calls * 1e6, 2))
        rp.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
