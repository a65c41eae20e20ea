"""Kernel time of ONE rank's share of a frame for N = 1, 2, 4, 8 (GPU; exploration tool).
# NOTE (round 3): VR_PIPELINE / VR_PAIR only act on an experiment build (make EXTRA=-DVR_EXPERIMENTS,
# VR_AMD_LIB pointing at it); the product library reads no environment (include/vr/vr_debug.h).

Renders rank 0's row-block shard (vr_render_device with rank 0 of N) of the C3 frame on one
device and reports the HIP-event kernel time: the per-rank GPU cost under strong scaling,
without the gather.  Ideal: time(N) = time(1) / N.
  python tools/shard_sweep.py [--shading 1] [--ert 1e-5] [--row-block 8] [--reps 30]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("volumetric-renderer_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, sub))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import synth  # noqa: E402
import vr_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shading", type=int, default=1)
    ap.add_argument("--ert", type=float, default=1e-5)
    ap.add_argument("--row-block", type=int, default=8)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--wave-shape", type=int, default=0)
    ap.add_argument("--pipeline", default="", help="VR_PIPELINE override: '', 0 or 1")
    ap.add_argument("--pair", default="", help="VR_PAIR override: '', 0 or 1")
    a = ap.parse_args()
    if a.pipeline:
        os.environ["VR_PIPELINE"] = a.pipeline
    if a.pair:
        os.environ["VR_PAIR"] = a.pair
    W, H = 1920, 1080
    rp = vr_amd.OffscreenPass(W, H)
    rp.generate_volume((512, 512, 512), np.float32, seed=2024)
    rp.transfer_function_changed(synth.tf2())
    cam = synth.camera("fill").to_vr_camera()
    p = vr_amd.default_params(shading=a.shading, ert_eps=a.ert, wave_shape=a.wave_shape)
    stream = torch.cuda.current_stream().cuda_stream
    res = {}
    for n in (1, 2, 4, 8):
        sr = vr_amd.shard_rows(H, a.row_block, n)
        out = torch.empty((sr, W), dtype=torch.int32, device="cuda")
        for _ in range(3):
            rp.render_device(cam, p, out.data_ptr(), vr_amd.OUT_RGBA8, a.row_block, 0, n, stream)
        torch.cuda.synchronize()
        rp.timing_reset()
        rp.timing_enable(True)
        for _ in range(a.reps):
            rp.render_device(cam, p, out.data_ptr(), vr_amd.OUT_RGBA8, a.row_block, 0, n, stream)
        ms, k = rp.timing_read()
        rp.timing_enable(False)
        res[n] = round(ms / k, 4)
    base = res[1]
    print(json.dumps(dict(args=vars(a), rank0_kernel_ms=res,
                          speedup={n: round(base / t, 2) for n, t in res.items()})))


if __name__ == "__main__":
    main()
