"""Minimal profiling workload: one configuration, K whole-frame launches through the C ABI.

Used under rocprofv3 (--kernel-trace --stats, or one --pmc group per run) so that every
counter pass replays a short process.  Prints the in-process HIP-event kernel time so the
profile's per-dispatch durations can be matched.  Frames go to a device buffer in one launch
each (vr_render_device): vr_render splits host-output frames into row bands.
  python tools/prof_run.py [--n 512] [--dtype float32] [--size 1920x1080] [--cam fill]
                           [--tf tf2] [--shading 1] [--ert 1e-5] [--frames 10] [--tile-order 0]
                           [--skip-empty 0] [--exact-gradient 0] [--knob name=value]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("volumetric-renderer_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, sub))

import numpy as np  # noqa: E402

import synth  # noqa: E402
import vr_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--cam", default="fill")
    ap.add_argument("--tf", default="tf2")
    ap.add_argument("--shading", type=int, default=1)
    ap.add_argument("--ert", type=float, default=1e-5)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--tile-order", type=int, default=0)
    ap.add_argument("--skip-empty", type=int, default=0)
    ap.add_argument("--wave-shape", type=int, default=0)
    ap.add_argument("--exact-gradient", type=int, default=0)
    ap.add_argument("--knob", action="append", default=[],
                    help="name=value: a vr_debug.h launch-policy knob, set before the upload "
                         "(e.g. u8_layout=1)")
    a = ap.parse_args()
    W, H = (int(x) for x in a.size.split("x"))
    rp = vr_amd.OffscreenPass(W, H)
    for kv in a.knob:
        k, v = kv.split("=")
        rp.set_knob(k, int(v))
    rp.generate_volume((a.n,) * 3, np.dtype(a.dtype), seed=2024)
    rp.transfer_function_changed(synth.TFS[a.tf]())
    cam = synth.camera(a.cam).to_vr_camera()
    p = vr_amd.default_params(shading=a.shading, ert_eps=a.ert, tile_order=a.tile_order,
                              skip_empty=a.skip_empty, wave_shape=a.wave_shape,
                              exact_gradient=a.exact_gradient)
    import torch
    frame = torch.empty((H, W), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    rp.render_device(cam, p, frame.data_ptr(), vr_amd.OUT_RGBA8, 16, 0, 1, s)
    torch.cuda.synchronize()
    rp.timing_enable(True)
    for _ in range(a.frames):
        rp.render_device(cam, p, frame.data_ptr(), vr_amd.OUT_RGBA8, 16, 0, 1, s)
    torch.cuda.synchronize()
    ms, n = rp.timing_read()
    st = rp.count_work(cam, p)
    print(json.dumps(dict(args=vars(a), kernel=rp.kernel_name(p), kernel_ms=ms / n, stats=st,
                          gsamples_s=st["samples"] / (ms / n * 1e-3) / 1e9)))


if __name__ == "__main__":
    main()
