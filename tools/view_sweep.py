"""Throughput of the ray-march kernel across view directions (GPU; exploration tool).

Renders one frame per camera K times through vr_render_device and prints the kernel time
(HIP events) and Gsamples/s per view, for the C3 volume by default.  Used to check the
layout model of tools/line_sim.py on hardware (view dependence of the gather cost).
"""
from __future__ import annotations

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

VIEWS = {
    "fill": dict(radius=1.6, rotate=None),
    "fill_oblique": dict(radius=1.6, rotate=(40.0, 25.0)),
    "side_x": dict(radius=1.6, rotate=(360.0, 0.0)),
    "top_z": dict(radius=1.6, rotate=(0.0, 360.0)),
    "diag": dict(radius=2.0, rotate=(180.0, 140.0)),
    "diag2": dict(radius=1.8, rotate=(120.0, 60.0)),
    "default": dict(radius=3.0, rotate=None),
    "far_oblique": dict(radius=3.2, rotate=(180.0, 80.0)),  # yaw 45, pitch 20 (round 6 grid)
    "far_side": dict(radius=2.4, rotate=(360.0, 80.0)),  # yaw 90, pitch 20: ray along x
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--tf", default="tf2")
    ap.add_argument("--shading", type=int, default=0)
    ap.add_argument("--ert", type=float, default=0.0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tile-order", type=int, default=0)
    ap.add_argument("--skip-empty", type=int, default=0)
    ap.add_argument("--wave-shape", type=int, default=0)
    ap.add_argument("--knob", action="append", default=[],
                    help="name=value: a vr_debug.h launch-policy knob (e.g. pipeline=1)")
    ap.add_argument("--inflight", type=int, default=1,
                    help="> 1: frames on this many streams, ms per frame from the wall clock")
    ap.add_argument("--views", default=",".join(VIEWS))
    args = ap.parse_args()
    W, H = (int(x) for x in args.size.split("x"))
    rp = vr_amd.OffscreenPass(W, H)
    for kv in args.knob:  # before the upload: layout knobs (u8_layout) apply to it
        k, v = kv.split("=")
        rp.set_knob(k, int(v))
    rp.generate_volume((args.n,) * 3, np.dtype(args.dtype), seed=2024)
    rp.transfer_function_changed(synth.TFS[args.tf]())
    out = torch.empty((H + 16, W), dtype=torch.int32, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(args.inflight)]
    outs = [torch.empty((H + 16, W), dtype=torch.int32, device="cuda") for _ in streams]
    stream = torch.cuda.current_stream().cuda_stream
    p = vr_amd.default_params(shading=args.shading, ert_eps=args.ert, tile_order=args.tile_order,
                              skip_empty=args.skip_empty, wave_shape=args.wave_shape,
                              frames_in_flight=args.inflight)
    res = {}
    for name in args.views.split(","):
        v = VIEWS[name]
        cam = vr_amd.make_camera(**v).to_vr_camera()
        st = rp.count_work(cam, p)
        for _ in range(3):
            rp.render_device(cam, p, out.data_ptr(), vr_amd.OUT_RGBA8, 16, 0, 1, stream)
        torch.cuda.synchronize()
        rp.timing_reset()
        rp.timing_enable(True)
        for _ in range(args.reps):
            rp.render_device(cam, p, out.data_ptr(), vr_amd.OUT_RGBA8, 16, 0, 1, stream)
        ms, n = rp.timing_read()
        rp.timing_enable(False)
        kms = ms / n
        if args.inflight > 1:  # wall-clock period of frames overlapping on the streams
            import time
            for i in range(3 * args.inflight):
                rp.render_device(cam, p, outs[i % len(outs)].data_ptr(), vr_amd.OUT_RGBA8, 16, 0, 1,
                                 streams[i % len(streams)].cuda_stream)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.reps):
                rp.render_device(cam, p, outs[i % len(outs)].data_ptr(), vr_amd.OUT_RGBA8, 16, 0, 1,
                                 streams[i % len(streams)].cuda_stream)
            torch.cuda.synchronize()
            kms = (time.perf_counter() - t0) / args.reps * 1e3
        res[name] = dict(kernel_ms=round(kms, 4), samples=st["samples"],
                         gsamples_s=round(st["samples"] / (kms * 1e-3) / 1e9, 2),
                         shaded=st["shaded_samples"], skipped=st["skipped_samples"],
                         fps=round(1e3 / kms, 1))
        print(name, json.dumps(res[name]), flush=True)
    print(json.dumps(dict(args=vars(args), views=res)))


if __name__ == "__main__":
    main()
