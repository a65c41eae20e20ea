"""A/B of tile orders (default: 4, adaptive, against 6, CU strips; ORDERS=4,6,3 to change)
on the C3 volume (512^3 f32, 1080p, TF-2), per view, shaded (Phong + ERT 1e-5) and unshaded,
serial frames and 3 in flight; two alternating rounds.  Prints one JSON line per measurement.
Usage: ORDERS=4,6 python tools/experiments/r05/order_ab.py [rounds] [views]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
for sub in ("volumetric-renderer_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, sub))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import synth  # noqa: E402
import vr_amd  # noqa: E402


def frames(rp, cam, p, n, inflight, W, H, outs, streams):
    t0 = time.perf_counter()
    for i in range(n):
        k = i % inflight
        rp.render_device(cam, p, outs[k].data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1, streams[k].cuda_stream)
        if inflight == 1:
            streams[0].synchronize()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


ORDERS = tuple(int(x) for x in os.environ.get("ORDERS", "4,6").split(","))


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    views = sys.argv[2].split(",") if len(sys.argv) > 2 else ["default", "fill", "diag"]
    W, H = 1920, 1080
    rp = vr_amd.OffscreenPass(W, H)
    rp.generate_volume((512, 512, 512), np.float32, seed=2024)
    rp.transfer_function_changed(synth.tf2())
    outs = [torch.empty((H, W), dtype=torch.int32, device="cuda") for _ in range(3)]
    streams = [torch.cuda.Stream() for _ in range(3)]
    for view in views:
        cam = synth.camera(view).to_vr_camera()
        for shading in (1, 0):
            for inflight in (1, 3):
                for rnd in range(rounds):
                    for order in ORDERS:
                        p = vr_amd.default_params(shading=shading, ert_eps=1e-5 if shading else 0.0,
                                                  frames_in_flight=inflight, tile_order=order)
                        frames(rp, cam, p, 60, inflight, W, H, outs, streams)  # warm + sort
                        ms = frames(rp, cam, p, 100 if inflight > 1 else 60, inflight, W, H, outs, streams)
                        print(json.dumps(dict(view=view, shading=shading, inflight=inflight, round=rnd,
                                              order=order, ms=round(ms, 4), kernel=rp.kernel_name(p))),
                              flush=True)
    rp.close()


if __name__ == "__main__":
    main()
