"""Launch-policy check along the orbit path (bench.orbit_cameras), C3 volume and params: for
every `stride`-th camera, the serial frame time (best of 3, structures built) of the policy's
own choice and of each forced alternative -- the binary16 field on the 8^3 bricks, the stencil
gradient on the 8^3 bricks, the oblique copy, the stencil copy (vr_debug.h knobs
VR_KNOB_GRAD_FIELD / VR_KNOB_ALT_GEOMETRY) -- as JSON lines.  Speed only: every variant renders
the frame the oracle pins for its gradient mode.
    python tools/orbit_policy.py [--frames 360] [--stride 4] [--shading 0] [--inflight 3]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import torch  # noqa: E402
import vr_amd  # noqa: E402

VARIANTS = {"auto": dict(grad_field=-1, alt_geometry=-1),
            "field_8cube": dict(grad_field=1, alt_geometry=0),
            "stencil_8cube": dict(grad_field=0, alt_geometry=0),
            "oblique_copy": dict(grad_field=0, alt_geometry=1),
            "stencil_copy": dict(grad_field=0, alt_geometry=4),
            "pair_lanes": dict(pair=1)}  # 2-4 lanes per ray on the 8^3 bricks (serial frames)
# unshaded frames read no gradient: the 8^3 bricks, the oblique copy or the plain copy
VARIANTS_UNSHADED = {"auto": dict(alt_geometry=-1), "bricks_8cube": dict(alt_geometry=0),
                     "oblique_copy": dict(alt_geometry=1), "plain_copy": dict(alt_geometry=3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=360)
    ap.add_argument("--stride", type=int, default=4)
    ap.add_argument("--shading", type=int, default=1)
    ap.add_argument("--inflight", type=int, default=1,
                    help="> 1: frames on this many streams, wall-clock ms per frame (12 frames)")
    ap.add_argument("--path", default="orbit", choices=("orbit", "grid"),
                    help="grid: yaw {0, 45, 90} x pitch {0 .. 85} x radius {1.6 .. 3.2} degrees")
    a = ap.parse_args()
    cfg = bench.CONFIGS["c3"]
    rp = bench.setup_pass(cfg, 0)
    rp.set_memory_budget(2 ** 64 - 1)
    p = vr_amd.default_params(shading=a.shading, ert_eps=cfg["ert"], frames_in_flight=a.inflight)
    streams = [torch.cuda.Stream() for _ in range(max(a.inflight, 1))]
    bufs = [torch.empty((cfg["H"], cfg["W"]), dtype=torch.int32, device="cuda") for _ in streams]
    variants = VARIANTS if a.shading else VARIANTS_UNSHADED
    frame = torch.empty((cfg["H"], cfg["W"]), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    if a.path == "grid":  # Camera::rotate takes mouse deltas at 0.25 degree each
        grid = [(y, pt, r) for y in (0.0, 45.0, 90.0) for pt in (0.0, 10.0, 20.0, 30.0, 60.0, 75.0, 85.0)
                for r in (1.6, 2.0, 2.4, 2.8, 3.2)]
        cams = [vr_amd.make_camera(radius=r, rotate=(4.0 * y, 4.0 * pt)).to_vr_camera() for y, pt, r in grid]
        tags = [dict(yaw=y, pitch=pt, radius=r) for y, pt, r in grid]
        idx = range(len(cams))
    else:
        cams = bench.orbit_cameras(a.frames)
        tags = [{} for _ in cams]
        idx = range(0, a.frames, a.stride)
    for i in idx:
        c = cams[i]
        st = rp.count_work(c, p, 8)
        row = dict(i=i, samples=st["samples"], shaded=st["shaded_samples"], view=[round(x, 4) for x in c.view[:12]],
                   **tags[i])
        for name, knobs in variants.items():
            for k in ("grad_field", "alt_geometry", "pair"):
                rp.set_knob(k, knobs.get(k, vr_amd.KNOB_AUTO[k]))
            best = 1e9
            if a.inflight > 1:  # the wall-clock period of frames overlapping on the streams
                for rep in range(3):
                    n = 12 if rep else 2 * a.inflight
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for f in range(n):
                        rp.render_device(c, p, bufs[f % a.inflight].data_ptr(), vr_amd.OUT_RGBA8, 8,
                                         0, 1, streams[f % a.inflight].cuda_stream)
                    torch.cuda.synchronize()
                    if rep:
                        best = min(best, (time.perf_counter() - t0) / n * 1e3)
            else:
                for _ in range(4):
                    t0 = time.perf_counter()
                    rp.render_device(c, p, frame.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1, s)
                    torch.cuda.synchronize()
                    best = min(best, (time.perf_counter() - t0) * 1e3)
            k = rp.kernel_name(p)
            row[name] = round(best, 4)
            row[name + "_kernel"] = k.split("march_kernel<")[-1].split(",")[0] if "march_kernel<" in k else k
        print(json.dumps(row), flush=True)
    rp.close()


if __name__ == "__main__":
    main()
