"""Host-output frame rate (vr_render into pageable host memory: the drop-in record() path,
PCIe inside the timed region), C3 by default.  python tools/host_output.py [--frames 100]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("volumetric-renderer_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, sub))

import numpy as np  # noqa: E402

import synth  # noqa: E402
import vr_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=100)
    ap.add_argument("--shading", type=int, default=1)
    ap.add_argument("--pinned", type=int, default=0, help="1: a page-locked host frame buffer")
    a = ap.parse_args()
    W, H = 1920, 1080
    rp = vr_amd.OffscreenPass(W, H)
    rp.generate_volume((512,) * 3, np.float32, seed=2024)
    rp.transfer_function_changed(synth.tf2())
    cam = synth.camera("fill").to_vr_camera()
    p = vr_amd.default_params(shading=a.shading, ert_eps=1e-5 if a.shading else 0.0)
    if a.pinned:
        import torch
        buf = torch.empty((H, W, 4), dtype=torch.uint8, pin_memory=True).numpy()
    else:
        buf = np.empty((H, W, 4), np.uint8)
    for _ in range(60):
        rp.render(cam, p, vr_amd.OUT_RGBA8, out=buf)
    t0 = time.perf_counter()
    for _ in range(a.frames):
        rp.render(cam, p, vr_amd.OUT_RGBA8, out=buf)
    dt = (time.perf_counter() - t0) / a.frames
    print(json.dumps(dict(lib=os.path.basename(os.path.dirname(os.environ.get("VR_AMD_LIB", "/lib/x"))),
                          pinned=a.pinned, shading=a.shading, ms=round(dt * 1e3, 4),
                          fps=round(1 / dt, 1))))


if __name__ == "__main__":
    main()
