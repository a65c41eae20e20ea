"""Serial frames (frames_in_flight 1) at the reference's default camera, C3 volume, shaded +
ERT: the launch policy's choice against lane groups (pair 1, 2 / 4 lanes) and other knobs.
ms per frame from device-synchronized loops (measurement script, round 5)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
for sub in ("", "volumetric-renderer_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, sub))
import bench  # noqa: E402
import synth  # noqa: E402
import vr_amd  # noqa: E402

cfg = bench.CONFIGS["c3_default"]
rp = bench.setup_pass(cfg, 0)
cam = synth.camera("default").to_vr_camera()
p = vr_amd.default_params(shading=1, ert_eps=1e-5, frames_in_flight=1)
W, H = cfg["W"], cfg["H"]
buf = torch.empty((H, W), dtype=torch.int32, device="cuda")
s = torch.cuda.Stream()
ref = None
out = []
variants = [dict(), dict(pair=1), dict(pair=1, pair_lanes=4), dict(pair=1, pair_lanes=2),
            dict(alt_geometry=0), dict(pipeline=0)]
for rnd in range(2):
    for kv in variants:
        with rp.knobs(**kv):
            for _ in range(60):
                rp.render_device(cam, p, buf.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1, s.cuda_stream)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 300
            for _ in range(n):
                rp.render_device(cam, p, buf.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1, s.cuda_stream)
                s.synchronize()  # serial: each frame complete before the next starts
            ms = (time.perf_counter() - t0) / n * 1e3
            img = buf.clone()
            if ref is None:
                ref = img
            same = bool(torch.equal(img, ref))
            name = rp.kernel_name(p)
        out.append(dict(round=rnd, knobs=kv, ms_per_frame=round(ms, 4), identical=same, kernel=name))
        print(json.dumps(out[-1]), flush=True)
rp.close()
