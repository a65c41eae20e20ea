"""Per-frame record of the orbit path (bench.orbit_cameras) on the C3 volume: for every camera,
the kernel the launch policy picks (vr_kernel_name), the executed samples, and the serial frame
time (best of 3 after the structures are built), as JSON lines.  Where the orbit's slow frames
come from.
    python tools/orbit_frames.py [--frames 360] [--stride 1]"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=360)
    ap.add_argument("--stride", type=int, default=1)
    a = ap.parse_args()
    cfg = bench.CONFIGS["c3"]
    rp = bench.setup_pass(cfg, 0)
    rp.set_memory_budget(2 ** 64 - 1)
    p = vr_amd.default_params(shading=cfg["shading"], ert_eps=cfg["ert"])
    frame = torch.empty((cfg["H"], cfg["W"]), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    cams = bench.orbit_cameras(a.frames)
    for i in range(0, a.frames, a.stride):
        c = cams[i]
        best = 1e9
        for _ in range(4):
            t0 = time.perf_counter()
            rp.render_device(c, p, frame.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1, s)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) * 1e3)
        st = rp.count_work(c, p, 8)
        k = rp.kernel_name(p)
        print(json.dumps(dict(i=i, ms=round(best, 4), samples=st["samples"], shaded=st["shaded_samples"],
                              ps_per_sample=round(best * 1e9 / max(st["samples"], 1), 3),
                              kernel=k.split("march_kernel<")[-1].split(">")[0] if "march_kernel<" in k else k,
                              view=[round(x, 3) for x in c.view[:12]])), flush=True)
    rp.close()


if __name__ == "__main__":
    main()
