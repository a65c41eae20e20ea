"""Where the sparse (far) views lose time, C3 volume and params: for a few views of the round-6
grid, the serial frame (best of 4, host-timed to the device's end), the same with lane groups
forced on and off (VR_KNOB_PAIR 1 / 0: 2-4 lanes per ray or one), and the wall-clock period
with 3 frames in flight (single lane, the policy, and lane groups forced),
plus the rays that hit the volume and the samples per such ray.  JSON lines.
    python tools/far_views.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import torch  # noqa: E402
import vr_amd  # noqa: E402

VIEWS = {"fill": (1.6, 0.0, 0.0), "default": (3.0, 0.0, 0.0), "far_oblique": (3.2, 45.0, 20.0),
         "far_side": (2.4, 90.0, 20.0), "mid_oblique": (2.4, 45.0, 30.0)}


def main():
    cfg = bench.CONFIGS["c3"]
    rp = bench.setup_pass(cfg, 0)
    rp.set_memory_budget(2 ** 64 - 1)
    H, W = cfg["H"], cfg["W"]
    frames = [torch.empty((H, W), dtype=torch.int32, device="cuda") for _ in range(3)]
    streams = [torch.cuda.Stream() for _ in range(3)]
    s0 = torch.cuda.current_stream().cuda_stream
    for name, (r, yaw, pitch) in VIEWS.items():
        cam = vr_amd.make_camera(radius=r, rotate=(4.0 * yaw, 4.0 * pitch)).to_vr_camera()
        p1 = vr_amd.default_params(shading=cfg["shading"], ert_eps=cfg["ert"])
        p3 = vr_amd.default_params(shading=cfg["shading"], ert_eps=cfg["ert"], frames_in_flight=3)
        st = rp.count_work(cam, p1, 8)
        row = dict(view=name, radius=r, yaw=yaw, pitch=pitch, samples=st["samples"],
                   rays=st.get("rays"), steps=st.get("steps"))

        def serial(params):
            best = 1e9
            for _ in range(5):
                t0 = time.perf_counter()
                rp.render_device(cam, params, frames[0].data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1, s0)
                torch.cuda.synchronize()
                best = min(best, (time.perf_counter() - t0) * 1e3)
            return round(best, 4)

        row["serial_ms"] = serial(p1)
        with rp.knobs(pair=1):
            row["serial_pair_ms"] = serial(p1)
        with rp.knobs(pair=1, pair_lanes=4):
            row["serial_pair4_ms"] = serial(p1)
        with rp.knobs(pair=0):
            row["serial_single_lane_ms"] = serial(p1)

        def inflight():
            for i in range(6):
                rp.render_device(cam, p3, frames[i % 3].data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1,
                                 streams[i % 3].cuda_stream)
            torch.cuda.synchronize()
            n = 30
            t0 = time.perf_counter()
            for i in range(n):
                rp.render_device(cam, p3, frames[i % 3].data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1,
                                 streams[i % 3].cuda_stream)
            torch.cuda.synchronize()
            return round((time.perf_counter() - t0) / n * 1e3, 4)

        row["inflight3_ms"] = inflight()
        with rp.knobs(pair=1):
            row["inflight3_pair_ms"] = inflight()
        print(json.dumps(row), flush=True)
    rp.close()


if __name__ == "__main__":
    main()
