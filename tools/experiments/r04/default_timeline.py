"""Where does a serial frame of the reference's default camera spend its time?  (round 4)

Experiment build (per-workgroup start/end, tile id, XCC id):
  make -C volumetric-renderer_amd LIBDIR=lib_wgt BUILDDIR=build_wgt EXTRA=-DVR_WG_TIMES
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_wgt/libvr_amd.so \
      python tools/experiments/r04/default_timeline.py OUT_DIR

C3 volume (512^3 f32), 1080p, TF-2, Phong + ERT; cameras: default (r = 3) and fill (r = 1.6).
Serial launches (one frame at a time).  Writes OUT_DIR/timeline_<cam>.npz (start/end us, tile,
xcc, hw_id) and prints a JSON summary per camera: span, workgroups, empty-tile cost, per-XCD last
end, and the end time of the longest tiles.
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
for sub in ("volumetric-renderer_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, sub))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import synth  # noqa: E402
import vr_amd  # noqa: E402


def grab(lib, rp, cam, p, W, H):
    out = torch.empty((H, W), dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(12):  # the adaptive order settles (re-ordered every 4 launches)
        rp.render_device(cam, p, out.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1, st)
    torch.cuda.synchronize()
    lib.vr_debug_wg_times(None, 0, None, 1)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    rp.render_device(cam, p, out.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1, st)
    ev1.record()
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * (4 * 131072))()
    n = C.c_uint(0)
    lib.vr_debug_wg_times(buf, 131072, C.byref(n), 0)
    t = np.frombuffer(buf, dtype=np.uint64, count=4 * n.value).reshape(-1, 4).copy()
    return t, ev0.elapsed_time(ev1)


def summary(t, ms, tiles_x):
    t0 = t[:, 0].astype(np.int64).min()
    s = (t[:, 0].astype(np.int64) - t0) * 0.01
    e = (t[:, 1].astype(np.int64) - t0) * 0.01
    tile = t[:, 2].astype(np.int64)
    xcc = (t[:, 3] >> np.uint64(32)).astype(np.int64)
    dur = e - s
    span = float(e.max())
    empty = dur < np.percentile(dur, 20) * 1.5
    order = np.argsort(-dur)
    top = order[: max(1, len(order) // 100)]
    per_xcd = {int(x): dict(wgs=int((xcc == x).sum()), last_end_us=round(float(e[xcc == x].max()), 1),
                            busy_us=round(float(dur[xcc == x].sum()), 1))
               for x in np.unique(xcc)}
    grid = np.linspace(0, span, 400)
    active = np.array([np.sum((s <= g) & (e > g)) for g in grid])
    return dict(event_ms=round(ms, 4), span_us=round(span, 1), workgroups=int(len(t)),
                dur_us=dict(p10=round(float(np.percentile(dur, 10)), 2), p50=round(float(np.median(dur)), 2),
                            p90=round(float(np.percentile(dur, 90)), 2), max=round(float(dur.max()), 1)),
                short_wgs=int(empty.sum()), short_wg_dur_us=round(float(dur[empty].mean()), 2),
                short_wgs_end_after_us=round(float(np.percentile(e[empty], 50)), 1),
                longest_1pct=dict(start_us=dict(max=round(float(s[top].max()), 1), mean=round(float(s[top].mean()), 1)),
                                  dur_us_mean=round(float(dur[top].mean()), 1),
                                  end_us_max=round(float(e[top].max()), 1),
                                  tiles_y=sorted(set(int(v) for v in (tile[top] // tiles_x)))[:20]),
                per_xcd=per_xcd,
                resident=dict(peak=int(active.max()), at_50pct_span=int(active[200]),
                              at_80pct=int(active[320]), at_90pct=int(active[360])))


def main():
    outd = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/timeline"
    os.makedirs(outd, exist_ok=True)
    lib = vr_amd.lib()
    fn = lib.vr_debug_wg_times
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_uint, C.POINTER(C.c_uint), C.c_int]
    W, H = 1920, 1080
    rp = vr_amd.OffscreenPass(W, H)
    rp.generate_volume((512, 512, 512), np.float32, seed=2024)
    rp.transfer_function_changed(synth.tf2())
    res = {}
    for camname in ("default", "fill"):
        cam = synth.camera(camname).to_vr_camera()
        for shading, ert in ((1, 1e-5), (0, 0.0)):
            p = vr_amd.default_params(shading=shading, ert_eps=ert)
            t, ms = grab(lib, rp, cam, p, W, H)
            key = f"{camname}_{'shaded' if shading else 'unshaded'}"
            np.savez_compressed(os.path.join(outd, f"timeline_{key}.npz"), t=t)
            res[key] = summary(t, ms, (W + 15) // 16)
            res[key]["kernel"] = rp.kernel_name(p)
            print(json.dumps({key: res[key]}), flush=True)
    with open(os.path.join(outd, "summary.json"), "w") as f:
        json.dump(res, f, indent=1)
    rp.close()


if __name__ == "__main__":
    main()
