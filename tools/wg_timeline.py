"""Workgroup timeline of one march launch (GPU; experiment build with -DVR_WG_TIMES).

  make -C volumetric-renderer_amd LIBDIR=lib_wgt BUILDDIR=build_wgt EXTRA=-DVR_WG_TIMES
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_wgt/libvr_amd.so python tools/wg_timeline.py

Records every workgroup's (start, end) wall clock (100 MHz) for one C3 frame (full frame and
rank 0's share at N = 8) and reports the launch span, workgroup durations, and how the
number of resident workgroups decays at the end (the tail a few long rays leave).
"""
import ctypes as C
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


def timeline(lib, rp, cam, p, nranks, W, H, rb=8):
    sr = vr_amd.shard_rows(H, rb, nranks)
    out = torch.empty((sr, W), dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        rp.render_device(cam, p, out.data_ptr(), vr_amd.OUT_RGBA8, rb, 0, nranks, stream)
    torch.cuda.synchronize()
    lib.vr_debug_wg_times(None, 0, None, 1)
    rp.render_device(cam, p, out.data_ptr(), vr_amd.OUT_RGBA8, rb, 0, nranks, stream)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * (4 * 131072))()
    n = C.c_uint(0)
    lib.vr_debug_wg_times(buf, 131072, C.byref(n), 0)
    # 4 words per workgroup: start, end, tile id, XCC_ID << 32 | HW_ID
    t = np.frombuffer(buf, dtype=np.uint64, count=4 * n.value).reshape(-1, 4)[:, :2].astype(np.int64)
    t0 = t[:, 0].min()
    s, e = (t[:, 0] - t0) * 0.01, (t[:, 1] - t0) * 0.01  # us
    span = e.max()
    dur = e - s
    grid = np.linspace(0, span, 200)
    active = np.array([(np.sum((s <= g) & (e > g))) for g in grid])
    peak = active.max()
    # time from which fewer than half the peak workgroups are resident
    half_from = grid[np.argmax((active < peak / 2) & (grid > grid[np.argmax(active)]))]
    return dict(nranks=nranks, workgroups=int(n.value), span_us=round(float(span), 1),
                wg_dur_us=dict(mean=round(float(dur.mean()), 1), p50=round(float(np.median(dur)), 1),
                               p99=round(float(np.percentile(dur, 99)), 1), max=round(float(dur.max()), 1)),
                peak_resident=int(peak), below_half_peak_from_us=round(float(half_from), 1),
                tail_fraction=round(float(1 - half_from / span), 3),
                busy_fraction=round(float(active.mean() / peak), 3))


def main():
    lib = vr_amd.lib()
    fn = lib.vr_debug_wg_times
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_uint, C.POINTER(C.c_uint), C.c_int]
    W, H = 1920, 1080
    rp = vr_amd.OffscreenPass(W, H)
    rp.generate_volume((512, 512, 512), np.float32, seed=2024)
    rp.transfer_function_changed(synth.tf2())
    cam = synth.camera("fill").to_vr_camera()
    res = []
    for shading, ert in ((1, 1e-5), (0, 0.0)):
        p = vr_amd.default_params(shading=shading, ert_eps=ert)
        for n in (1, 8):
            r = timeline(lib, rp, cam, p, n, W, H)
            r["shading"] = shading
            res.append(r)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
