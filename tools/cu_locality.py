"""Which tiles share a CU while they run (GPU; experiment build with -DVR_WG_TIMES).

  make -C volumetric-renderer_amd LIBDIR=lib_wgt BUILDDIR=build_wgt EXTRA=-DVR_WG_TIMES
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_wgt/libvr_amd.so python tools/cu_locality.py

One C3 frame (fill view, Phong + ERT, 3 frames in flight before it) with every workgroup's
start/end wall clock, tile and hardware id (XCC_ID, HW_ID: SE / SH / CU).  For each workgroup,
the workgroups resident on the same CU at its midpoint and their distance in tiles (Chebyshev):
the L1 a 16x16-pixel tile's four wavefronts share is shared with those tiles too, so tiles
close together on one CU would reuse each other's brick lines.
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


def main():
    lib = vr_amd.lib()
    fn = lib.vr_debug_wg_times
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_uint, C.POINTER(C.c_uint), C.c_int]
    W, H = 1920, 1080
    rp = vr_amd.OffscreenPass(W, H)
    rp.generate_volume((512, 512, 512), np.float32, seed=2024)
    rp.transfer_function_changed(synth.tf2())
    cam = synth.camera(sys.argv[1] if len(sys.argv) > 1 else "fill").to_vr_camera()
    p = vr_amd.default_params(shading=1, ert_eps=1e-5, frames_in_flight=1)
    out = torch.empty((H, W), dtype=torch.int32, device="cuda")
    for _ in range(8):
        rp.render_device(cam, p, out.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1)
    torch.cuda.synchronize()
    fn(None, 0, None, 1)
    rp.render_device(cam, p, out.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * (4 * 131072))()
    n = C.c_uint(0)
    fn(buf, 131072, C.byref(n), 0)
    a = np.frombuffer(buf, dtype=np.uint64, count=4 * n.value).reshape(-1, 4)
    s, e = a[:, 0].astype(np.int64), a[:, 1].astype(np.int64)
    tile = (a[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    wg = (a[:, 2] >> np.uint64(32)).astype(np.int64)
    xcc = (a[:, 3] >> np.uint64(32)).astype(np.int64)
    hw = (a[:, 3] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    cu_key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    tiles_x = (W + 15) // 16
    tx, ty = tile % tiles_x, tile // tiles_x
    mid = (s + e) // 2
    dists, counts = [], []
    for i in range(len(tile)):
        m = (cu_key == cu_key[i]) & (s <= mid[i]) & (e > mid[i])
        m[i] = False
        counts.append(int(m.sum()))
        if m.any():
            d = np.maximum(np.abs(tx[m] - tx[i]), np.abs(ty[m] - ty[i]))
            dists.append(float(np.median(d)))
    ncu = len(np.unique(cu_key))
    # the dispatch order on one CU: tiles of consecutive workgroups there
    order_d = []
    for k in np.unique(cu_key)[:64]:
        idx = np.where(cu_key == k)[0]
        idx = idx[np.argsort(s[idx])]
        if len(idx) > 1:
            order_d.extend(np.maximum(np.abs(np.diff(tx[idx])), np.abs(np.diff(ty[idx]))).tolist())
    res = dict(workgroups=int(n.value), cus=int(ncu), per_cu_mean=round(len(tile) / max(ncu, 1), 1),
               coresident_mean=round(float(np.mean(counts)), 2),
               coresident_tile_distance=dict(p10=float(np.percentile(dists, 10)),
                                             median=float(np.median(dists)),
                                             p90=float(np.percentile(dists, 90))),
               consecutive_on_cu_tile_distance=dict(median=float(np.median(order_d)),
                                                    p90=float(np.percentile(order_d, 90))),
               xcc_values=sorted(set(xcc.tolist()))[:8], se_values=sorted(set(se.tolist())),
               cu_ids=sorted(set(cu.tolist())))
    # the dispatcher: per XCD, the CU each workgroup id went to, in id order (first 4 XCDs'
    # first 80 workgroups), and whether workgroups of one XCD visit its CUs round-robin
    disp = {}
    for x in range(8):
        idx = np.where(xcc == x)[0]
        idx = idx[np.argsort(wg[idx])]
        disp[x] = dict(wg_mod8=sorted(set((wg[idx] % 8).tolist())),
                       first_cus=[int(k) % 1024 for k in cu_key[idx][:80]])
    res["dispatch"] = {k: disp[k] for k in (0, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
