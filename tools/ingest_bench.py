"""NRRD ingest -> device, measured on the GPU box.

For the BASELINE volumes C2 (256^3 u8), C3 (512^3 f32) and C4 (1024^3 u8), written as raw
detached NRRDs to $TMPDIR (so the files sit in the page cache: parse rates are from memory):

  nrrd_parse      vr_nrrd_load: this repo's reader, the file's native element type
  upload+brick    vr_set_volume: host -> device copy + on-device bricking (synchronous, as
                  volume_dataset_changed)
  brick (device)  vr_set_volume_device from a device-resident linear volume: the bricking
                  kernel alone, against the HBM roofline (bytes = linear read + bricked write)
  reference parse NrrdFileParser::parse through the reference's own NrrdIO (oracle/_ref,
                  built from its sources): parse + float conversion + min/max on the host,
                  the CPU side of the reference's ingest (its Vulkan staging upload of the
                  float volume cannot run here)

  python tools/ingest_bench.py [--configs c2,c3,c4] [--reps 3]
"""
import argparse
import ctypes as C
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("volumetric-renderer_amd", "tools", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, sub))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import synth  # noqa: E402
import vr_amd  # noqa: E402

HBM_PEAK_GBS = 8000.0


def volume(name):
    if name == "c2":
        return synth.ct_head(256, 1234)
    if name == "c3":
        return synth.gaussians_numpy((512, 512, 512), seed=2024)
    n = 1024  # c4: u8 pattern (content does not change ingest cost)
    z = np.arange(n, dtype=np.uint32)
    return ((z[:, None, None] * 7 + z[None, :, None] * 13 + z[None, None, :] * 3) % 251).astype(np.uint8)


def best(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c3,c4")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    L = vr_amd.lib()
    import pyoracle
    ref_ok = pyoracle.nrrdio_available()
    tmp = tempfile.mkdtemp(prefix="vr_ingest_")
    gpu = torch.cuda.is_available()
    rp = vr_amd.OffscreenPass(64, 64, device=0) if gpu else None
    out = {}
    for name in a.configs.split(","):
        vol = volume(name)
        nz, ny, nx = vol.shape
        path = os.path.join(tmp, f"{name}.nhdr")
        vr_amd.write_nrrd_raw(path, vol)
        src_bytes = vol.nbytes
        vmin, vmax = float(vol.min()), float(vol.max())
        dt = vr_amd.NP_TO_DTYPE[vol.dtype]
        r = dict(dims=[nx, ny, nz], dtype=vol.dtype.name, file_bytes=src_bytes)

        def parse():
            ds = vr_amd.vr_dataset()
            if L.vr_nrrd_load(path.encode(), C.byref(ds)) != 0:
                raise RuntimeError(L.vr_host_last_error().decode())
            L.vr_dataset_free(C.byref(ds))
        t = best(parse, a.reps)
        r["nrrd_parse_s"] = round(t, 4)
        r["nrrd_parse_gbs"] = round(src_bytes / t / 1e9, 2)

        if gpu:
            data = np.ascontiguousarray(vol)

            def upload():
                rc = L.vr_set_volume(rp._ctx, data.ctypes.data, dt, nx, ny, nz, vmin, vmax)
                if rc != 0:
                    raise RuntimeError(L.vr_last_error(rp._ctx).decode())
            t = best(upload, a.reps)
            r["upload_brick_s"] = round(t, 4)
            r["upload_brick_gbs"] = round(src_bytes / t / 1e9, 2)
            brick_bytes = rp.volume_bytes()
            r["bricked_bytes"] = brick_bytes

            dev = torch.from_numpy(data).to("cuda")
            torch.cuda.synchronize()

            def brick():
                rp.volume_dataset_changed_device(dev.data_ptr(), data.dtype, (nx, ny, nz), vmin, vmax)
                torch.cuda.synchronize()
            t = best(brick, a.reps)
            r["brick_device_s"] = round(t, 5)
            r["brick_device_hbm_gbs"] = round((src_bytes + brick_bytes) / t / 1e9, 1)
            r["brick_device_hbm_frac"] = round((src_bytes + brick_bytes) / t / 1e9 / HBM_PEAK_GBS, 3)
            del dev
            if vol.dtype == np.float32:
                # the first shaded frame after a volume change builds the f32 difference field
                # (3 x the bricked density, written once): first minus second frame time
                cam = vr_amd.make_camera(radius=2.0).to_vr_camera()
                p = vr_amd.default_params(shading=1)
                fr = torch.empty((64, 64), dtype=torch.int32, device="cuda")

                def frame():
                    t0 = time.perf_counter()
                    rp.render_device(cam, p, fr.data_ptr(), vr_amd.OUT_RGBA8, 16, 0, 1, 0)
                    torch.cuda.synchronize()
                    return time.perf_counter() - t0
                t1, t2 = frame(), frame()
                field_bytes = brick_bytes * 3
                r["grad_field_build_s"] = round(t1 - t2, 5)
                r["grad_field_hbm_gbs"] = round((brick_bytes + field_bytes) / (t1 - t2) / 1e9, 1)

        if ref_ok:
            pyoracle.nrrdio_load(path)  # load the library once
            NR = pyoracle._NREF

            def ref():
                dims = (C.c_uint32 * 3)()
                typ = C.c_int()
                fp = C.POINTER(C.c_float)()
                lo, hi = C.c_float(), C.c_float()
                if NR.nref_load(path.encode(), dims, C.byref(typ), C.byref(fp), C.byref(lo), C.byref(hi)):
                    raise RuntimeError("nref_load failed")
                NR.nref_free(fp)
            t = best(ref, a.reps)
            r["reference_parse_s"] = round(t, 4)
            r["reference_parse_gbs"] = round(src_bytes / t / 1e9, 2)
            r["reference_float_bytes"] = nx * ny * nz * 4
        out[name] = r
        print(name, json.dumps(r), flush=True)
        os.remove(path)
        raw = path[:-5] + ".raw"
        if os.path.exists(raw):
            os.remove(raw)
    if rp:
        rp.close()
    print(json.dumps(dict(ingest=out, reference_nrrdio=ref_ok)))


if __name__ == "__main__":
    main()
