"""Slab-march counters (experiment build lib_stats, -DVR_SLAB_STATS): slabs staged, elements
staged, samples served from LDS and from the bricks, for one frame of a bench config."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
for sub in ("", "volumetric-renderer_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, sub))
os.environ["VR_SLAB"] = "1"
import bench  # noqa: E402
import synth  # noqa: E402
import vr_amd  # noqa: E402

lib = vr_amd.lib()
f = lib.vr_debug_slab_stats
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
out = (C.c_ulonglong * 4)()
for cfg_name in sys.argv[1:] or ["c3", "c3_ref"]:
    cfg = bench.CONFIGS[cfg_name]
    rp = bench.setup_pass(cfg, 0)
    cam = synth.camera(cfg["cam"])
    p = vr_amd.default_params(shading=cfg["shading"], ert_eps=cfg["ert"], frames_in_flight=1)
    for _ in range(6):
        rp.render(cam, p)
    f(out, 1)
    rp.render(cam, p)
    f(out, 1)
    work = rp.count_work(cam.to_vr_camera(), p)
    print(json.dumps(dict(config=cfg_name, slabs=out[0], elements=out[1], lds_samples=out[2],
                          brick_samples=out[3], samples=work["samples"],
                          tiles=((cfg["W"] + 15) // 16) * ((cfg["H"] + 15) // 16))), flush=True)
    rp.close()
