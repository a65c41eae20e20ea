"""Lane occupancy of the march (experiment): lane-steps (the normal counting kernel) against
64 x each wavefront's longest ray (a -DVR_EXP_WAVE_STEPS=1 build, VR_AMD_LIB_WS), per view.
GPU box: python tools/experiments/r01_r02/lane_occupancy.py"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CODE = r'''
import sys, json, os
sys.path.insert(0, os.path.join("%s", "volumetric-renderer_amd")); sys.path.insert(0, os.path.join("%s", "tools"))
import numpy as np, synth, vr_amd
from view_sweep import VIEWS
rp = vr_amd.OffscreenPass(1920, 1080)
rp.generate_volume((512,) * 3, np.float32, seed=2024)
rp.transfer_function_changed(synth.TFS["tf2"]())
out = {}
for shading, ert in ((1, 1e-5), (0, 0.0)):
    p = vr_amd.default_params(shading=shading, ert_eps=ert)
    for name, v in VIEWS.items():
        out[f"{name}/s{shading}"] = rp.count_work(vr_amd.make_camera(**v).to_vr_camera(), p)["steps"]
print(json.dumps(out))
''' % (ROOT, ROOT)


def run(lib):
    env = dict(os.environ, VR_AMD_LIB=lib)
    r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, check=True)
    return json.loads(r.stdout.strip().splitlines()[-1])


lane = run(os.path.join(ROOT, "volumetric-renderer_amd", "lib", "libvr_amd.so"))
wave = run(os.path.join(ROOT, "volumetric-renderer_amd", "lib_ws", "libvr_amd.so"))
for k in lane:
    print(k.ljust(20), "lane-steps", lane[k], "wave-steps x64", wave[k], "occupancy", round(lane[k] / wave[k], 3))
