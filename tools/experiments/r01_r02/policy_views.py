"""Which march kernel the launch policy picks per view (unshaded and shaded), C3 volume."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "volumetric-renderer_amd")); sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np, torch, synth, vr_amd
from view_sweep import VIEWS
rp = vr_amd.OffscreenPass(1920, 1080)
rp.generate_volume((512,) * 3, np.float32, seed=2024)
rp.transfer_function_changed(synth.TFS["tf2"]())
out = torch.empty((1080 + 16, 1920), dtype=torch.int32, device="cuda")
for sh in (0, 1):
    p = vr_amd.default_params(shading=sh, ert_eps=1e-5 if sh else 0.0, frames_in_flight=3)
    for name, v in VIEWS.items():
        cam = vr_amd.make_camera(**v).to_vr_camera()
        rp.render_device(cam, p, out.data_ptr(), vr_amd.OUT_RGBA8, 16, 0, 1, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        print(f"shading={sh} {name:13s} {rp.kernel_name(p)}")
