import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for sub in ("volumetric-renderer_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, sub))
import numpy as np, torch, synth, vr_amd
W, H = 96, 80
rp = vr_amd.OffscreenPass(W, H)
cam = synth.camera("fill_oblique").to_vr_camera()
vol = synth.gaussians_numpy((41, 37, 45), seed=5).astype(np.float32)
rp.volume_dataset_changed(synth.dataset(vol))
rp.transfer_function_changed(synth.tf_band(0.1, 0.9))
for nranks in (1, 2, 4):
    for rank in range(nranks):
        sr = vr_amd.shard_rows(H, 8, nranks)
        res = {}
        for fif in (0, 3):
            for pair in ("", "0", "1"):
                if pair: os.environ["VR_PAIR"] = pair
                else: os.environ.pop("VR_PAIR", None)
                p = vr_amd.default_params(shading=1, ert_eps=1e-5, frames_in_flight=fif)
                o = torch.zeros((sr, W), dtype=torch.int32, device="cuda")
                rp.render_device(cam, p, o.data_ptr(), vr_amd.OUT_RGBA8, 8, rank, nranks, 0)
                torch.cuda.synchronize()
                res[(fif, pair)] = o.cpu().numpy()
        base = res[(0, "0")]
        for k, v in res.items():
            d = np.argwhere(v != base)
            print(nranks, rank, k, len(d), d[:3].tolist())
