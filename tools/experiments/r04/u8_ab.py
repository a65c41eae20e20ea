"""C4-class A/B of a library build (VR_AMD_LIB) on 8-bit volumes: 1024^3 u8 (plain 7x8x8 bricks,
the pipelined kernel), 2048^2, TF-2, unshaded; views fill / default / diag; 3 frames in flight and
serial.  Prints JSON lines with ms per frame and a hash of the last frame (byte identity across
builds).  Usage: VR_AMD_LIB=... python tools/experiments/r04/u8_ab.py TAG [dims] [W]"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
for sub in ("volumetric-renderer_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import synth  # noqa: E402
import vr_amd  # noqa: E402


def main():
    tag = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    W = H = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
    rp = vr_amd.OffscreenPass(W, H)
    rp.generate_volume((n, n, n), np.uint8, seed=7)
    rp.transfer_function_changed(synth.tf2())
    outs = [torch.empty((H, W), dtype=torch.int32, device="cuda") for _ in range(3)]
    streams = [torch.cuda.Stream() for _ in range(3)]
    for view in ("fill", "default", "diag"):
        cam = synth.camera(view).to_vr_camera()
        for inflight in (3, 1):
            p = vr_amd.default_params(frames_in_flight=inflight)
            for rep in range(2):
                nf = 60 if inflight > 1 else 30
                for phase in ("warm", "time"):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for i in range(nf):
                        k = i % inflight
                        rp.render_device(cam, p, outs[k].data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1,
                                         streams[k].cuda_stream)
                        if inflight == 1:
                            streams[0].synchronize()
                    torch.cuda.synchronize()
                    ms = (time.perf_counter() - t0) / nf * 1e3
                h = hashlib.sha256(outs[(nf - 1) % inflight].cpu().numpy().tobytes()).hexdigest()[:16]
                st = rp.count_work(cam, p)
                print(json.dumps(dict(tag=tag, view=view, inflight=inflight, rep=rep, ms=round(ms, 4),
                                      gsamples=round(st["samples"] / ms / 1e6, 1), frame=h,
                                      kernel=rp.kernel_name(p))), flush=True)
    rp.close()


if __name__ == "__main__":
    main()
