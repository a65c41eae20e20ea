"""Host enqueue cost per frame of the library's frame paths, against the device frame period
of an N = 8 rank share (C3, 3 frames in flight).  If the host needs longer to enqueue a frame
than the device needs to render it, an N = 8 rank is host-bound.

  render_device share : vr_render_device of rank 0's 1/8 row share, 3 streams round-robin
  dist one-rank       : vr_dist_render (render -> ncclGather -> assemble) on a one-rank
                        communicator (the full frame: the only RCCL group one GPU can hold)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for sub in ("volumetric-renderer_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, sub))
import torch  # noqa: E402

import synth  # noqa: E402
import vr_amd  # noqa: E402

W, H, N = 1920, 1080, 8
torch.cuda.set_device(0)
rp = vr_amd.OffscreenPass(W, H, device=0)
rp.generate_volume((512, 512, 512), seed=2024)
rp.transfer_function_changed(synth.TFS["tf2"]())
cam = synth.camera("fill").to_vr_camera()
p = vr_amd.default_params(shading=1, ert_eps=1e-5, frames_in_flight=3)
sr = vr_amd.shard_rows(H, 8, N)
streams = [torch.cuda.Stream() for _ in range(3)]
outs = [torch.empty((sr, W), dtype=torch.int32, device="cuda") for _ in range(3)]


def share(i):
    rp.render_device(cam, p, outs[i % 3].data_ptr(), vr_amd.OUT_RGBA8, 8, 0, N,
                     streams[i % 3].cuda_stream)


for i in range(30):
    share(i)
torch.cuda.synchronize()
for n in (100, 1000):
    t0 = time.perf_counter()
    for i in range(n):
        share(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"render_device 1/{N} share x{n}: host {1e6 * (t1 - t0) / n:.1f} us/frame, "
          f"device period {1e6 * (t2 - t0) / n:.1f} us/frame", flush=True)

df = vr_amd.DistFrames(rp, vr_amd.dist_unique_id(), 1, 0, row_block=8, frames_in_flight=3)
frame = torch.empty((H, W), dtype=torch.int32, device="cuda")
s = torch.cuda.Stream()
for _ in range(10):
    df.render(cam, p, frame.data_ptr(), s.cuda_stream)
df.synchronize()
torch.cuda.synchronize()
for n in (20, 200):
    t0 = time.perf_counter()
    for _ in range(n):
        df.render(cam, p, frame.data_ptr(), s.cuda_stream)
    t1 = time.perf_counter()
    df.synchronize()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"vr_dist_render one-rank full frame x{n}: host {1e6 * (t1 - t0) / n:.1f} us/frame, "
          f"device period {1e6 * (t2 - t0) / n:.1f} us/frame", flush=True)
df.close()
rp.close()
