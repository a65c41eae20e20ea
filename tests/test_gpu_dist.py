"""GPU: the library's multi-GPU frame path (include/vr/vr_dist.h) on a one-rank RCCL
communicator, the only one a single device can hold.  Render -> ncclGather -> assemble runs
stream-ordered over 1-3 frames in flight, and every assembled frame must equal the
single-GPU render of the same camera byte for byte.  The multi-rank logic is the same code
with nranks > 1; the CPU gloo tests (test_multirank.py) cover the row-block layout, and the
driver's 8-GPU run checks it with bench.py's frame_check."""
import numpy as np
import pytest

import synth
import vr_amd

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("inflight", [1, 3])
def test_dist_frames_one_rank_equal_single_gpu_render(gpu, inflight):
    import torch
    W, H = 120, 88
    rp = vr_amd.OffscreenPass(W, H, device=0)
    try:
        rp.volume_dataset_changed(synth.dataset(synth.gaussians_numpy((29, 33, 31), seed=4)))
        rp.transfer_function_changed(synth.tf_color())
        df = vr_amd.DistFrames(rp, vr_amd.dist_unique_id(), 1, 0, row_block=8,
                               frames_in_flight=inflight)
        stream = torch.cuda.Stream()
        cams = [vr_amd.make_camera(radius=2.0, rotate=(37.0 * k, 11.0 * k)).to_vr_camera()
                for k in range(5)]
        for shading in (0, 1):
            p = vr_amd.default_params(shading=shading, ert_eps=1e-5)
            frames = [torch.zeros((H, W), dtype=torch.int32, device="cuda") for _ in cams]
            for cam, fr in zip(cams, frames):
                df.render(cam, p, fr.data_ptr(), stream.cuda_stream)
            stream.synchronize()
            df.synchronize()
            for k, (cam, fr) in enumerate(zip(cams, frames)):
                ref = rp.render(cam, p, vr_amd.OUT_RGBA8).view(np.int32).reshape(H, W)
                assert np.array_equal(fr.cpu().numpy(), ref), (shading, k)
        # one frame buffer reused by consecutive frames: the last frame wins, intact
        one = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        p = vr_amd.default_params(shading=1)
        for cam in cams:
            df.render(cam, p, one.data_ptr(), stream.cuda_stream)
        stream.synchronize()
        ref = rp.render(cams[-1], p, vr_amd.OUT_RGBA8).view(np.int32).reshape(H, W)
        assert np.array_equal(one.cpu().numpy(), ref)
        with pytest.raises(RuntimeError, match="frame_dev"):
            df.render(cams[0], p, 0, stream.cuda_stream)
        # a resized context needs a new vr_dist
        rp.framebuffer_size_changed(W + 8, H)
        with pytest.raises(RuntimeError, match="resized"):
            df.render(cams[0], p, one.data_ptr(), stream.cuda_stream)
        df.close()
    finally:
        rp.close()
