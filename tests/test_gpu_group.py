"""GPU: the multi-device context (vr_create_mask, vr.h) -- SURVEY.md §8b's `device_mask`
boundary, the reference's single-threaded host driving several GPUs through the same calls.

On the one-GPU test box the mask holds device 0 only: the frame still goes the whole
multi-device way (member context, slot pipeline, ncclCommInitAll communicator, ncclGather,
assembly, frame-worker issue), and every frame must equal the one-device context's bytes.
The N = 2/3 member schedule runs on host threads in tests/test_sched_host.py."""
import numpy as np
import pytest

import synth
import vr_amd

pytestmark = pytest.mark.gpu


def _scene(rp, vol, tf, W, H):
    rp.framebuffer_size_changed(W, H)
    rp.volume_dataset_changed(synth.dataset(vol))
    rp.transfer_function_changed(tf)


def test_mask_one_device_frames_equal_single_device(gpu):
    import torch
    W, H = 130, 97
    vol = synth.gaussians_numpy((41, 37, 45), seed=31).astype(np.float32)
    tf = synth.tf_band(0.15, 0.9)
    one = vr_amd.OffscreenPass(W, H, device=0)
    grp = vr_amd.OffscreenPass(W, H, device_mask=0x1)
    try:
        assert grp.device_mask == 1 and one.device_mask == 1
        for rp in (one, grp):
            _scene(rp, vol, tf, W, H)
        assert np.array_equal(grp.read_volume(), one.read_volume())
        for camname in ("rotA", "fill_oblique", "default"):
            cam = synth.camera(camname).to_vr_camera()
            for shading, skip in ((0, 0), (1, 0), (1, 1)):
                p = vr_amd.default_params(shading=shading, skip_empty=skip, ert_eps=1e-5)
                for fmt in (vr_amd.OUT_RGBA8, vr_amd.OUT_RGBA32F):
                    a = one.render(cam, p, fmt)
                    b = grp.render(cam, p, fmt)
                    assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), (camname, shading, skip, fmt)
                assert grp.count_work(cam, p) == one.count_work(cam, p)
        # frames in flight across the members, one caller stream and one frame buffer (as
        # bench.py drives it): every frame equals the one-device frame
        cam = synth.camera("fill_oblique").to_vr_camera()
        ref = torch.empty((H, W), dtype=torch.int32, device="cuda")
        p1 = vr_amd.default_params(shading=1, ert_eps=1e-5)
        one.render_device(cam, p1, ref.data_ptr(), vr_amd.OUT_RGBA8, 16, 0, 1)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        for f in (1, 3, 4):
            pf = vr_amd.default_params(shading=1, ert_eps=1e-5, frames_in_flight=f)
            outs = [torch.zeros((H, W), dtype=torch.int32, device="cuda") for _ in range(5)]
            frame = torch.zeros((H, W), dtype=torch.int32, device="cuda")
            for o in outs:  # the caller copies each frame out on its stream before the next
                grp.render_device(cam, pf, frame.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1, s.cuda_stream)
                with torch.cuda.stream(s):
                    o.copy_(frame)
            torch.cuda.synchronize()
            for i, o in enumerate(outs):
                assert torch.equal(o, ref), (f, i)
        # resize, slicing and TF changes reach every member
        grp.framebuffer_size_changed(77, 61)
        one.framebuffer_size_changed(77, 61)
        for rp in (one, grp):
            rp.slicing_changed((0.1, 0.0, 0.2), (0.9, 0.8, 1.0))
            rp.transfer_function_changed(synth.tf_color())
        for shading in (0, 1):
            p = vr_amd.default_params(shading=shading)
            cam = synth.camera("rotB").to_vr_camera()
            assert np.array_equal(one.render(cam, p).view(np.uint32), grp.render(cam, p).view(np.uint32))
        with pytest.raises(RuntimeError, match="whole frames"):
            grp.render_device(cam, vr_amd.default_params(), ref.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 2)
    finally:
        grp.close()
        one.close()


def test_mask_generated_and_u8_volumes(gpu):
    """Generated volumes (vr_generate_volume) and 8-bit uploads replicate to the members."""
    W, H = 96, 72
    grp = vr_amd.OffscreenPass(W, H, device_mask=0x1)
    one = vr_amd.OffscreenPass(W, H, device=0)
    try:
        for rp in (one, grp):
            rp.generate_volume((48, 40, 44), np.uint8, seed=5)
            rp.transfer_function_changed(synth.tf2())
        assert grp.volume_bytes() == one.volume_bytes()
        cam = synth.camera("fill").to_vr_camera()
        for shading in (0, 1):
            p = vr_amd.default_params(shading=shading)
            assert np.array_equal(one.render(cam, p), grp.render(cam, p))
        ct = synth.ct_head(64, seed=3)
        for rp in (one, grp):
            rp.volume_dataset_changed(synth.dataset(ct))
        p = vr_amd.default_params()
        assert np.array_equal(one.render(cam, p), grp.render(cam, p))
    finally:
        grp.close()
        one.close()


def test_mask_rejects_missing_devices_and_dist(gpu):
    import torch
    n = torch.cuda.device_count()
    with pytest.raises(RuntimeError, match=f"device {n} of device_mask"):
        vr_amd.OffscreenPass(32, 32, device_mask=(1 << (n + 1)) - 1)
    with pytest.raises(RuntimeError, match="empty"):
        vr_amd.OffscreenPass(32, 32, device_mask=0)
    grp = vr_amd.OffscreenPass(32, 32, device_mask=0x1)
    try:
        with pytest.raises(RuntimeError, match="distributes its own frames"):
            vr_amd.DistFrames(grp, bytes(vr_amd.DIST_ID_BYTES), 1, 0)
    finally:
        grp.close()
