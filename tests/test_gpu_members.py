"""GPU: the multi-device path with more than one member on the one GPU of the test box
(vr_debug_create_members, include/vr/vr_debug.h) -- VERDICT r4 item 3.

A context whose member list names device 0 twice (or three times) runs on hardware what an
8-GPU vr_create_mask context runs: the frame-worker threads (one per member beyond 0), the
volume replication (peer copy, here device to itself), per-member slot pipelines and row
shares, the exchange of shards onto member 0 and the block-cyclic assembly.  RCCL holds one
rank per device, so the shards travel by the copy exchange (stream-ordered device copies with
host handshakes between the member threads).  Every frame must equal the one-device
context's bytes -- the reference renders a frame on one thread and one device
(/root/reference/src/application.cpp:59-95) -- and a failing member must end in VR_EIO, not
a hang."""
import numpy as np
import pytest

import synth
import vr_amd

pytestmark = pytest.mark.gpu


def _scene(rp, vol, tf):
    rp.volume_dataset_changed(synth.dataset(vol))
    rp.transfer_function_changed(tf)


@pytest.mark.parametrize("members", [(0, 0), (0, 0, 0)])
def test_members_on_one_device_equal_single_device(gpu, members):
    import torch
    W, H = 131, 203  # several 8-row blocks per member, a ragged last block
    vol = synth.gaussians_numpy((41, 37, 45), seed=77).astype(np.float32)
    tf = synth.tf_band(0.12, 0.92)
    one = vr_amd.OffscreenPass(W, H, device=0)
    grp = vr_amd.OffscreenPass(W, H, members=members, exchange=vr_amd.EXCHANGE_COPY)
    try:
        for rp in (one, grp):
            _scene(rp, vol, tf)
        # replicate_volume ran: every member reads the same bricks
        assert np.array_equal(grp.read_volume(), one.read_volume())
        grp.timing_enable(True)
        for camname in ("rotA", "fill_oblique", "default"):
            cam = synth.camera(camname).to_vr_camera()
            for shading in (0, 1):
                p = vr_amd.default_params(shading=shading, ert_eps=1e-5)
                for fmt in (vr_amd.OUT_RGBA8, vr_amd.OUT_RGBA32F):
                    a = one.render(cam, p, fmt)
                    b = grp.render(cam, p, fmt)
                    assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), (camname, shading, fmt)
        # frames in flight through every member's slot pipeline, one caller stream and one
        # frame buffer copied out after each frame (bench.py's pattern)
        cam = synth.camera("fill_oblique").to_vr_camera()
        ref = torch.empty((H, W), dtype=torch.int32, device="cuda")
        one.render_device(cam, vr_amd.default_params(shading=1, ert_eps=1e-5), ref.data_ptr(),
                          vr_amd.OUT_RGBA8, 16, 0, 1)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        for f in (1, 3, 8):
            pf = vr_amd.default_params(shading=1, ert_eps=1e-5, frames_in_flight=f)
            outs = [torch.zeros((H, W), dtype=torch.int32, device="cuda") for _ in range(11)]
            frame = torch.zeros((H, W), dtype=torch.int32, device="cuda")
            for o in outs:
                grp.render_device(cam, pf, frame.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1, s.cuda_stream)
                with torch.cuda.stream(s):
                    o.copy_(frame)
            torch.cuda.synchronize()
            for i, o in enumerate(outs):
                assert torch.equal(o, ref), (f, i)
        # per-member timing: one entry per member, every member rendered every frame
        rows = [grp.timing_member(m) for m in range(len(members))]
        assert all(r["device"] == 0 for r in rows)
        nframes = rows[0]["frames"]
        assert nframes > 0 and all(r["frames"] == nframes for r in rows), rows
        assert all(r["render_ms"] > 0 and r["kernel_ms"] > 0 for r in rows), rows
        assert rows[0]["assemble_ms"] > 0
        # weighted row shares rebuild the pipelines; frames stay byte-identical
        for w0, w in ((1, 2), (3, 1), (7, 8)):
            grp.set_row_share(w0, w)
            p = vr_amd.default_params(shading=1)
            cam = synth.camera("rotB").to_vr_camera()
            assert np.array_equal(one.render(cam, p).view(np.uint32),
                                  grp.render(cam, p).view(np.uint32)), (w0, w)
        # resize, slicing and TF changes reach every member
        for rp in (one, grp):
            rp.framebuffer_size_changed(77, 61)
            rp.slicing_changed((0.1, 0.0, 0.2), (0.9, 0.8, 1.0))
            rp.transfer_function_changed(synth.tf_color())
        for shading in (0, 1):
            p = vr_amd.default_params(shading=shading)
            cam = synth.camera("rotB").to_vr_camera()
            assert np.array_equal(one.render(cam, p).view(np.uint32), grp.render(cam, p).view(np.uint32))
    finally:
        grp.close()
        one.close()


def test_members_u8_and_generated_volumes(gpu):
    W, H = 96, 72
    grp = vr_amd.OffscreenPass(W, H, members=(0, 0), exchange=vr_amd.EXCHANGE_COPY)
    one = vr_amd.OffscreenPass(W, H, device=0)
    try:
        for rp in (one, grp):
            rp.generate_volume((48, 40, 44), np.uint8, seed=5)
            rp.transfer_function_changed(synth.tf2())
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


@pytest.mark.parametrize("member,frame", [(1, 2), (0, 1), (2, 0)])
def test_member_failure_ends_in_eio_without_hang(gpu, member, frame):
    """A member whose enqueue fails (injected) aborts the exchange: the frame calls report
    VR_EIO (-5) within a few frames, and closing the context returns."""
    import torch
    W, H = 64, 80
    grp = vr_amd.OffscreenPass(W, H, members=(0, 0, 0), exchange=vr_amd.EXCHANGE_COPY)
    try:
        _scene(grp, synth.gaussians_numpy((24, 20, 28), seed=3), synth.tf_color())
        cam = synth.camera("fill").to_vr_camera()
        p = vr_amd.default_params(shading=1, frames_in_flight=3)
        frame_buf = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        grp.render_device(cam, p, frame_buf.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1)  # builds pipelines
        torch.cuda.synchronize()
        grp.fail_member(member, frame + 1)  # pipeline frame numbers count from the build
        with pytest.raises(RuntimeError, match=r"\(-5\)"):
            for _ in range(frame + 8):
                grp.render_device(cam, p, frame_buf.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1)
            grp.render(cam, p)  # synchronous: reports a worker's failure at the latest
        # still failing afterwards (the exchange is aborted), and close() returns
        with pytest.raises(RuntimeError):
            grp.render(cam, p)
    finally:
        grp.close()
    torch.cuda.synchronize()


def test_members_reject_rccl_for_a_repeated_device(gpu):
    with pytest.raises(RuntimeError, match="listed twice"):
        vr_amd.OffscreenPass(32, 32, members=(0, 0), exchange=vr_amd.EXCHANGE_RCCL)
    with pytest.raises(RuntimeError, match="not present"):
        vr_amd.OffscreenPass(32, 32, members=(0, 99))
    one = vr_amd.OffscreenPass(32, 32, device=0)
    try:
        with pytest.raises(RuntimeError, match="not a multi-device"):
            one.fail_member(0, 0)
    finally:
        one.close()


def test_dist_rejects_a_row_share_changed_after_creation(gpu):
    """vr_dist sized its shards for the share at creation; a later
    vr_set_row_share must be refused, not overflow the shard buffers."""
    import torch
    W, H = 64, 48
    rp = vr_amd.OffscreenPass(W, H, device=0)
    try:
        rp.volume_dataset_changed(synth.dataset(synth.gaussians_numpy((16, 16, 16), seed=1)))
        df = vr_amd.DistFrames(rp, vr_amd.dist_unique_id(), 1, 0, row_block=8, frames_in_flight=2)
        fr = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        cam = synth.camera("fill").to_vr_camera()
        p = vr_amd.default_params()
        df.render(cam, p, fr.data_ptr())
        df.synchronize()
        rp.set_row_share(3, 5)
        with pytest.raises(RuntimeError, match="row share changed"):
            df.render(cam, p, fr.data_ptr())
        rp.set_row_share(1, 1)
        df.render(cam, p, fr.data_ptr())  # back to the creation share: accepted
        df.synchronize()
        df.close()
    finally:
        rp.close()


def test_members_random_sequence_of_frames_shares_and_flights(gpu):
    """A seeded random sequence on 4 members of device 0 (copy exchange): frames in flight
    1..8, row shares, output formats, cameras and TF changes interleaved; after every burst
    each frame equals the one-device context's bytes (pipeline rebuilds, slot reuse and the
    exchange's handshakes under changing shapes)."""
    import torch
    rng = np.random.default_rng(505)
    W, H = 120, 90
    vol = synth.gaussians_numpy((36, 40, 32), seed=12).astype(np.float32)
    one = vr_amd.OffscreenPass(W, H, device=0)
    grp = vr_amd.OffscreenPass(W, H, members=(0, 0, 0, 0), exchange=vr_amd.EXCHANGE_COPY)
    try:
        tfs = [synth.tf_color(), synth.tf_band(0.1, 0.9), synth.tf2()]
        for rp in (one, grp):
            _scene(rp, vol, tfs[0])
        s = torch.cuda.Stream()
        for burst in range(12):
            if burst % 4 == 3:
                tf = tfs[int(rng.integers(len(tfs)))]
                for rp in (one, grp):
                    rp.transfer_function_changed(tf)
            w0, w = int(rng.integers(1, 5)), int(rng.integers(1, 5))
            grp.set_row_share(w0, w)
            f = int(rng.integers(1, 9))
            cam = vr_amd.make_camera(radius=float(rng.uniform(1.4, 3.0)),
                                     rotate=(float(rng.uniform(0, 360)), float(rng.uniform(-60, 60)))).to_vr_camera()
            p = vr_amd.default_params(shading=int(rng.integers(2)), ert_eps=1e-5, frames_in_flight=f)
            fmt = vr_amd.OUT_RGBA8 if rng.integers(2) else vr_amd.OUT_RGBA32F
            words = 1 if fmt == vr_amd.OUT_RGBA8 else 4
            ref = torch.empty((H, W * words), dtype=torch.int32, device="cuda")
            one.render_device(cam, p, ref.data_ptr(), fmt, 16, 0, 1)
            torch.cuda.synchronize()
            frame = torch.zeros((H, W * words), dtype=torch.int32, device="cuda")
            outs = [torch.zeros_like(frame) for _ in range(int(rng.integers(3, 10)))]
            for o in outs:
                grp.render_device(cam, p, frame.data_ptr(), fmt, 8, 0, 1, s.cuda_stream)
                with torch.cuda.stream(s):
                    o.copy_(frame)
            torch.cuda.synchronize()
            for i, o in enumerate(outs):
                assert torch.equal(o, ref), (burst, i, f, (w0, w), fmt)
    finally:
        grp.close()
        one.close()
