"""GPU (round 4): cases the earlier suites did not reach.

* The binary16 difference field's scale comes from the stored data's own range, never from the
  caller's vmin/vmax: a Dataset whose min/max is a display window narrower than the
  data (the reference always takes min/max from the data, nrrd_file_parser.cpp:39-40, but the
  boundary accepts any) must not clamp large central differences.
"""
import numpy as np
import pytest

import pyoracle
import synth
import vr_amd

pytestmark = pytest.mark.gpu


def _bits_equal(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return int((a.view(np.uint32) != b.view(np.uint32)).any(axis=-1).sum())


def _step_volume():
    """A float block of 3000.5 in zeros plus fractional noise: central differences up to ~3000
    at the block faces, not integers (so the volume stays f32 and reads the field)."""
    rng = np.random.default_rng(4)
    vol = rng.uniform(0.0, 0.75, size=(26, 30, 28)).astype(np.float32)
    vol[6:20, 8:22, 7:21] += np.float32(3000.5)
    return vol


@pytest.mark.parametrize("window", [(0.0, 2000.0), (0.0, 1.0), (-10.0, 400.0)])
def test_half_field_scale_from_data_not_window(gpu, window):
    vol = _step_volume()
    W, H = 72, 56
    rp = vr_amd.OffscreenPass(W, H, device=0)
    try:
        ds = vr_amd.Dataset((vol.shape[2], vol.shape[1], vol.shape[0]), window[0], window[1], vol)
        rp.volume_dataset_changed(ds)
        assert rp.volume_info()[2] == 4  # f32 storage
        tf = synth.tf_color()
        rp.transfer_function_changed(tf)
        cam = synth.camera("fill").to_vr_camera()
        p = vr_amd.default_params(shading=1)
        with rp.knobs(grad_field=1):  # every view reads the field
            img = rp.render(cam, p, vr_amd.OUT_RGBA32F)
            assert "F32H" in rp.kernel_name(p)
        half, st = pyoracle.Scene.from_params(vol, window[0], window[1], tf, cam, W, H, p,
                                              grad_f16=True).render()
        exact, _ = pyoracle.Scene.from_params(vol, window[0], window[1], tf, cam, W, H, p).render()
        assert st["shaded_samples"] > 0
        assert _bits_equal(img, half) == 0
        # no clamped differences: the binary16 frame stays as close to the exact one as on
        # ordinary volumes (a window-derived scale of 2^15 or 2^5 would clamp the block's faces)
        d = img.astype(np.float64) - exact
        assert float(np.sqrt(np.mean(d * d))) < 1e-4 and float(np.abs(d).max()) < 5e-3
        # the oracle restating a window-derived scale would NOT match (the case is exercised)
        wrong = pyoracle.Scene.from_params(vol, window[0], window[1], tf, cam, W, H, p, grad_f16=True)
        wrong.s.grad_range_set = 0
        bad, _ = wrong.render()
        assert _bits_equal(img, bad) > 0
    finally:
        rp.close()


# ---- weighted row shares (vr_set_row_share) -------------------------------------------------

@pytest.mark.parametrize("share", [(1, 1), (1, 2), (3, 4), (2, 1), (7, 8)])
def test_row_share_shards_assemble_exactly(gpu, share):
    """Every rank's shard under a weighted split (rank 0 lighter or heavier), gathered
    rank-major and assembled, equals the single-rank frame bit for bit; the shards' work sums to
    the frame's; the shard rows follow vr_dist.py's restatement."""
    import torch
    import vr_dist
    W, H = 70, 53
    rp = vr_amd.OffscreenPass(W, H, device=0)
    try:
        vol = synth.gaussians_numpy((24, 24, 24), seed=5)
        rp.volume_dataset_changed(synth.dataset(vol))
        rp.transfer_function_changed(synth.tf_color())
        cam = synth.camera("rotB").to_vr_camera()
        p = vr_amd.default_params(shading=1)
        full = torch.empty((H, W), dtype=torch.int32, device="cuda")
        rp.render_device(cam, p, full.data_ptr(), vr_amd.OUT_RGBA8, 16, 0, 1)
        rp.set_row_share(*share)
        assert rp.row_share() == share
        for nranks, rb in ((2, 16), (3, 8), (8, 4), (5, 1)):
            sr = rp.shard_rows(H, rb, nranks)
            assert sr == vr_dist.shard_rows(H, rb, nranks, share)
            gathered = torch.zeros((nranks, sr, W), dtype=torch.int32, device="cuda")
            for r in range(nranks):
                rp.render_device(cam, p, gathered[r].data_ptr(), vr_amd.OUT_RGBA8, rb, r, nranks)
            out = torch.empty((H, W), dtype=torch.int32, device="cuda")
            rp.assemble_rows(gathered.data_ptr(), out.data_ptr(), vr_amd.OUT_RGBA8, rb, nranks)
            torch.cuda.synchronize()
            assert torch.equal(out, full), (share, nranks, rb)
            tot = {k: 0 for k in ("rays", "samples", "shaded_samples", "steps", "skipped_samples")}
            for r in range(nranks):
                for k, v in rp.count_work(cam, p, rb, r, nranks).items():
                    tot[k] += v
            assert tot == rp.count_work(cam, p)
        # vr_render's host bands keep their own split whatever the share
        img = rp.render(cam, p, vr_amd.OUT_RGBA8)
        assert np.array_equal(img.view(np.int32).reshape(H, W), full.cpu().numpy())
    finally:
        rp.close()


def test_mask_context_row_share_and_member_timing(gpu):
    """A multi-device context (device 0 here) with a weighted share renders the one-device frame
    byte for byte, and vr_debug_timing_member reports the member's kernel, render, gather and
    assembly spans for the frames timed."""
    import torch
    W, H = 96, 72
    vol = synth.gaussians_numpy((32, 28, 24), seed=2)
    one = vr_amd.OffscreenPass(W, H, device=0)
    grp = vr_amd.OffscreenPass(W, H, device_mask=0x1)
    try:
        for r in (one, grp):
            r.volume_dataset_changed(synth.dataset(vol))
            r.transfer_function_changed(synth.tf_color())
        cam = synth.camera("fill_oblique").to_vr_camera()
        p = vr_amd.default_params(shading=1, frames_in_flight=3)
        ref = one.render(cam, p, vr_amd.OUT_RGBA8)
        grp.set_row_share(3, 4)
        grp.timing_reset()
        grp.timing_enable(True)
        frame = torch.empty((H, W), dtype=torch.int32, device="cuda")
        s = torch.cuda.Stream()
        for _ in range(5):
            grp.render_device(cam, p, frame.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1, s.cuda_stream)
        s.synchronize()
        t = grp.timing_member(0)
        grp.timing_enable(False)
        assert t["device"] == 0 and t["frames"] == 5
        assert t["kernel_ms"] > 0 and t["render_ms"] >= t["kernel_ms"] * 0.5
        assert t["gather_ms"] > 0 and t["assemble_ms"] > 0
        with pytest.raises(RuntimeError):
            grp.timing_member(1)
        assert np.array_equal(frame.cpu().numpy(), ref.view(np.int32).reshape(H, W))
        assert np.array_equal(grp.render(cam, p, vr_amd.OUT_RGBA8), ref)
    finally:
        grp.close()
        one.close()


# ---- derived-structure memory budget and preparation ----------------------------------------

def _views():
    return {"fill": synth.camera("fill").to_vr_camera(),
            "default": synth.camera("default").to_vr_camera(),
            "diag": synth.camera("diag").to_vr_camera()}


def test_memory_budget_zero_and_unlimited_render_the_same_frames(gpu):
    """Budget 0 keeps only the bricks (no difference field, no alternative copies, no skip-empty
    classification); every frame equals the unlimited budget's bit for bit (exact gradient), and
    with the binary16 default the budget-0 shaded frame is the exact-gradient oracle's."""
    W, H = 120, 90
    vol = synth.gaussians_numpy((64, 60, 66), seed=31).astype(np.float32)
    tf = synth.tf_band(0.15, 0.9)
    rp = vr_amd.OffscreenPass(W, H, device=0)
    try:
        rp.volume_dataset_changed(synth.dataset(vol))
        rp.transfer_function_changed(tf)
        frames = {}
        for budget in (2 ** 64 - 1, 0):
            rp.set_memory_budget(budget)
            for name, cam in _views().items():
                for shading in (0, 1):
                    for skip in (0, 1):
                        p = vr_amd.default_params(shading=shading, ert_eps=1e-5, skip_empty=skip,
                                                  exact_gradient=1)
                        frames[(budget, name, shading, skip)] = rp.render(cam, p, vr_amd.OUT_RGBA32F)
            m = rp.memory_report()
            if budget == 0:
                assert m["derived_bytes"] == 0 and m["budget_bytes"] == 0
                assert m["field_bytes"] == m["oblique_copy_bytes"] == m["stencil_copy_bytes"] == 0
            else:
                assert m["derived_bytes"] > 0 and m["volume_bytes"] == rp.volume_bytes()
        for (b, name, shading, skip), img in frames.items():
            if b == 0:
                ref = frames[(2 ** 64 - 1, name, shading, skip)]
                assert _bits_equal(img, ref) == 0, (name, shading, skip)
        # binary16 default under budget 0: the stencil (exact) gradient, i.e. the f32 oracle
        cam = _views()["fill"]
        p = vr_amd.default_params(shading=1, ert_eps=1e-5)
        img = rp.render(cam, p, vr_amd.OUT_RGBA32F)
        assert "F32H" not in rp.kernel_name(p)
        ref, _ = pyoracle.Scene.from_params(vol, float(vol.min()), float(vol.max()), tf, cam, W, H,
                                            p).render()
        assert _bits_equal(img, ref) == 0
    finally:
        rp.close()


def test_budget_between_copies_evicts_and_prepare_builds_ahead(gpu):
    """A budget that holds one alternative copy but not two: crossing from the diagonal (oblique
    copy) to the default camera (stencil copy) evicts the first, frames stay exact.  vr_prepare
    builds what the next view reads outside a frame, and reports it."""
    W, H = 120, 90
    vol = synth.gaussians_numpy((64, 60, 66), seed=32).astype(np.float32)
    tf = synth.tf_band(0.15, 0.9)
    rp = vr_amd.OffscreenPass(W, H, device=0)
    try:
        rp.volume_dataset_changed(synth.dataset(vol))
        rp.transfer_function_changed(tf)
        v = _views()
        # frames in flight: the throughput kernels (serial frames this small take the lane-pair
        # kernel, which reads the 8^3 bricks and wants no alternative copy)
        p = vr_amd.default_params(shading=1, ert_eps=1e-5, exact_gradient=1, frames_in_flight=3)
        rp.prepare(v["diag"], p)
        m = rp.memory_report()
        assert m["oblique_copy_bytes"] > 0 and m["stencil_copy_bytes"] == 0
        rp.prepare(v["default"], p)
        m2 = rp.memory_report()
        assert m2["stencil_copy_bytes"] > 0 and m2["oblique_copy_bytes"] > 0
        one = max(m2["oblique_copy_bytes"], m2["stencil_copy_bytes"])
        rp.set_memory_budget(one + (1 << 20))  # lower: frees everything, one copy fits
        assert rp.memory_report()["derived_bytes"] == 0
        for name in ("diag", "default", "diag"):
            img = rp.render(v[name], p, vr_amd.OUT_RGBA32F)
            m3 = rp.memory_report()
            assert m3["derived_bytes"] <= one + (1 << 20)
            ref, _ = pyoracle.Scene.from_params(vol, float(vol.min()), float(vol.max()), tf,
                                                v[name], W, H, p).render()
            assert _bits_equal(img, ref) == 0, name
        assert m3["oblique_copy_bytes"] > 0 and m3["stencil_copy_bytes"] == 0  # evicted
    finally:
        rp.close()


# (The wavefront work queue, tile_order 5, measured 2-4x slower in round 5, is in
# tools/experiments/r05_pruned/ with its test; tile_order 5 now runs as 4, test_gpu_parity.py.)
