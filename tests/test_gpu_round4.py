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
