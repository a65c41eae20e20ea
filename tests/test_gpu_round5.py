"""GPU: round-5 additions to the boundary (vr.h ABI 8).

* The default derived-structure budget: VR_MEMORY_BUDGET_DEFAULT is 5x
  the bricked volume's bytes (4x in ABI 8), so a camera that crosses every view class keeps at
  most the difference field and the copies a shaded orbit visits, with frames unchanged.  The reference holds one
  volume image (/root/reference/src/rendering/offscreen_pass.cpp:940-989); this bounds what
  the library adds beside it.
"""
import numpy as np
import pytest

import pyoracle
import synth
import vr_amd

pytestmark = pytest.mark.gpu

BUDGET_DEFAULT = 2 ** 64 - 2
BUDGET_UNLIMITED = 2 ** 64 - 1


def _bits_equal(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return int((a.view(np.uint32) != b.view(np.uint32)).any(axis=-1).sum())


def test_default_budget_is_bounded_and_frames_unchanged(gpu):
    W, H = 160, 120
    vol = synth.gaussians_numpy((64, 60, 66), seed=41).astype(np.float32)
    tf = synth.tf_band(0.15, 0.9)
    rp = vr_amd.OffscreenPass(W, H, device=0)
    try:
        rp.volume_dataset_changed(synth.dataset(vol))
        rp.transfer_function_changed(tf)
        m0 = rp.memory_report()
        bricks = m0["volume_bytes"]
        assert 5 * bricks <= m0["budget_bytes"] <= 5 * bricks + bricks // 16 + (1 << 20), m0
        cams = {k: synth.camera(k).to_vr_camera() for k in ("fill", "default", "diag", "rotA")}
        frames = {}
        for budget in (BUDGET_DEFAULT, BUDGET_UNLIMITED):
            rp.set_memory_budget(0)  # start from the bricks alone
            rp.set_memory_budget(budget)
            for name, cam in cams.items():
                for shading in (0, 1):
                    for skip in (0, 1):
                        p = vr_amd.default_params(shading=shading, ert_eps=1e-5, skip_empty=skip,
                                                  exact_gradient=1, frames_in_flight=3)
                        frames[budget, name, shading, skip] = rp.render(cam, p, vr_amd.OUT_RGBA32F)
                        m = rp.memory_report()
                        if budget == BUDGET_DEFAULT:
                            assert m["derived_bytes"] <= m["budget_bytes"], (name, m)
            if budget == BUDGET_UNLIMITED:
                assert rp.memory_report()["budget_bytes"] == BUDGET_UNLIMITED
        for (b, name, shading, skip), img in frames.items():
            if b == BUDGET_DEFAULT:
                assert _bits_equal(img, frames[BUDGET_UNLIMITED, name, shading, skip]) == 0, \
                    (name, shading, skip)
        # and against the oracle, on the default budget's last view
        rp.set_memory_budget(BUDGET_DEFAULT)
        p = vr_amd.default_params(shading=1, ert_eps=1e-5, exact_gradient=1)
        img = rp.render(cams["fill"], p, vr_amd.OUT_RGBA32F)
        ref, _ = pyoracle.Scene.from_params(vol, float(vol.min()), float(vol.max()), tf,
                                            cams["fill"], W, H, p).render()
        assert _bits_equal(img, ref) == 0
    finally:
        rp.close()
