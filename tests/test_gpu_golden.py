"""The committed golden scenes (tests/golden/scenes.npz: inputs, the C oracle's RGBA and exact
work counters, made by tools/make_golden.py and pinned on the CPU against the independent
float64 restatement in test_oracle.py) rendered on the GPU through the C ABI: every pixel
equals the stored image bit for bit and the work counters are equal.  Shaded scenes run with
vr_params.exact_gradient = 1 (the fixtures hold exact f32 differences) and, with the default
binary16 field, stay within the parity tolerance of the same fixture."""
import os

import numpy as np
import pytest

import vr_amd

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def scenes():
    z = np.load(os.path.join(GOLD, "scenes.npz"))
    return z, sorted({k.split("/")[0] for k in z.files})


def test_golden_scenes_on_the_gpu(gpu):
    z, names = scenes()
    assert len(names) >= 6
    rp = vr_amd.OffscreenPass(8, 8)
    try:
        for n in names:
            W, H = (int(x) for x in z[n + "/size"])
            vol = z[n + "/vol"]
            smin, smax = z[n + "/slice"]
            shading = int(z[n + "/shading"])
            rp.framebuffer_size_changed(W, H)
            v32 = vol.astype(np.float32)
            rp.volume_dataset_changed(vr_amd.Dataset(vol.shape[::-1], float(v32.min()),
                                                     float(v32.max()), vol))
            rp.transfer_function_changed(np.asarray(z[n + "/tf"], dtype=np.uint32))
            rp.slicing_changed(smin, smax)
            cam = vr_amd.vr_camera()
            for i in range(16):
                cam.view[i] = float(z[n + "/view"][i])
            for i in range(3):
                cam.position[i] = float(z[n + "/pos"][i])
            want = z[n + "/img"]
            p = vr_amd.default_params(shading=shading, exact_gradient=1)
            img = rp.render(cam, p, vr_amd.OUT_RGBA32F)
            assert np.array_equal(img.view(np.uint32), want.view(np.uint32)), n
            cw = rp.count_work(cam, p)
            assert [cw[k] for k in ("rays", "samples", "shaded_samples", "steps")] == \
                list(z[n + "/stats"]), n
            if shading:
                h = rp.render(cam, vr_amd.default_params(shading=1), vr_amd.OUT_RGBA32F)
                d = h.astype(np.float64) - want
                assert np.sqrt(np.mean(d * d)) <= 1e-4 and np.abs(d).max() <= 2e-3, n
            rp.slicing_changed((0, 0, 0), (1, 1, 1))
    finally:
        rp.close()
