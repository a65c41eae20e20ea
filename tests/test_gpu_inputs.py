"""GPU: the hot path's input producers feeding a rendered frame.

* f4: CSV z-slices through vr_csv_load (the restated CsvFileParser, min/max seeded at 0) ->
  volume_dataset_changed -> HIP render, against the CPU oracle on the same Dataset.
* f2: the golden TF texels (tests/golden/tf_golden.json, an independent restatement of
  gradient.cpp + ImGui packing) are what the product's Gradient hands to
  transfer_function_changed, and a frame rendered with them matches the oracle."""
import json
import os

import numpy as np
import pytest

import pyoracle
import synth
import vr_amd

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _parity(rp, vol, vmin, vmax, tf, cam, W, H, p):
    img = rp.render(cam, p, vr_amd.OUT_RGBA32F)
    half = "F32H" in rp.kernel_name(p)  # binary16 difference field: restated by the oracle
    ref, st = pyoracle.Scene.from_params(vol, vmin, vmax, tf, cam, W, H, p, grad_f16=half).render()
    d = img.astype(np.float64) - ref
    assert float(np.sqrt(np.mean(d * d))) <= 1e-4 and np.abs(d).max() <= 2e-3
    assert np.array_equal(img.view(np.uint32), ref.astype(np.float32).view(np.uint32))
    assert rp.count_work(cam, p) == st
    return st


def test_csv_slices_to_rendered_frame(gpu, tmp_path):
    W, H = 96, 80
    vol = synth.gaussians_numpy((20, 18, 14), seed=9) * np.float32(3.0) - np.float32(0.5)
    paths = []
    for z in range(vol.shape[0]):
        p = tmp_path / f"slice{z:03d}.csv"
        p.write_text("\n".join(",".join(repr(float(v)) for v in row) for row in vol[z]) + "\n")
        paths.append(str(p))
    ds = vr_amd.load_csv(paths)
    assert ds.dims == (vol.shape[2], vol.shape[1], vol.shape[0])
    assert np.array_equal(ds.data, vol)
    assert ds.vmin == min(0.0, float(vol.min())) and ds.vmax == max(0.0, float(vol.max()))
    rp = vr_amd.OffscreenPass(W, H)
    rp.volume_dataset_changed(ds)
    tf = synth.tf_color()
    rp.transfer_function_changed(tf)
    for camname, shading in (("rotA", 0), ("fill_oblique", 1)):
        cam = synth.camera(camname).to_vr_camera()
        st = _parity(rp, ds.data, ds.vmin, ds.vmax, tf, cam, W, H, vr_amd.default_params(shading=shading))
        assert st["samples"] > 0
    rp.close()


@pytest.mark.parametrize("name", ["tf1_256", "tf2_256", "tf_color_7"])
def test_golden_tf_texels_to_rendered_frame(gpu, name):
    W, H = 80, 64
    gold = json.load(open(os.path.join(GOLD, "tf_golden.json")))[name]
    texels = np.array(gold["texels"], dtype=np.uint32)
    if name == "tf1_256":
        assert np.array_equal(synth.tf1(), texels)
    if name == "tf2_256":
        assert np.array_equal(synth.tf2(), texels)
    vol = synth.gaussians_numpy((24, 20, 16), seed=2024)
    rp = vr_amd.OffscreenPass(W, H)
    rp.volume_dataset_changed(synth.dataset(vol))
    rp.transfer_function_changed(texels)
    cam = synth.camera("fill").to_vr_camera()
    _parity(rp, vol, float(vol.min()), float(vol.max()), texels, cam, W, H,
            vr_amd.default_params(shading=1, ert_eps=1e-5))
    rp.close()
