"""GPU: randomized parity sweep.  Seeded random scenes over the whole parameter space -- volume
dims (odd, anisotropic, single-brick and multi-brick), element types, camera orbits and radii
(including inside the near-clip range), TFs, slicing boxes, shading, ERT, empty-space skipping,
work placement, frame sizes up to 320x300 (host readback in row bands) -- each rendered by the
HIP kernel and checked against the CPU oracle with the documented tolerance (RMSE <= 1e-4,
max <= 2e-3) and exact work counters."""
import numpy as np
import pytest

import pyoracle
import synth
import vr_amd

pytestmark = pytest.mark.gpu

DTYPES = [np.float32, np.uint8, np.uint16, np.int16, np.int8, np.float64, np.int32]


def scene(seed):
    rng = np.random.default_rng(1000 + seed)
    dims = tuple(int(x) for x in rng.integers(3, 41, size=3))
    base = synth.gaussians_numpy(dims[::-1], seed=seed)
    dt = DTYPES[seed % len(DTYPES)]
    if np.issubdtype(dt, np.integer):
        info = np.iinfo(dt)
        lo, hi = max(info.min, -3000), min(info.max, 50000)
        vol = (lo + base / base.max() * (hi - lo)).round().astype(dt)
    else:
        vol = (base * rng.uniform(0.5, 20.0) - rng.uniform(0, 1)).astype(dt)
    tf = [synth.tf0, synth.tf1, synth.tf2, synth.tf_color, synth.tf_band][seed % 5]()
    radius = float(rng.choice([0.9, 1.3, 1.6, 2.2, 3.5]))
    rot = (float(rng.uniform(-400, 400)), float(rng.uniform(-400, 400)))
    cam = vr_amd.make_camera(radius=radius, rotate=rot).to_vr_camera()
    if rng.random() < 0.4:
        a = rng.uniform(0.0, 0.45, size=3)
        b = rng.uniform(0.55, 1.0, size=3)
        sl = (tuple(float(x) for x in a), tuple(float(x) for x in b))
    else:
        sl = ((0.0, 0.0, 0.0), (1.0, 1.0, 1.0))
    p = vr_amd.default_params(shading=int(rng.random() < 0.5),
                              ert_eps=float(rng.choice([0.0, 0.0, 1e-5, 1e-3])),
                              skip_empty=int(rng.random() < 0.5),
                              wave_shape=int(rng.integers(0, 4)),
                              tile_order=int(rng.integers(0, 4)))
    W, H = int(rng.integers(24, 97)), int(rng.integers(16, 81))
    if seed >= 64:  # frames of >= 256 rows: vr_render's row bands with overlapped readback
        W, H = int(rng.integers(200, 321)), int(rng.integers(256, 300))
    return vol, tf, cam, sl, p, W, H


@pytest.fixture(scope="module")
def rp(gpu):
    r = vr_amd.OffscreenPass(32, 32)
    yield r
    r.close()


@pytest.mark.parametrize("seed", range(72))
def test_random_scene_matches_oracle(rp, seed):
    vol, tf, cam, (smin, smax), p, W, H = scene(seed)
    rp.framebuffer_size_changed(W, H)
    ds = synth.dataset(vol)
    rp.volume_dataset_changed(ds)
    rp.transfer_function_changed(tf)
    rp.slicing_changed(smin, smax)
    img = rp.render(cam, p, vr_amd.OUT_RGBA32F)
    sc = pyoracle.Scene.from_params(vol.astype(np.float32), ds.vmin, ds.vmax, tf, cam, W, H, p,
                                    smin, smax)
    ref, st = sc.render()
    d = img.astype(np.float64) - ref
    rmse, mx = float(np.sqrt(np.mean(d * d))), float(np.abs(d).max())
    assert rmse <= 1e-4 and mx <= 2e-3, f"seed {seed}: rmse {rmse:.3e} max {mx:.3e}"
    cw = rp.count_work(cam, p)
    # the oracle never skips: its samples are the kernel's fetched + skipped samples
    assert cw["rays"] == st["rays"] and cw["steps"] == st["steps"]
    assert cw["shaded_samples"] == st["shaded_samples"]
    assert cw["samples"] + cw["skipped_samples"] == st["samples"]
    if not p.skip_empty:
        assert cw["skipped_samples"] == 0
    rp.slicing_changed((0, 0, 0), (1, 1, 1))
