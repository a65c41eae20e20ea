"""GPU: randomized parity sweep.  Seeded random scenes over the whole parameter space -- volume
dims (odd, anisotropic, single-brick and multi-brick), element types, camera orbits and radii
(including inside the near-clip range), TFs, slicing boxes, shading, ERT, empty-space skipping,
work placement, frames in flight (kernel choice), frame sizes up to 320x300 (host readback in row bands) -- each rendered by the
HIP kernel and checked against the CPU oracle: within the documented tolerance (RMSE <= 1e-4,
max <= 2e-3), then bit for bit, with exact work counters.  Seeds 64-119 render frames of >= 256 rows
(vr_render's row bands with overlapped readback); seeds 120-279 multi-brick volumes of 48-130
voxels per axis, where oblique and sparse views read the alternative brick copies and shaded f32
dense-row views the binary16 difference field."""
import numpy as np
import pytest

import pyoracle
import synth
import vr_amd

pytestmark = pytest.mark.gpu

DTYPES = [np.float32, np.uint8, np.uint16, np.int16, np.int8, np.float64, np.int32]


def scene(seed):
    rng = np.random.default_rng(1000 + seed)
    big = seed >= 120  # multi-brick volumes: the alternative copies and the difference field
    dims = tuple(int(x) for x in rng.integers(48, 131, size=3)) if big else \
        tuple(int(x) for x in rng.integers(3, 41, size=3))
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
    if big and rng.random() < 0.5:  # axis-aligned: the default, side and top views (sparse
        # at small frames: more than 0.8 voxels per pixel step)
        rot = [(0.0, 0.0), (360.0, 0.0), (0.0, 360.0)][int(rng.integers(0, 3))]
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
                              tile_order=int(rng.integers(0, 4)),
                              frames_in_flight=int(rng.integers(0, 4)))
    W, H = int(rng.integers(24, 97)), int(rng.integers(16, 81))
    if seed >= 64:  # frames of >= 256 rows: vr_render's row bands with overlapped readback
        W, H = int(rng.integers(200, 321)), int(rng.integers(256, 300))
    if big:
        W, H = int(rng.integers(40, 257)), int(rng.integers(32, 200))
    return vol, tf, cam, sl, p, W, H


KERNELS = {}  # march kernel name -> seeds that ran it (the sweep's layout coverage)


@pytest.fixture(scope="module")
def rp(gpu):
    r = vr_amd.OffscreenPass(32, 32)
    yield r
    r.close()


@pytest.mark.parametrize("seed", range(280))
def test_random_scene_matches_oracle(rp, seed):
    vol, tf, cam, (smin, smax), p, W, H = scene(seed)
    rp.framebuffer_size_changed(W, H)
    ds = synth.dataset(vol)
    rp.volume_dataset_changed(ds)
    rp.transfer_function_changed(tf)
    rp.slicing_changed(smin, smax)
    img = rp.render(cam, p, vr_amd.OUT_RGBA32F)
    # a shaded f32 frame that reads the binary16 difference field: the oracle restates its
    # rounding (kernel tag F32H); every other frame is the exact f32 restatement
    kname = rp.kernel_name(p)
    KERNELS.setdefault(kname, []).append(seed)
    half = "F32H" in kname
    sc = pyoracle.Scene.from_params(vol.astype(np.float32), ds.vmin, ds.vmax, tf, cam, W, H, p,
                                    smin, smax, grad_f16=half)
    ref, st = sc.render()
    d = img.astype(np.float64) - ref
    rmse, mx = float(np.sqrt(np.mean(d * d))), float(np.abs(d).max())
    assert rmse <= 1e-4 and mx <= 2e-3, f"seed {seed}: rmse {rmse:.3e} max {mx:.3e}"
    # and bit for bit: the kernel performs the oracle's IEEE operations in the same order
    assert np.array_equal(img, ref.astype(np.float32)), \
        f"seed {seed}: {int((img != ref.astype(np.float32)).any(axis=-1).sum())} pixels differ"
    cw = rp.count_work(cam, p)
    # the oracle never skips: its samples are the kernel's fetched + skipped samples
    assert cw["rays"] == st["rays"] and cw["steps"] == st["steps"]
    assert cw["shaded_samples"] == st["shaded_samples"]
    assert cw["samples"] + cw["skipped_samples"] == st["samples"]
    if not p.skip_empty:
        assert cw["skipped_samples"] == 0
    rp.slicing_changed((0, 0, 0), (1, 1, 1))


def test_random_sweep_covered_the_layouts():
    """Runs after the sweep: the scenes reached every f32 brick copy the launch policy picks, the
    binary16 field and the
    8-bit yz-quads (plain 8-bit bricks start at 2^25 voxels, past the oracle's budget here:
    test_byte_layouts_plain_and_quad_identical renders them)."""
    names = "\n".join(f"{k}: {len(v)}" for k, v in sorted(KERNELS.items()))
    print(names)
    for tag in ("vr::F32H", "vr::F32Alt", "vr::F32S", "vr::F32P", "Quad8<unsigned char>"):
        assert any(tag in k for k in KERNELS), f"no scene ran {tag}:\n{names}"
