"""CPU: the oracle itself — pinned by closed-form KATs, an independent
float64 restatement (oracle/ref_numpy.py) and the committed golden fixtures."""
import json
import os

import numpy as np
import pytest

import pyoracle
import ref_numpy
import synth
import vr_amd

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_kat_b4_trilinear():
    kat = json.load(open(os.path.join(GOLD, "kat_b4.json")))
    v = np.array(kat["volume_zyx"], np.float32)
    for k in kat["trilinear"]:
        got = pyoracle.trilinear(v, k["pos"])
        assert got == pytest.approx(k["expect"], abs=1e-6), k
        ref = ref_numpy.trilinear(np.pad(v.astype(np.float64), 1), np.array([2, 2, 2.0]),
                                  np.array([k["pos"]], np.float64))[0]
        assert ref == pytest.approx(k["expect"], abs=1e-12), k


def test_kat_b4_tf_decode_before_filter():
    kat = json.load(open(os.path.join(GOLD, "kat_b4.json")))
    tf = np.array(kat["tf_texels"], np.uint32)
    for k in kat["tf"]:
        s = pyoracle.tf_sample(tf, k["t"])
        assert s[:3] == pytest.approx([k["expect_rgb"]] * 3, abs=1e-6), k
        assert s[3] == pytest.approx(k["expect_a"], abs=1e-6)
    # decoding after the lerp would give srgb_to_linear(0.5) ~ 0.214
    assert abs(pyoracle.tf_sample(tf, 0.5)[0] - 0.214) > 0.2


def test_srgb_decode_table():
    tf = np.arange(256, dtype=np.uint32) * 0x00010101 | 0x80000000
    lut = pyoracle.tf_decode(tf)
    c = np.arange(256) / 255.0
    want = np.where(c <= 0.04045, c / 12.92, ((c + 0.055) / 1.055) ** 2.4)
    assert np.allclose(lut[:, 0], want, atol=1e-7)
    assert np.all(lut[:, 3] == np.float32(128) / np.float32(255))


def test_golden_scenes_bit_exact_and_restatement():
    z = np.load(os.path.join(GOLD, "scenes.npz"))
    names = sorted({k.split("/")[0] for k in z.files})
    assert len(names) >= 6
    for n in names:
        W, H = (int(x) for x in z[n + "/size"])
        smin, smax = z[n + "/slice"]
        sc = pyoracle.Scene(z[n + "/vol"], float(z[n + "/vol"].min()), float(z[n + "/vol"].max()),
                            z[n + "/tf"], z[n + "/view"], z[n + "/pos"], W, H, smin=smin, smax=smax,
                            shading=int(z[n + "/shading"]))
        img, st = sc.render()
        assert np.array_equal(img, z[n + "/img"]), n
        assert [st[k] for k in ("rays", "samples", "shaded_samples", "steps")] == list(z[n + "/stats"])
        ref = ref_numpy.render(z[n + "/vol"], float(z[n + "/vol"].min()), float(z[n + "/vol"].max()),
                               z[n + "/tf"], z[n + "/view"], z[n + "/pos"], W, H, smin, smax,
                               shading=bool(int(z[n + "/shading"])))
        d = img.astype(np.float64) - ref
        assert np.sqrt(np.mean(d * d)) < 1e-5 and np.abs(d).max() < 5e-4, n


@pytest.mark.parametrize("camname", ["default", "rotA", "rotB", "fill", "fill_oblique"])
def test_oracle_vs_float64_restatement(camname):
    vol = synth.gaussians_numpy((14, 11, 17), seed=21)
    tf = synth.tf_color()
    cam = synth.camera(camname).to_vr_camera()
    for shading in (0, 1):
        p = vr_amd.default_params(shading=shading)
        sc = pyoracle.Scene.from_params(vol, float(vol.min()), float(vol.max()), tf, cam, 40, 30, p)
        img, _ = sc.render()
        ref = ref_numpy.render(vol, float(vol.min()), float(vol.max()), tf, list(cam.view),
                               list(cam.position), 40, 30, shading=bool(shading))
        d = img.astype(np.float64) - ref
        # float32 position accumulation vs float64: a ray may take one more/less sample at
        # its exit face; one such sample moves a pixel by < 2e-3
        assert np.sqrt(np.mean(d * d)) < 3e-5 and np.abs(d).max() < 2e-3


def test_kat_b1_b2_b3_on_oracle():
    vol = synth.gaussians_numpy((12, 12, 12), seed=1)
    cam = synth.camera("rotA").to_vr_camera()
    p = vr_amd.default_params()
    W, H = 32, 24
    # B2 transparent TF -> clear everywhere
    sc = pyoracle.Scene.from_params(vol, float(vol.min()), float(vol.max()),
                                    np.array([0x00FFFFFF], np.uint32), cam, W, H, p)
    img, st = sc.render()
    assert np.all(img == np.array([0.11, 0.11, 0.11, 1.0], np.float32))
    assert st["rays"] > 0 and st["samples"] > 0
    # B3 startup TF: first in-slab sample is opaque white -> exactly (1,1,1,1) or clear
    sc = pyoracle.Scene.from_params(np.zeros((1, 1, 1), np.float32), 0.0, 1.0, synth.tf0(), cam, W, H, p)
    img, st = sc.render()
    white = np.all(img == 1.0, axis=2)
    clear = np.all(img == np.array([0.11, 0.11, 0.11, 1], np.float32), axis=2)
    # edge-grazing rays with no in-slab sample keep the clear colour
    assert np.all(white | clear) and 0 < white.sum() <= st["rays"]
    assert st["samples"] == white.sum()  # exact ERT at T == 0 after the first sample
    # B1 constant TF: per pixel T = (1-a)^k with k = samples on that ray
    a8 = 64
    tf = np.array([(a8 << 24) | 0x00808080], np.uint32)
    sc = pyoracle.Scene.from_params(vol, float(vol.min()), float(vol.max()), tf, cam, W, H, p)
    img, st = sc.render()
    a = np.float64(np.float32(a8) / np.float32(255))
    alpha = img[..., 3].astype(np.float64)
    # out.a = A^2 - A + 1, A = 1 - (1-a)^k: enumerate k
    kk = np.arange(0, 400)
    Ak = 1 - (1 - a) ** kk
    ak = Ak * Ak - Ak + 1
    c = pyoracle.tf_decode(tf)[0, 0]
    rk = c * Ak * Ak + 0.11 * (1 - Ak)
    best = (np.abs(alpha[..., None] - ak) + np.abs(img[..., 0][..., None] - rk)).argmin(axis=2)
    assert np.allclose(img[..., 0], rk[best], atol=3e-6)
    assert np.allclose(alpha, ak[best], atol=3e-6)


def test_step_count_constant():
    # volume.frag:29-31: int(1.8 / 0.005) in float32 == 360 > max chord sqrt(3)/0.005 = 346.4
    assert int(np.float32(1.8) / np.float32(0.005)) == 360


def test_row_range_rendering_matches_full():
    vol = synth.gaussian_blob(12)
    cam = synth.camera("rotB").to_vr_camera()
    p = vr_amd.default_params(shading=1)
    sc = pyoracle.Scene.from_params(vol, float(vol.min()), float(vol.max()), synth.tf_color(), cam, 30, 20, p)
    full, st = sc.render()
    part, st2 = sc.render(5, 9)
    assert np.array_equal(full[5:9], part[5:9])
    assert np.isnan(part[:5]).all() and np.isnan(part[9:]).all()
    assert st2["samples"] < st["samples"]


def test_u8_voxel_source_equals_float_copy():
    """The oracle's u8 voxel source (used for multi-GiB u8 volumes, e.g. C5) renders exactly
    what the reference's float Dataset of the same voxels renders (float(u8) is exact)."""
    import vr_amd
    rng = np.random.default_rng(4)
    vol = rng.integers(0, 256, size=(13, 11, 9), dtype=np.uint8)
    cam = vr_amd.make_camera(radius=2.0, rotate=(100.0, 60.0)).to_vr_camera()
    for shading in (0, 1):
        p = vr_amd.default_params(shading=shading)
        a, sa = pyoracle.Scene.from_params(vol, 0.0, 255.0, synth.tf_color(), cam, 40, 30, p).render()
        b, sb = pyoracle.Scene.from_params(vol.astype(np.float32), 0.0, 255.0, synth.tf_color(),
                                           cam, 40, 30, p).render()
        assert np.array_equal(a, b) and sa == sb


def test_round_f16_is_ieee_binary16():
    """oracle.c or_round_f16 (the device's f32 -> binary16 conversion of the difference field,
    DESIGN.md §3) equals IEEE binary16 round-to-nearest-even (numpy's float16), subnormals,
    ties and the largest finite value included."""
    rng = np.random.default_rng(3)
    mags = 10.0 ** rng.uniform(-9, 4.8, 60000)
    xs = (rng.choice([-1.0, 1.0], mags.size) * mags).astype(np.float32)
    ties = (np.arange(1, 3000, dtype=np.float32) + np.float32(0.5)) * np.float32(2.0 ** -24)
    edge = np.array([0.0, -0.0, 65504.0, -65504.0, 65503.9, 2.0 ** -14, 2.0 ** -24, 2.0 ** -25,
                     3 * 2.0 ** -26, 1.0 + 2.0 ** -11, 1.0 + 3 * 2.0 ** -11, 6.1e-5], np.float32)
    xs = np.concatenate([xs[np.abs(xs) <= 65504], ties, edge])
    got = np.array([pyoracle.round_f16(float(x)) for x in xs], np.float32)
    want = xs.astype(np.float16).astype(np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert np.isnan(pyoracle.round_f16(float("nan")))


def test_field_scale_log2_matches_the_library():
    """The binary16 field's scale exponent: the oracle's restatement equals the library's
    field_scale_log2 (vr_internal.h, compiled here on the host) and the definition."""
    import subprocess
    import tempfile
    pairs = [(0.0, 1.0), (-1000.0, 3000.0), (0.0, 0.0), (0.0, 255.0), (-128.0, 127.0),
             (0.0, 65504.0), (0.0, 65505.0), (1e-7, 3e-7), (-1e30, 1e30), (5.0, 5.0),
             (-3.5, -1.25), (0.0, 1e-30), (0.0, float("inf")), (2.0, 1.0)]
    src = ('#include "vr_internal.h"\n#include <cstdio>\nint main(){float p[][2]={'
           + ",".join("{%s,%s}" % tuple("INFINITY" if v == float("inf") else f"{v!r}f" for v in ab)
                      for ab in pairs)
           + '};for(auto&q:p)std::printf("%d\\n",vr::field_scale_log2(q[0],q[1]));}\n')
    csrc = os.path.join(os.path.dirname(vr_amd.__file__), "csrc")
    with tempfile.TemporaryDirectory() as d:
        with open(os.path.join(d, "t.cpp"), "w") as f:
            f.write(src)
        subprocess.run(["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-std=c++17",
                        "-I", csrc, os.path.join(d, "t.cpp"), "-o", os.path.join(d, "t")],
                       check=True, capture_output=True)
        lib_k = [int(x) for x in subprocess.run([os.path.join(d, "t")], capture_output=True,
                                                text=True, check=True).stdout.split()]
    for (a, b), k in zip(pairs, lib_k):
        assert pyoracle.field_scale_log2(a, b) == k, (a, b)
        B = max(b, 0.0) - min(a, 0.0)
        if B > 0 and np.isfinite(B) and B * 2.0 ** -120 <= 65504 and B * 2.0 ** 120 > 65504:
            assert B * 2.0 ** k <= 65504 < B * 2.0 ** (k + 1), (a, b, k)


@pytest.mark.parametrize("scale", [1.0, 4000.0, 1e-6])
def test_oracle_binary16_gradient_mode(scale):
    """oracle.c's binary16 field mode (grad_f16) against the independent float64 restatement of
    the same rounding (ref_numpy grad_f16, numpy float16), and against the exact mode: within
    the parity tolerance, and not identical."""
    vol = (synth.gaussians_numpy((14, 11, 17), seed=21) * scale).astype(np.float32)
    vmin, vmax = float(vol.min()), float(vol.max())
    tf = synth.tf_color()
    cam = synth.camera("fill_oblique").to_vr_camera()
    p = vr_amd.default_params(shading=1)
    h, _ = pyoracle.Scene.from_params(vol, vmin, vmax, tf, cam, 40, 30, p, grad_f16=True).render()
    x, _ = pyoracle.Scene.from_params(vol, vmin, vmax, tf, cam, 40, 30, p).render()
    ref = ref_numpy.render(vol, vmin, vmax, tf, list(cam.view), list(cam.position), 40, 30,
                           shading=True, grad_f16=True)
    d = h.astype(np.float64) - ref
    assert np.sqrt(np.mean(d * d)) < 3e-5 and np.abs(d).max() < 2e-3
    e = h.astype(np.float64) - x
    assert np.sqrt(np.mean(e * e)) <= 1e-4 and np.abs(e).max() <= 2e-3
    assert not np.array_equal(h, x)
