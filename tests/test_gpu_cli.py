"""GPU: the headless C++ CLI (host/vr_cli.cpp over include/vr/offscreen_pass_hip.hpp, the
reference-shaped C++ shim) renders exactly the frame the ctypes path renders, for a
synthetic volume and for an NRRD file, with and without empty-space skipping."""
import os
import subprocess

import numpy as np
import pytest

import synth
import vr_amd

pytestmark = pytest.mark.gpu

CLI = os.path.join(os.path.dirname(vr_amd.LIB_PATH), "vr_cli")


def read_ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(b"\n", 3)
    assert parts[0] == b"P6" and parts[2] == b"255"
    w, h = (int(x) for x in parts[1].split())
    return np.frombuffer(parts[3], np.uint8).reshape(h, w, 3)


def run_cli(*args):
    r = subprocess.run([CLI, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout


@pytest.mark.parametrize("skip,mask", [(False, None), (True, None), (False, "0x1")])
def test_cli_synthetic_matches_ctypes(gpu, tmp_path, skip, mask):
    W, H = 96, 64
    out = str(tmp_path / "f.ppm")
    args = ["synthetic:40", out, "--size", f"{W}x{H}", "--radius", "2", "--rotate", "100,60",
            "--tf", "demo", "--shading"]
    run_cli(*args, *(["--skip-empty"] if skip else []), *(["--device-mask", mask] if mask else []))
    img = read_ppm(out)
    rp = vr_amd.OffscreenPass(W, H)
    rp.generate_volume((40, 40, 40), np.float32, seed=2024)
    rp.transfer_function_changed(synth.tf2())
    cam = vr_amd.make_camera(radius=2.0, rotate=(100.0, 60.0)).to_vr_camera()
    ref = rp.render(cam, vr_amd.default_params(shading=1), vr_amd.OUT_RGBA8)
    rp.close()
    assert np.array_equal(img, ref[..., :3])


def test_cli_nrrd_file_matches_ctypes(gpu, tmp_path):
    W, H = 80, 72
    vol = (synth.gaussians_numpy((24, 20, 28), seed=4) * 9000).astype(np.uint16)
    path = str(tmp_path / "v.nhdr")
    vr_amd.write_nrrd_raw(path, vol)
    out = str(tmp_path / "f.ppm")
    run_cli(path, out, "--size", f"{W}x{H}", "--radius", "1.6", "--tf", "demo")
    img = read_ppm(out)
    rp = vr_amd.OffscreenPass(W, H)
    rp.volume_dataset_changed(vr_amd.load_nrrd(path))
    rp.transfer_function_changed(synth.tf2())
    ref = rp.render(vr_amd.make_camera(radius=1.6).to_vr_camera(), vr_amd.default_params(),
                    vr_amd.OUT_RGBA8)
    rp.close()
    assert np.array_equal(img, ref[..., :3])
