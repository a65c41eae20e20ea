"""Synthetic inputs of BASELINE.json's configurations — test/bench data only.

Volumes (numpy, (nz, ny, nx), x fastest, Dataset semantics):
  C1 gaussian_blob(64):  f32, v = exp(-|p-c|^2 / (2 sigma^2)), c = 31.5, sigma = 64/6
  C2 ct_head(256):       u8 ellipsoidal skull shell 200-255 + soft tissue 60-100 + 3 Gaussian
                         "ventricles" (low) + uniform noise +-8, seed 1234
  C3 gaussians(512):     f32 sum of 32 Gaussians + 0.05 value noise — generated ON DEVICE by
                         vr_generate_volume(kind 0, seed 2024); `gaussians_numpy` restates that
                         generator for small sizes (tests)
Transfer functions (via the Gradient restatement, exactly as the reference UI produces them):
  TF-0 startup 1-texel 0xFFFFFFFF (offscreen_pass.cpp:119)
  TF-1 default Gradient().discretize(256) (opaque black->white ramp)
  TF-2 black->white, alpha markers (0,0) (0.14,0) (1,1) (the demo GIF's TF)
Cameras: default (r = 3, q = 180 deg about z), rotate((100,60)) at r = 2, rotate((-300,-150))
at r = 2, frame-filling r = 1.6.
"""
from __future__ import annotations

import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(_HERE), "volumetric-renderer_amd"))
import vr_amd  # noqa: E402


def gaussian_blob(n=64):
    c = (n - 1) / 2.0
    sigma = n / 6.0
    i = np.arange(n, dtype=np.float64)
    g = np.exp(-((i - c) ** 2) / (2 * sigma * sigma))
    v = g[:, None, None] * g[None, :, None] * g[None, None, :]
    return v.astype(np.float32)


def ct_head(n=256, seed=1234):
    rng = np.random.default_rng(seed)
    ax = (np.arange(n, dtype=np.float32) + 0.5) / n * 2 - 1  # [-1, 1]
    z, y, x = np.meshgrid(ax, ax, ax, indexing="ij")
    r_outer = np.sqrt((x / 0.80) ** 2 + (y / 0.92) ** 2 + (z / 0.85) ** 2)
    r_inner = np.sqrt((x / 0.72) ** 2 + (y / 0.84) ** 2 + (z / 0.77) ** 2)
    vol = np.zeros((n, n, n), np.float32)
    soft = r_inner < 1.0
    vol[soft] = 60 + 40 * (1 - r_inner[soft])
    skull = (r_outer < 1.0) & (r_inner >= 1.0)
    vol[skull] = 200 + 55 * np.clip((1 - r_outer[skull]) * 8, 0, 1)
    for cx, cy, cz, s in ((-0.2, 0.1, 0.1, 0.12), (0.2, 0.1, 0.1, 0.12), (0.0, -0.25, -0.05, 0.09)):
        d2 = (x - cx) ** 2 + (y - cy) ** 2 + (z - cz) ** 2
        vol -= 50 * np.exp(-d2 / (2 * s * s)) * soft
    vol += rng.uniform(-8, 8, size=vol.shape).astype(np.float32)
    return np.clip(np.rint(vol), 0, 255).astype(np.uint8)


def _splitmix_uniforms(seed, count):
    """splitmix64 -> floats in [0,1), as vr_api.hip SplitMix (float32 arithmetic)."""
    s = seed & 0xFFFFFFFFFFFFFFFF
    out = []
    M = 0xFFFFFFFFFFFFFFFF
    for _ in range(count):
        s = (s + 0x9E3779B97F4A7C15) & M
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z = z ^ (z >> 31)
        out.append(np.float32(z >> 40) * np.float32(1.0 / 16777216.0))
    return out


def gaussian_params(dims, seed, ng=32):
    """(ng, 5) float32: cx, cy, cz, k = 1/(2 sigma^2), amp in voxel units (vr_generate_volume)."""
    u = iter(_splitmix_uniforms(seed, ng * 5))
    d = [np.float32(x) for x in dims]
    nmin = min(d)
    prm = []
    for _ in range(ng):
        c = [d[a] * (np.float32(0.15) + np.float32(0.7) * next(u)) for a in range(3)]
        sigma = nmin * (np.float32(0.04) + np.float32(0.10) * next(u))
        k = np.float32(1.0) / (np.float32(2.0) * sigma * sigma)
        amp = np.float32(0.3) + np.float32(0.7) * next(u)
        prm.append(c + [k, amp])
    return np.array(prm, dtype=np.float32)


def hash01(x, y, z):
    x = x.astype(np.uint32)
    y = y.astype(np.uint32)
    z = z.astype(np.uint32)
    with np.errstate(over="ignore"):
        h = (x * np.uint32(73856093)) ^ (y * np.uint32(19349663)) ^ (z * np.uint32(83492791))
        h ^= h >> np.uint32(13)
        h *= np.uint32(0x5BD1E995)
        h ^= h >> np.uint32(15)
    return (h & np.uint32(0xFFFFFF)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def gaussians_numpy(dims, seed=2024, dtype=np.float32):
    """Restatement of vr_generate_volume kind 0 (float64 exp: agrees to ~1e-6 relative)."""
    nx, ny, nz = dims
    prm = gaussian_params(dims, seed)
    z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    acc = np.zeros((nz, ny, nx), np.float64)
    for cx, cy, cz, k, amp in prm.astype(np.float64):
        acc += amp * np.exp(-k * ((x - cx) ** 2 + (y - cy) ** 2 + (z - cz) ** 2))
    acc += 0.05 * hash01(x, y, z)
    scale = {np.dtype(np.float32): 1.0, np.dtype(np.uint8): 160.0, np.dtype(np.uint16): 40000.0}[np.dtype(dtype)]
    v = acc * scale
    if np.dtype(dtype) == np.float32:
        return v.astype(np.float32)
    hi = 255 if np.dtype(dtype) == np.uint8 else 65535
    return np.clip(np.rint(v), 0, hi).astype(dtype)


def dataset(vol):
    v = vol.astype(np.float32)
    return vr_amd.Dataset((vol.shape[2], vol.shape[1], vol.shape[0]), float(v.min()), float(v.max()), vol)


# ---- transfer functions ----
def tf0():
    return np.array([0xFFFFFFFF], dtype=np.uint32)


def tf1():
    return vr_amd.Gradient().discretize(256)


def tf2():
    g = vr_amd.Gradient()
    g.set_alpha_marker(0, 0.0, 0.0)           # first marker's opacity 100% -> 0%
    i = g.add_alpha_marker(0.14, g.sample(0.14)[3])
    g.set_alpha_marker(i, 0.14, 0.0)
    return g.discretize(256)


def tf_color():
    """A coloured TF with partial opacity everywhere (exercises every channel)."""
    g = vr_amd.Gradient()
    g.set_color_marker(0, 0.0, (0.1, 0.2, 0.9))
    g.set_color_marker(1, 1.0, (1.0, 0.9, 0.2))
    i = g.add_color_marker(0.5, (0.9, 0.1, 0.1))
    g.set_color_marker(i, 0.5, (0.9, 0.1, 0.1))
    g.set_alpha_marker(0, 0.0, 0.02)
    g.set_alpha_marker(1, 1.0, 0.35)
    return g.discretize(256)


def tf_band(lo=0.3, hi=0.8, n=256):
    """Coloured TF, opaque only inside [lo, hi] (alpha exactly 0 outside): empty-space skipping
    has transparent texels on BOTH sides of the visible band."""
    t = (np.arange(n) + 0.5) / n
    r = np.round(255 * t).astype(np.uint32)
    g = np.round(255 * (1 - t)).astype(np.uint32)
    b = np.full(n, 160, np.uint32)
    a = np.where((t >= lo) & (t <= hi), np.round(255 * np.sin(np.pi * (t - lo) / (hi - lo)) ** 2), 0)
    return (r | (g << 8) | (b << 16) | (a.astype(np.uint32) << 24)).astype(np.uint32)


TFS = {"tf0": tf0, "tf1": tf1, "tf2": tf2, "tfc": tf_color, "tfband": tf_band}


# ---- cameras ----
CAMERAS = {
    "default": dict(radius=3.0, rotate=None),
    "rotA": dict(radius=2.0, rotate=(100.0, 60.0)),
    "rotB": dict(radius=2.0, rotate=(-300.0, -150.0)),
    "fill": dict(radius=1.6, rotate=None),
    "fill_oblique": dict(radius=1.6, rotate=(40.0, 25.0)),
    # the diagonal view of the view sweeps (tools/view_sweep.py): rays cross brick rows and slabs
    "diag": dict(radius=2.0, rotate=(180.0, 140.0)),
    # the near plane (0.198 in glm's [-1, 1] clip form) cuts the cube's front face
    "near": dict(radius=0.65, rotate=None),
}


def camera(name):
    return vr_amd.make_camera(**CAMERAS[name])
