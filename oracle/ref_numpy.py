"""Independent float64 numpy restatement of the reference ray-march — TEST INFRASTRUCTURE ONLY.

Written directly from the reference sources, not from oracle.c, to cross-check the C oracle:
  res/shaders/volume.frag:21-52            loop, strict slab test, composite
  src/rendering/offscreen_pass.cpp:1152-1171 perspectiveRH(40 deg, W/H, 0.1, 10) * Rx(90) * S(-1,1,1)
  offscreen_pass.cpp:1014-1039 / :1125-1150 border trilinear / clamp-to-edge sRGB TF
  offscreen_pass.cpp:715-725, :170-173      blend over the clear colour
Everything is float64 (camera, rays, accumulation), so agreement with the float32 C oracle is
to rounding (tests/test_oracle.py states the tolerance), not bit-exact.
"""
from __future__ import annotations

import numpy as np


def projection(width, height, fovy_deg=40.0, zn=0.1, zf=10.0):
    f = np.radians(fovy_deg)
    aspect = width / height
    th = np.tan(f / 2)
    P = np.zeros((4, 4))
    P[0, 0] = 1 / (aspect * th)
    P[1, 1] = 1 / th
    P[2, 2] = -(zf + zn) / (zf - zn)
    P[3, 2] = -1.0
    P[2, 3] = -(2 * zf * zn) / (zf - zn)
    Rx = np.eye(4)  # rotate 90 deg about x (exact)
    Rx[1, 1], Rx[1, 2], Rx[2, 1], Rx[2, 2] = 0.0, -1.0, 1.0, 0.0
    S = np.diag([-1.0, 1.0, 1.0, 1.0])
    return P @ Rx @ S


def srgb_to_linear(c):
    c = np.asarray(c, dtype=np.float64)
    return np.where(c <= 0.04045, c / 12.92, ((c + 0.055) / 1.055) ** 2.4)


def decode_tf(tf):
    tf = np.asarray(tf, dtype=np.uint64)
    r = (tf & 0xFF) / 255.0
    g = ((tf >> 8) & 0xFF) / 255.0
    b = ((tf >> 16) & 0xFF) / 255.0
    a = ((tf >> 24) & 0xFF) / 255.0
    return np.stack([srgb_to_linear(r), srgb_to_linear(g), srgb_to_linear(b), a], axis=1)


def trilinear(volp, N, pos):
    """volp: volume zero-padded by 1 on every side, shape (nz+2, ny+2, nx+2); pos (n,3) in [0,1]."""
    u = pos * N - 0.5
    i0 = np.floor(u)
    a = u - i0
    i = i0.astype(np.int64) + 1  # padded index
    x, y, z = i[:, 0], i[:, 1], i[:, 2]
    ax, ay, az = a[:, 0], a[:, 1], a[:, 2]
    v = lambda dx, dy, dz: volp[z + dz, y + dy, x + dx]
    c00 = v(0, 0, 0) * (1 - ax) + v(1, 0, 0) * ax
    c10 = v(0, 1, 0) * (1 - ax) + v(1, 1, 0) * ax
    c01 = v(0, 0, 1) * (1 - ax) + v(1, 0, 1) * ax
    c11 = v(0, 1, 1) * (1 - ax) + v(1, 1, 1) * ax
    c0 = c00 * (1 - ay) + c10 * ay
    c1 = c01 * (1 - ay) + c11 * ay
    return c0 * (1 - az) + c1 * az


def tf_sample(lut, t):
    n = lut.shape[0]
    u = np.clip(t * n - 0.5, -1.0, float(n))
    u = np.where(np.isnan(u), -1.0, u)
    f = np.floor(u)
    w = (u - f)[:, None]
    i0 = np.clip(f.astype(np.int64), 0, n - 1)
    i1 = np.clip(f.astype(np.int64) + 1, 0, n - 1)
    return lut[i0] * (1 - w) + lut[i1] * w


def render(vol, vmin, vmax, tf, view, cam_pos, width, height, smin=(0, 0, 0), smax=(1, 1, 1),
           step=0.005, ray_dist=1.8, clear=(0.11, 0.11, 0.11, 1.0), shading=False,
           ka=0.3, kd=0.7, ks=0.25, spec_power=16, grad_f16=False):
    """grad_f16: the device's binary16 difference field (vr_params.exact_gradient = 0): each
    per-voxel central difference D (float32) becomes float16(clip(D * 2^k, +-65504)), numpy's
    round-to-nearest-even, k the largest power of two with (max(vmax,0) - min(vmin,0)) 2^k <=
    65504 -- restated here independently of oracle.c's or_round_f16."""
    vol32 = np.asarray(vol, dtype=np.float32)
    vol = np.asarray(vol, dtype=np.float64)
    nz, ny, nx = vol.shape
    N = np.array([nx, ny, nz], dtype=np.float64)
    volp = np.pad(vol, 2)  # 2 zero layers: index shift +2 below
    V = np.asarray(view, dtype=np.float64).reshape(4, 4).T  # column-major -> row-major
    PV = projection(width, height) @ V
    inv = np.linalg.inv(PV)
    px, py = np.meshgrid(np.arange(width), np.arange(height))
    x = (px.ravel() + 0.5) / width * 2 - 1
    y = (py.ravel() + 0.5) / height * 2 - 1
    h0 = inv @ np.stack([x, y, np.zeros_like(x), np.ones_like(x)])
    h1 = inv @ np.stack([x, y, np.ones_like(x), np.ones_like(x)])
    p0 = (h0[:3] / h0[3]).T
    d = (h1[:3] / h1[3]).T - p0
    with np.errstate(divide="ignore", invalid="ignore"):
        t1 = (-0.5 - p0) / d
        t2 = (0.5 - p0) / d
    lo = np.minimum(t1, t2)
    hi = np.maximum(t1, t2)
    te = lo.max(axis=1)
    tx = hi.min(axis=1)
    covered = (te < tx) & (te >= 0) & (te <= 1)
    entry = p0 + te[:, None] * d
    cam = np.asarray(cam_pos, dtype=np.float64)
    dirs = entry - cam
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    pos = entry + 0.5
    axis = lo.argmax(axis=1)  # entry face: its coordinate is exactly 0 or 1
    rows = np.arange(pos.shape[0])
    pos[rows, axis] = np.where(d[rows, axis] > 0, 0.0, 1.0)
    lut = decode_tf(tf)
    smin = np.asarray(smin, np.float64)
    smax = np.asarray(smax, np.float64)

    dfield = None
    if grad_f16:
        B = max(float(vmax), 0.0) - min(float(vmin), 0.0)
        k = 0
        if B > 0 and np.isfinite(B):
            while k > -120 and B * 2.0 ** k > 65504.0:
                k -= 1
            while k < 120 and B * 2.0 ** (k + 1) <= 65504.0:
                k += 1
        vp32 = np.pad(vol32, 3)  # D at padded index + 2 needs one more layer
        dfield = []
        for ax_ in range(3):
            sl_p = [slice(1, -1)] * 3
            sl_m = [slice(1, -1)] * 3
            # numpy axes (z, y, x): volume axis ax_ is numpy axis 2 - ax_
            sl_p[2 - ax_] = slice(2, None)
            sl_m[2 - ax_] = slice(0, -2)
            D = (vp32[tuple(sl_p)] - vp32[tuple(sl_m)]).astype(np.float32) * np.float32(2.0 ** k)
            D = np.where(np.isnan(D), D, np.clip(D, -65504.0, 65504.0)).astype(np.float32)
            dfield.append(D.astype(np.float16).astype(np.float64))

    n = pos.shape[0]
    T = np.ones(n)
    Cc = np.zeros((n, 3))
    alive = covered.copy()
    for _ in range(int(np.float32(ray_dist) / np.float32(step))):
        inb = np.all((pos <= 1) & (pos >= 0), axis=1)
        alive &= inb
        if not alive.any():
            break
        slab = alive & np.all((pos < smax) & (pos > smin), axis=1)
        idx = np.nonzero(slab)[0]
        if idx.size:
            p = pos[idx]
            u = p * N - 0.5
            i0 = np.floor(u).astype(np.int64) + 2
            a = u - np.floor(u)

            def cell(ii, src=None):
                src = volp if src is None else src
                xx, yy, zz = ii[:, 0], ii[:, 1], ii[:, 2]
                ax, ay, az = a[:, 0], a[:, 1], a[:, 2]
                v = lambda dx, dy, dz: src[zz + dz, yy + dy, xx + dx]
                c00 = v(0, 0, 0) * (1 - ax) + v(1, 0, 0) * ax
                c10 = v(0, 1, 0) * (1 - ax) + v(1, 1, 0) * ax
                c01 = v(0, 0, 1) * (1 - ax) + v(1, 0, 1) * ax
                c11 = v(0, 1, 1) * (1 - ax) + v(1, 1, 1) * ax
                return (c00 * (1 - ay) + c10 * ay) * (1 - az) + (c01 * (1 - ay) + c11 * ay) * az

            dens = cell(i0)
            with np.errstate(divide="ignore", invalid="ignore"):
                t = (dens - vmin) / (vmax - vmin)
            s = tf_sample(lut, t)
            rgb = s[:, :3].copy()
            alpha = s[:, 3]
            if shading:
                g = np.zeros((idx.size, 3))
                for ax_ in range(3):
                    e = np.zeros(3, np.int64)
                    e[ax_] = 1
                    if grad_f16:
                        g[:, ax_] = cell(i0, dfield[ax_]) * N[ax_]
                    else:
                        g[:, ax_] = (cell(i0 + e) - cell(i0 - e)) * N[ax_]
                g2 = (g * g).sum(axis=1)
                ok = (alpha > 0) & (g2 > 0)
                with np.errstate(divide="ignore", invalid="ignore"):
                    ndl = np.abs((g * dirs[idx]).sum(axis=1) / np.sqrt(g2))
                shade = ka + kd * ndl
                spec = ks * ndl ** spec_power
                rgb = np.where(ok[:, None], rgb * shade[:, None] + spec[:, None], rgb)
            Cc[idx] += (rgb * alpha[:, None]) * T[idx, None]
            T[idx] *= (1 - alpha)
        pos = pos + dirs * step
    A = 1 - T
    out = np.empty((n, 4))
    out[:, :3] = Cc * A[:, None] + np.asarray(clear[:3]) * (1 - A)[:, None]
    out[:, 3] = A * A + clear[3] * (1 - A)
    out[~covered] = np.asarray(clear)
    return out.reshape(height, width, 4)
