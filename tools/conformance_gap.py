"""How far can a conformant Vulkan run of the reference move a pixel away from the oracle?

CPU only (oracle/liboracle.so; TEST/MEASUREMENT INFRASTRUCTURE).  The oracle fixes several
implementation-defined freedoms of the reference's Vulkan pipeline by choice.  Each is restated
as a variant of `or_render_rows` (oracle.h `conf_weight_bits` / `OR_CONF_*`):

  w8 / w4   LINEAR-filter texel coordinates (3D volume and 1D TF) on a 2^-8 / 2^-4 grid:
            subTexelPrecisionBits, typical hardware / the spec minimum
            (samplers: /root/reference/src/rendering/offscreen_pass.cpp:1014-1039,1125-1150)
  fma       FMA contraction of ray_pos += ray_dir*step_size and C.rgb += (rgb*a)*T, which the
            SPIR-V permits (no NoContraction; res/shaders/volume.frag:44-47,
            tests/test_spirv_facts.py)
  clip_zo   glm's [0, 1] clip form (offscreen_pass.cpp:3,1166)
  raster    entry attributes from a rasteriser model (float clip coordinates, 8-bit sub-pixel
            snapping, float perspective-correct barycentrics) instead of the exact intersection
  gpu_math  d*rcp(range) and v*rsqrt(dot(v,v)) for the shader's division and normalize()
  conf8     w8 + fma + raster + gpu_math: one plausible conformant implementation
  conf4     w4 + fma + raster + gpu_math: the same at the spec-minimum filter precision

Each is compared with the oracle (all variants off), over every pixel x 4 channels of the
float RGBA after the blend and of the RGBA8 output:
  rmse, max |d|, RGBA8 max LSB, fraction of pixels whose RGBA8 differs, covered-ray delta.

Scenes (BASELINE.json configs, reference semantics = no shading, no ERT, TF-2):
  C1 64^3 f32 @ 256^2 (fill camera r = 1.6), C2 256^3 u8 CT head @ 1024^2 (fill),
  C3 512^3 f32 @ 1920x1080 at r = 1.6 and at the reference's default camera (r = 3), and the
  headline C3 (Phong + ERT 1e-5, exact f32 gradient) at r = 1.6; plus C1 with the camera 0.15
  from the cube (r = 0.65), where the near plane cuts it and the clip form decides coverage.

Usage: python tools/conformance_gap.py [--out profiles/r04/conformance] [--scenes c1,c2,...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("oracle", "tools", "volumetric-renderer_amd"):
    sys.path.insert(0, os.path.join(ROOT, sub))
import pyoracle  # noqa: E402
import synth  # noqa: E402
import vr_amd  # noqa: E402

F, Z, R, G = pyoracle.CONF_FMA, pyoracle.CONF_CLIP_ZO, pyoracle.CONF_RASTER, pyoracle.CONF_GPU_MATH
VARIANTS = [
    ("w8", 8, 0), ("w4", 4, 0), ("fma", 0, F), ("clip_zo", 0, Z), ("raster", 0, R),
    ("gpu_math", 0, G), ("conf8", 8, F | R | G), ("conf4", 4, F | R | G),
]


def gaussians_separable(dims, seed=2024):
    """The C3 volume (synth.gaussians_numpy / vr_generate_volume kind 0) with each Gaussian as
    an outer product of per-axis float64 exponentials (same parameters; equal to the direct
    form within float64 rounding, so within 1 ulp of float32)."""
    nx, ny, nz = dims
    acc = np.zeros((nz, ny, nx), np.float64)
    for cx, cy, cz, k, amp in synth.gaussian_params(dims, seed).astype(np.float64):
        ex = np.exp(-k * (np.arange(nx) - cx) ** 2)
        ey = np.exp(-k * (np.arange(ny) - cy) ** 2)
        ez = amp * np.exp(-k * (np.arange(nz) - cz) ** 2)
        acc += ez[:, None, None] * (ey[:, None] * ex[None, :])[None]
    for z in range(nz):  # the value noise, one slice at a time (bounded memory)
        yy, xx = np.meshgrid(np.arange(ny), np.arange(nx), indexing="ij")
        acc[z] += 0.05 * synth.hash01(xx, yy, np.full_like(xx, z))
    return acc.astype(np.float32)


def scenes(names):
    out = []
    if "c1" in names:
        out.append(("C1 64^3 f32 @ 256^2, fill", synth.gaussian_blob(64), 256, 256, "fill", 0))
    if "c1near" in names:  # the near plane cuts the cube (camera 0.15 from the front face)
        out.append(("C1 near camera (r = 0.65, front face 0.15 away: NO clip plane 0.198, ZO 0.1)", synth.gaussian_blob(64),
                    256, 256, "near", 0))
    if "c2" in names:
        out.append(("C2 256^3 u8 CT head @ 1024^2, fill", synth.ct_head(256, 1234), 1024, 1024,
                    "fill", 0))
    if any(n.startswith("c3") for n in names):
        vol = gaussians_separable((512, 512, 512))
        if "c3" in names:
            out.append(("C3 512^3 f32 @ 1920x1080, fill (r = 1.6)", vol, 1920, 1080, "fill", 0))
        if "c3d" in names:
            out.append(("C3 512^3 f32 @ 1920x1080, default camera (r = 3)", vol, 1920, 1080,
                        "default", 0))
        if "c3s" in names:
            out.append(("C3 headline: Phong + ERT 1e-5, exact gradient, fill", vol, 1920, 1080,
                        "fill", 1))
    return out


def rgba8(x):
    return np.rint(np.clip(x, 0.0, 1.0) * 255.0).astype(np.int32)


def compare(ref, img, st_ref, st):
    d = img.astype(np.float64) - ref.astype(np.float64)
    q = np.abs(rgba8(img) - rgba8(ref))
    return dict(rmse=float(np.sqrt(np.mean(d * d))), max_abs=float(np.abs(d).max()),
                rgba8_max_lsb=int(q.max()),
                rgba8_pixels_differing=float(np.mean(q.max(axis=-1) > 0)),
                covered_ray_delta=int(st["rays"]) - int(st_ref["rays"]))


def run(names, threads=0, log=print):
    rows = []
    for title, vol, W, H, camname, shading in scenes(names):
        cam = synth.camera(camname).to_vr_camera()
        p = vr_amd.default_params(shading=shading)
        if shading:
            p.ert_eps = 1e-5
        fv = vol.astype(np.float32)
        sc = pyoracle.Scene.from_params(vol, float(fv.min()), float(fv.max()), synth.tf2(), cam,
                                        W, H, p)
        t0 = time.time()
        ref, st_ref = sc.render(nthreads=threads)
        row = dict(scene=title, width=W, height=H, shading=shading, rays=int(st_ref["rays"]),
                   samples=int(st_ref["samples"]), oracle_s=round(time.time() - t0, 2),
                   variants={})
        for name, wb, fl in VARIANTS:
            try:
                img, st = sc.conformance(wb, fl).render(nthreads=threads)
            except RuntimeError:  # OR_CONF_RASTER: the scene needs near-plane clipping
                row["variants"][name] = None
                log(f"{title:58s} {name:9s} n/a (rasteriser model without clipping)")
                continue
            row["variants"][name] = compare(ref, img, st_ref, st)
            v = row["variants"][name]
            log(f"{title:58s} {name:9s} rmse {v['rmse']:.3e}  max {v['max_abs']:.3e}  "
                f"lsb {v['rgba8_max_lsb']}  px {100 * v['rgba8_pixels_differing']:.3f}%  "
                f"rays {v['covered_ray_delta']:+d}")
        sc.conformance(0, 0)
        rows.append(row)
    return rows


def markdown(rows):
    names = [v[0] for v in VARIANTS]
    lines = ["| scene | " + " | ".join(names) + " |", "|---" * (len(names) + 1) + "|"]
    for r in rows:
        cells = []
        for n in names:
            v = r["variants"][n]
            if v is None:
                cells.append("n/a")
                continue
            cells.append(f"{v['rmse']:.1e} / {v['max_abs']:.1e} / {v['rgba8_max_lsb']}")
        lines.append(f"| {r['scene']} | " + " | ".join(cells) + " |")
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r04", "conformance"))
    ap.add_argument("--scenes", default="c1,c1near,c2,c3,c3d,c3s")
    ap.add_argument("--threads", type=int, default=0)
    a = ap.parse_args()
    rows = run(a.scenes.split(","), a.threads)
    os.makedirs(a.out, exist_ok=True)
    doc = dict(what="RMSE / max |d| over float RGBA (all pixels x 4 channels) and RGBA8 LSB of "
                    "each conformance variant against the oracle (tools/conformance_gap.py)",
               threads=a.threads or pyoracle.max_threads(), scenes=rows)
    with open(os.path.join(a.out, "conformance_gap.json"), "w") as f:
        json.dump(doc, f, indent=1)
    md = markdown(rows)
    with open(os.path.join(a.out, "conformance_gap.md"), "w") as f:
        f.write("rmse / max |d| / RGBA8 max LSB against the oracle\n\n" + md + "\n")
    print(md)


if __name__ == "__main__":
    main()
