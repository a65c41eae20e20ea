"""Cache-line footprint model of the ray-march gathers (design tool, CPU only).

For a sample of 8x8-pixel wavefront tiles, march the 64 rays in lock-step exactly as one
wavefront does and, for every load instruction the kernel would issue, count the distinct
cache lines the 64 lanes touch.  The L1 (TCP) access rate is the measured limiter of the
kernel (profiles/r01/pmc_*), so "lines per wave-instruction x instructions per sample" is the
figure of merit for a volume layout.  Layouts are given as functions (x, y, z) -> element
offset, voxel size and the loads a sample issues.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import ref_numpy  # noqa: E402


def rays(view, cam_pos, W, H, px, py):
    V = np.asarray(view, dtype=np.float64).reshape(4, 4).T
    inv = np.linalg.inv(ref_numpy.projection(W, H) @ V)
    x = (px + 0.5) / W * 2 - 1
    y = (py + 0.5) / H * 2 - 1
    h0 = inv @ np.stack([x, y, np.zeros_like(x), np.ones_like(x)])
    h1 = inv @ np.stack([x, y, np.ones_like(x), np.ones_like(x)])
    p0 = (h0[:3] / h0[3]).T
    d = (h1[:3] / h1[3]).T - p0
    with np.errstate(divide="ignore", invalid="ignore"):
        t1 = (-0.5 - p0) / d
        t2 = (0.5 - p0) / d
    lo = np.minimum(t1, t2).max(axis=1)
    hi = np.maximum(t1, t2).min(axis=1)
    ok = (lo < hi) & (lo >= 0) & (lo <= 1)
    e = p0 + lo[:, None] * d
    dirs = e - np.asarray(cam_pos)
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    return ok, e + 0.5, dirs


# ---- layouts: each returns a list of per-lane byte-address arrays, one per load instruction --
def brick_apron(B, vb, pair_x=True):
    S = B + 1

    def fn(i, j, k, nb):
        pi, pj, pk = i + 2, j + 2, k + 2
        b = ((pk // B) * nb + (pj // B)) * nb + (pi // B)
        base = (b * S ** 3 + ((pk % B) * S + (pj % B)) * S + (pi % B)) * vb
        loads = []
        for dz in (0, 1):
            for dy in (0, 1):
                o = base + (dz * S * S + dy * S) * vb
                if pair_x:
                    loads.append((o, 2 * vb))
                else:
                    loads.append((o, vb))
                    loads.append((o + vb, vb))
        return loads
    return fn


def brick_apron_zpair(B, vb):
    """Each stored element holds (v(z), v(z+1)): one 4*vb-byte load gets x-pair x z-pair."""
    S = B + 1

    def fn(i, j, k, nb):
        pi, pj, pk = i + 2, j + 2, k + 2
        b = ((pk // B) * nb + (pj // B)) * nb + (pi // B)
        base = (b * S ** 3 + ((pk % B) * S + (pj % B)) * S + (pi % B)) * 2 * vb
        return [(base, 4 * vb), (base + S * 2 * vb, 4 * vb)]
    return fn


def brick_apron_yzquad(B, vb):
    """Each stored element holds v(y..y+1, z..z+1): one 8*vb-byte run at x gets the whole
    2x2x2 footprint (f32: two dwordx4; u16: one dwordx4; u8: one dwordx2)."""
    S = B + 1

    def fn(i, j, k, nb):
        pi, pj, pk = i + 2, j + 2, k + 2
        b = ((pk // B) * nb + (pj // B)) * nb + (pi // B)
        base = (b * S ** 3 + ((pk % B) * S + (pj % B)) * S + (pi % B)) * 4 * vb
        w = 8 * vb
        if w <= 16:
            return [(base, w)]
        return [(base, 16), (base + 16, 16)]
    return fn


def linear(vb, n):
    def fn(i, j, k, nb):
        loads = []
        for dz in (0, 1):
            for dy in (0, 1):
                o = ((np.clip(k + dz, 0, n - 1) * n + np.clip(j + dy, 0, n - 1)) * n + np.clip(i, 0, n - 1)) * vb
                loads.append((o, 2 * vb))
        return loads
    return fn


def simulate(layout, n, vb, view, pos, W=1920, H=1080, ntiles=300, seed=0, line=128, tile=(8, 8)):
    """tile: the wavefront's pixel footprint (tw, th), tw * th = 64 lanes."""
    rng = np.random.default_rng(seed)
    nb = (n + 3) // 4 + 1  # >= bricks per axis for any brick size >= 4 (indices stay unique)
    tw, th = tile
    tot_instr = 0
    tot_lines = 0
    samples = 0
    tiles = 0
    while tiles < ntiles:
        tx = rng.integers(0, W // tw)
        ty = rng.integers(0, H // th)
        px, py = np.meshgrid(np.arange(tw) + tx * tw, np.arange(th) + ty * th)
        ok, pos0, dirs = rays(view, pos, W, H, px.ravel().astype(float), py.ravel().astype(float))
        if ok.sum() < 32:
            continue
        tiles += 1
        p = pos0.copy()
        alive = ok.copy()
        for _ in range(360):
            alive &= np.all((p >= 0) & (p <= 1), axis=1)
            if not alive.any():
                break
            u = p[alive] * n - 0.5
            i0 = np.floor(u).astype(np.int64)
            loads = layout(i0[:, 0], i0[:, 1], i0[:, 2], nb)
            for addr, width in loads:
                first = addr // line
                last = (addr + width - 1) // line
                tot_lines += len(np.unique(np.concatenate([first, last])))
                tot_instr += 1
            samples += int(alive.sum())
            p = p + dirs * 0.005
    return dict(lines_per_instr=tot_lines / tot_instr, instr_per_wave_step=tot_instr / max(1, tiles),
                lines_per_sample=tot_lines / samples, samples=samples)


def tile_shapes(n=512, ntiles=60):
    """Lines per wave-level load of the shipped layouts for wavefront tile shapes 8x8, 16x4,
    4x16, 32x2 over the sweep views."""
    sys.path.insert(0, os.path.join(ROOT, "volumetric-renderer_amd"))
    import synth
    cams = {"fill": synth.camera("fill"), "fill_oblique": synth.camera("fill_oblique"),
            "side_x": synth.vr_amd.make_camera(radius=1.6, rotate=(360.0, 0.0)),
            "top_z": synth.vr_amd.make_camera(radius=1.6, rotate=(0.0, 360.0)),
            "diag": synth.vr_amd.make_camera(radius=2.0, rotate=(180.0, 140.0)),
            "default": synth.camera("default")}
    layouts = {"f32 zpair": (brick_apron_zpair(8, 4), 4), "u8 yzquad": (brick_apron_yzquad(8, 1), 1)}
    for cname, cam in cams.items():
        vc = cam.to_vr_camera()
        for lname, (fn, vb) in layouts.items():
            row = []
            for t in ((8, 8), (16, 4), (4, 16), (32, 2)):
                r = simulate(fn, n, vb, list(vc.view), list(vc.position), ntiles=ntiles, tile=t)
                row.append(f"{t[0]}x{t[1]} {r['lines_per_sample']:.3f}")
            print(f"{cname:13s} {lname:10s} lines/sample: " + "  ".join(row), flush=True)


if __name__ == "__main__":
    sys.path.insert(0, os.path.join(ROOT, "volumetric-renderer_amd"))
    import synth
    if len(sys.argv) > 1 and sys.argv[1] == "tiles":
        tile_shapes()
        sys.exit(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    cams = {"fill": synth.camera("fill"), "fill_oblique": synth.camera("fill_oblique"),
            "side_x": synth.vr_amd.make_camera(radius=1.6, rotate=(360.0, 0.0)),
            "top_z": synth.vr_amd.make_camera(radius=1.6, rotate=(0.0, 360.0))}
    layouts = {
        "brick16+apron f32 (current, dwordx2)": (brick_apron(16, 4), 4),
        "brick8+apron f32 (dwordx2)": (brick_apron(8, 4), 4),
        "brick4+apron f32 (dwordx2)": (brick_apron(4, 4), 4),
        "brick16+apron f32 zpair (dwordx4 x2)": (brick_apron_zpair(16, 4), 4),
        "brick8+apron f32 zpair (dwordx4 x2)": (brick_apron_zpair(8, 4), 4),
        "brick4+apron f32 zpair (dwordx4 x2)": (brick_apron_zpair(4, 4), 4),
    }
    for cname, cam in cams.items():
        vc = cam.to_vr_camera()
        for lname, (fn, vb) in layouts.items():
            r = simulate(fn, n, vb, list(vc.view), list(vc.position), ntiles=60)
            print(f"{cname:13s} {lname:40s} lines/instr {r['lines_per_instr']:6.2f}  "
                  f"lines/sample {r['lines_per_sample']:.3f}")


# ---- plain 8-bit layouts (round 2: cutting the yz-quad's 4x duplication) --------------------
def brick_plain_u8(B, pad_to=4):
    """u8 voxels one per element in (B+1)^3-element bricks (apron), brick stride rounded up to
    pad_to bytes.  A sample = 2 x 16-B loads at 4-aligned addresses: floor4(e) covers rows
    (y, z) and (y+1, z) at x, x+1 (offsets e, e+1, e+S, e+S+1 all < floor4(e) + 16 when
    S <= 12); the second the same at z+1."""
    S = B + 1
    stride = (S ** 3 + pad_to - 1) // pad_to * pad_to

    def fn(i, j, k, nb):
        pi, pj, pk = i + 2, j + 2, k + 2
        b = ((pk // B) * nb + (pj // B)) * nb + (pi // B)
        e = b * stride + ((pk % B) * S + (pj % B)) * S + (pi % B)
        e2 = e + S * S
        return [(e & ~3, 16), (e2 & ~3, 16)]
    return fn, stride / B ** 3


def views_u8(n=256, ntiles=60, W=1024, H=1024):
    sys.path.insert(0, os.path.join(ROOT, "volumetric-renderer_amd"))
    import synth
    cams = {"fill": synth.camera("fill"), "fill_oblique": synth.camera("fill_oblique"),
            "side_x": synth.vr_amd.make_camera(radius=1.6, rotate=(360.0, 0.0)),
            "diag": synth.vr_amd.make_camera(radius=2.0, rotate=(180.0, 140.0)),
            "default": synth.camera("default")}
    p8, f8 = brick_plain_u8(8)
    p4, f4 = brick_plain_u8(4, 128)
    layouts = {"yzquad8 (1 x dwordx2)": (brick_apron_yzquad(8, 1), 4 * (9 / 8) ** 3),
               f"plain8 (2 x dwordx4)": (p8, f8), f"plain4/128B (2 x dwordx4)": (p4, f4)}
    for cname, cam in cams.items():
        vc = cam.to_vr_camera()
        for lname, (fn, foot) in layouts.items():
            r = simulate(fn, n, 1, list(vc.view), list(vc.position), W=W, H=H, ntiles=ntiles, tile=(16, 4))
            print(f"{cname:13s} {lname:28s} x{foot:.2f}  lines/instr {r['lines_per_instr']:6.2f}  "
                  f"lines/sample {r['lines_per_sample']:.3f}", flush=True)


# ---- round 4: what TCP counts per wave-level load, and lane-pair sharing ---------------------
def tcp_counts(addr, width, lanes_on=None, sector=64, line=128):
    """For one wave-level load (64 lane addresses, `width` bytes each): three candidate counts
    of TCP_TOTAL_CACHE_ACCESSES -- distinct 128-B lines of the wave (H0), distinct lines per
    quarter-wave summed (H2), distinct 64-B sectors per quarter-wave summed (H1)."""
    a = np.asarray(addr)
    on = np.ones(len(a), bool) if lanes_on is None else np.asarray(lanes_on)
    first_l, last_l = a // line, (a + width - 1) // line
    first_s, last_s = a // sector, (a + width - 1) // sector
    h0 = len(np.unique(np.concatenate([first_l[on], last_l[on]])))
    h1 = h2 = 0
    for q in range(4):
        m = on.copy()
        m[:] = False
        m[q * 16:(q + 1) * 16] = on[q * 16:(q + 1) * 16]
        if m.any():
            h2 += len(np.unique(np.concatenate([first_l[m], last_l[m]])))
            h1 += len(np.unique(np.concatenate([first_s[m], last_s[m]])))
    return h0, h1, h2


def tcp_model(view_name="fill", n=512, W=1920, H=1080, ntiles=40, seed=0, vb=4):
    """C3's density gathers (f32 z-pairs in 8^3 bricks, 16x4 wavefronts, 2 x 16-B loads per
    sample) under the three counting hypotheses, and the share of x-neighbour lane pairs
    (l, l ^ 1) whose cells are the same cell (VR_F32_SHARE) or in the same row pair of a brick
    (the 8-bit plain layout's VR_U8_SHARE=1 criterion)."""
    sys.path.insert(0, os.path.join(ROOT, "volumetric-renderer_amd"))
    import synth
    vc = synth.camera(view_name).to_vr_camera()
    view, pos = list(vc.view), list(vc.position)
    layout = brick_apron_zpair(8, vb)
    rng = np.random.default_rng(seed)
    nb = (n + 3) // 4 + 1
    tw, th = 16, 4
    tot = np.zeros(3)
    loads = 0
    pairs = same_cell = 0
    tiles = 0
    while tiles < ntiles:
        tx, ty = rng.integers(0, W // tw), rng.integers(0, H // th)
        px, py = np.meshgrid(np.arange(tw) + tx * tw, np.arange(th) + ty * th)
        ok, pos0, dirs = rays(view, pos, W, H, px.ravel().astype(float), py.ravel().astype(float))
        if ok.sum() < 32:
            continue
        tiles += 1
        p = np.clip(pos0.copy(), 0.0, 1.0)  # the entry-face snap (pixel_ray)
        alive = ok.copy()
        for _ in range(360):
            alive &= np.all((p >= 0) & (p <= 1), axis=1)
            if not alive.any():
                break
            i0 = np.floor(np.clip(p, 0, 1) * n - 0.5).astype(np.int64)
            for addr, width in layout(i0[:, 0], i0[:, 1], i0[:, 2], nb):
                tot += tcp_counts(addr, width, alive)
                loads += 1
            cell = (i0[:, 2] * (n + 8) + i0[:, 1]) * (n + 8) + i0[:, 0]
            both = alive[0::2] & alive[1::2]
            pairs += int(both.sum())
            same_cell += int(((cell[0::2] == cell[1::2]) & both).sum())
            p = p + dirs * 0.005
    return dict(view=view_name, wave_loads=loads, h0_lines_per_wave=tot[0] / loads,
                h1_sectors_per_quarter=tot[1] / loads, h2_lines_per_quarter=tot[2] / loads,
                pair_same_cell=same_cell / max(1, pairs))


# ---- round 5: the reading td_mask settled (TCP accesses = active 4-lane quads x 64-B sectors) --
def quad_sectors(addr, width, lanes_on, sector=64):
    """L1 accesses of one wave-level load under the measured reading of
    TCP_TOTAL_CACHE_ACCESSES (profiles/r05/m3/td_pmc.json): per 4-lane quad with an active
    lane, the distinct 64-B sectors its active lanes' `width`-byte loads touch."""
    a = np.asarray(addr)
    on = np.asarray(lanes_on)
    tot = 0
    for q in range(len(a) // 4):
        m = on[q * 4:(q + 1) * 4]
        if not m.any():
            continue
        aa = a[q * 4:(q + 1) * 4][m]
        tot += len(np.unique(np.concatenate([aa // sector, (aa + width - 1) // sector])))
    return tot


def quad_model(view_name, layout, n, W, H, lane_xy=lambda l: (l & 15, l >> 4), ntiles=20, seed=0):
    """Mean quad_sectors per wave-level load of `layout` ((i, j, k, nb) -> [(addr, width)])
    over random 16x4 wavefront strips of the view; lane_xy maps a lane to its pixel in the
    strip (the kernel's 16x4 raster by default).  C3 fill: 24.1 (measured ~22); C4: 23.8 (21.4)."""
    sys.path.insert(0, os.path.join(ROOT, "volumetric-renderer_amd"))
    import synth
    vc = synth.camera(view_name).to_vr_camera()
    view, pos = list(vc.view), list(vc.position)
    rng = np.random.default_rng(seed)
    nb = (n + 3) // 4 + 1
    lx = np.array([lane_xy(l)[0] for l in range(64)])
    ly = np.array([lane_xy(l)[1] for l in range(64)])
    tot = loads = tiles = 0
    while tiles < ntiles:
        tx, ty = rng.integers(0, W // 16), rng.integers(0, H // 4)
        ok, pos0, dirs = rays(view, pos, W, H, (lx + tx * 16).astype(float), (ly + ty * 4).astype(float))
        if ok.sum() < 32:
            continue
        tiles += 1
        p = np.clip(pos0.copy(), 0.0, 1.0)
        alive = ok.copy()
        for _ in range(360):
            alive &= np.all((p >= 0) & (p <= 1), axis=1)
            if not alive.any():
                break
            i0 = np.floor(np.clip(p, 0, 1) * n - 0.5).astype(np.int64)
            for addr, width in layout(i0[:, 0], i0[:, 1], i0[:, 2], nb):
                tot += quad_sectors(addr, width, alive)
                loads += 1
            p = p + dirs * 0.005
    return tot / max(1, loads)


def zpair_geom(BX, BY, BZ, vb=4):
    """f32 z-pairs in BX x BY x BZ-cell bricks (the -DVR_BRICK_CELLS geometries)."""
    EX, EY, EZ = BX + 1, BY + 1, BZ + 1

    def fn(i, j, k, nb):
        pi, pj, pk = i + 2, j + 2, k + 2
        b = ((pk // BZ) * nb + (pj // BY)) * nb + (pi // BX)
        base = (b * EX * EY * EZ + ((pk % BZ) * EY + (pj % BY)) * EX + (pi % BX)) * 2 * vb
        return [(base, 4 * vb), (base + EX * 2 * vb, 4 * vb)]
    return fn


def tile_box_model(view_name="fill", n=512, W=1920, H=1080, K=8, ntiles=40, seed=1):
    """Cells in the box a 16x16-pixel tile's rays sample over a stage of K steps (the LDS
    staging a tile-stage would need): median / p90 / max over stages."""
    sys.path.insert(0, os.path.join(ROOT, "volumetric-renderer_amd"))
    import synth
    vc = synth.camera(view_name).to_vr_camera()
    view, pos = list(vc.view), list(vc.position)
    rng = np.random.default_rng(seed)
    sizes, tiles = [], 0
    while tiles < ntiles:
        tx, ty = rng.integers(0, W // 16), rng.integers(0, H // 16)
        px, py = np.meshgrid(np.arange(16) + tx * 16, np.arange(16) + ty * 16)
        ok, p0, d = rays(view, pos, W, H, px.ravel().astype(float), py.ravel().astype(float))
        if ok.sum() < 200:
            continue
        tiles += 1
        p0, d = np.clip(p0[ok], 0, 1), d[ok]
        for s in range(0, 360 // K):
            ks = np.arange(s * K, (s + 1) * K)
            P = p0[:, None, :] + ks[None, :, None] * d[:, None, :] * 0.005
            inb = np.all((P >= 0) & (P <= 1), axis=2)
            if not inb.any():
                break
            u = np.floor(P[inb] * n - 0.5)
            sizes.append(float(np.prod(u.max(0) + 1 - u.min(0) + 1)))
    s = np.array(sizes)
    return dict(K=K, median=float(np.median(s)), p90=float(np.percentile(s, 90)), max=float(s.max()))
