"""GPU: round-6 additions to the boundary (vr.h ABI 9).

* Derived structures under a memory budget: a structure
  that does not fit evicts the least recently read others, one at a time; an evicted structure is
  released stream-ordered after the frames in flight on the context's other streams (frame
  fences), never with a device synchronisation on the frame path; every frame whose view wanted
  a structure the budget refused is counted (vr_memory_info.downgrades / last_downgrade) -- the
  reference never degrades silently, it throws (/root/reference/src/rendering/offscreen_pass.cpp:
  328-331).  Frames stay bit-identical to the unlimited budget's.
"""
import numpy as np
import pytest
import torch

import synth
import vr_amd

pytestmark = pytest.mark.gpu

BUDGET_DEFAULT = 2 ** 64 - 2
BUDGET_UNLIMITED = 2 ** 64 - 1
FIELD, OBLIQUE, PLAIN, STENCIL, SKIP = 1, 2, 3, 4, 5


def _bits_equal(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return int((a.view(np.uint32) != b.view(np.uint32)).any(axis=-1).sum())


def _pass(W=160, H=120, seed=61):
    vol = synth.gaussians_numpy((64, 60, 66), seed=seed).astype(np.float32)
    rp = vr_amd.OffscreenPass(W, H, device=0)
    rp.volume_dataset_changed(synth.dataset(vol))
    rp.transfer_function_changed(synth.tf_band(0.15, 0.9))
    return rp


def _views():
    return {k: synth.camera(k).to_vr_camera() for k in ("fill", "diag", "default")}


def test_forced_downgrade_is_reported(gpu):
    """Budget 0: the fill view's difference field and the diagonal's oblique copy are refused;
    each such frame is counted with the refused structure, and an unlimited budget counts none."""
    rp = _pass()
    try:
        v = _views()
        p = vr_amd.default_params(shading=1, ert_eps=1e-5, frames_in_flight=3)
        m0 = rp.memory_report()
        assert m0["downgrades"] == 0 and m0["last_downgrade"] == 0
        rp.set_memory_budget(0)
        rp.render(v["fill"], p, vr_amd.OUT_RGBA32F)
        m1 = rp.memory_report()
        # vr_render renders 4 row bands of >= 256-row frames, one launch here (120 rows)
        assert m1["downgrades"] == 1 and m1["last_downgrade"] == FIELD, m1
        assert m1["derived_bytes"] == 0
        rp.render(v["diag"], p, vr_amd.OUT_RGBA32F)
        m2 = rp.memory_report()
        assert m2["downgrades"] == 2 and m2["last_downgrade"] == OBLIQUE, m2
        rp.render(v["fill"], vr_amd.default_params(shading=1, skip_empty=1, exact_gradient=1,
                                                   frames_in_flight=3), vr_amd.OUT_RGBA32F)
        m3 = rp.memory_report()
        assert m3["downgrades"] == 3 and m3["last_downgrade"] in (SKIP, FIELD), m3
        rp.set_memory_budget(BUDGET_UNLIMITED)
        for name in ("fill", "diag", "default"):
            rp.render(v[name], p, vr_amd.OUT_RGBA32F)
        m4 = rp.memory_report()
        assert m4["downgrades"] == m3["downgrades"] and m4["builds"] > m3["builds"], m4
    finally:
        rp.close()


def test_least_recently_read_structure_is_evicted_and_frames_unchanged(gpu):
    """A budget that holds the field and one copy, not all three: fill (field) -> diag (oblique
    copy) -> default (stencil copy) evicts the field, the least recently read; back to fill
    evicts the oblique copy.  Every frame equals the unlimited budget's bit for bit (exact
    gradient), and the evictions are counted."""
    rp = _pass()
    try:
        v = _views()
        p = vr_amd.default_params(shading=1, ert_eps=1e-5, exact_gradient=1, frames_in_flight=3)
        rp.set_memory_budget(BUDGET_UNLIMITED)  # the references: every structure resident
        ref = {k: rp.render(c, p, vr_amd.OUT_RGBA32F) for k, c in v.items()}
        m = rp.memory_report()
        F, O, S = m["field_bytes"], m["oblique_copy_bytes"], m["stencil_copy_bytes"]
        assert F > 0 and O > 0 and S > 0, dict(m)
        skip = m["skip_bytes"]
        budget = F + max(O, S) + skip + (1 << 16)
        assert budget < F + O + S + skip
        rp.set_memory_budget(budget)  # lower: the device drains, everything is freed
        e0 = rp.memory_report()["evictions"]
        seq = [("fill", dict(field=True)), ("diag", dict(field=True, oblique=True)),
               ("default", dict(oblique=True, stencil=True)), ("fill", dict(field=True, stencil=True))]
        for i, (name, held) in enumerate(seq):
            img = rp.render(v[name], p, vr_amd.OUT_RGBA32F)
            assert _bits_equal(img, ref[name]) == 0, (i, name)
            m = rp.memory_report()
            assert m["derived_bytes"] <= m["budget_bytes"], m
            assert (m["field_bytes"] > 0) == held.get("field", False), (i, name, m)
            assert (m["oblique_copy_bytes"] > 0) == held.get("oblique", False), (i, name, m)
            assert (m["stencil_copy_bytes"] > 0) == held.get("stencil", False), (i, name, m)
        assert rp.memory_report()["evictions"] - e0 == 2
    finally:
        rp.close()


def test_evictions_under_frames_in_flight_keep_frames_exact(gpu):
    """Frames on three streams, enqueued back to back with no host wait, through views that evict
    each other's structures almost every frame (a budget of one copy): each eviction is ordered
    after the frames in flight on the other streams (frame fences), so every frame is still the
    unlimited budget's, byte for byte."""
    W, H = 160, 120
    rp = _pass(W, H, seed=62)
    try:
        v = _views()
        p = vr_amd.default_params(shading=1, ert_eps=1e-5, exact_gradient=1, frames_in_flight=3)
        order = ["fill", "diag", "default", "diag", "fill", "default"] * 5
        ref = {}
        for k, c in v.items():
            buf = torch.empty((H, W), dtype=torch.int32, device="cuda")
            rp.render_device(c, p, buf.data_ptr(), vr_amd.OUT_RGBA8, 16, 0, 1)
            torch.cuda.synchronize()
            ref[k] = buf.clone()
        m = rp.memory_report()
        one = max(m["oblique_copy_bytes"], m["stencil_copy_bytes"], m["field_bytes"])
        rp.set_memory_budget(one + m["skip_bytes"] + (1 << 16))
        e0 = rp.memory_report()["evictions"]
        streams = [torch.cuda.Stream() for _ in range(3)]
        outs = [torch.empty((H, W), dtype=torch.int32, device="cuda") for _ in order]
        for i, name in enumerate(order):
            rp.render_device(v[name], p, outs[i].data_ptr(), vr_amd.OUT_RGBA8, 16, 0, 1,
                             streams[i % 3].cuda_stream)
        torch.cuda.synchronize()
        for i, name in enumerate(order):
            assert torch.equal(outs[i], ref[name]), (i, name)
        assert rp.memory_report()["evictions"] - e0 >= len(order) // 2
    finally:
        rp.close()


def test_default_budget_orbit_counts(gpu):
    """A short orbit of the reference's camera drag (bench.orbit_cameras) under the default
    budget: the history counters move as structures are built, and no frame is downgraded."""
    import bench
    rp = _pass(W=192, H=108, seed=63)
    try:
        p = vr_amd.default_params(shading=1, ert_eps=1e-5, frames_in_flight=3)
        m0 = rp.memory_report()
        buf = torch.empty((108, 192), dtype=torch.int32, device="cuda")
        for cam in bench.orbit_cameras(90)[::3]:
            rp.render_device(cam, p, buf.data_ptr(), vr_amd.OUT_RGBA8, 16, 0, 1)
        torch.cuda.synchronize()
        m1 = rp.memory_report()
        assert m1["builds"] > m0["builds"]
        assert m1["downgrades"] == m0["downgrades"]
        assert m1["derived_bytes"] <= m1["budget_bytes"]
    finally:
        rp.close()


def test_member_host_profile(gpu):
    """vr_debug_host_profile_member (tools/host_cost.cpp's mask-path rows): every member of a
    3-member context on device 0 counts every frame it enqueued, across a pipeline rebuild
    (frames in flight 1 -> 3), with positive host time in its render and its total; a
    one-device context refuses with VR_EINVAL."""
    import torch
    W, H = 96, 80
    vol = synth.gaussians_numpy((40, 36, 44), seed=64).astype(np.float32)
    grp = vr_amd.OffscreenPass(W, H, members=(0, 0, 0), exchange=vr_amd.EXCHANGE_COPY)
    one = vr_amd.OffscreenPass(W, H, device=0)
    try:
        grp.volume_dataset_changed(synth.dataset(vol))
        grp.transfer_function_changed(synth.tf_band(0.15, 0.9))
        grp.host_profile_enable(True)
        cam = synth.camera("fill").to_vr_camera()
        frame = torch.empty((H, W), dtype=torch.int32, device="cuda")
        n = 0
        for fif in (1, 3):
            p = vr_amd.default_params(shading=1, ert_eps=1e-5, frames_in_flight=fif)
            for _ in range(7):
                grp.render_device(cam, p, frame.data_ptr(), vr_amd.OUT_RGBA8, 8, 0, 1)
                n += 1
        rows = [grp.host_profile_member(m) for m in range(3)]
        for m, r in enumerate(rows):
            assert r["frames"] == n, (m, r)
            assert r["render_us"] > 0 and r["total_us"] >= r["render_us"], (m, r)
        assert rows[0]["assemble_us"] > 0 and rows[1]["assemble_us"] == 0, rows
        assert grp.host_profile_member(1)["frames"] == 0  # read clears
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError):
            one.host_profile_enable(True)
    finally:
        grp.close()
        one.close()


def test_layout_policy_by_ray_axis_and_row_alignment(gpu):
    """vr_api.hip want_alt / use_grad_field (round 6, profiles/r06/policy/): on sparse views
    (> 0.8 voxels per pixel; r = 3 here) the stencil / plain copy only when the image rows follow
    the bricks' rows, the oblique copy when they cross them (the orbit's slowest frames before);
    the binary16 field for sparse row-aligned views whose ray runs along z; the oblique copy for
    rays along x.  Every choice renders the 8^3 bricks' frame byte for byte (exact gradient)."""
    W, H = 192, 120
    rp = _pass(W, H, seed=65)
    try:
        cams = {"default": vr_amd.make_camera(radius=3.0),                       # ray y, rows along x
                "top_far": vr_amd.make_camera(radius=3.0, rotate=(0.0, 340.0)),  # ray z, rows along x
                "side_far": vr_amd.make_camera(radius=3.0, rotate=(360.0, 80.0)),  # ray x, rows along y
                "side_near": vr_amd.make_camera(radius=1.6, rotate=(360.0, 0.0))}  # ray x, dense
        want = {  # (shading, exact_gradient) -> tag per view; None: the 8^3 bricks, no field
            (1, 0): {"default": "F32S", "top_far": "F32H", "side_far": "F32Alt", "side_near": "F32Alt"},
            (1, 1): {"default": "F32S", "top_far": "F32S", "side_far": "F32Alt", "side_near": "F32Alt"},
            (0, 0): {"default": "F32P", "top_far": "F32P", "side_far": "F32Alt", "side_near": "F32Alt"}}
        for (shading, exact), tags in want.items():
            p = vr_amd.default_params(shading=shading, ert_eps=1e-5, exact_gradient=exact,
                                      frames_in_flight=3)
            for name, oc in cams.items():
                cam = oc.to_vr_camera()
                img = rp.render(cam, p, vr_amd.OUT_RGBA32F)
                tag = tags[name]
                kname = rp.kernel_name(p)
                assert tag in kname, (shading, exact, name, kname)
                if tag != "F32H":  # the same frame as the 8^3 bricks with the stencil gradient
                    with rp.knobs(grad_field=0, alt_geometry=0):
                        ref = rp.render(cam, p, vr_amd.OUT_RGBA32F)
                    assert _bits_equal(img, ref) == 0, (shading, exact, name)
    finally:
        rp.close()
