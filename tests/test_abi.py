"""CPU: the C-ABI library loads and exports every entry point include/vr/*.h declares.
No compute calls here (no GPU in the build container)."""
import ctypes as C
import os
import re
import subprocess

import pytest

import vr_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    src = open(os.path.join(ROOT, "include", "vr", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(vr_[a-z0-9_]+)\s*\(", src))
    return names


def exported():
    out = subprocess.run(["nm", "-D", "--defined-only", vr_amd.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


@pytest.mark.parametrize("header", ["vr.h", "vr_host.h", "vr_dist.h", "vr_debug.h"])
def test_every_declared_symbol_is_exported(header):
    names = declared(header)
    assert len(names) >= 2
    missing = names - exported()
    assert not missing, missing


def test_binding_lists_cover_headers():
    assert declared("vr.h") == set(vr_amd.ABI_SYMBOLS)
    assert declared("vr_host.h") == set(vr_amd.HOST_SYMBOLS)
    assert declared("vr_dist.h") == set(vr_amd.DIST_SYMBOLS)
    assert declared("vr_debug.h") == set(vr_amd.DEBUG_SYMBOLS)


def test_product_never_reads_the_environment():
    """Launch-policy overrides go through vr_debug.h knobs; the library reads the process
    environment only in experiment builds (#ifdef VR_EXPERIMENTS)."""
    csrc = os.path.join(ROOT, "volumetric-renderer_amd", "csrc")
    for name in sorted(os.listdir(csrc)):
        depth, guarded = 0, []
        for line in open(os.path.join(csrc, name)):
            s = line.strip()
            if s.startswith("#if"):
                guarded.append("VR_EXPERIMENTS" in s)
            elif s.startswith("#endif") and guarded:
                guarded.pop()
            elif "getenv" in s and not any(guarded):
                raise AssertionError(f"{name}: getenv outside #ifdef VR_EXPERIMENTS: {s}")


def test_library_loads_and_pure_entry_points():
    L = vr_amd.lib()
    assert L.vr_abi_version() == 9
    p = vr_amd.default_params()
    assert p.step == pytest.approx(0.005) and p.ray_dist == pytest.approx(1.8)
    assert list(p.clear_color) == pytest.approx([0.11, 0.11, 0.11, 1.0])
    assert p.ert_eps == 0.0 and p.shading == 0
    # row-block sharding arithmetic
    assert vr_amd.shard_rows(1080, 16, 1) == 1088
    assert vr_amd.shard_rows(1080, 16, 8) == 144
    assert vr_amd.shard_rows(53, 1, 5) == 11
    assert vr_amd.shard_rows(10, 0, 2) == 0
    # external-memory import: argument checks come before any HIP call
    mem, ptr = C.c_void_p(), C.c_void_p()
    assert L.vr_import_memory_fd(None, 3, 64, 0, C.byref(mem), C.byref(ptr)) == -22
    assert L.vr_release_external_memory(None, None) == -22
    # ABI 7 entry points: argument checks before any HIP call
    assert L.vr_set_row_share(None, 1, 1) == -22
    assert L.vr_set_memory_budget(None, 0) == -22
    assert L.vr_memory_report(None, None) == -22
    assert L.vr_shard_rows_ctx(None, 1080, 8, 8) == 0
    assert L.vr_debug_timing_member(None, 0, None) == -22


def test_struct_layouts_match_header():
    # sizes of the ABI structs as declared in vr.h (no padding surprises across the boundary)
    assert C.sizeof(vr_amd.vr_camera) == 4 * (16 + 3 + 3)
    assert C.sizeof(vr_amd.vr_params) == 4 * (3 + 1 + 4 + 3 + 1 + 6)
    assert C.sizeof(vr_amd.vr_stats) == 40
    src = open(os.path.join(ROOT, "include", "vr", "vr.h")).read()
    test = r"""
#include "vr/vr.h"
#include <stdio.h>
#include <stddef.h>
#include "vr/vr_debug.h"
int main(void) { printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(vr_camera), sizeof(vr_params),
  sizeof(vr_stats), offsetof(vr_params, spec_power), offsetof(vr_params, skip_empty), offsetof(vr_params, frames_in_flight), offsetof(vr_params, exact_gradient), offsetof(vr_params, depth_zero_to_one),
  sizeof(vr_memory_info), sizeof(vr_member_timing), offsetof(vr_member_timing, kernel_ms)); return 0; }
"""
    tmp = os.path.join("/tmp", "vr_abi_layout")
    with open(tmp + ".c", "w") as f:
        f.write(test)
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), tmp + ".c", "-o", tmp], check=True)
    out = subprocess.run([tmp], capture_output=True, text=True, check=True).stdout.split()
    assert [int(x) for x in out] == [C.sizeof(vr_amd.vr_camera), C.sizeof(vr_amd.vr_params),
                                     C.sizeof(vr_amd.vr_stats), vr_amd.vr_params.spec_power.offset,
                                     vr_amd.vr_params.skip_empty.offset,
                                     vr_amd.vr_params.frames_in_flight.offset,
                                     vr_amd.vr_params.exact_gradient.offset,
                                     vr_amd.vr_params.depth_zero_to_one.offset,
                                     C.sizeof(vr_amd.vr_memory_info), C.sizeof(vr_amd.vr_member_timing),
                                     vr_amd.vr_member_timing.kernel_ms.offset]
    assert "VR_ABI_VERSION 9" in src


def test_create_without_device_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    with pytest.raises(RuntimeError, match="vr_create failed"):
        vr_amd.OffscreenPass(8, 8)


def test_dist_entry_points_reject_bad_arguments():
    """vr_dist.h argument checks (no communicator is created, no device touched)."""
    L = vr_amd.lib()
    assert L.vr_dist_create(None, None, 2, 0, 8, 3) is None
    assert b"NULL" in L.vr_dist_last_error(None)
    assert L.vr_dist_unique_id(None) == -22
    p = vr_amd.default_params()
    cam = vr_amd.make_camera().to_vr_camera()
    assert L.vr_dist_render(None, C.byref(cam), C.byref(p), None, None) == -22
    assert L.vr_dist_synchronize(None) == -22
    L.vr_dist_destroy(None)  # no-op


def test_no_cpu_fallback_in_product():
    """The product path never routes through the oracle or any CPU renderer."""
    for path in ("volumetric-renderer_amd/vr_amd.py", "volumetric-renderer_amd/csrc/vr_api.hip",
                 "volumetric-renderer_amd/csrc/vr_kernels.hip", "volumetric-renderer_amd/host/vr_host.cpp",
                 "volumetric-renderer_amd/csrc/vr_dist.cpp"):
        txt = open(os.path.join(ROOT, path)).read()
        for needle in ("pyoracle", "liboracle", "oracle.h", "import oracle", "ref_numpy", "or_render"):
            assert needle not in txt, (path, needle)
    out = subprocess.run(["nm", "-D", vr_amd.LIB_PATH], capture_output=True, text=True).stdout
    assert "or_render_rows" not in out


def test_stale_pmc_traffic_is_never_used():
    """bench.py's roofline divides measured HBM bytes (profiles/pmc_traffic.json) by its frame
    period only when the entry was measured on this kernel, these kernel sources
    (vr_amd.kernel_code_hash) and this volume layout: any mismatch gives traffic None and a
    "stale: ..." status in the bench line, never old bytes."""
    import json
    import bench
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    e = d["c3"]
    assert e["hbm_bytes_per_launch"] > 0 and e["layout"].startswith("st4:")
    good = dict(world=e["n_gpus"], kernel=e["kernel"], layout=e["layout"])
    byts, _, status = bench.load_traffic("c3", **good)
    if e.get("code_hash") == vr_amd.kernel_code_hash():
        assert status == "ok" and byts == float(e["hbm_bytes_per_launch"])
    else:
        assert byts is None and status.startswith("stale: code_hash")
    for k, v in (("world", e["n_gpus"] + 1), ("kernel", "other"), ("layout", "st4:1")):
        byts, _, status = bench.load_traffic("c3", **dict(good, **{k: v}))
        assert byts is None and status.startswith("stale:"), (k, status)
    assert bench.load_traffic("no_such_config", **good)[2].startswith("missing:")


def test_committed_pmc_traffic_matches_the_kernel_code():
    """profiles/pmc_traffic.json was measured on this library's device code: every config entry
    carries the current vr_amd.kernel_code_hash (the .hip_fatbin bytes), so a kernel change
    cannot leave a stale roofline behind (re-measure with tools/measure_round.sh on the GPU).
    No xfail: a stale entry fails here; host-only edits do not move the hash."""
    import json
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    now = vr_amd.kernel_code_hash()
    for cfg in ("c3", "c3_default", "c3_ref", "c2", "c4", "c5"):
        assert cfg in d, f"no PMC traffic for {cfg}"
        e = d[cfg]
        assert e.get("code_hash") == now, (cfg, e.get("code_hash"), now)
        assert e["hbm_bytes_per_launch"] > 0
    for cfg in ("c3", "c3_default", "c3_ref"):
        assert d[cfg]["layout"].startswith("st4:")
