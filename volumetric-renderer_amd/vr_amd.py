"""ctypes binding of the MI355X ray-marcher's C ABI (include/vr/vr.h, include/vr/vr_host.h).

Python here is plumbing for tests and the benchmark; the product is lib/libvr_amd.so (HIP
kernels for gfx950 + the C ABI).  The class `OffscreenPass` mirrors the reference's
`Vol::Rendering::OffscreenPass` API (src/rendering/offscreen_pass.h:40-54): same method names,
argument meaning and error behaviour (failures raise RuntimeError, as the reference throws
std::runtime_error).  There is NO CPU fallback: if the shared library is missing this module
raises at import-time use, and every render goes through the HIP kernels.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# VR_AMD_LIB selects an experiment build (make LIBDIR=... EXTRA=...); default: lib/
LIB_PATH = os.environ.get("VR_AMD_LIB") or os.path.join(HERE, "lib", "libvr_amd.so")

# enum vr_dtype
DTYPE_I8, DTYPE_U8, DTYPE_I16, DTYPE_U16, DTYPE_I32, DTYPE_U32 = 1, 2, 3, 4, 5, 6
DTYPE_I64, DTYPE_U64, DTYPE_F32, DTYPE_F64 = 7, 8, 9, 10
NP_TO_DTYPE = {
    np.dtype(np.int8): DTYPE_I8, np.dtype(np.uint8): DTYPE_U8,
    np.dtype(np.int16): DTYPE_I16, np.dtype(np.uint16): DTYPE_U16,
    np.dtype(np.int32): DTYPE_I32, np.dtype(np.uint32): DTYPE_U32,
    np.dtype(np.int64): DTYPE_I64, np.dtype(np.uint64): DTYPE_U64,
    np.dtype(np.float32): DTYPE_F32, np.dtype(np.float64): DTYPE_F64,
}
DTYPE_TO_NP = {v: k for k, v in NP_TO_DTYPE.items()}
STORAGE_BYTES = {0: 1, 1: 1, 2: 2, 3: 2, 4: 4}  # vr::StorageType -> bytes per voxel

OUT_RGBA8, OUT_RGBA32F = 0, 1


class vr_camera(C.Structure):
    _fields_ = [("view", C.c_float * 16), ("position", C.c_float * 3),
                ("fovy_deg", C.c_float), ("znear", C.c_float), ("zfar", C.c_float)]


class vr_params(C.Structure):
    _fields_ = [("step", C.c_float), ("ray_dist", C.c_float), ("ert_eps", C.c_float),
                ("shading", C.c_int32), ("clear_color", C.c_float * 4),
                ("ambient", C.c_float), ("diffuse", C.c_float), ("specular", C.c_float),
                ("spec_power", C.c_int32), ("tile_order", C.c_int32),
                ("skip_empty", C.c_int32), ("wave_shape", C.c_int32),
                ("frames_in_flight", C.c_int32), ("exact_gradient", C.c_int32),
                ("depth_zero_to_one", C.c_int32)]


class vr_stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("samples", C.c_uint64),
                ("shaded_samples", C.c_uint64), ("steps", C.c_uint64),
                ("skipped_samples", C.c_uint64)]


class vr_orbit_camera(C.Structure):
    _fields_ = [("center", C.c_float * 3), ("orientation", C.c_float * 4),
                ("radius", C.c_float)]


class vr_memory_info(C.Structure):  # vr.h (ABI 7; history fields ABI 9)
    _fields_ = [(n, C.c_uint64) for n in (
        "volume_bytes", "field_bytes", "oblique_copy_bytes", "plain_copy_bytes",
        "stencil_copy_bytes", "skip_bytes", "derived_bytes", "budget_bytes",
        "builds", "evictions", "downgrades", "last_downgrade")]


class vr_dist_host_profile(C.Structure):  # vr_dist.h
    _fields_ = [("frames", C.c_uint64)] + [(n, C.c_double) for n in (
        "render_us", "gather_us", "assemble_us", "record_us", "wait_us", "total_us")]


# vr.h enum vr_derived (vr_memory_info.last_downgrade)
DERIVED = {1: "field", 2: "oblique_copy", 3: "plain_copy", 4: "stencil_copy", 5: "skip"}


class vr_member_timing(C.Structure):  # vr_debug.h (ABI 7)
    _fields_ = [("device", C.c_int32), ("frames", C.c_uint64), ("kernel_ms", C.c_double),
                ("render_ms", C.c_double), ("gather_ms", C.c_double), ("assemble_ms", C.c_double)]


class vr_dataset(C.Structure):
    _fields_ = [("dims", C.c_uint32 * 3), ("dtype", C.c_int), ("data", C.c_void_p),
                ("vmin", C.c_float), ("vmax", C.c_float)]


# Every entry point include/vr/vr.h and include/vr/vr_host.h declare (checked by the CPU tests).
ABI_SYMBOLS = [
    "vr_abi_version", "vr_params_default", "vr_create", "vr_destroy", "vr_last_error",
    "vr_create_mask", "vr_get_device_mask",
    "vr_resize", "vr_get_size", "vr_get_device", "vr_set_volume", "vr_set_volume_device", "vr_generate_volume",
    "vr_volume_bytes", "vr_debug_read_volume", "vr_debug_read_volume_native", "vr_debug_volume_info",
    "vr_set_transfer_function", "vr_set_slicing", "vr_render", "vr_render_device",
    "vr_shard_rows", "vr_assemble_rows", "vr_count_work", "vr_timing_enable",
    "vr_timing_read", "vr_timing_reset", "vr_kernel_name",
    "vr_import_memory_fd", "vr_release_external_memory",
    "vr_set_row_share", "vr_get_row_share", "vr_shard_rows_ctx",
    "vr_set_memory_budget", "vr_memory_report", "vr_prepare",
]
HOST_SYMBOLS = [
    "vr_cam_init", "vr_cam_rotate", "vr_cam_zoom", "vr_cam_position", "vr_cam_view",
    "vr_cam_to_camera", "vr_gradient_create", "vr_gradient_destroy",
    "vr_gradient_add_color_marker", "vr_gradient_add_alpha_marker",
    "vr_gradient_remove_color_marker", "vr_gradient_remove_alpha_marker",
    "vr_gradient_set_alpha_marker", "vr_gradient_set_color_marker", "vr_gradient_marker_count",
    "vr_gradient_sample", "vr_gradient_discretize", "vr_nrrd_load", "vr_nrrd_write_raw",
    "vr_csv_load", "vr_dataset_free", "vr_host_last_error",
]

DIST_SYMBOLS = [
    "vr_dist_unique_id", "vr_dist_create", "vr_dist_render", "vr_dist_synchronize",
    "vr_dist_last_error", "vr_dist_destroy", "vr_dist_timing_enable", "vr_dist_timing_read",
    "vr_dist_host_profile_enable", "vr_dist_host_profile_read",
]
DIST_ID_BYTES = 128  # include/vr/vr_dist.h VR_DIST_ID_BYTES
DEBUG_SYMBOLS = ["vr_debug_set_knob", "vr_debug_get_knob", "vr_debug_timing_member",
                 "vr_debug_create_members", "vr_debug_fail_member",
                 "vr_debug_host_profile_enable", "vr_debug_host_profile_member"]
# include/vr/vr_debug.h enum vr_exchange (multi-device contexts: how shards reach member 0)
EXCHANGE_RCCL, EXCHANGE_COPY = 0, 1
# include/vr/vr_debug.h enum vr_knob (launch-policy overrides: speed only, never results)
KNOBS = {"pipeline": 1, "pair": 2, "pair_lanes": 3, "grad_field": 4, "u8_layout": 6,
         "tile_order": 7, "narrow": 8, "alt_geometry": 9}
KNOB_AUTO = {"pipeline": -1, "pair": -1, "pair_lanes": 0, "grad_field": -1,
             "u8_layout": -1, "tile_order": 0, "narrow": 1, "alt_geometry": -1}

ABI_VERSION = 9  # include/vr/vr.h VR_ABI_VERSION
_LIB = None


def lib() -> C.CDLL:
    """Load lib/libvr_amd.so (fails loudly: there is no fallback path)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C volumetric-renderer_amd` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
    # PyTorch ships its own libamdhip64.so.7 / libhsa-runtime64.so.1 under the same sonames as
    # /opt/rocm's.  Whichever loads first serves the whole process, and torch's CUDA init
    # failed ("No HIP GPUs are available") once this library had brought in /opt/rocm's
    # runtime and initialised it.  Load torch first when it is installed, so the process
    # runs one runtime that both use (the one the GPU tests and bench.py run on).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, u32, f32, i32 = C.c_void_p, C.c_uint32, C.c_float, C.c_int
    sig = {
        "vr_abi_version": (i32, []),
        "vr_params_default": (None, [C.POINTER(vr_params)]),
        "vr_create": (vp, [i32, u32, u32]),
        "vr_destroy": (None, [vp]),
        "vr_last_error": (C.c_char_p, [vp]),
        "vr_resize": (i32, [vp, u32, u32]),
        "vr_get_size": (i32, [vp, C.POINTER(u32), C.POINTER(u32)]),
        "vr_get_device": (i32, [vp, C.POINTER(i32)]),
        "vr_create_mask": (vp, [u32, u32, u32]),
        "vr_get_device_mask": (i32, [vp, C.POINTER(u32)]),
        "vr_dist_unique_id": (i32, [vp]),
        "vr_dist_create": (vp, [vp, vp, i32, i32, u32, i32]),
        "vr_dist_render": (i32, [vp, C.POINTER(vr_camera), C.POINTER(vr_params), vp, vp]),
        "vr_dist_synchronize": (i32, [vp]),
        "vr_dist_last_error": (C.c_char_p, [vp]),
        "vr_dist_destroy": (None, [vp]),
        "vr_dist_timing_enable": (i32, [vp, i32]),
        "vr_dist_host_profile_enable": (i32, [vp, i32]),
        "vr_dist_host_profile_read": (i32, [vp, C.POINTER(vr_dist_host_profile)]),
        "vr_dist_timing_read": (i32, [vp, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                      C.POINTER(C.c_uint64)]),
        "vr_set_volume": (i32, [vp, vp, i32, u32, u32, u32, f32, f32]),
        "vr_set_volume_device": (i32, [vp, vp, i32, u32, u32, u32, f32, f32, vp]),
        "vr_generate_volume": (i32, [vp, i32, i32, u32, u32, u32, u32, C.POINTER(f32), C.POINTER(f32)]),
        "vr_volume_bytes": (C.c_uint64, [vp]),
        "vr_debug_read_volume": (i32, [vp, vp]),
        "vr_debug_read_volume_native": (i32, [vp, vp]),
        "vr_debug_volume_info": (i32, [vp, C.POINTER(u32), C.POINTER(f32), C.POINTER(i32)]),
        "vr_set_transfer_function": (i32, [vp, C.POINTER(u32), u32]),
        "vr_set_slicing": (i32, [vp, C.POINTER(f32), C.POINTER(f32)]),
        "vr_render": (i32, [vp, C.POINTER(vr_camera), C.POINTER(vr_params), vp, i32]),
        "vr_render_device": (i32, [vp, C.POINTER(vr_camera), C.POINTER(vr_params), vp, i32, u32, u32, u32, vp]),
        "vr_shard_rows": (u32, [u32, u32, u32]),
        "vr_assemble_rows": (i32, [vp, vp, vp, i32, u32, u32, vp]),
        "vr_count_work": (i32, [vp, C.POINTER(vr_camera), C.POINTER(vr_params), u32, u32, u32, C.POINTER(vr_stats)]),
        "vr_timing_enable": (i32, [vp, i32]),
        "vr_timing_read": (i32, [vp, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
        "vr_timing_reset": (i32, [vp]),
        "vr_kernel_name": (C.c_char_p, [vp, C.POINTER(vr_params)]),
        "vr_import_memory_fd": (C.c_int, [vp, C.c_int, C.c_uint64, C.c_uint64, C.POINTER(vp),
                                          C.POINTER(vp)]),
        "vr_release_external_memory": (C.c_int, [vp, vp]),
        "vr_debug_set_knob": (i32, [vp, i32, i32]),
        "vr_debug_timing_member": (i32, [vp, i32, C.POINTER(vr_member_timing)]),
        "vr_debug_host_profile_enable": (i32, [vp, i32]),
        "vr_debug_host_profile_member": (i32, [vp, i32, C.POINTER(vr_dist_host_profile)]),
        "vr_set_row_share": (i32, [vp, u32, u32]),
        "vr_get_row_share": (i32, [vp, C.POINTER(u32), C.POINTER(u32)]),
        "vr_shard_rows_ctx": (u32, [vp, u32, u32, u32]),
        "vr_set_memory_budget": (i32, [vp, C.c_uint64]),
        "vr_memory_report": (i32, [vp, C.POINTER(vr_memory_info)]),
        "vr_prepare": (i32, [vp, C.POINTER(vr_camera), C.POINTER(vr_params)]),
        "vr_debug_get_knob": (i32, [vp, i32, C.POINTER(i32)]),
        "vr_debug_create_members": (vp, [C.POINTER(i32), i32, u32, u32, i32]),
        "vr_debug_fail_member": (i32, [vp, i32, C.c_uint64]),
        "vr_cam_init": (None, [C.POINTER(vr_orbit_camera)]),
        "vr_cam_rotate": (None, [C.POINTER(vr_orbit_camera), f32, f32]),
        "vr_cam_zoom": (None, [C.POINTER(vr_orbit_camera), f32]),
        "vr_cam_position": (None, [C.POINTER(vr_orbit_camera), C.POINTER(f32)]),
        "vr_cam_view": (None, [C.POINTER(vr_orbit_camera), C.POINTER(f32)]),
        "vr_cam_to_camera": (None, [C.POINTER(vr_orbit_camera), C.POINTER(vr_camera)]),
        "vr_gradient_create": (vp, []),
        "vr_gradient_destroy": (None, [vp]),
        "vr_gradient_add_color_marker": (i32, [vp, f32, f32, f32, f32]),
        "vr_gradient_add_alpha_marker": (i32, [vp, f32, f32]),
        "vr_gradient_remove_color_marker": (i32, [vp, C.c_size_t]),
        "vr_gradient_remove_alpha_marker": (i32, [vp, C.c_size_t]),
        "vr_gradient_set_alpha_marker": (i32, [vp, C.c_size_t, f32, f32]),
        "vr_gradient_set_color_marker": (i32, [vp, C.c_size_t, f32, f32, f32, f32]),
        "vr_gradient_marker_count": (C.c_size_t, [vp, i32]),
        "vr_gradient_sample": (None, [vp, f32, C.POINTER(f32)]),
        "vr_gradient_discretize": (i32, [vp, C.c_size_t, C.POINTER(u32)]),
        "vr_nrrd_load": (i32, [C.c_char_p, C.POINTER(vr_dataset)]),
        "vr_nrrd_write_raw": (i32, [C.c_char_p, vp, i32, C.POINTER(u32)]),
        "vr_csv_load": (i32, [C.POINTER(C.c_char_p), C.c_size_t, C.POINTER(vr_dataset)]),
        "vr_dataset_free": (None, [C.POINTER(vr_dataset)]),
        "vr_host_last_error": (C.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.vr_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH} has ABI {L.vr_abi_version()}, this binding expects "
                           f"{ABI_VERSION}: rebuild it")
    _LIB = L
    return L


def default_params(**overrides) -> vr_params:
    p = vr_params()
    lib().vr_params_default(C.byref(p))
    for k, v in overrides.items():
        if k == "clear_color":
            for i in range(4):
                p.clear_color[i] = v[i]
        else:
            setattr(p, k, v)
    return p


# --------------------------------------------------------------------------------------
# Inputs that feed the pass (C++ restatements in host/vr_host.cpp)
# --------------------------------------------------------------------------------------
class OrbitCamera:
    """Vol::Scene::Camera (src/scene/camera.cpp:7-48), via vr_cam_*."""

    def __init__(self):
        self._c = vr_orbit_camera()
        lib().vr_cam_init(C.byref(self._c))

    def rotate(self, dx: float, dy: float) -> "OrbitCamera":
        lib().vr_cam_rotate(C.byref(self._c), dx, dy)
        return self

    def zoom(self, delta: float) -> "OrbitCamera":
        lib().vr_cam_zoom(C.byref(self._c), delta)
        return self

    def set_radius(self, r: float) -> "OrbitCamera":
        self._c.radius = r
        return self

    @property
    def radius(self) -> float:
        return float(self._c.radius)

    def get_position(self) -> np.ndarray:
        out = (C.c_float * 3)()
        lib().vr_cam_position(C.byref(self._c), out)
        return np.array(out[:], dtype=np.float32)

    def get_view(self) -> np.ndarray:
        out = (C.c_float * 16)()
        lib().vr_cam_view(C.byref(self._c), out)
        return np.array(out[:], dtype=np.float32)

    def to_vr_camera(self) -> vr_camera:
        cam = vr_camera()
        lib().vr_cam_to_camera(C.byref(self._c), C.byref(cam))
        return cam


def make_camera(radius: float = 3.0, rotate=None) -> OrbitCamera:
    cam = OrbitCamera()
    if rotate is not None:
        cam.rotate(float(rotate[0]), float(rotate[1]))
    cam.set_radius(radius)
    return cam


class Gradient:
    """Vol::UI::Components::Gradient (src/ui/components/gradient.cpp), via vr_gradient_*."""

    def __init__(self):
        self._g = lib().vr_gradient_create()

    def __del__(self):
        if getattr(self, "_g", None):
            lib().vr_gradient_destroy(self._g)
            self._g = None

    def add_color_marker(self, loc, rgb) -> int:
        return lib().vr_gradient_add_color_marker(self._g, loc, *[float(x) for x in rgb])

    def add_alpha_marker(self, loc, a) -> int:
        return lib().vr_gradient_add_alpha_marker(self._g, loc, float(a))

    def remove_color_marker(self, i) -> bool:
        return bool(lib().vr_gradient_remove_color_marker(self._g, i))

    def remove_alpha_marker(self, i) -> bool:
        return bool(lib().vr_gradient_remove_alpha_marker(self._g, i))

    def set_alpha_marker(self, i, loc, a) -> int:
        return lib().vr_gradient_set_alpha_marker(self._g, i, loc, float(a))

    def set_color_marker(self, i, loc, rgb) -> int:
        return lib().vr_gradient_set_color_marker(self._g, i, loc, *[float(x) for x in rgb])

    def marker_count(self, alpha: bool) -> int:
        return int(lib().vr_gradient_marker_count(self._g, 1 if alpha else 0))

    def sample(self, loc) -> np.ndarray:
        out = (C.c_float * 4)()
        lib().vr_gradient_sample(self._g, loc, out)
        return np.array(out[:], dtype=np.float32)

    def discretize(self, count: int = 256) -> np.ndarray:
        out = (C.c_uint32 * count)()
        if lib().vr_gradient_discretize(self._g, count, out) != 0:
            raise RuntimeError("discretize failed")
        return np.array(out[:], dtype=np.uint32)


@dataclass
class Dataset:
    """Vol::Data::Dataset (src/data/dataset.h:9-13), kept in the file's native dtype."""
    dims: tuple
    vmin: float
    vmax: float
    data: np.ndarray  # shape (nz, ny, nx), native dtype, x fastest


def _take_dataset(ds: vr_dataset) -> Dataset:
    dims = tuple(int(x) for x in ds.dims)
    npdt = DTYPE_TO_NP[ds.dtype]
    n = dims[0] * dims[1] * dims[2]
    buf = (C.c_char * (n * npdt.itemsize)).from_address(ds.data)
    # one copy out of the library's buffer, which is freed below
    arr = np.frombuffer(buf, dtype=npdt).reshape(dims[2], dims[1], dims[0]).copy()
    out = Dataset(dims, float(ds.vmin), float(ds.vmax), arr)
    lib().vr_dataset_free(C.byref(ds))
    return out


def load_nrrd(path: str) -> Dataset:
    """NrrdFileParser::parse (nrrd_file_parser.cpp:21-47); raises RuntimeError like the reference."""
    ds = vr_dataset()
    rc = lib().vr_nrrd_load(path.encode(), C.byref(ds))
    if rc != 0:
        raise RuntimeError(lib().vr_host_last_error().decode())
    return _take_dataset(ds)


def load_csv(paths: Sequence[str]) -> Dataset:
    """CsvFileParser::parse (csv_file_parser.cpp:14-50)."""
    arr = (C.c_char_p * len(paths))(*[p.encode() for p in paths])
    ds = vr_dataset()
    rc = lib().vr_csv_load(arr, len(paths), C.byref(ds))
    if rc != 0:
        raise RuntimeError(lib().vr_host_last_error().decode())
    return _take_dataset(ds)


def write_nrrd_raw(nhdr_path: str, data: np.ndarray) -> None:
    """Write data (nz, ny, nx) as a detached raw NRRD pair (nhdr + raw)."""
    data = np.ascontiguousarray(data)
    dims = (C.c_uint32 * 3)(data.shape[2], data.shape[1], data.shape[0])
    rc = lib().vr_nrrd_write_raw(nhdr_path.encode(), data.ctypes.data, NP_TO_DTYPE[data.dtype], dims)
    if rc != 0:
        raise RuntimeError(lib().vr_host_last_error().decode())


# --------------------------------------------------------------------------------------
# The pass
# --------------------------------------------------------------------------------------
class OffscreenPass:
    """Mirror of Vol::Rendering::OffscreenPass (offscreen_pass.h:40-54) over the C ABI."""

    def __init__(self, width: int, height: int, device: int = 0, device_mask: Optional[int] = None,
                 members: Optional[Sequence[int]] = None, exchange: int = EXCHANGE_COPY):
        """device: the HIP device (vr_create); device_mask: render every frame across these
        devices instead (vr_create_mask, bit d = device d); members: an explicit member list
        whose devices may repeat (vr_debug_create_members, the one-GPU rehearsal), with the
        shards reaching member 0 by `exchange` (EXCHANGE_COPY or EXCHANGE_RCCL)."""
        L = lib()
        self.n_members = len(members) if members is not None else (
            1 if device_mask is None else bin(device_mask).count("1"))
        if members is not None:
            devs = (C.c_int * len(members))(*members)
            self._ctx = L.vr_debug_create_members(devs, len(members), width, height, exchange)
            what = "vr_debug_create_members"
        elif device_mask is None:
            self._ctx = L.vr_create(device, width, height)
            what = "vr_create"
        else:
            self._ctx = L.vr_create_mask(device_mask, width, height)
            what = "vr_create_mask"
        if not self._ctx:
            raise RuntimeError(f"{what} failed: {L.vr_last_error(None).decode()}")

    # -- lifecycle --
    def close(self):
        if getattr(self, "_ctx", None):
            lib().vr_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown: module globals may already be gone
            pass

    def _check(self, rc: int, what: str):
        if rc != 0:
            raise RuntimeError(f"{what} failed ({rc}): {lib().vr_last_error(self._ctx).decode()}")

    @property
    def device_mask(self) -> int:
        m = C.c_uint32()
        self._check(lib().vr_get_device_mask(self._ctx, C.byref(m)), "vr_get_device_mask")
        return int(m.value)

    @property
    def size(self):
        w, h = C.c_uint32(), C.c_uint32()
        self._check(lib().vr_get_size(self._ctx, C.byref(w), C.byref(h)), "vr_get_size")
        return int(w.value), int(h.value)

    # -- reference setters --
    def framebuffer_size_changed(self, width: int, height: int):
        self._check(lib().vr_resize(self._ctx, width, height), "framebuffer_size_changed")

    def volume_dataset_changed(self, dataset: Dataset):
        data = np.ascontiguousarray(dataset.data)
        nx, ny, nz = dataset.dims
        assert data.size == nx * ny * nz, "dataset dims do not match data"
        self._check(lib().vr_set_volume(self._ctx, data.ctypes.data, NP_TO_DTYPE[data.dtype],
                                        nx, ny, nz, float(dataset.vmin), float(dataset.vmax)),
                    "volume_dataset_changed")

    def volume_dataset_changed_device(self, ptr: int, dtype, dims, vmin, vmax, stream: int = 0):
        nx, ny, nz = dims
        self._check(lib().vr_set_volume_device(self._ctx, C.c_void_p(ptr), NP_TO_DTYPE[np.dtype(dtype)],
                                               nx, ny, nz, float(vmin), float(vmax),
                                               C.c_void_p(stream or None)),
                    "volume_dataset_changed(device)")

    def generate_volume(self, dims, dtype=np.float32, seed: int = 2024, kind: int = 0):
        lo, hi = C.c_float(), C.c_float()
        self._check(lib().vr_generate_volume(self._ctx, kind, NP_TO_DTYPE[np.dtype(dtype)],
                                             dims[0], dims[1], dims[2], seed,
                                             C.byref(lo), C.byref(hi)), "vr_generate_volume")
        return float(lo.value), float(hi.value)

    def read_volume(self, native: bool = False) -> np.ndarray:
        """The resident volume as (nz, ny, nx) float32, or (native=True) in its storage type
        (uint8/int8/uint16/int16/float32: 1/4 of the host memory for 8-bit volumes)."""
        dims, mm, st = self.volume_info()
        shape = (dims[2], dims[1], dims[0])
        if native:
            out = np.empty(shape, dtype=(np.uint8, np.int8, np.uint16, np.int16, np.float32)[st])
            self._check(lib().vr_debug_read_volume_native(self._ctx, out.ctypes.data),
                        "vr_debug_read_volume_native")
            return out
        out = np.empty(shape, dtype=np.float32)
        self._check(lib().vr_debug_read_volume(self._ctx, out.ctypes.data), "vr_debug_read_volume")
        return out

    def volume_info(self):
        dims = (C.c_uint32 * 3)()
        mm = (C.c_float * 2)()
        st = C.c_int()
        self._check(lib().vr_debug_volume_info(self._ctx, dims, mm, C.byref(st)), "vr_debug_volume_info")
        return tuple(dims[:]), (float(mm[0]), float(mm[1])), int(st.value)

    def volume_bytes(self) -> int:
        return int(lib().vr_volume_bytes(self._ctx))

    def slicing_changed(self, vmin, vmax):
        a = (C.c_float * 3)(*[float(x) for x in vmin])
        b = (C.c_float * 3)(*[float(x) for x in vmax])
        self._check(lib().vr_set_slicing(self._ctx, a, b), "slicing_changed")

    def transfer_function_changed(self, data):
        arr = np.ascontiguousarray(np.asarray(data, dtype=np.uint32))
        ptr = arr.ctypes.data_as(C.POINTER(C.c_uint32))
        self._check(lib().vr_set_transfer_function(self._ctx, ptr, int(arr.size)),
                    "transfer_function_changed")

    # -- record/render --
    def render(self, camera: OrbitCamera, params: Optional[vr_params] = None,
               out_format: int = OUT_RGBA32F, out: Optional[np.ndarray] = None) -> np.ndarray:
        """Synchronous full frame into host memory: (H, W, 4) float32 or uint8 (into `out`
        when given, e.g. a buffer reused frame after frame)."""
        w, h = self.size
        p = params if params is not None else default_params()
        cam = camera.to_vr_camera() if isinstance(camera, OrbitCamera) else camera
        dt = np.float32 if out_format == OUT_RGBA32F else np.uint8
        if out is None:
            out = np.empty((h, w, 4), dtype=dt)
        elif out.shape != (h, w, 4) or out.dtype != dt or not out.flags.c_contiguous:
            raise ValueError(f"out must be a C-contiguous ({h}, {w}, 4) {np.dtype(dt).name} array")
        self._check(lib().vr_render(self._ctx, C.byref(cam), C.byref(p), out.ctypes.data, out_format),
                    "render")
        return out

    def render_device(self, camera, params, out_ptr: int, out_format: int = OUT_RGBA8,
                      row_block: int = 16, rank: int = 0, nranks: int = 1, stream: int = 0):
        cam = camera.to_vr_camera() if isinstance(camera, OrbitCamera) else camera
        self._check(lib().vr_render_device(self._ctx, C.byref(cam), C.byref(params),
                                           C.c_void_p(out_ptr), out_format, row_block, rank,
                                           nranks, C.c_void_p(stream or None)), "render_device")

    def assemble_rows(self, gathered_ptr: int, out_ptr: int, out_format: int, row_block: int,
                      nranks: int, stream: int = 0):
        self._check(lib().vr_assemble_rows(self._ctx, C.c_void_p(gathered_ptr), C.c_void_p(out_ptr),
                                           out_format, row_block, nranks, C.c_void_p(stream or None)),
                    "assemble_rows")

    def count_work(self, camera, params, row_block=16, rank=0, nranks=1) -> dict:
        cam = camera.to_vr_camera() if isinstance(camera, OrbitCamera) else camera
        st = vr_stats()
        self._check(lib().vr_count_work(self._ctx, C.byref(cam), C.byref(params), row_block, rank,
                                        nranks, C.byref(st)), "count_work")
        return dict(rays=st.rays, samples=st.samples, shaded_samples=st.shaded_samples,
                    steps=st.steps, skipped_samples=st.skipped_samples)

    def timing_enable(self, on: bool = True):
        self._check(lib().vr_timing_enable(self._ctx, 1 if on else 0), "timing_enable")

    def timing_read(self):
        ms, n = C.c_double(), C.c_uint64()
        self._check(lib().vr_timing_read(self._ctx, C.byref(ms), C.byref(n)), "timing_read")
        return float(ms.value), int(n.value)

    def timing_reset(self):
        self._check(lib().vr_timing_reset(self._ctx), "timing_reset")

    def kernel_name(self, params) -> str:
        return lib().vr_kernel_name(self._ctx, C.byref(params)).decode()

    def timing_member(self, member: int) -> dict:
        """vr_debug_timing_member: one device's summed kernel / render / gather / assembly ms."""
        t = vr_member_timing()
        self._check(lib().vr_debug_timing_member(self._ctx, member, C.byref(t)), "timing_member")
        return dict(device=int(t.device), frames=int(t.frames), kernel_ms=float(t.kernel_ms),
                    render_ms=float(t.render_ms), gather_ms=float(t.gather_ms),
                    assemble_ms=float(t.assemble_ms))

    # -- ABI 7: row shares, derived-structure memory, preparation --
    def fail_member(self, member: int, frame: int):
        """vr_debug_fail_member: member's enqueue of pipeline frame `frame` fails (VR_EIO)."""
        self._check(lib().vr_debug_fail_member(self._ctx, member, frame), "vr_debug_fail_member")

    def set_row_share(self, first_weight: int, other_weight: int):
        self._check(lib().vr_set_row_share(self._ctx, first_weight, other_weight), "set_row_share")

    def row_share(self):
        a, b = C.c_uint32(), C.c_uint32()
        self._check(lib().vr_get_row_share(self._ctx, C.byref(a), C.byref(b)), "row_share")
        return int(a.value), int(b.value)

    def shard_rows(self, height: int, row_block: int, nranks: int) -> int:
        return int(lib().vr_shard_rows_ctx(self._ctx, height, row_block, nranks))

    def set_memory_budget(self, nbytes: int):
        self._check(lib().vr_set_memory_budget(self._ctx, C.c_uint64(nbytes)), "set_memory_budget")

    def memory_report(self) -> dict:
        m = vr_memory_info()
        self._check(lib().vr_memory_report(self._ctx, C.byref(m)), "memory_report")
        return {n: int(getattr(m, n)) for n, _ in vr_memory_info._fields_}

    def prepare(self, camera, params):
        cam = camera.to_vr_camera() if isinstance(camera, OrbitCamera) else camera
        self._check(lib().vr_prepare(self._ctx, C.byref(cam), C.byref(params)), "prepare")

    # -- include/vr/vr_debug.h: launch-policy overrides for tests (speed only, never results) --
    def host_profile_enable(self, on: bool = True):
        """vr_debug_host_profile_enable (multi-device contexts): per-member host enqueue time."""
        self._check(lib().vr_debug_host_profile_enable(self._ctx, int(bool(on))), "host_profile_enable")

    def host_profile_member(self, member: int) -> dict:
        """vr_debug_host_profile_member: member's host microseconds per frame, by step."""
        h = vr_dist_host_profile()
        self._check(lib().vr_debug_host_profile_member(self._ctx, member, C.byref(h)),
                    "host_profile_member")
        n = max(int(h.frames), 1)
        return dict(frames=int(h.frames), **{k: getattr(h, k) / n for k, _ in vr_dist_host_profile._fields_[1:]})

    def set_knob(self, name: str, value: int):
        self._check(lib().vr_debug_set_knob(self._ctx, KNOBS[name], int(value)), f"set_knob({name})")

    def get_knob(self, name: str) -> int:
        v = C.c_int()
        self._check(lib().vr_debug_get_knob(self._ctx, KNOBS[name], C.byref(v)), f"get_knob({name})")
        return int(v.value)

    @contextlib.contextmanager
    def knobs(self, **kw):
        """Set knobs for the duration of a with-block (auto values restored after)."""
        for k, v in kw.items():
            self.set_knob(k, v)
        try:
            yield self
        finally:
            for k in kw:
                self.set_knob(k, KNOB_AUTO[k])


def dist_unique_id() -> bytes:
    """Rank 0: a fresh RCCL communicator id (vr_dist_unique_id) to send to every rank."""
    buf = C.create_string_buffer(DIST_ID_BYTES)
    rc = lib().vr_dist_unique_id(buf)
    if rc:
        raise RuntimeError(f"vr_dist_unique_id failed ({rc}): {lib().vr_dist_last_error(None).decode()}")
    return buf.raw


class DistFrames:
    """Multi-GPU frames of one OffscreenPass over RCCL (include/vr/vr_dist.h): this rank's
    row blocks -> ncclGather to rank 0 -> de-interleave there, all stream-ordered, with
    `frames_in_flight` frames in flight.  Every rank constructs it together (it blocks until
    all `nranks` have joined) with the same communicator id."""

    def __init__(self, rp: "OffscreenPass", uid: bytes, nranks: int, rank: int,
                 row_block: int = 8, frames_in_flight: int = 3):
        if len(uid) != DIST_ID_BYTES:
            raise ValueError("communicator id must be DIST_ID_BYTES bytes")
        self.rank, self.nranks = rank, nranks
        self._rp = rp  # keeps the context alive
        self._d = lib().vr_dist_create(rp._ctx, C.create_string_buffer(uid, DIST_ID_BYTES),
                                       nranks, rank, row_block, frames_in_flight)
        if not self._d:
            raise RuntimeError(f"vr_dist_create failed: {lib().vr_dist_last_error(None).decode()}")

    def _check(self, rc: int, what: str):
        if rc:
            raise RuntimeError(f"{what} failed ({rc}): {lib().vr_dist_last_error(self._d).decode()}")

    def render(self, camera, params, frame_ptr: int = 0, stream: int = 0):
        """Enqueue one frame; rank 0's RGBA8 frame (H x W x 4 bytes at frame_ptr) is complete
        once `stream` passes this point."""
        cam = camera.to_vr_camera() if isinstance(camera, OrbitCamera) else camera
        self._check(lib().vr_dist_render(self._d, C.byref(cam), C.byref(params),
                                         C.c_void_p(frame_ptr or None), C.c_void_p(stream or None)),
                    "vr_dist_render")

    def synchronize(self):
        self._check(lib().vr_dist_synchronize(self._d), "vr_dist_synchronize")

    def timing_enable(self, on: bool = True):
        self._check(lib().vr_dist_timing_enable(self._d, 1 if on else 0), "vr_dist_timing_enable")

    def host_profile(self, enable=None):
        """Host microseconds per frame of each step vr_dist_render enqueues (vr_dist.h host
        profile), averaged since the last read, and the frames counted; enable=True/False
        switches the profiling first (then returns None)."""
        if enable is not None:
            self._check(lib().vr_dist_host_profile_enable(self._d, 1 if enable else 0),
                        "vr_dist_host_profile_enable")
            return None
        h = vr_dist_host_profile()
        self._check(lib().vr_dist_host_profile_read(self._d, C.byref(h)), "vr_dist_host_profile_read")
        n = max(int(h.frames), 1)
        return dict(frames=int(h.frames), **{k: getattr(h, k) / n for k, _ in vr_dist_host_profile._fields_[1:]})

    def timing_read(self):
        """(render ms, gather ms, frames) summed over the frames since timing was enabled (or
        last read): HIP events around this rank's render and its ncclGather."""
        r, g, n = C.c_double(), C.c_double(), C.c_uint64()
        self._check(lib().vr_dist_timing_read(self._d, C.byref(r), C.byref(g), C.byref(n)),
                    "vr_dist_timing_read")
        return r.value, g.value, n.value

    def close(self):
        if getattr(self, "_d", None):
            lib().vr_dist_destroy(self._d)
            self._d = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


KERNEL_SOURCES = ("csrc/vr_kernels.hip", "csrc/vr_internal.h", "csrc/vr_exact_math.h", "Makefile")


def kernel_source_hash() -> str:
    """sha256 (16 hex digits) of the kernel sources (round 4's key; kept for the record)."""
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(HERE, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _elf_sections(b: bytes, base: int = 0):
    import struct
    shoff = struct.unpack_from("<Q", b, base + 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, base + 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", b, base + shoff + i * shentsize) for i in range(shnum)]
    names = base + secs[shstrndx][4]
    return [(b[names + s[0]:b.index(b"\0", names + s[0])],) + s for s in secs]


def kernel_code_hash(path: Optional[str] = None) -> str:
    """sha256 (16 hex digits) of the frame kernels' machine code in the library: every
    instantiation of march_kernel, march_pair_kernel (lane groups: small row shares) and
    order_tiles_kernel (the adaptive tile order inside a frame) -- gfx950 code bytes and kernel
    descriptor (register counts, LDS, kernarg size; the descriptor's layout-dependent
    code-entry offset zeroed), read from the code object in the `.hip_fatbin` ELF section.
    Keys measured per-kernel figures (the PMC traffic bench.py's roofline reads) to the machine
    code they were measured on: host-only edits and changes to other kernels leave it
    unchanged, any change to a kernel a frame launches moves it (the build is deterministic;
    ADVICE r5: the pair and tile-order kernels were not hashed before)."""
    import hashlib
    import re
    import struct
    b = open(path or LIB_PATH, "rb").read()
    fb = [s for s in _elf_sections(b) if s[0] == b".hip_fatbin"]
    if not fb:
        raise RuntimeError(f"{path or LIB_PATH} has no .hip_fatbin section")
    fat = b[fb[0][5]:fb[0][5] + fb[0][6]]
    syms = []
    for p in (m.start() for m in re.finditer(b"__CLANG_OFFLOAD_BUNDLE__", fat)):
        q = p + 32
        for _ in range(struct.unpack_from("<Q", fat, p + 24)[0]):
            off, size, tl = struct.unpack_from("<QQQ", fat, q)
            triple = fat[q + 24:q + 24 + tl]
            q += 24 + tl
            if b"gfx950" not in triple:
                continue
            co = fat[p + off:p + off + size]
            secs = _elf_sections(co)
            st = next(s for s in secs if s[0] == b".symtab")
            strt = next(s for s in secs if s[0] == b".strtab")
            for i in range(st[6] // 24):
                nm, _, _, shndx, val, sz = struct.unpack_from("<IBBHQQ", co, st[5] + i * 24)
                name = co[strt[5] + nm:co.index(b"\0", strt[5] + nm)]
                frame_kernel = any(k in name for k in (b"12march_kernel", b"17march_pair_kernel",
                                                         b"18order_tiles_kernel"))
                if frame_kernel and 0 < shndx < len(secs) and sz > 0:
                    sec = secs[shndx]
                    code = bytearray(co[sec[5] + val - sec[4]:sec[5] + val - sec[4] + sz])
                    if name.endswith(b".kd") and len(code) >= 24:
                        code[16:24] = bytes(8)  # kernel_code_entry_byte_offset
                    syms.append((name, bytes(code)))
    if not syms:
        raise RuntimeError(f"{path or LIB_PATH}: no march_kernel code in the gfx950 code object")
    h = hashlib.sha256()
    for name, code in sorted(syms):
        h.update(name)
        h.update(code)
    return h.hexdigest()[:16]


def shard_rows(height: int, row_block: int, nranks: int) -> int:
    return int(lib().vr_shard_rows(height, row_block, nranks))


def unorm8(img: np.ndarray) -> np.ndarray:
    """Float RGBA -> R8G8B8A8_UNORM exactly as the kernel stores it: (u8)(clamp*255 + 0.5)."""
    v = np.clip(np.nan_to_num(img.astype(np.float32), nan=0.0), np.float32(0), np.float32(1))
    return np.floor(v * np.float32(255.0) + np.float32(0.5)).astype(np.uint8)
