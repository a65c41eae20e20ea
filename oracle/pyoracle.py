"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference ray-march (oracle/oracle.c).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the checker or the
reported CPU baseline, never as the thing measured or shipped.

Parity status: pinned by the closed-form KATs of SURVEY.md Appendix B and by an independent
float64 numpy restatement (oracle/ref_numpy.py); pixel parity against the real Vulkan
reference is unpinned (no Vulkan here, no reference outputs exist) — see DESIGN.md.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
NREF_PATH = os.path.join(HERE, "_ref", "libnrrdref.so")


class or_scene(C.Structure):
    _fields_ = [
        ("vol", C.POINTER(C.c_float)), ("nx", C.c_int32), ("ny", C.c_int32), ("nz", C.c_int32),
        ("vmin", C.c_float), ("vmax", C.c_float),
        ("tf", C.POINTER(C.c_uint32)), ("tf_n", C.c_int32),
        ("smin", C.c_float * 3), ("smax", C.c_float * 3),
        ("view", C.c_float * 16), ("cam_pos", C.c_float * 3),
        ("fovy_deg", C.c_float), ("znear", C.c_float), ("zfar", C.c_float),
        ("width", C.c_int32), ("height", C.c_int32),
        ("step", C.c_float), ("ray_dist", C.c_float), ("ert_eps", C.c_float),
        ("shading", C.c_int32), ("clear", C.c_float * 4),
        ("ka", C.c_float), ("kd", C.c_float), ("ks", C.c_float), ("spec_power", C.c_int32),
        ("vol_u8", C.POINTER(C.c_uint8)),
        ("grad_f16", C.c_int32),
        ("conf_weight_bits", C.c_int32), ("conf_flags", C.c_int32),
        ("grad_range_set", C.c_int32), ("grad_range", C.c_float * 2),
    ]


# conformance-study variants (oracle.h OR_CONF_*; tools/conformance_gap.py)
CONF_FMA, CONF_CLIP_ZO, CONF_RASTER, CONF_GPU_MATH = 1, 2, 4, 8


class or_stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("samples", C.c_uint64),
                ("shaded_samples", C.c_uint64), ("steps", C.c_uint64)]


_LIB = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.or_render_rows.restype = C.c_int
        L.or_render_rows.argtypes = [C.POINTER(or_scene), C.c_void_p, C.c_int, C.c_int, C.c_int,
                                     C.POINTER(or_stats)]
        L.or_render_row_list.restype = C.c_int
        L.or_render_row_list.argtypes = [C.POINTER(or_scene), C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                         C.POINTER(or_stats)]
        L.or_trilinear.restype = C.c_float
        L.or_trilinear.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float, C.c_float]
        L.or_tf_decode.restype = None
        L.or_tf_decode.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.or_tf_sample.restype = None
        L.or_tf_sample.argtypes = [C.c_void_p, C.c_int, C.c_float, C.c_void_p]
        L.or_pixel_ray.restype = C.c_int
        L.or_pixel_ray.argtypes = [C.POINTER(or_scene), C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_max_threads.restype = C.c_int
        _LIB = L
    return _LIB


class Scene:
    """Inputs of one oracle render; field meaning as include/vr/vr.h."""

    def __init__(self, vol, vmin, vmax, tf, view, cam_pos, width, height, smin=(0, 0, 0),
                 smax=(1, 1, 1), step=0.005, ray_dist=1.8, ert_eps=0.0, shading=0,
                 clear=(0.11, 0.11, 0.11, 1.0), ka=0.3, kd=0.7, ks=0.25, spec_power=16,
                 fovy_deg=40.0, znear=0.1, zfar=10.0, grad_f16=False, conf_weight_bits=0,
                 conf_flags=0):
        # (nz, ny, nx); u8 volumes are kept as u8 (float(v) is exact: same samples, 1/4 the
        # host memory of a float copy, e.g. C5's 2048^3)
        if np.asarray(vol).dtype == np.uint8:
            self.vol = np.ascontiguousarray(vol)
        else:
            self.vol = np.ascontiguousarray(vol, dtype=np.float32)
        self.tf = np.ascontiguousarray(np.asarray(tf, dtype=np.uint32))
        s = or_scene()
        if self.vol.dtype == np.uint8:
            s.vol_u8 = self.vol.ctypes.data_as(C.POINTER(C.c_uint8))
        else:
            s.vol = self.vol.ctypes.data_as(C.POINTER(C.c_float))
        s.nz, s.ny, s.nx = self.vol.shape
        s.vmin, s.vmax = float(vmin), float(vmax)
        s.tf = self.tf.ctypes.data_as(C.POINTER(C.c_uint32))
        s.tf_n = int(self.tf.size)
        for a in range(3):
            s.smin[a] = float(smin[a])
            s.smax[a] = float(smax[a])
            s.cam_pos[a] = float(cam_pos[a])
        for i in range(16):
            s.view[i] = float(view[i])
        s.fovy_deg, s.znear, s.zfar = fovy_deg, znear, zfar
        s.width, s.height = int(width), int(height)
        s.step, s.ray_dist, s.ert_eps = step, ray_dist, ert_eps
        s.shading = int(shading)
        for i in range(4):
            s.clear[i] = float(clear[i])
        s.ka, s.kd, s.ks, s.spec_power = ka, kd, ks, int(spec_power)
        s.grad_f16 = 1 if grad_f16 else 0
        if grad_f16:  # the device scales the binary16 field by the stored data's own range
            lo, hi = (float(np.min(self.vol)), float(np.max(self.vol))) if self.vol.size else (0.0, 0.0)
            s.grad_range_set = 1
            s.grad_range[0], s.grad_range[1] = lo, hi
        s.conf_weight_bits = int(conf_weight_bits)
        s.conf_flags = int(conf_flags)
        self.s = s

    def conformance(self, weight_bits=0, flags=0):
        """Switch the conformance-study variant (oracle.h OR_CONF_*); (0, 0) is the oracle."""
        self.s.conf_weight_bits = int(weight_bits)
        self.s.conf_flags = int(flags)
        return self

    @classmethod
    def from_params(cls, vol, vmin, vmax, tf, camera, width, height, params, smin=(0, 0, 0),
                    smax=(1, 1, 1), grad_f16=False):
        """Build from a vr_amd vr_camera / vr_params pair (same meaning as the C ABI).
        grad_f16: restate the device's binary16 difference field (a shaded f32 frame with
        params.exact_gradient == 0 whose kernel reads the field: kernel tag F32H in
        vr_kernel_name)."""
        return cls(vol, vmin, vmax, tf, list(camera.view), list(camera.position), width, height,
                   smin=smin, smax=smax, step=params.step, ray_dist=params.ray_dist,
                   ert_eps=params.ert_eps, shading=params.shading,
                   clear=list(params.clear_color), ka=params.ambient, kd=params.diffuse,
                   ks=params.specular, spec_power=params.spec_power,
                   fovy_deg=camera.fovy_deg or 40.0, znear=camera.znear or 0.1,
                   zfar=camera.zfar or 10.0, grad_f16=grad_f16,
                   conf_flags=CONF_CLIP_ZO if getattr(params, "depth_zero_to_one", 0) else 0)

    def render(self, row0=0, row1=None, nthreads=0):
        """Float RGBA (H, W, 4) and work stats; rows outside [row0, row1) are left at NaN."""
        H, W = self.s.height, self.s.width
        row1 = H if row1 is None else row1
        out = np.full((H, W, 4), np.nan, dtype=np.float32)
        st = or_stats()
        rc = lib().or_render_rows(C.byref(self.s), out.ctypes.data, row0, row1, nthreads, C.byref(st))
        if rc != 0:
            raise RuntimeError(f"or_render_rows failed ({rc})")
        return out, dict(rays=st.rays, samples=st.samples, shaded_samples=st.shaded_samples,
                         steps=st.steps, skipped_samples=0)  # the reference never skips

    def render_rows(self, rows, out=None, nthreads=0):
        """Render an arbitrary list of rows (OpenMP over the list) into `out` (H, W, 4)."""
        H, W = self.s.height, self.s.width
        if out is None:
            out = np.full((H, W, 4), np.nan, dtype=np.float32)
        rows = np.ascontiguousarray(np.asarray(rows, dtype=np.int32))
        st = or_stats()
        rc = lib().or_render_row_list(C.byref(self.s), out.ctypes.data, rows.ctypes.data,
                                      int(rows.size), nthreads, C.byref(st))
        if rc != 0:
            raise RuntimeError(f"or_render_row_list failed ({rc})")
        return out, dict(rays=st.rays, samples=st.samples, shaded_samples=st.shaded_samples,
                         steps=st.steps, skipped_samples=0)  # the reference never skips

    def pixel_ray(self, px, py):
        tex = np.zeros(3, np.float32)
        frag = np.zeros(3, np.float32)
        d = np.zeros(3, np.float32)
        ok = lib().or_pixel_ray(C.byref(self.s), px, py, tex.ctypes.data, frag.ctypes.data, d.ctypes.data)
        return bool(ok), tex, frag, d


def trilinear(vol, p):
    vol = np.ascontiguousarray(vol, dtype=np.float32)
    nz, ny, nx = vol.shape
    return float(lib().or_trilinear(vol.ctypes.data, nx, ny, nz, p[0], p[1], p[2]))


def tf_decode(tf):
    tf = np.ascontiguousarray(np.asarray(tf, dtype=np.uint32))
    out = np.empty((tf.size, 4), np.float32)
    lib().or_tf_decode(tf.ctypes.data, int(tf.size), out.ctypes.data)
    return out


def tf_sample(tf, t):
    tf = np.ascontiguousarray(np.asarray(tf, dtype=np.uint32))
    out = np.empty(4, np.float32)
    lib().or_tf_sample(tf.ctypes.data, int(tf.size), float(t), out.ctypes.data)
    return out


def field_scale_log2(vmin, vmax):
    lib().or_field_scale_log2.restype = C.c_int
    lib().or_field_scale_log2.argtypes = [C.c_float, C.c_float]
    return int(lib().or_field_scale_log2(vmin, vmax))


def round_f16(x):
    lib().or_round_f16.restype = C.c_float
    lib().or_round_f16.argtypes = [C.c_float]
    return float(lib().or_round_f16(x))


def max_threads():
    return int(lib().or_max_threads())


# ---- reference NrrdIO loader (oracle/_ref, built from the reference's own sources) ----
_NREF = None


def nrrdio_available():
    return os.path.exists(NREF_PATH)


def nrrdio_load(path):
    """NrrdFileParser::parse through the reference's NrrdIO: (dims, nrrd_type, float data, min, max)."""
    global _NREF
    if _NREF is None:
        L = C.CDLL(NREF_PATH)
        L.nref_load.restype = C.c_int
        L.nref_load.argtypes = [C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_int),
                                C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.nref_free.restype = None
        L.nref_free.argtypes = [C.POINTER(C.c_float)]
        _NREF = L
    dims = (C.c_uint32 * 3)()
    typ = C.c_int()
    data = C.POINTER(C.c_float)()
    lo, hi = C.c_float(), C.c_float()
    rc = _NREF.nref_load(path.encode(), dims, C.byref(typ), C.byref(data), C.byref(lo), C.byref(hi))
    if rc != 0:
        return rc, None
    n = dims[0] * dims[1] * dims[2]
    arr = np.ctypeslib.as_array(data, shape=(n,)).copy().reshape(dims[2], dims[1], dims[0])
    _NREF.nref_free(data)
    return 0, dict(dims=tuple(dims[:]), nrrd_type=typ.value, data=arr, vmin=lo.value, vmax=hi.value)
