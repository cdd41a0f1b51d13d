"""ctypes binding of libwgt.so — the C-ABI declared in include/wgt_api.h.

The product has no CPU fallback: if libwgt.so is missing, loading fails loudly;
if no HIP device is present, wgt_create returns an error.  Build with
`python -c "import __graft_entry__ as g; g.build()"` or `make -C webgputracer_amd`.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WGT_LIB_PATH") or os.path.join(PKG_DIR, "libwgt.so")  # override: A/B runs

# Byte layouts of include/wgt_api.h (= the reference GPU buffers)
QUAD_DTYPE = np.dtype([("pos", "<f4", 4), ("right", "<f4", 4), ("up", "<f4", 4), ("norm", "<f4", 4),
                       ("w", "<f4", 3), ("d", "<f4"), ("col", "<f4", 3), ("emissive", "<f4")])
SPHERE_DTYPE = np.dtype([("center", "<f4", 3), ("radius", "<f4"), ("col", "<f4", 3), ("emissive", "<f4")])
TRI_DTYPE = np.dtype([("v0", "<f4", 4), ("e1", "<f4", 4), ("e2", "<f4", 4), ("face_norm", "<f4", 4),
                      ("col", "<f4", 3), ("emissive", "<f4")])
CAMERA_DTYPE = np.dtype([("origin", "<f4", 3), ("pad0", "<f4"), ("target", "<f4", 3), ("pad1", "<f4"),
                         ("aspect", "<f4"), ("fovy", "<f4"), ("spp", "<u4"), ("seed", "<u4")])
TILE_DTYPE = np.dtype([("x0", "<u4"), ("y0", "<u4"), ("seed", "<u4"), ("frame", "<u4")])
assert QUAD_DTYPE.itemsize == 96 and SPHERE_DTYPE.itemsize == 32
assert TRI_DTYPE.itemsize == 80 and CAMERA_DTYPE.itemsize == 48 and TILE_DTYPE.itemsize == 16

API_VERSION = 2  # WGT_API_VERSION of include/wgt_api.h
WGT_OK, WGT_E_INVALID, WGT_E_HIP, WGT_E_NOSCENE, WGT_E_IO, WGT_E_NOMEM = 0, -1, -2, -3, -4, -5
NO_HIT = 0xFFFFFFFF


class WgtStats(ctypes.Structure):
    _fields_ = [("queries", ctypes.c_uint64), ("traced_rays", ctypes.c_uint64), ("samples", ctypes.c_uint64),
                ("nan_rays", ctypes.c_uint64), ("node_visits", ctypes.c_uint64), ("tri_tests", ctypes.c_uint64),
                ("pixels", ctypes.c_uint64), ("loop_wave_iters", ctypes.c_uint64),
                ("loop_lane_iters", ctypes.c_uint64), ("trav_wave_steps", ctypes.c_uint64),
                ("trav_lane_steps", ctypes.c_uint64), ("cyc_service", ctypes.c_uint64),
                ("cyc_trav", ctypes.c_uint64), ("kernel_ms", ctypes.c_float),
                ("trace_ms", ctypes.c_float), ("shade_ms", ctypes.c_float), ("iterations", ctypes.c_uint32),
                ("cyc_refill", ctypes.c_uint64), ("cyc_finalise", ctypes.c_uint64),
                ("cyc_shade", ctypes.c_uint64), ("cyc_camera", ctypes.c_uint64), ("cyc_quads", ctypes.c_uint64),
                ("cyc_root", ctypes.c_uint64), ("stack_spills", ctypes.c_uint64),
                ("stack_refills", ctypes.c_uint64), ("stack_overflows", ctypes.c_uint64),
                ("top_node_visits", ctypes.c_uint64), ("cyc_node_steps", ctypes.c_uint64),
                ("cyc_top_steps", ctypes.c_uint64), ("cyc_tri_steps", ctypes.c_uint64),
                ("quad_ref_scans", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class WgtSceneInfo(ctypes.Structure):
    _fields_ = [("n_lights", ctypes.c_uint32), ("n_quads", ctypes.c_uint32), ("n_spheres", ctypes.c_uint32),
                ("n_tris", ctypes.c_uint32), ("bvh_nodes", ctypes.c_uint32), ("bvh_leaves", ctypes.c_uint32),
                ("bvh_max_depth", ctypes.c_uint32), ("bvh_max_leaf", ctypes.c_uint32),
                ("device_bytes", ctypes.c_uint64), ("sah_cost", ctypes.c_double), ("bvh_width", ctypes.c_uint32),
                ("bvh_stack", ctypes.c_uint32), ("bvh2_nodes", ctypes.c_uint32), ("bvh2_depth", ctypes.c_uint32),
                ("bvh_compact", ctypes.c_uint32), ("bvh_compact_step", ctypes.c_float), ("ps_waves", ctypes.c_uint32),
                ("ps_park", ctypes.c_uint32), ("ps_stack", ctypes.c_uint32), ("node_form", ctypes.c_uint32),
                ("ps_resident", ctypes.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# Every symbol include/wgt_api.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "wgt_create", "wgt_destroy", "wgt_last_error", "wgt_version", "wgt_build_id", "wgt_device_count",
    "wgt_upload_scene", "wgt_scene_info_get", "wgt_render_tile", "wgt_render_tiles_async",
    "wgt_render_tiles_stats", "wgt_render_tiles_profile", "wgt_trace_rays", "wgt_trace_rays_async", "wgt_sync", "wgt_selftest_math", "wgt_stream",
    "wgt_pipeline_stream",
    "wgt_scene_cornell", "wgt_make_triangles", "wgt_load_obj", "wgt_procedural_mesh",
    "wgt_write_obj", "wgt_write_png", "wgt_bvh_build", "wgt_bvh_build_compact",
    "wgt_render_frames",
]

_lib = None


class WgtError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"wgt error {code}: {msg}")
        self.code = code


def lib():
    """Load libwgt.so (raises if it was not built: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built; run __graft_entry__.build() (no CPU fallback exists)")
    # One HIP runtime per process: torch ships its own libamdhip64.so.7.  Loaded
    # first, it is the one libwgt.so binds to (same SONAME), so device pointers and
    # streams from torch and from libwgt.so belong to one runtime; loaded after
    # libwgt.so's /opt/rocm copy, torch's would initialise a second runtime, which
    # fails ("No HIP GPUs are available").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    P, U32, I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    sig = {
        "wgt_create": (I, [I, ctypes.POINTER(P)]),
        "wgt_destroy": (None, [P]),
        "wgt_last_error": (ctypes.c_char_p, [P]),
        "wgt_version": (I, []),
        "wgt_build_id": (ctypes.c_char_p, []),
        "wgt_device_count": (I, [ctypes.POINTER(I)]),
        "wgt_upload_scene": (I, [P, P, U32, P, U32, P, U32, P, U32]),
        "wgt_scene_info_get": (I, [P, ctypes.POINTER(WgtSceneInfo)]),
        "wgt_render_tile": (I, [P, P, U32, U32, U32, U32, U32, U32, P, P, P, P]),
        "wgt_render_tiles_async": (I, [P, P, U32, U32, U32, U32, P, U32, P, P, P, P]),
        "wgt_render_tiles_stats": (I, [P, P, U32, U32, U32, U32, P, U32, P]),
        "wgt_render_tiles_profile": (I, [P, P, U32, U32, U32, U32, P, U32, P]),
        "wgt_trace_rays": (I, [P, P, U32, P, P]),
        "wgt_trace_rays_async": (I, [P, P, U32, P, P, P]),
        "wgt_sync": (I, [P]),
        "wgt_selftest_math": (I, [P, U32, U32, P]),
        "wgt_stream": (P, [P]),
        "wgt_pipeline_stream": (P, [P, U32]),
        "wgt_scene_cornell": (I, [P, ctypes.POINTER(U32), P, ctypes.POINTER(U32), P, ctypes.POINTER(U32)]),
        "wgt_make_triangles": (I, [P, U32, P, I, P, P]),
        "wgt_load_obj": (I, [ctypes.c_char_p, P, P, I, P, ctypes.POINTER(U32)]),
        "wgt_procedural_mesh": (I, [I, U32, U32, P, ctypes.POINTER(U32)]),
        "wgt_write_obj": (I, [ctypes.c_char_p, P, U32]),
        "wgt_write_png": (I, [ctypes.c_char_p, P, U32, U32]),
        "wgt_bvh_build": (I, [P, U32, P, U32, P, ctypes.POINTER(WgtSceneInfo)]),
        "wgt_render_frames": (I, [P, P, U32, U32, P, U32, P, P]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("WGT_LIB_PATH") and not hasattr(L, name):
            continue  # an older build loaded for same-box A/B timing
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.wgt_version() != API_VERSION:  # the structs above mirror this version of include/wgt_api.h
        raise ImportError(f"{LIB_PATH}: ABI version {L.wgt_version()}, this wrapper mirrors {API_VERSION}")
    _lib = L
    return L


def ptr(a):
    """Host numpy array -> void* (None passes NULL)."""
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.c_void_p)


def check(rc, ctx=None):
    if rc != WGT_OK:
        msg = lib().wgt_last_error(ctx)
        raise WgtError(rc, msg.decode() if msg else "")
    return rc
