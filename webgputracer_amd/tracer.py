"""Python face of the C-ABI (include/wgt_api.h), used by tests and bench.py.

Mirrors the reference's host objects for the path-tracing hot path:
  Scene::Scene (scene.cpp:14-36)            -> cornell_scene(), mesh_scene()
  Scene::LoadObj (scene.cpp:56-131)         -> load_obj()
  Camera::Update (camera.cpp:64-70)         -> camera_param()
  Renderer::InitDevice / OnRender dispatch  -> Context.render_tile / render_tiles_async
  sample_hit (path_tracer.wgsl:290-310)     -> Context.trace_rays
The C++ mirror (include/wgt/{scene,camera,renderer}.h) is the same API for C++ callers.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import (CAMERA_DTYPE, QUAD_DTYPE, SPHERE_DTYPE, TILE_DTYPE, TRI_DTYPE, WgtSceneInfo, WgtStats,
                   WGT_E_HIP, WgtError, check, lib, ptr)

COL_WHITE = np.array([0.73, 0.73, 0.73], np.float32)  # color_util.h:8
MESH_KINDS = {"bunny": (0, 69451), "sponza": (1, 262267)}


def cornell_scene():
    """The reference Cornell box (scene.cpp:14-36): (lights[1], quads[17], spheres[1])."""
    L = lib()
    lights, quads, spheres = np.zeros(4, QUAD_DTYPE), np.zeros(32, QUAD_DTYPE), np.zeros(4, SPHERE_DTYPE)
    nl, nq, ns = ctypes.c_uint32(4), ctypes.c_uint32(32), ctypes.c_uint32(4)
    check(L.wgt_scene_cornell(ptr(lights), ctypes.byref(nl), ptr(quads), ctypes.byref(nq), ptr(spheres),
                              ctypes.byref(ns)))
    return lights[:nl.value].copy(), quads[:nq.value].copy(), spheres[:ns.value].copy()


def make_triangles(verts, col=COL_WHITE, emissive=False, translation=(0.0, 0.0, 0.0)):
    """Triangle ctor (triangle.cpp:3-16) on verts (n, 3, 3) after Vertex::Translate."""
    v = np.ascontiguousarray(verts, np.float32).reshape(-1, 9)
    out = np.zeros(len(v), TRI_DTYPE)
    c = np.ascontiguousarray(col, np.float32).reshape(3)
    t = np.ascontiguousarray(translation, np.float32).reshape(3)
    check(lib().wgt_make_triangles(ptr(v), len(v), ptr(c), int(emissive), ptr(t), ptr(out)))
    return out


def load_obj(path, col=COL_WHITE, translation=(0.0, 0.0, 0.0), emissive=False):
    """Scene::LoadObj (scene.cpp:56-65) through the own OBJ reader."""
    L = lib()
    c = np.ascontiguousarray(col, np.float32).reshape(3)
    t = np.ascontiguousarray(translation, np.float32).reshape(3)
    n = ctypes.c_uint32(0)
    check(L.wgt_load_obj(str(path).encode(), ptr(c), ptr(t), int(emissive), None, ctypes.byref(n)))
    out = np.zeros(n.value, TRI_DTYPE)
    check(L.wgt_load_obj(str(path).encode(), ptr(c), ptr(t), int(emissive), ptr(out), ctypes.byref(n)))
    return out[:n.value]


def write_obj(path, tris):
    check(lib().wgt_write_obj(str(path).encode(), ptr(np.ascontiguousarray(tris)), len(tris)))


def write_png(path, rgba8):
    rgba8 = np.ascontiguousarray(rgba8, np.uint8)
    h, w = rgba8.shape[:2]
    check(lib().wgt_write_png(str(path).encode(), ptr(rgba8), w, h))


def procedural_mesh(kind: str, target_tris: int | None = None, seed: int = 1):
    """Deterministic stand-in for an absent asset (kind: 'bunny' | 'sponza')."""
    k, default = MESH_KINDS[kind]
    target = default if target_tris is None else int(target_tris)
    L = lib()
    n = ctypes.c_uint32(0)
    check(L.wgt_procedural_mesh(k, target, seed, None, ctypes.byref(n)))
    out = np.zeros(n.value, TRI_DTYPE)
    check(L.wgt_procedural_mesh(k, target, seed, ptr(out), ctypes.byref(n)))
    return out[:n.value]


def mesh_scene(kind: str, target_tris: int | None = None, seed: int = 1, obj_path: str | None = None):
    """Mesh configs (BASELINE configs 3-5): reference light + the 5 Cornell walls +
    the mesh (the two inner boxes removed) + the dummy sphere."""
    lights, quads, spheres = cornell_scene()
    tris = load_obj(obj_path) if obj_path else procedural_mesh(kind, target_tris, seed)
    return lights, quads[:5].copy(), spheres, tris


def bvh_build(tris):
    """Host-only BVH build (wgt_bvh_build): (info, nodes (n, 8, 4) f32, leaf-ordered tris (n, 4, 4) f32)."""
    tris = np.ascontiguousarray(tris, TRI_DTYPE)
    L = lib()
    info = WgtSceneInfo()
    check(L.wgt_bvh_build(ptr(tris), len(tris), None, 0, None, ctypes.byref(info)))
    nodes = np.zeros((info.bvh_nodes, 8, 4), np.float32)
    recs = np.zeros((len(tris), 4, 4), np.float32)
    check(L.wgt_bvh_build(ptr(tris), len(tris), ptr(nodes), info.bvh_nodes, ptr(recs), ctypes.byref(info)))
    return info.as_dict(), nodes, recs


def bvh_build_compact(tris):
    """Host-only compact form of the same tree (wgt_bvh_build_compact):
    (cnodes (n, 16) u32, crefs (n, 4) i32, step)."""
    tris = np.ascontiguousarray(tris, TRI_DTYPE)
    L = lib()
    info = WgtSceneInfo()
    check(L.wgt_bvh_build(ptr(tris), len(tris), None, 0, None, ctypes.byref(info)))
    cn = np.zeros((info.bvh_nodes, 16), np.uint32)
    cr = np.zeros((info.bvh_nodes, 4), np.int32)
    step = ctypes.c_float(0.0)
    check(L.wgt_bvh_build_compact(ptr(tris), len(tris), ptr(cn), ptr(cr), info.bvh_nodes, ctypes.byref(step)))
    return cn, cr, step.value


def camera_param(aspect: float, spp: int, seed: int, fovy: float = 40.0):
    """Camera::Update (camera.cpp:64-70) with an explicit seed instead of RandSeed()."""
    cam = np.zeros(1, CAMERA_DTYPE)
    cam["origin"] = (278.0, 278.0, -800.0)
    cam["target"] = (278.0, 278.0, 0.0)
    cam["aspect"] = np.float32(aspect)
    cam["fovy"] = np.float32(fovy)
    cam["spp"] = spp
    cam["seed"] = seed & 0xFFFFFFFF
    return cam


def build_id() -> str:
    """The loaded library's kernel build id (wgt_build_id: hash of the HIP sources and flags)."""
    return lib().wgt_build_id().decode()


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib().wgt_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


class Context:
    """A HIP device context (wgt_ctx): owns the stream and the scene in HBM."""

    def __init__(self, device: int = 0):
        self._L = lib()
        h = ctypes.c_void_p()
        check(self._L.wgt_create(device, ctypes.byref(h)))
        self.h = h
        self.device = device
        self.n_prims = 0

    def close(self):
        if getattr(self, "h", None):
            self._L.wgt_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        return check(rc, self.h)

    def upload_scene(self, lights, quads, spheres, tris=None):
        lights = np.ascontiguousarray(lights, QUAD_DTYPE)
        quads = np.ascontiguousarray(quads, QUAD_DTYPE)
        spheres = np.ascontiguousarray(spheres, SPHERE_DTYPE)
        tris = np.zeros(0, TRI_DTYPE) if tris is None else np.ascontiguousarray(tris, TRI_DTYPE)
        self._check(self._L.wgt_upload_scene(self.h, ptr(lights), len(lights), ptr(quads), len(quads),
                                             ptr(spheres), len(spheres), ptr(tris) if len(tris) else None,
                                             len(tris)))
        self.n_prims = len(lights) + len(quads) + len(tris) + len(spheres)

    def scene_info(self):
        info = WgtSceneInfo()
        self._check(self._L.wgt_scene_info_get(self.h, ctypes.byref(info)))
        return info.as_dict()

    def render_tile(self, cam, W, H, x0=0, y0=0, tw=None, th=None, want=("u8", "f32", "hit"), stats=False):
        tw = W if tw is None else tw
        th = H if th is None else th
        u8 = np.zeros((th, tw, 4), np.uint8) if "u8" in want else None
        f32 = np.zeros((th, tw, 4), np.float32) if "f32" in want else None
        hit = np.zeros((th, tw), np.uint32) if "hit" in want else None
        st = WgtStats() if stats else None
        cam = np.ascontiguousarray(cam, CAMERA_DTYPE)
        self._check(self._L.wgt_render_tile(self.h, ptr(cam), W, H, x0, y0, tw, th, ptr(u8), ptr(f32), ptr(hit),
                                            ctypes.byref(st) if st is not None else None))
        return {"u8": u8, "f32": f32, "hit": hit, "stats": st.as_dict() if st is not None else None}

    def render_frames(self, cam, W, H, seeds, stats=False):
        """n whole frames in one launch (wgt_render_frames): (n, H, W, 4) uint8 (+ stats)."""
        seeds = np.ascontiguousarray(seeds, np.uint32)
        out = np.zeros((len(seeds), H, W, 4), np.uint8)
        st = WgtStats() if stats else None
        cam = np.ascontiguousarray(cam, CAMERA_DTYPE)
        self._check(self._L.wgt_render_frames(self.h, ptr(cam), W, H, ptr(seeds), len(seeds), ptr(out),
                                              ctypes.byref(st) if st is not None else None))
        return (out, st.as_dict()) if stats else out

    def render_tiles_async(self, cam, W, H, tw, th, d_tiles, n_tiles, d_u8=0, d_f32=0, d_hit=0, stream=0):
        """Device-pointer launch (ints are raw device addresses, 0 = NULL)."""
        cam = np.ascontiguousarray(cam, CAMERA_DTYPE)
        self._check(self._L.wgt_render_tiles_async(self.h, ptr(cam), W, H, tw, th, ctypes.c_void_p(d_tiles),
                                                   n_tiles, ctypes.c_void_p(d_u8 or None),
                                                   ctypes.c_void_p(d_f32 or None), ctypes.c_void_p(d_hit or None),
                                                   ctypes.c_void_p(stream or None)))

    def render_tiles_stats(self, cam, W, H, tw, th, d_tiles, n_tiles):
        st = WgtStats()
        cam = np.ascontiguousarray(cam, CAMERA_DTYPE)
        self._check(self._L.wgt_render_tiles_stats(self.h, ptr(cam), W, H, tw, th, ctypes.c_void_p(d_tiles),
                                                   n_tiles, ctypes.byref(st)))
        return st.as_dict()

    def render_tiles_profile(self, cam, W, H, tw, th, d_tiles, n_tiles):
        st = WgtStats()
        cam = np.ascontiguousarray(cam, CAMERA_DTYPE)
        self._check(self._L.wgt_render_tiles_profile(self.h, ptr(cam), W, H, tw, th, ctypes.c_void_p(d_tiles),
                                                     n_tiles, ctypes.byref(st)))
        return st.as_dict()

    def trace_rays(self, start, direction):
        start = np.asarray(start, np.float32).reshape(-1, 3)
        direction = np.asarray(direction, np.float32).reshape(-1, 3)
        n = len(start)
        soa = np.ascontiguousarray(np.concatenate([start.T, direction.T], axis=0), np.float32)
        prim = np.zeros(n, np.uint32)
        dist = np.zeros(n, np.float32)
        self._check(self._L.wgt_trace_rays(self.h, ptr(soa), n, ptr(prim), ptr(dist)))
        return prim, dist

    def trace_rays_async(self, d_rays, n, d_prim, d_dist, stream=0):
        self._check(self._L.wgt_trace_rays_async(self.h, ctypes.c_void_p(d_rays), n, ctypes.c_void_p(d_prim),
                                                 ctypes.c_void_p(d_dist), ctypes.c_void_p(stream or None)))

    def stream(self) -> int:
        return self._L.wgt_stream(self.h) or 0

    def pipeline_stream(self, i: int) -> int:
        """The context's i-th pipeline stream (own hardware queue; frames issued round-robin overlap)."""
        s = self._L.wgt_pipeline_stream(self.h, i)
        if not s:
            raise WgtError(WGT_E_HIP, (self._L.wgt_last_error(self.h) or b"").decode())
        return s

    def sync(self):
        self._check(self._L.wgt_sync(self.h))

    def selftest_math(self, n: int, seed: int = 1):
        """-> dict of wgt_selftest_math's counts (include/wgt_api.h)."""
        counts = np.zeros(8, np.uint64)
        self._check(self._L.wgt_selftest_math(self.h, n, seed, counts.ctypes.data_as(ctypes.c_void_p)))
        keys = ("sqrt_tests", "sqrt_rn_bad", "div_tests", "div_rn_bad", "sqrt_fast_tests", "sqrt_fast_bad",
                "compiler_sqrt_bad", "compiler_div_bad")
        return dict(zip(keys, (int(c) for c in counts)))


def tile_grid(W: int, H: int, T: int, seed: int = 0, frame: int = 0):
    """All T x T tiles of a W x H frame, row-major (x0, y0, seed, frame)."""
    ys, xs = np.meshgrid(np.arange(0, H, T, dtype=np.uint32), np.arange(0, W, T, dtype=np.uint32), indexing="ij")
    tiles = np.zeros(xs.size, TILE_DTYPE)
    tiles["x0"] = xs.ravel()
    tiles["y0"] = ys.ravel()
    tiles["seed"] = seed & 0xFFFFFFFF
    tiles["frame"] = frame
    return tiles
