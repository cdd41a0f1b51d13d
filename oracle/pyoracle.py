"""ctypes binding for the CPU oracle (oracle/wgt_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.  The oracle is a
literal restatement of resources/shader/path_tracer.wgsl (reference); parity is
UNPINNED by the reference (it has no tests/fixtures).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")

# Byte layouts -- identical to the product's wgt_api.h types.
QUAD_DTYPE = np.dtype([("pos", "<f4", 4), ("right", "<f4", 4), ("up", "<f4", 4), ("norm", "<f4", 4),
                       ("w", "<f4", 3), ("d", "<f4"), ("col", "<f4", 3), ("emissive", "<f4")])
SPHERE_DTYPE = np.dtype([("center", "<f4", 3), ("radius", "<f4"), ("col", "<f4", 3), ("emissive", "<f4")])
TRI_DTYPE = np.dtype([("v0", "<f4", 4), ("e1", "<f4", 4), ("e2", "<f4", 4), ("fn", "<f4", 4),
                      ("col", "<f4", 3), ("emissive", "<f4")])
CAMERA_DTYPE = np.dtype([("origin", "<f4", 3), ("pad0", "<f4"), ("target", "<f4", 3), ("pad1", "<f4"),
                         ("aspect", "<f4"), ("fovy", "<f4"), ("spp", "<u4"), ("seed", "<u4")])
assert QUAD_DTYPE.itemsize == 96 and SPHERE_DTYPE.itemsize == 32
assert TRI_DTYPE.itemsize == 80 and CAMERA_DTYPE.itemsize == 48

CNT_QUERIES, CNT_TRACED, CNT_SAMPLES, CNT_NAN_RAYS = 0, 1, 2, 3
NO_HIT = 0xFFFFFFFF

_lib = None


def build() -> None:
    """Compile the oracle with its Makefile (gcc; no GPU needed)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def use_build(name: str = "liboracle.so"):
    """Select the oracle build to load (bench.py's cpu_baseline times liboracle_v3.so,
    the same source built for x86-64-v3); resets the loaded library."""
    global _lib, _LIB_PATH
    _lib = None
    _LIB_PATH = os.path.join(_HERE, "build", name)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        L.o_sin.restype = ctypes.c_float
        L.o_sin.argtypes = [ctypes.c_float]
        L.o_cos.restype = ctypes.c_float
        L.o_cos.argtypes = [ctypes.c_float]
        L.o_tan.restype = ctypes.c_float
        L.o_tan.argtypes = [ctypes.c_float]
        L.o_radians.restype = ctypes.c_float
        L.o_radians.argtypes = [ctypes.c_float]
        L.o_rand_seq.restype = ctypes.c_uint32
        L.o_rand_seq.argtypes = [ctypes.c_uint32, ctypes.c_int, P]
        L.o_cornell_scene.argtypes = [P, P, P, P, P, P]
        L.o_make_quad.argtypes = [P, P, P, P, ctypes.c_int, P]
        L.o_make_triangle.argtypes = [P, P, P, P, ctypes.c_int, P]
        L.o_camera_param.argtypes = [ctypes.c_float, ctypes.c_uint32, ctypes.c_uint32, P]
        L.o_scene_create.restype = P
        L.o_scene_create.argtypes = [P, ctypes.c_int, P, ctypes.c_int, P, ctypes.c_int, P, ctypes.c_int]
        L.o_scene_destroy.argtypes = [P]
        L.o_trace.argtypes = [P, ctypes.c_int, P, P, P, P, ctypes.c_int]
        L.o_trace_tris.argtypes = [P, ctypes.c_int, P, P, P, P, ctypes.c_int]
        L.o_render.restype = ctypes.c_int
        L.o_render.argtypes = [P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.c_uint32, ctypes.c_uint32, P, P, P, P, ctypes.c_int]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def rand_seq(seed: int, n: int):
    out = np.zeros(n, np.float32)
    final = lib().o_rand_seq(seed & 0xFFFFFFFF, n, _p(out))
    return out, final


def cornell_scene():
    """Scene::Scene (scene.cpp:14-36) restated: (lights, quads, spheres) structured arrays."""
    lights = np.zeros(4, QUAD_DTYPE)
    quads = np.zeros(32, QUAD_DTYPE)
    spheres = np.zeros(4, SPHERE_DTYPE)
    nl, nq, ns = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    lib().o_cornell_scene(_p(lights), ctypes.byref(nl), _p(quads), ctypes.byref(nq), _p(spheres),
                          ctypes.byref(ns))
    return lights[:nl.value].copy(), quads[:nq.value].copy(), spheres[:ns.value].copy()


def make_triangles(v0, v1, v2, col, emissive=False):
    """Triangle ctor (triangle.cpp:3-16) for arrays of vertices (n,3)."""
    v0 = np.ascontiguousarray(v0, np.float32)
    v1 = np.ascontiguousarray(v1, np.float32)
    v2 = np.ascontiguousarray(v2, np.float32)
    col = np.ascontiguousarray(col, np.float32).reshape(3)
    out = np.zeros(len(v0), TRI_DTYPE)
    L = lib()
    for i in range(len(v0)):
        L.o_make_triangle(_p(v0[i]), _p(v1[i]), _p(v2[i]), _p(col), int(emissive),
                          ctypes.c_void_p(out.ctypes.data + i * TRI_DTYPE.itemsize))
    return out


def camera_param(aspect: float, spp: int, seed: int):
    cam = np.zeros(1, CAMERA_DTYPE)
    lib().o_camera_param(ctypes.c_float(aspect), spp, seed & 0xFFFFFFFF, _p(cam))
    return cam


class OracleScene:
    def __init__(self, lights, quads, spheres, tris=None):
        self._keep = [np.ascontiguousarray(a) for a in (lights, quads, spheres)]
        tris = np.zeros(0, TRI_DTYPE) if tris is None else np.ascontiguousarray(tris)
        self._keep.append(tris)
        self.n_lights, self.n_quads, self.n_spheres, self.n_tris = len(lights), len(quads), len(spheres), len(tris)
        self._L = lib()  # the build this scene was created with (use_build may switch later)
        self.h = self._L.o_scene_create(_p(self._keep[0]), len(lights), _p(self._keep[1]), len(quads),
                                      _p(self._keep[2]), len(spheres), _p(tris), len(tris))

    def close(self):
        if self.h:
            self._L.o_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render(self, cam, W, H, x0=0, y0=0, tw=None, th=None, nthreads=0, want=("f32", "u8", "hit")):
        tw = W if tw is None else tw
        th = H if th is None else th
        f32 = np.zeros((th, tw, 4), np.float32) if "f32" in want else None
        u8 = np.zeros((th, tw, 4), np.uint8) if "u8" in want else None
        hit = np.zeros((th, tw), np.uint32) if "hit" in want else None
        cnt = np.zeros(8, np.uint64)
        rc = self._L.o_render(self.h, _p(cam), W, H, x0, y0, tw, th, _p(f32), _p(u8), _p(hit), _p(cnt),
                            nthreads)
        if rc != 0:
            raise RuntimeError(f"o_render failed: {rc}")
        return {"f32": f32, "u8": u8, "hit": hit, "counters": cnt}

    def trace(self, start, direction, brute=False):
        start = np.ascontiguousarray(start, np.float32)
        direction = np.ascontiguousarray(direction, np.float32)
        n = len(start)
        pid = np.zeros(n, np.uint32)
        dist = np.zeros(n, np.float32)
        self._L.o_trace(self.h, n, _p(start), _p(direction), _p(pid), _p(dist), int(brute))
        return pid, dist

    def trace_tris(self, start, direction, brute=False):
        start = np.ascontiguousarray(start, np.float32)
        direction = np.ascontiguousarray(direction, np.float32)
        n = len(start)
        tid = np.zeros(n, np.uint32)
        t = np.zeros(n, np.float32)
        self._L.o_trace_tris(self.h, n, _p(start), _p(direction), _p(tid), _p(t), int(brute))
        return tid, t
