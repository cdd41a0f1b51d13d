"""webgputracer_amd — MI355X-native (gfx950) path-tracing hot path of kugimasa/WebGPUTracer.

The per-pixel path tracer of resources/shader/path_tracer.wgsl re-built as hand-written
HIP kernels behind a C-ABI (include/wgt_api.h, libwgt.so), with a BVH + Moller-Trumbore
triangle extension, tile sharding over GPUs and an RCCL gather (webgputracer_amd.dist).
"""
from .tracer import (Context, build_id, bvh_build, bvh_build_compact, camera_param, cornell_scene, device_count, load_obj,
                     make_triangles, mesh_scene, procedural_mesh, tile_grid, write_obj, write_png)

__all__ = ["Context", "build_id", "bvh_build", "bvh_build_compact", "camera_param", "cornell_scene", "device_count", "load_obj",
           "make_triangles", "mesh_scene", "procedural_mesh", "tile_grid", "write_obj", "write_png"]
