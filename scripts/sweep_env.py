"""Time one render per env setting (one process, one GPU), min of REPS.
  python scripts/sweep_env.py scene W H spp "K=V,K=V;K=V;..."   """
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import webgputracer_amd as w  # noqa: E402

scene, W, H, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
envs = [e for e in sys.argv[5].split(";")]
ctx = w.Context(0)
ctx.upload_scene(*(w.cornell_scene() if scene == "cornell" else w.mesh_scene(scene)))
cam = w.camera_param(W / H, spp, 0)
ref = None
base = dict(os.environ)
for env in envs:
    os.environ.clear()
    os.environ.update(base)
    for kv in filter(None, env.split(",")):
        k, v = kv.split("=")
        os.environ[k] = v
    if os.environ.get("REUPLOAD"):  # builder knobs: rebuild the BVH under this env
        ctx.upload_scene(*(w.cornell_scene() if scene == "cornell" else w.mesh_scene(scene)))
    runs = [ctx.render_tile(cam, W, H, want=("u8",), stats=True) for _ in range(int(os.environ.get("REPS", "2")))]
    st = runs[0]["stats"]
    same = ref is None or np.array_equal(runs[0]["u8"], ref)
    ref = runs[0]["u8"] if ref is None else ref
    print(json.dumps({"scene": scene, "spp": spp, "env": env, "ms": round(min(r["stats"]["kernel_ms"] for r in runs), 2),
                      "trav_util": round(st["trav_lane_steps"] / max(64 * st["trav_wave_steps"], 1), 3),
                      "wave_steps": st["trav_wave_steps"], "nodes": st["node_visits"], "tris": st["tri_tests"],
                      "bvh": {k: v for k, v in ctx.scene_info().items() if k in ("bvh_nodes", "bvh_stack",
                              "bvh_max_depth", "sah_cost")}, "identical": bool(same)}), flush=True)
ctx.close()
