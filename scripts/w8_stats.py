"""Counters of one instrumented render per node form (round 5, the wide form):
  python scripts/w8_stats.py scene W H spp  (WGT_CNODE values in W8_FORMS, default "2 4")"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import webgputracer_amd as w  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "sponza"
W, H, spp = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1920, 1080, 16)
ctx = w.Context(0)
for cn in os.environ.get("W8_FORMS", "2 4").split():
    os.environ["WGT_CNODE"] = cn
    ctx.upload_scene(*w.mesh_scene(scene))
    info = ctx.scene_info()
    st = ctx.render_tile(w.camera_param(W / H, spp, 0), W, H, want=(), stats=True)["stats"]
    r = max(st["traced_rays"], 1)
    print(json.dumps({"scene": scene, "cnode": cn, "node_form": info["node_form"], "ps_resident": info["ps_resident"], 
                      "kernel_ms": round(st["kernel_ms"], 3), "nodes_per_ray": round(st["node_visits"] / r, 4),
                      "tris_per_ray": round(st["tri_tests"] / r, 4),
                      "tri_groups_pushed_per_ray": round(st["stack_spills"] / r, 4),
                      "tri_groups_popped_per_ray": round(st["stack_refills"] / r, 4),
                      "simt_bvh": round(st["trav_lane_steps"] / max(64 * st["trav_wave_steps"], 1), 4),
                      "w8": {k: info[k] for k in ("w8_groups", "w8_depth", "w8_stack", "w8_nodes", "w8_leaves")}}),
          flush=True)
ctx.close()
