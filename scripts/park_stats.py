"""Spill/refill counts of the parked persistent kernel on one
sponza / bunny 1080p frame at 16 spp, at the default LDS stack and at smaller ones
(WGT_PS_CAP, read at scene upload), with the frame time of each."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import webgputracer_amd as w  # noqa: E402

for kind in ("sponza", "bunny"):
    scene = w.mesh_scene(kind)
    ctx = w.Context(0)
    for cap in ("", "12", "8"):
        if cap:
            os.environ["WGT_PS_CAP"] = cap
        else:
            os.environ.pop("WGT_PS_CAP", None)
        ctx.upload_scene(*scene)
        info = ctx.scene_info()
        cam = w.camera_param(16 / 9, 16, 0)
        r = ctx.render_tile(cam, 1920, 1080, stats=True)
        st = r["stats"]
        t = ctx.render_tile(cam, 1920, 1080, stats=True)["stats"]["kernel_ms"]
        print(json.dumps({"scene": kind, "ps_stack": info["ps_stack"], "bvh_stack": info["bvh_stack"],
                          "traced_rays": st["traced_rays"], "node_visits": st["node_visits"],
                          "spills": st["stack_spills"], "refills": st["stack_refills"],
                          "spills_per_mray": round(st["stack_spills"] / st["traced_rays"] * 1e6, 2),
                          "kernel_ms_16spp": round(t, 3)}), flush=True)
    ctx.close()
