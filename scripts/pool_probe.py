"""Pool-kernel probe: the instrumented pass (stats) of a 1080p frame with WGT_POOL set,
printing traversal / service SIMT utilisation, wave cycles per phase and the pool events
the STATS build counts in the wgt_stats cycle fields (wgt_pool.hip: adopt = rays taken
from tickets, miss = failed claims, park = own rays parked at a traversal exit, return =
adopted rays written back, stash = finished own rays moved to a ticket, phases = service
passes per wave; without the pool those fields hold the region cycles of k_render_ps).
  WGT_POOL=6 python scripts/pool_probe.py [scene] [spp]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import webgputracer_amd as w  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "sponza"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
W, H = 1920, 1080
ctx = w.Context(0)
ctx.upload_scene(*w.mesh_scene(scene))
tiles = w.tile_grid(W, H, W)
dev = torch.device("cuda", 0)
d_t = torch.from_numpy(tiles.view(np.uint8).copy()).to(dev)
cam = w.camera_param(W / H, spp, 0)
st = ctx.render_tiles_stats(cam, W, H, W, H, d_t.data_ptr(), len(tiles))
pr = ctx.render_tiles_profile(cam, W, H, W, H, d_t.data_ptr(), len(tiles))
pr = ctx.render_tiles_profile(cam, W, H, W, H, d_t.data_ptr(), len(tiles))
pool = os.environ.get("WGT_POOL", "0")
out = {"scene": scene, "spp": spp, "pool": pool, "ms": round(pr["kernel_ms"], 3),
       "trav_util": round(st["trav_lane_steps"] / max(64 * st["trav_wave_steps"], 1), 4),
       "svc_util": round(st["loop_lane_iters"] / max(64 * st["loop_wave_iters"], 1), 4),
       "trav_wave_steps": st["trav_wave_steps"], "svc_wave_iters": st["loop_wave_iters"],
       "nodes": st["node_visits"], "tris": st["tri_tests"], "traced": st["traced_rays"],
       "cyc_service": st["cyc_service"], "cyc_trav": st["cyc_trav"]}
if pool == "0":  # k_render_ps: wave cycles per service-phase region (STATS, WGT_REGION)
    out["svc_regions"] = {k[4:]: round(st[k] / max(st["cyc_service"], 1), 4) for k in
                          ("cyc_refill", "cyc_finalise", "cyc_shade", "cyc_camera", "cyc_quads", "cyc_root")}
    out["svc_cyc_per_pass"] = round(st["cyc_service"] / max(st["loop_wave_iters"], 1), 1)
    out["trav_cyc_per_step"] = round(st["cyc_trav"] / max(st["trav_wave_steps"], 1), 1)
else:
    out.update({"adopt": st["cyc_refill"], "miss": st["cyc_finalise"], "park": st["cyc_shade"],
                "return": st["cyc_camera"], "stash": st["cyc_quads"], "phases": st["cyc_root"]})
print(json.dumps(out), flush=True)
ctx.close()
