"""Where the traversal phase's time goes by BVH level (bound the LDS node-tile
lever before building it).  One instrumented pass (wgt_render_tiles_stats: the STATS kernel,
s_memtime around every traversal step) over
  * the whole frame (the steady state and its drain), and
  * rank 0's share of the frame split over N GPUs (dist.shard_tiles; fewer pixels than lanes),
printing per pass: the share of node visits at levels 1-2 (the root's children and grandchildren;
the root is tested in the service phase), the share of node-step cycles spent in steps whose
visiting lanes are all at levels 1-2 (what an LDS copy of those levels could shorten: a step waits
for its slowest lane), and the node / triangle step shares of the traversal phase's cycles.

  python scripts/level_stats.py [--scene sponza] [--n 8] [--spp 64]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="sponza")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--n", type=int, default=8)
    a = ap.parse_args()
    import torch

    import webgputracer_amd as w
    from webgputracer_amd import dist as wd

    W, H, T = a.width, a.height, a.tile
    ctx = w.Context(0)
    ctx.upload_scene(*w.mesh_scene(a.scene))
    info = ctx.scene_info()
    dev = torch.device("cuda", 0)
    cam = w.camera_param(W / H, a.spp, 0)
    out = []
    for name, tiles in (("frame", wd.shard_tiles(W, H, T, [(0, 0)], 0, 1)),
                        (f"share_1_of_{a.n}", wd.shard_tiles(W, H, T, [(0, 0)], 0, a.n))):
        d_t = torch.from_numpy(tiles.view(np.uint8).copy()).to(dev)
        st = ctx.render_tiles_stats(cam, W, H, T, T, d_t.data_ptr(), len(tiles))
        trav = max(st["cyc_trav"], 1)
        out.append({"pass": name, "tiles": len(tiles), "node_visits": st["node_visits"],
                    "top_node_visits": st["top_node_visits"],
                    "top_visit_frac": round(st["top_node_visits"] / max(st["node_visits"], 1), 4),
                    "node_step_cyc_frac_of_trav": round(st["cyc_node_steps"] / trav, 4),
                    "tri_step_cyc_frac_of_trav": round(st["cyc_tri_steps"] / trav, 4),
                    "top_only_step_cyc_frac_of_node_steps": round(st["cyc_top_steps"] / max(st["cyc_node_steps"], 1), 4),
                    "top_only_step_cyc_frac_of_trav": round(st["cyc_top_steps"] / trav, 4),
                    "trav_frac_of_wave_cycles": round(st["cyc_trav"] / max(st["cyc_trav"] + st["cyc_service"], 1), 4),
                    "quad_ref_scans_per_ray": round(st["quad_ref_scans"] / max(st["traced_rays"], 1), 6)})
    print(json.dumps({"scene": a.scene, "frame": f"{W}x{H}/{a.spp}spp", "bvh_nodes": info["bvh_nodes"],
                      "node_form": info["node_form"], "passes": out}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
