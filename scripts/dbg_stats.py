"""Debug: STATS counters of a 100x60/9spp bunny render after a given call sequence.
  python scripts/dbg_stats.py SEQ   (SEQ: comma list of kf0 kf1 kf2 s0 s1)"""
import json
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, ROOT)
import webgputracer_amd as w  # noqa: E402

ctx = w.Context(0)
L, Q, S, T = w.mesh_scene("bunny")
out = []
for step in sys.argv[1].split(","):
    for k in ("WGT_PQ_LPT", "WGT_KERNEL", "WGT_WF_RAYS", "WGT_WF_CHUNK"):
        os.environ.pop(k, None)
    if step.startswith("kf"):
        os.environ.update({"WGT_KERNEL": step[2], "WGT_WF_RAYS": "2", "WGT_WF_CHUNK": "256"})
        W, H, spp, seed, a = 72, 40, 4, 21, 16 / 9
    else:
        os.environ["WGT_PQ_LPT"] = step[1]
        W, H, spp, seed, a = 100, 60, 9, 3, 5 / 3
    ctx.upload_scene(L, Q, S, T)
    g = ctx.render_tile(w.camera_param(a, spp, seed), W, H, stats=True)
    out.append((step, g["stats"]["pixels"]))
print(json.dumps({"seq": sys.argv[1], "pixels": out}), flush=True)
