"""Sweep the phase-split thresholds of the persistent kernel (one process, one GPU).
  python scripts/sweep_ps.py [scene W H spp]"""
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import webgputracer_amd as w  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "bunny"
W, H, spp = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1920, 1080, 64)
ctx = w.Context(0)
ctx.upload_scene(*w.mesh_scene(scene))
cam = w.camera_param(W / H, spp, 0)
grid = [(t, s) for t, s in itertools.product(
    [int(v) for v in os.environ.get("PS_T", "16,24,32,40,48").split(",")],
    [int(v) for v in os.environ.get("PS_S", "4,8,12,16").split(",")]) if s < t]
for t, s in [(24, 8)] + grid:
    os.environ["WGT_PS_TO_TRAV"], os.environ["WGT_PS_TO_SERVICE"] = str(t), str(s)
    ms = min(ctx.render_tile(cam, W, H, want=("u8",), stats=True)["stats"]["kernel_ms"] for _ in range(2))
    print(json.dumps({"scene": scene, "to_trav": t, "to_service": s, "ms": round(ms, 2)}), flush=True)
ctx.close()
