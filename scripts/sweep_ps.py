"""Sweep the phase-split thresholds / kernel choice on one GPU (one process).
  python scripts/sweep_ps.py [scene] [W H spp]"""
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
ref = None
configs = [("1", None, None)] + [("0", str(x), str(y)) for x, y in itertools.product([24, 32, 40, 48, 56], [8, 16, 24])
                                   if y < x]
for kern, x, y in configs:
    os.environ["WGT_KERNEL"] = kern
    if x:
        os.environ["WGT_PS_TO_TRAV"], os.environ["WGT_PS_TO_SERVICE"] = x, y
    ctx.render_tile(cam, W, H, want=("u8",))  # warm
    r = ctx.render_tile(cam, W, H, want=("u8",), stats=True)
    st = r["stats"]
    same = ref is None or (r["u8"] == ref).all()
    ref = r["u8"] if ref is None else ref
    print(json.dumps({"kernel": kern, "to_trav": x, "to_service": y, "ms": round(st["kernel_ms"], 2),
                      "Mrays_s": round(st["traced_rays"] / st["kernel_ms"] / 1e3, 1),
                      "svc_util": round(st["loop_lane_iters"] / max(64 * st["loop_wave_iters"], 1), 3),
                      "trav_util": round(st["trav_lane_steps"] / max(64 * st["trav_wave_steps"], 1), 3),
                      "identical": bool(same)}), flush=True)
ctx.close()
