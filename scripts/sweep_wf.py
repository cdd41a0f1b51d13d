"""Compare kernels and sweep wavefront knobs on one GPU (one process).
  python scripts/sweep_wf.py [scene] [W H spp]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import webgputracer_amd as w  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "bunny"
W, H, spp = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1920, 1080, 64)
ctx = w.Context(0)
ctx.upload_scene(*(w.cornell_scene() if scene == "cornell" else w.mesh_scene(scene)))
cam = w.camera_param(W / H, spp, 0)
print(json.dumps(ctx.scene_info()), flush=True)
ref = None
configs = [{"WGT_KERNEL": "1"}, {"WGT_KERNEL": "2"}]
for rays in ("1", "2", "4", "8"):
    configs.append({"WGT_KERNEL": "0", "WGT_WF_RAYS": rays})
for chunk in ("256", "512", "1024"):
    for refill in ("8", "16", "32"):
        configs.append({"WGT_KERNEL": "0", "WGT_WF_CHUNK": chunk, "WGT_WF_REFILL": refill})
only = os.environ.get("SWEEP_ONLY")  # e.g. "2": only that kernel, default knobs
if only:
    configs = [{"WGT_KERNEL": k} for k in only.split(",")]
base_env = dict(os.environ)
for cfg in configs:
    os.environ.clear()
    os.environ.update(base_env)
    os.environ.update(cfg)
    r = ctx.render_tile(cam, W, H, want=("u8",), stats=True)
    st = r["stats"]
    for _ in range(int(os.environ.get("REPS", "1")) - 1):  # min over reps (single frames vary ~2%)
        st["kernel_ms"] = min(st["kernel_ms"], ctx.render_tile(cam, W, H, want=("u8",), stats=True)["stats"]["kernel_ms"])
    same = ref is None or np.array_equal(r["u8"], ref)
    ref = r["u8"] if ref is None else ref
    print(json.dumps({**cfg, "ms": round(st["kernel_ms"], 2), "trace_ms": round(st["trace_ms"], 2),
                      "shade_ms": round(st["shade_ms"], 2), "iters": st["iterations"],
                      "Mrays_s": round(st["traced_rays"] / st["kernel_ms"] / 1e3, 1),
                      "svc_util": round(st["loop_lane_iters"] / max(64 * st["loop_wave_iters"], 1), 3),
                      "trav_util": round(st["trav_lane_steps"] / max(64 * st["trav_wave_steps"], 1), 3),
                      "svc_frac": round(st["cyc_service"] / max(st["cyc_service"] + st["cyc_trav"], 1), 3),
                      "svc_cyc_per_iter": round(st["cyc_service"] / max(st["loop_wave_iters"], 1), 1),
                      "trav_cyc_per_step": round(st["cyc_trav"] / max(st["trav_wave_steps"], 1), 1),
                      "wave_iters": st["loop_wave_iters"], "wave_steps": st["trav_wave_steps"],
                      "nodes": st["node_visits"], "tris": st["tri_tests"], "rays": st["traced_rays"],
                      "svc_regions": {k[4:]: round(st[k] / max(st["cyc_service"], 1), 3) for k in
                                      ("cyc_refill", "cyc_finalise", "cyc_shade", "cyc_camera", "cyc_quads",
                                       "cyc_root")},
                      "identical": bool(same)}), flush=True)
ctx.close()
