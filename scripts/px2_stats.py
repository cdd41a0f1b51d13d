"""STATS counters and timing of the persistent kernel per variant (round 5, two pixels per lane).
  python scripts/px2_stats.py SCENE SPP VARIANT...   (VARIANT: name=K:V,K:V or name=)"""
import json
import os
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, ROOT)
import webgputracer_amd as w  # noqa: E402

scene, spp = sys.argv[1], int(sys.argv[2])
ctx = w.Context(0)
L, Q, S, T = w.mesh_scene(scene)
cam = w.camera_param(16 / 9, spp, 1)
for v in sys.argv[3:]:
    name, envs = v.split("=", 1)
    keys = []
    for e in filter(None, envs.split(",")):
        k, val = e.split(":")
        os.environ[k] = val
        keys.append(k)
    ctx.upload_scene(L, Q, S, T)
    info = ctx.scene_info()
    g = ctx.render_tile(cam, 1920, 1080, stats=True)
    ctx.render_tile(cam, 1920, 1080)
    t0 = time.perf_counter()
    for _ in range(3):
        ctx.render_tile(cam, 1920, 1080)
    ms = (time.perf_counter() - t0) / 3 * 1e3
    st = g["stats"]
    out = {"variant": name, "ms": round(ms, 2), "ps_waves": info["ps_waves"], "ps_resident": info.get("ps_resident")}
    out.update({k: (round(v, 3) if isinstance(v, float) else int(v)) for k, v in st.items()})
    tr = max(out.get("traced_rays", 1), 1)
    out["svc_iters_per_ray"] = round(out["loop_wave_iters"] * 64 / tr, 3)
    out["trav_wave_steps_per_ray"] = round(out["trav_wave_steps"] * 64 / tr, 3)
    out["simt_loop"] = round(out["loop_lane_iters"] / max(64 * out["loop_wave_iters"], 1), 4)
    out["simt_trav"] = round(out["trav_lane_steps"] / max(64 * out["trav_wave_steps"], 1), 4)
    out["cyc_svc_frac"] = round(out["cyc_service"] / max(out["cyc_service"] + out["cyc_trav"], 1), 4)
    if info["ps_waves"] == 4:  # k_render_ps2's STATS fields (wgt_kernels.hip)
        waves = max(int(info.get("ps_resident") or 1), 1)
        out["life_frac"] = round(out["cyc_refill"] / max(waves * out["cyc_root"], 1), 4)
        out["svc_loop_iters_per_wave"] = round(out["cyc_camera"] / waves, 1)
        out["trav_swaps_per_ray"] = round(out["stack_spills"] / tr, 4)
        out["svc_swaps_per_ray"] = round(out["stack_refills"] / tr, 4)
    print(json.dumps(out), flush=True)
    for k in keys:
        os.environ.pop(k)
