"""Where the parked kernel's time goes: the instrumented pass's wave cycles
per phase and per service region (s_memtime, k_render_ps STATS) for WGT_PARK=0 and 1, sponza and
bunny 1080p at 16 spp, with the frame time of the uninstrumented launch (best of 3)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import webgputracer_amd as w  # noqa: E402

KEYS = ("cyc_service", "cyc_trav", "cyc_refill", "cyc_finalise", "cyc_shade", "cyc_camera", "cyc_quads", "cyc_root")
for kind in ("sponza", "bunny"):
    scene = w.mesh_scene(kind)
    ctx = w.Context(0)
    cam = w.camera_param(16 / 9, 16, 0)
    for park in ("0", "1", "0", "1"):
        os.environ["WGT_PARK"] = park
        os.environ["WGT_PS_CAP"] = "17"
        ctx.upload_scene(*scene)
        st = [ctx.render_tile(cam, 1920, 1080, want=("u8",), stats=True)["stats"] for _ in range(3)]
        s = st[0]
        tot = s["cyc_service"] + s["cyc_trav"]
        print(json.dumps({"scene": kind, "park": int(park), "kernel_ms": min(x["kernel_ms"] for x in st),
                          "wave_steps": s["trav_wave_steps"], "svc_passes": s["loop_wave_iters"],
                          **{k: round(s[k] / tot, 4) for k in KEYS}, "cyc_total": tot}), flush=True)
    ctx.close()
