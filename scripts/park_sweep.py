"""Frame time of the persistent kernel against its LDS bytes per wave:
the parked kernel at LDS stacks of 20 down to 12 entries (11 parked words + 3 B per entry per lane:
6,656 down to 5,120 B per wave) and the whole-stack kernel (6,144 B), sponza 1080p at 64 spp, each
the best of 3 isolated frames (event pair around the launch)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import webgputracer_amd as w  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "sponza"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
scene = w.mesh_scene(kind)
ctx = w.Context(0)
cam = w.camera_param(16 / 9, spp, 0)
for park, cap in [("0", ""), ("1", "20"), ("1", "19"), ("1", "18"), ("1", "17"), ("1", "16"), ("1", "14"),
                  ("1", "12"), ("0", "")]:
    os.environ["WGT_PARK"] = park
    if cap:
        os.environ["WGT_PS_CAP"] = cap
    else:
        os.environ.pop("WGT_PS_CAP", None)
    ctx.upload_scene(*scene)
    info = ctx.scene_info()
    ts = [ctx.render_tile(cam, 1920, 1080, want=("u8",), stats=True)["stats"] for _ in range(3)]
    lds = info["ps_stack"] * 64 * 3 + (11 * 64 * 4 if info["ps_park"] else 0)
    print(json.dumps({"scene": kind, "spp": spp, "park": info["ps_park"], "ps_stack": info["ps_stack"],
                      "lds_bytes_per_wave": lds, "kernel_ms": [round(s["kernel_ms"], 3) for s in ts],
                      "spills": ts[0]["stack_spills"], "refills": ts[0]["stack_refills"]}), flush=True)
ctx.close()
