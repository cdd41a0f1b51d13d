"""One render of a scene (profiling child).

  python scripts/render_once.py SCENE SPP            (1920x1080)
  python scripts/render_once.py SCENE W H SPP        (the older form, still accepted)

SCENE: sponza | bunny | cornell."""
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import webgputracer_amd as w  # noqa: E402

args = sys.argv[1:]
if len(args) == 2:
    scene, W, H, spp = args[0], 1920, 1080, int(args[1])
elif len(args) == 4:
    scene, W, H, spp = args[0], int(args[1]), int(args[2]), int(args[3])
else:
    raise SystemExit(__doc__)
ctx = w.Context(0)
if scene == "cornell":
    ctx.upload_scene(*w.cornell_scene())
else:
    ctx.upload_scene(*w.mesh_scene(scene))
ctx.render_tile(w.camera_param(W / H, spp, 1), W, H)
print("done", flush=True)
