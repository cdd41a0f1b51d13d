"""One render through the C-ABI (for rocprofv3 runs).
  python scripts/render_once.py [scene] [W H spp]   (kernel/knobs via WGT_* env)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import webgputracer_amd as w  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "bunny"
W, H, spp = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1920, 1080, 64)
ctx = w.Context(0)
ctx.upload_scene(*w.mesh_scene(scene)) if scene != "cornell" else ctx.upload_scene(*w.cornell_scene())
r = ctx.render_tile(w.camera_param(W / H, spp, 0), W, H, want=("u8",))
ctx.close()
print("rendered", scene, W, H, spp)
