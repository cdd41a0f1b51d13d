"""Tail timeline of one persistent-kernel launch (needs a build with the WGT_DUMP_TAIL
instrumentation): per wave, the s_memrealtime (100 MHz) when the queue first ran dry
for it, when its live lanes fell to <= 32 and <= 8, and when it exited.
  WGT_LIB_PATH=ab/x_tail.so python scripts/tail_timeline.py [scene W H spp]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import webgputracer_amd as w  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "bunny"
W, H, spp = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1920, 1080, 256)
ctx = w.Context(0)
ctx.upload_scene(*w.mesh_scene(scene))
cam = w.camera_param(W / H, spp, 0)
path = "/tmp/wgt_tail.bin"
os.environ["WGT_DUMP_TAIL"] = path
for rep in range(2):
    r = ctx.render_tile(cam, W, H, want=("u8",))
a = np.fromfile(path, np.uint32).reshape(-1, 4).astype(np.int64)
t0 = a[:, 0][a[:, 0] > 0].min()
rel = (a - t0) / 100.0  # microseconds -> ms below
rel = rel / 1000.0
ex, t32, t8, tend = rel[:, 0], rel[:, 1], rel[:, 2], rel[:, 3]
q = lambda v: [round(float(np.percentile(v, p)), 2) for p in (0, 10, 50, 90, 99, 100)]
print(json.dumps({"scene": scene, "spp": spp, "waves": len(a),
                  "exhaust_ms_pct_0_10_50_90_99_100": q(ex), "le32_ms": q(t32), "le8_ms": q(t8), "exit_ms": q(tend)}))
ctx.close()
