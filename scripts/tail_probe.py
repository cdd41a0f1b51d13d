"""Tail probe: time one launch over the frame's tiles (N copies, each copy a different
frame id, so different seeds) for N = 1, 2, 4.  T(N) = a + b*N; the intercept a is
the launch tail (the last wave rounds running partly empty), b the steady per-frame cost.
  python scripts/tail_probe.py [scene] [W H spp T]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import webgputracer_amd as w  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "bunny"
W, H, spp, T = (int(v) for v in sys.argv[2:6]) if len(sys.argv) > 5 else (1920, 1080, 64, 8)
ctx = w.Context(0)
ctx.upload_scene(*w.mesh_scene(scene))
cam = w.camera_param(W / H, spp, 0)
dev = torch.device("cuda", 0)
stream = torch.cuda.Stream(device=dev)
torch.cuda.set_stream(stream)
envs = [e for e in os.environ.get("TAIL_ENVS", "").split(";") if e] or [""]
for env in envs:
  for kv in env.split(","):
    if kv:
        k, v = kv.split("=")
        os.environ[k] = v
  res = {}
  for n in (1, 2, 4):
    tiles = np.concatenate([w.tile_grid(W, H, T, seed=f, frame=f) for f in range(n)])
    d_tiles = torch.from_numpy(tiles.view(np.uint8).copy()).to(dev)
    out = torch.zeros((len(tiles), T, T, 4), dtype=torch.uint8, device=dev)
    times = []
    for rep in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        ctx.render_tiles_async(cam, W, H, T, T, d_tiles.data_ptr(), len(tiles), d_u8=out.data_ptr(),
                               stream=stream.cuda_stream)
        b.record(stream)
        torch.cuda.synchronize()
        times.append(a.elapsed_time(b))
    res[n] = min(times)
    print(json.dumps({"scene": scene, "env": env, "copies": n, "waves": len(tiles), "ms": round(res[n], 2)}),
          flush=True)
  slope, icpt = np.polyfit([1, 2, 4], [res[1], res[2], res[4]], 1)
  print(json.dumps({"scene": scene, "env": env, "spp": spp, "per_frame_ms": round(float(slope), 2),
                    "tail_ms": round(float(icpt), 2), "tail_frac_of_1": round(float(icpt / res[1]), 3)}),
        flush=True)
ctx.close()
