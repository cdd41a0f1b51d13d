"""ms per frame of K frames issued back to back on the context's pipeline streams (2 in flight),
and of one frame alone, for the library in WGT_LIB_PATH.
  python scripts/pipeline_ab.py scene W H spp K"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import webgputracer_amd as w  # noqa: E402

scene, W, H, spp, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
T = 32
dev = torch.device("cuda", 0)
ctx = w.Context(0)
ctx.upload_scene(*w.mesh_scene(scene))
cam = w.camera_param(W / H, spp, 0)
tiles = w.tile_grid(W, H, T, seed=0)
d_tiles = torch.from_numpy(tiles.view(np.uint8).copy()).to(dev)
outs = [torch.zeros((len(tiles), T, T, 4), dtype=torch.uint8, device=dev) for _ in range(2)]
streams = [ctx.pipeline_stream(i) for i in range(2)]
for k in range(2):
    ctx.render_tiles_async(cam, W, H, T, T, d_tiles.data_ptr(), len(tiles), d_u8=outs[k].data_ptr(), stream=streams[k])
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(K):
    ctx.render_tiles_async(cam, W, H, T, T, d_tiles.data_ptr(), len(tiles), d_u8=outs[k % 2].data_ptr(),
                           stream=streams[k % 2])
torch.cuda.synchronize()
pipe = (time.perf_counter() - t0) / K * 1e3
t0 = time.perf_counter()
ctx.render_tiles_async(cam, W, H, T, T, d_tiles.data_ptr(), len(tiles), d_u8=outs[0].data_ptr(), stream=streams[0])
torch.cuda.synchronize()
alone = (time.perf_counter() - t0) * 1e3
print(json.dumps({"lib": os.path.basename(os.environ.get("WGT_LIB_PATH", "libwgt.so")), "scene": scene, "spp": spp,
                  "frames": K, "ms_per_frame_pipelined": round(pipe, 2), "ms_alone": round(alone, 2)}), flush=True)
ctx.close()
