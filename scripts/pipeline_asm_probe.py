"""Does bench.py's N=1 frame assembly (dist.ShardedFrames.gather: one index op after each launch, on the
launch's stream) delay the next frame of the pipeline?  ms per frame of K frames issued back to back on
the context's two pipeline streams, without the assembly, with it on the launch's stream, and with it
on a third stream (the next launch into the same buffer waits on it through an event).
  python scripts/pipeline_asm_probe.py scene W H spp K"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import webgputracer_amd as w  # noqa: E402
from webgputracer_amd.dist import assemble_index  # noqa: E402

scene, W, H, spp, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
T = 32
dev = torch.device("cuda", 0)
ctx = w.Context(0)
ctx.upload_scene(*w.mesh_scene(scene))
cam = w.camera_param(W / H, spp, 0)
tiles = w.tile_grid(W, H, T, seed=0)
d_tiles = torch.from_numpy(tiles.view(np.uint8).copy()).to(dev)
idx = torch.from_numpy(assemble_index(tiles, W, H, T, [0])).to(dev)
outs = [torch.zeros((len(tiles), T, T, 4), dtype=torch.uint8, device=dev) for _ in range(2)]
streams = [torch.cuda.ExternalStream(ctx.pipeline_stream(i), device=dev) for i in range(2)]
side = torch.cuda.Stream(device=dev)


def run(mode):
    done = [None, None]
    imgs = None
    for k in range(K):
        s = streams[k % 2]
        with torch.cuda.stream(s):
            if done[k % 2] is not None:
                s.wait_event(done[k % 2])
            ctx.render_tiles_async(cam, W, H, T, T, d_tiles.data_ptr(), len(tiles), d_u8=outs[k % 2].data_ptr(),
                                   stream=s.cuda_stream)
            if mode == "same":
                imgs = outs[k % 2].reshape(-1, 4)[idx]
            elif mode == "side":
                ev = torch.cuda.Event()
                ev.record(s)
                side.wait_event(ev)
                with torch.cuda.stream(side):
                    imgs = outs[k % 2].reshape(-1, 4)[idx]
                    done[k % 2] = torch.cuda.Event()
                    done[k % 2].record(side)
    return imgs


for mode in ("none", "same", "side", "none", "same", "side"):
    run(mode)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(mode)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / K * 1e3
    print(json.dumps({"scene": scene, "spp": spp, "frames": K, "assembly": mode, "ms_per_frame": round(ms, 2)}),
          flush=True)
ctx.close()
