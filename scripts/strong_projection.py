"""Projected strong-scaling efficiency of C4 (one 1080p/256spp frame split over N GPUs) from
one GPU: rank r of N renders only its share of the frame's 32x32 tiles
(dist.shard_tiles(W, H, 32, [(0, 0)], r, N), bench.py --scaling strong), timed alone on an
idle device (HIP events around the launch on the context stream, after one warm-up), for
every r.  A rank's launch pays the same end-of-launch drain as a whole frame (each pixel's
samples are a serial RNG chain, path_tracer.wgsl:378, 381-395) at 1/N of the work, so
  efficiency(N) = T_full / (N * max_r T_r)
is what N ranks of the real job would reach without the gather (which adds ~1 MB per peer).

  python scripts/strong_projection.py [--scene sponza] [--reps 2] [--ns 2 4 8] > out.jsonl
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="sponza")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--ns", type=int, nargs="+", default=[2, 4, 8])
    a = ap.parse_args()
    import torch

    import webgputracer_amd as w
    from webgputracer_amd import dist as wd

    W, H, T = a.width, a.height, a.tile
    ctx = w.Context(0)
    ctx.upload_scene(*w.mesh_scene(a.scene))
    dev = torch.device("cuda", 0)
    cam = w.camera_param(W / H, a.spp, 0)
    stream = torch.cuda.Stream(device=dev)

    def timed(tiles):
        d_t = torch.from_numpy(tiles.view(np.uint8).copy()).to(dev)
        out = torch.zeros((len(tiles), T, T, 4), dtype=torch.uint8, device=dev)
        best = None
        for k in range(a.reps + 1):  # the first launch warms up
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(stream)
            ctx.render_tiles_async(cam, W, H, T, T, d_t.data_ptr(), len(tiles), d_u8=out.data_ptr(),
                                   stream=stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            if k > 0:
                best = ms if best is None else min(best, ms)
        return best

    full = timed(wd.shard_tiles(W, H, T, [(0, 0)], 0, 1))
    print(json.dumps({"scene": a.scene, "n": 1, "rank_ms": [round(full, 3)], "full_ms": round(full, 3),
                      "efficiency": 1.0, "build_id": w.build_id(),
                      "pool": os.environ.get("WGT_POOL", "0")}), flush=True)
    for n in a.ns:
        ms = [timed(wd.shard_tiles(W, H, T, [(0, 0)], r, n)) for r in range(n)]
        print(json.dumps({"scene": a.scene, "n": n, "rank_ms": [round(x, 3) for x in ms], "full_ms": round(full, 3),
                          "max_rank_ms": round(max(ms), 3), "efficiency": round(full / (n * max(ms)), 4),
                          "build_id": w.build_id(), "pool": os.environ.get("WGT_POOL", "0")}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
