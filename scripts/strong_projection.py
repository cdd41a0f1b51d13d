"""Projected strong-scaling efficiency of C4 (one 1080p/256spp frame split over N GPUs) from
one GPU: rank r of N renders only its share of the frame's 32x32 tiles
(dist.shard_tiles(W, H, 32, [(0, 0)], r, N), bench.py --scaling strong), timed alone on an
idle device (HIP events around the launch on the context stream, after one warm-up), for
every r.  A rank's launch pays the same end-of-launch drain as a whole frame (each pixel's
samples are a serial RNG chain, path_tracer.wgsl:378, 381-395) at 1/N of the work, so
  efficiency(N) = T_full / (N * max_r T_r)
is what N ranks of the real job would reach without the gather (which adds ~1 MB per peer).

--frames K --pipeline P: a job of K frames instead, each split over the N GPUs (bench.py
--scaling strong): rank r renders its share of frame k on the context's pipeline stream k % P,
P frames in flight, timed from the first launch to the last one's end (host clock between two
device synchronisations), so a rank pays one drain per job instead of one per frame.  At N = 8
a rank's share of a 1080p frame (259k pixels) is fewer pixels than the device holds lanes
(6144 waves x 64), which P frames in flight make up for.

  python scripts/strong_projection.py [--scene sponza] [--reps 2] [--ns 2 4 8] [--frames 8 --pipeline 4]
"""
import argparse
import json
import os
import sys
import time

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
    ap.add_argument("--frames", type=int, default=1, help="frames per job (1: one launch per rank, alone)")
    ap.add_argument("--pipeline", type=int, default=1, help="frames in flight (1..4) when --frames > 1")
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

    def timed_job(rank, n):
        P = max(1, min(a.pipeline, 4))
        streams = [ctx.pipeline_stream(i) for i in range(P)]
        d_ts = [torch.from_numpy(wd.shard_tiles(W, H, T, [(k, k + 1)], rank, n).view(np.uint8).copy()).to(dev)
                for k in range(a.frames)]
        nt = len(d_ts[0]) // wd.TILE_DTYPE.itemsize
        outs = [torch.zeros((nt, T, T, 4), dtype=torch.uint8, device=dev) for _ in range(P)]
        best = None
        for rep in range(a.reps + 1):  # the first job warms up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k, d_t in enumerate(d_ts):
                ctx.render_tiles_async(cam, W, H, T, T, d_t.data_ptr(), nt, d_u8=outs[k % P].data_ptr(),
                                       stream=streams[k % P])
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / a.frames
            if rep > 0:
                best = ms if best is None else min(best, ms)
        return best

    if a.frames > 1:
        full = timed_job(0, 1)
        base = {"scene": a.scene, "frames": a.frames, "pipeline": a.pipeline, "build_id": w.build_id()}
        print(json.dumps({**base, "n": 1, "rank_ms_per_frame": [round(full, 3)], "efficiency": 1.0}), flush=True)
        for n in a.ns:
            ms = [timed_job(r, n) for r in range(n)]
            print(json.dumps({**base, "n": n, "rank_ms_per_frame": [round(x, 3) for x in ms],
                              "full_ms_per_frame": round(full, 3), "max_rank_ms_per_frame": round(max(ms), 3),
                              "efficiency": round(full / (n * max(ms)), 4)}), flush=True)
        ctx.close()
        return

    full = timed(wd.shard_tiles(W, H, T, [(0, 0)], 0, 1))
    print(json.dumps({"scene": a.scene, "n": 1, "rank_ms": [round(full, 3)], "full_ms": round(full, 3),
                      "efficiency": 1.0, "build_id": w.build_id()}), flush=True)
    for n in a.ns:
        ms = [timed(wd.shard_tiles(W, H, T, [(0, 0)], r, n)) for r in range(n)]
        print(json.dumps({"scene": a.scene, "n": n, "rank_ms": [round(x, 3) for x in ms], "full_ms": round(full, 3),
                          "max_rank_ms": round(max(ms), 3), "efficiency": round(full / (n * max(ms)), 4),
                          "build_id": w.build_id()}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
