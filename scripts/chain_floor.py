"""The serial per-pixel sample chain's floor under strong scaling.

Each pixel's 256 samples are one serial RNG chain (path_tracer.wgsl:378, 381-395): the state a
sample starts from depends on how many rand() draws every earlier sample of the pixel made, so a
pixel runs on one lane from its first sample to its last.  A rank of a frame split over N = 8 GPUs
holds 259k pixels for the device's 393k lanes, so its launch ends with its slowest pixels' chains.

This script measures, on one GPU:
  1. every 32x32 tile of the frame rendered alone at --probe-spp (16 waves on an idle device: no
     wave shares a SIMD), to rank the tiles by cost;
  2. the --top most expensive tiles rendered alone at the full spp: the time of a tile alone is its
     slowest 8x8 block's chain at the least contention a launch can give it -- the chain floor;
  3. the N-way shares of the frame (dist.shard_tiles, rank r of N), each rendered alone, as
     scripts/strong_projection.py does.
It prints one JSON line: the floor, each share's time and the share's slowest tile alone, so that
the projected efficiency T_full / (N max_r T_r) can be read against the floor's T_full / (N floor).

  python scripts/chain_floor.py [--scene sponza] [--n 8] [--top 12]
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
    ap.add_argument("--probe-spp", type=int, default=16)
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    import torch

    import webgputracer_amd as w
    from webgputracer_amd import dist as wd

    W, H, T = a.width, a.height, a.tile
    ctx = w.Context(0)
    ctx.upload_scene(*w.mesh_scene(a.scene))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)

    def timed(tiles, spp, reps=1):
        cam = w.camera_param(W / H, spp, 0)
        d_t = torch.from_numpy(tiles.view(np.uint8).copy()).to(dev)
        out = torch.zeros((len(tiles), T, T, 4), dtype=torch.uint8, device=dev)
        best = None
        for k in range(reps + 1):  # the first launch warms up
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(stream)
            ctx.render_tiles_async(cam, W, H, T, T, d_t.data_ptr(), len(tiles), d_u8=out.data_ptr(),
                                   stream=stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            if k > 0:
                ms = e0.elapsed_time(e1)
                best = ms if best is None else min(best, ms)
        return best

    full = wd.shard_tiles(W, H, T, [(0, 0)], 0, 1)
    t_full = timed(full, a.spp)
    # 1. rank the tiles by their cost alone at the probe spp
    probe = np.array([timed(full[i:i + 1], a.probe_spp, reps=1) for i in range(len(full))])
    order = np.argsort(-probe)
    # 2. the most expensive tiles alone at the full spp: the chain floor
    top = [(int(i), round(timed(full[i:i + 1], a.spp, reps=2), 3)) for i in order[:a.top]]
    floor = max(ms for _, ms in top)
    # 3. the N-way shares alone, and each share's slowest tile (by the probe) alone
    shares = []
    key = {(int(t["x0"]), int(t["y0"])): i for i, t in enumerate(full)}
    for r in range(a.n):
        tl = wd.shard_tiles(W, H, T, [(0, 0)], r, a.n)
        idx = [key[(int(t["x0"]), int(t["y0"]))] for t in tl]
        worst = max(idx, key=lambda i: probe[i])
        shares.append({"rank": r, "tiles": len(tl), "ms": round(timed(tl, a.spp, reps=2), 3),
                       "slowest_tile_alone_ms": round(timed(full[worst:worst + 1], a.spp, reps=1), 3)})
    t_max = max(s["ms"] for s in shares)
    print(json.dumps({"scene": a.scene, "frame": f"{W}x{H}/{a.spp}spp", "full_frame_ms": round(t_full, 3),
                      "n": a.n, "shares": shares, "projected_efficiency": round(t_full / (a.n * t_max), 4),
                      "chain_floor_ms": floor, "top_tiles_alone_ms": top,
                      "efficiency_at_floor": round(t_full / (a.n * floor), 4),
                      "share_over_floor": round(t_max / floor, 4),
                      "probe": {"spp": a.probe_spp, "tile_ms_min_median_max": [round(float(probe.min()), 3),
                                                                               round(float(np.median(probe)), 3),
                                                                               round(float(probe.max()), 3)]}}),
          flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
