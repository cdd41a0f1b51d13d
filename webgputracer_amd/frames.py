"""Multi-frame launcher (BASELINE config C5): a frame range
rendered by one process per GPU, frames dealt round-robin, no collective.

Replaces the reference's machine split (settings/run.py:11-24: frames 1-320 on
one host, 321-600 on another, each running `WebGPUTracer --frame s e`,
main.cpp:17-33) inside one node.  `--frame s e` means the frames
i = s-1 ... e-1 written as "%03d.png" % i (Renderer::OnCompute's loop
`for (i = start_frame - 1; i < end_frame; ++i) OnRender(i)`, render.cpp:437-439,
and the file name of OnRender, render.cpp:493-497), so `--frame 1 600` writes
000.png ... 599.png; rank r of N renders the frames i with (i - (s-1)) % N == r.
The camera is static (Camera::Update ignores t, camera.cpp:64-70), so frames
differ only by their seed: seed = frame index i (the reference draws
std::random_device, util.h:43-47; the C++ CLI's --fixed-seed uses the same i).

Frames are rendered B per launch (one full-frame tile per frame, each with its
frame's seed), so the persistent kernel's end-of-launch drain is paid once per B
frames instead of once per frame, and consecutive launches alternate over the
context's two pipeline streams: batch k+1 starts in batch k's
drain, while the host encodes batch k-1's PNGs.  Every frame is bit-identical to a
single-frame render.

  python -m webgputracer_amd.frames --frame 1 600 --spp 64 --scene bunny --batch 4 --out out/
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
      -m webgputracer_amd.frames --frame 1 600 --spp 64 --batch 4 --out out/
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from .tracer import Context, camera_param, cornell_scene, mesh_scene, write_png


def frame_indices(start: int, end: int):
    """The frame indices `--frame start end` renders: start-1 ... end-1
    (render.cpp:437, `for (uint32_t i = start_frame - 1; i < end_frame; ++i)`)."""
    if start < 1 or end < start:
        return []
    return list(range(start - 1, end))


def frames_of_rank(start: int, end: int, rank: int, world: int):
    """Frame indices of `--frame start end` (frame_indices) dealt to `rank`:
    round-robin, as even as the range allows."""
    return [f for k, f in enumerate(frame_indices(start, end)) if k % world == rank]


def _cpu_share() -> int:
    """CPUs this process may use, capped by OMP_NUM_THREADS where the launcher sets it."""
    n = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(n, omp) if omp > 0 else n


def batches(frames, batch: int):
    return [frames[i:i + batch] for i in range(0, len(frames), max(batch, 1))]


class FrameRenderer:
    """Renders batches of whole frames on one GPU: render() is one synchronous launch
    per batch (wgt_render_frames); stream() pipelines the batches (a launch per batch
    on the context's pipeline streams)."""

    def __init__(self, ctx: Context, W: int, H: int, spp: int):
        self.ctx, self.W, self.H, self.spp = ctx, W, H, spp
        self.cam = camera_param(W / H, spp, 0)  # per-frame seeds override cam.seed

    def render(self, frames):
        """{frame: (H, W, 4) uint8} for the batch `frames`, seed = frame index."""
        out = self.ctx.render_frames(self.cam, self.W, self.H, np.asarray(frames, np.uint32))
        return {f: out[j] for j, f in enumerate(frames)}

    def stream(self, frame_batches, depth: int = 2):
        """Yield (batch, {frame: (H, W, 4) uint8}) for each batch of `frame_batches`, in
        order.  Batch k renders on pipeline stream k % depth into buffer set k % depth;
        it is issued before batch k-1 is handed out, so the device always has the next
        launch queued behind the running one.  Host copies are made on the batch's own
        stream once its launch is done (no pinned buffers: torch's host allocator would
        outlive the context's streams)."""
        import torch

        from ._lib import TILE_DTYPE

        dev = torch.device("cuda", self.ctx.device)
        W, H = self.W, self.H
        nmax = max((len(b) for b in frame_batches), default=0)
        if nmax == 0:
            return
        streams = [torch.cuda.ExternalStream(self.ctx.pipeline_stream(i), device=dev) for i in range(depth)]
        d_out = [torch.empty((nmax, H, W, 4), dtype=torch.uint8, device=dev) for _ in range(depth)]
        pending = []
        for k, b in enumerate(frame_batches):
            j = k % depth
            if len(pending) == depth:  # the oldest batch in flight holds set j: hand it out first
                yield self._finish(pending.pop(0), streams, d_out)
            s = streams[j]
            t = np.zeros(len(b), TILE_DTYPE)  # one full-frame tile per frame (wgt_render_frames' list)
            t["seed"] = np.asarray(b, np.uint32)
            t["frame"] = np.arange(len(b), dtype=np.uint32)
            with torch.cuda.stream(s):
                d_tiles = torch.from_numpy(t.view(np.uint8).copy()).to(dev)
                self.ctx.render_tiles_async(self.cam, W, H, W, H, d_tiles.data_ptr(), len(b),
                                            d_u8=d_out[j].data_ptr(), stream=s.cuda_stream)
                d_tiles.record_stream(s)
            pending.append((k, b))
        while pending:
            yield self._finish(pending.pop(0), streams, d_out)

    @staticmethod
    def _finish(kb, streams, d_out):
        import torch

        k, b = kb
        j = k % len(streams)
        with torch.cuda.stream(streams[j]):  # ordered after batch k's launch on its stream
            imgs = d_out[j][:len(b)].cpu().numpy()
        return b, {f: imgs[i] for i, f in enumerate(b)}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--frame", nargs=2, type=int, default=[1, 1], metavar=("START", "END"))
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--scene", default="bunny", help="bunny | sponza | cornell | obj:<path>")
    ap.add_argument("--batch", type=int, default=4,
                    help="frames per launch (4 with 2 in flight: 33.0 frames/s, 31.6 at 8, 31.1 at 1; "
                         "profiles/configs/r02_c5_frames.jsonl)")
    ap.add_argument("--pipeline", type=int, default=2, help="batches in flight (1..4, DESIGN.md §4.2a)")
    ap.add_argument("--out", default=None, help="directory for NNN.png (none: render only)")
    ap.add_argument("--png-threads", type=int, default=0,
                    help="PNG encoder threads (0: this process's CPU share, capped by OMP_NUM_THREADS and 16)")
    a = ap.parse_args(argv)
    if a.frame[0] < 1 or a.frame[1] < a.frame[0]:
        ap.error("bad frame range")  # the C++ CLI's check (csrc/main.cpp)
    if not 1 <= a.pipeline <= 4:
        ap.error("--pipeline must be 1..4 (the context has 4 pipeline streams)")
    if a.batch < 1:
        ap.error("--batch must be >= 1")

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    import torch

    # one process per GPU; ranks beyond the visible GPUs share them (rehearsals, tests)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    if a.scene == "cornell":
        scene = cornell_scene()
    elif a.scene.startswith("obj:"):
        scene = mesh_scene("bunny", obj_path=a.scene[4:])
    else:
        scene = mesh_scene(a.scene)
    ctx = Context(local)
    ctx.upload_scene(*scene)
    fr = FrameRenderer(ctx, a.width, a.height, a.spp)
    mine = frames_of_rank(a.frame[0], a.frame[1], rank, world)
    if a.out:
        os.makedirs(a.out, exist_ok=True)
    # PNG encoding (zlib on the host, ~0.5 s per 1080p frame) runs on a thread pool while the GPU
    # renders the next batches (wgt_write_png is a ctypes call: it releases the GIL); at most
    # 4 frames per writer are held
    workers = max(1, a.png_threads or min(_cpu_share(), 16))
    pool = ThreadPoolExecutor(max_workers=workers) if a.out else None
    pending = collections.deque()
    t0 = time.perf_counter()
    for b, imgs in fr.stream(batches(mine, a.batch), depth=a.pipeline):
        if a.out:
            for f in b:  # render.cpp:494-497
                pending.append(pool.submit(write_png, os.path.join(a.out, f"{f:03d}.png"), imgs[f]))
            while len(pending) > 4 * workers:
                pending.popleft().result()
    while pending:
        pending.popleft().result()
    dt = time.perf_counter() - t0
    if pool:
        pool.shutdown()
    torch.cuda.synchronize()
    print(json.dumps({"rank": rank, "world": world, "frames": len(mine), "batch": a.batch, "pipeline": a.pipeline,
                      "seconds": round(dt, 3),
                      "frames_per_s": round(len(mine) / dt, 3) if dt > 0 else None}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
