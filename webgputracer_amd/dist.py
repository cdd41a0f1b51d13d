"""Tile sharding of frames over GPUs + the final gather (RCCL over xGMI).

The reference distributes only whole frame ranges over machines via SSH
(settings/run.py:11-24: frames 1-320 local, 321-600 remote, no data exchange).
Here one process per GPU renders an interleaved share of the T x T tiles of a
batch of frames, and rank 0 gathers the tiles and assembles the frames:

  * pixel (x, y) of frame f depends only on (x, y, W, H, seed_f, scene)
    (path_tracer.wgsl:378), so ANY partition reproduces the single-GPU frame bit
    for bit; tiles are dealt along a Morton (Z-order) curve over the tile grid: each
    run of N consecutive curve positions (neighbouring tiles, whose costs are alike)
    gives every rank one tile, the ranks rotated per run so that over N runs every
    rank takes every place in a run once, in a hashed order that no lattice of the
    tile grid lines up with; the expensive and the cheap (escaping, NaN-absorbed)
    regions spread evenly (row-major dealing, t % N, left ranks 19% apart at N = 8
    on the sponza frame);
  * weak scaling: a step renders N frames on N GPUs, i.e. one frame's worth of
    tiles per GPU; the only collective is one gather per step
    (torch.distributed backend "nccl" = RCCL on ROCm; "gloo" in CPU tests).
"""
from __future__ import annotations

import numpy as np

from ._lib import TILE_DTYPE


def frame_tiles(W: int, H: int, T: int):
    """(x0, y0) of every T x T tile of a W x H frame, row-major."""
    ys, xs = np.meshgrid(np.arange(0, H, T, dtype=np.uint32), np.arange(0, W, T, dtype=np.uint32), indexing="ij")
    return np.stack([xs.ravel(), ys.ravel()], axis=1)


def curve_positions(W: int, H: int, T: int):
    """Position of every tile of frame_tiles(W, H, T) along the Morton curve over the tile grid
    (ties impossible: distinct tiles have distinct codes)."""
    xy = frame_tiles(W, H, T) // T
    code = np.zeros(len(xy), np.uint64)
    for b in range(16):  # interleave the bits of the tile column (even) and row (odd)
        code |= ((xy[:, 0].astype(np.uint64) >> b) & 1) << (2 * b)
        code |= ((xy[:, 1].astype(np.uint64) >> b) & 1) << (2 * b + 1)
    pos = np.empty(len(xy), np.int64)
    pos[np.argsort(code, kind="stable")] = np.arange(len(xy))
    return pos


def _hash32(x):
    """The murmur3 32-bit finaliser, elementwise."""
    h = np.asarray(x, np.uint64) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    return h


def run_rotations(n_runs: int, world: int):
    """Rotation of the ranks for each run of `world` curve positions: the runs of each group of
    `world` consecutive runs take the rotations 0 .. world-1 once each, in an order hashed from the
    run index, so over a group every rank takes every place in a run once (no place's cost stays
    with one rank) and no lattice of the tile grid lines up with the order."""
    g = np.arange(n_runs, dtype=np.int64)
    order = np.lexsort((_hash32(g), g // world))  # by group, then by hash within the group
    rot = np.empty(n_runs, np.int64)
    rot[order] = np.arange(n_runs) % world  # groups are contiguous in `order`, each of size world
    # (the last group may be partial: its runs still take distinct rotations)
    return rot


def tile_ranks(W: int, H: int, T: int, j: int, world: int):
    """Rank of every tile of frame_tiles(W, H, T) in the j-th frame of a batch: the tile at curve
    position p (run p // world) goes to rank (p + j + run_rotations(...)[p // world]) % world."""
    pos = curve_positions(W, H, T)
    rot = run_rotations(int(pos.max()) // world + 1 if len(pos) else 0, world)
    return (pos + j + rot[pos // world]) % world


def shard_tiles(W: int, H: int, T: int, frames, rank: int, world: int):
    """Tile list (TILE_DTYPE) of `rank` for the batch `frames` (list of (frame_id, seed)), in
    row-major tile order, dealt by tile_ranks."""
    xy = frame_tiles(W, H, T)
    out = []
    for j, (fid, seed) in enumerate(frames):
        sel = np.nonzero(tile_ranks(W, H, T, j, world) == rank)[0]
        t = np.zeros(len(sel), TILE_DTYPE)
        t["x0"] = xy[sel, 0]
        t["y0"] = xy[sel, 1]
        t["seed"] = seed & 0xFFFFFFFF
        t["frame"] = fid
        out.append(t)
    return np.concatenate(out) if out else np.zeros(0, TILE_DTYPE)


def max_tiles_per_rank(W: int, H: int, T: int, n_frames: int, world: int) -> int:
    n = len(frame_tiles(W, H, T))
    return max(len(shard_tiles(W, H, T, [(j, j) for j in range(n_frames)], r, world)) for r in range(world))


def assemble(tiles: np.ndarray, data, W: int, H: int, T: int, frame_ids, xp=np):
    """Scatter compact tiles data[k] (T, T, C) of tile list `tiles` into frames.
    Works with numpy or torch (pass xp=torch and torch tensors)."""
    C = data.shape[-1]
    frames = {}
    for fid in frame_ids:
        frames[int(fid)] = xp.zeros((H, W, C), dtype=data.dtype) if xp is np else \
            xp.zeros((H, W, C), dtype=data.dtype, device=data.device)
    for k in range(len(tiles)):
        fid = int(tiles["frame"][k])
        if fid not in frames:
            continue
        x0, y0 = int(tiles["x0"][k]), int(tiles["y0"][k])
        w, h = min(T, W - x0), min(T, H - y0)
        frames[fid][y0:y0 + h, x0:x0 + w] = data[k, :h, :w]
    return frames


def assemble_index(tiles: np.ndarray, W: int, H: int, T: int, frame_ids):
    """Gather index for assembling frames in one indexing op: for the tile list
    `tiles` (compact buffer data[k] of shape (T, T, C), flattened to rows of C),
    returns idx of shape (len(frame_ids), H, W) with frames[i] = data.reshape(-1, C)[idx[i]].
    Same result as assemble(); computed once on the host, used every step."""
    fpos = {int(f): i for i, f in enumerate(frame_ids)}
    idx = np.zeros((len(frame_ids), H, W), np.int64)
    ly, lx = np.meshgrid(np.arange(T), np.arange(T), indexing="ij")
    for k in range(len(tiles)):
        fid = int(tiles["frame"][k])
        if fid not in fpos:
            continue
        x0, y0 = int(tiles["x0"][k]), int(tiles["y0"][k])
        w, h = min(T, W - x0), min(T, H - y0)
        idx[fpos[fid], y0:y0 + h, x0:x0 + w] = (k * T + ly[:h, :w]) * T + lx[:h, :w]
    return idx


def pad_tiles(tiles: np.ndarray, n: int):
    """Pad a tile list to n entries (pad tiles have frame = 0xffffffff and are ignored by assemble)."""
    if len(tiles) >= n:
        return tiles
    pad = np.zeros(n - len(tiles), TILE_DTYPE)
    pad["frame"] = 0xFFFFFFFF
    if len(tiles):
        pad["x0"], pad["y0"], pad["seed"] = tiles["x0"][0], tiles["y0"][0], tiles["seed"][0]
    return np.concatenate([tiles, pad])


def gather_tiles(local, rank: int, world: int, dist, dst: int = 0, collective: bool = False):
    """Gather equally-sized per-rank tile buffers to `dst` (RCCL gather over xGMI on
    GPUs, gloo on CPU).  Returns the list of buffers on dst, None elsewhere.  One rank
    returns its buffer as it is unless `collective` (the call then goes through the
    process group's gather, as at N > 1)."""
    if world == 1 and not collective:
        return [local]
    if rank == dst:
        bufs = [local.new_empty(local.shape) for _ in range(world)]
        dist.gather(local, gather_list=bufs, dst=dst)
        return bufs
    dist.gather(local, dst=dst)
    return None


class ShardedFrames:
    """One rank's share of a step (bench.py's N>1 path, and its GPU test): the
    step's frames cut into T x T tiles dealt along the Morton curve (shard_tiles), one
    tile-list launch into a compact device buffer (wgt_render_tiles_async), one
    gather to rank 0 (RCCL over xGMI with backend "nccl"; gloo gathers host
    copies) and rank 0's assembly with a single index op built once here.

    frames: list of (frame id, seed).  want: "u8" (rgba8, always) and optionally
    "f32" (radiance before quantisation, gathered the same way).  depth: output
    buffer sets, one per step in flight: consecutive steps launched on different
    streams (the context's pipeline streams) overlap on the device, so step k
    renders into set k % depth (launch(stream, slot), gather(slot)).

    Decoupled gathers (gather_async, round 5): the gather and rank 0's assembly of
    step k run on a stream of their own once step k's launch has finished, and only
    the launch that next writes the same buffer set waits for them (wait_slot).  A
    render launch therefore never queues behind a collective whose kernels wait for
    CUs the next frame's persistent grid holds, and no rank's launch k + 2 is tied to
    the slowest rank's drain of k + 1 (with depth >= 2 x the frames in flight, the
    gather of a set has a whole step to finish before its set is written again).
    collective: go through the process group's gather even with one rank (tests)."""

    def __init__(self, ctx, cam, W, H, T, frames, rank, world, dist, device, backend="nccl", want=("u8",),
                 depth=1, collective=False):
        import torch

        self.ctx, self.cam, self.W, self.H, self.T = ctx, cam, W, H, T
        self.frames, self.rank, self.world, self.dist = list(frames), rank, world, dist
        self.backend, self.device, self.collective = backend, device, collective
        # one rank (no collective): each frame is one W x H tile, whose compact output is the frame
        # itself, row-major: nothing to gather and nothing to assemble
        self.whole = world == 1 and not collective
        self.tw, self.th = (W, H) if self.whole else (T, T)
        if self.whole:
            self.tiles = np.zeros(len(self.frames), TILE_DTYPE)
            self.tiles["seed"] = [seed & 0xFFFFFFFF for _, seed in self.frames]
            self.tiles["frame"] = [fid for fid, _ in self.frames]
            self.n_max = len(self.frames)
        else:
            self.tiles = shard_tiles(W, H, T, self.frames, rank, world)
            self.n_max = max_tiles_per_rank(W, H, T, len(self.frames), world)
        self.d_tiles = torch.from_numpy(self.tiles.view(np.uint8).copy()).to(device)
        self.bufsets = []
        for _ in range(max(depth, 1)):
            b = {"u8": torch.zeros((self.n_max, self.th, self.tw, 4), dtype=torch.uint8, device=device)}
            if "f32" in want:
                b["f32"] = torch.zeros((self.n_max, self.th, self.tw, 4), dtype=torch.float32, device=device)
            self.bufsets.append(b)
        self.bufs = self.bufsets[0]
        self.gather_stream = None  # created on the first gather_async
        self.done = [None] * len(self.bufsets)  # per set: an event after the gather that last read it
        self.frame_ids = [f for f, _ in self.frames]
        self.asm_idx = None
        if rank == 0 and not self.whole:
            layout = self.tiles if world == 1 else np.concatenate(
                [pad_tiles(shard_tiles(W, H, T, self.frames, r, world), self.n_max) for r in range(world)])
            self.asm_idx = torch.from_numpy(assemble_index(layout, W, H, T, self.frame_ids)).to(device)

    def stats(self):
        """Instrumented pass over this rank's tiles (exact counters; untimed)."""
        return self.ctx.render_tiles_stats(self.cam, self.W, self.H, self.tw, self.th, self.d_tiles.data_ptr(),
                                           len(self.tiles))

    def launch(self, stream=0, slot=0):
        """Render this rank's tiles into buffer set `slot` (asynchronous, ordered on `stream`, a raw
        hipStream_t)."""
        bufs = self.bufsets[slot]
        f32 = bufs.get("f32")
        self.ctx.render_tiles_async(self.cam, self.W, self.H, self.tw, self.th, self.d_tiles.data_ptr(),
                                    len(self.tiles), d_u8=bufs["u8"].data_ptr(),
                                    d_f32=f32.data_ptr() if f32 is not None else 0, stream=stream)

    def gather(self, slot=0):
        """Gather every rank's tiles of buffer set `slot` to rank 0 and assemble (on torch's current
        stream, which must be the one the launch ran on): {kind: {frame id: (H, W, 4) tensor}} on
        rank 0, None elsewhere.

        Lifetime: when one rank renders whole frames (`whole`, N = 1 without a collective) the
        tensors are VIEWS of buffer set `slot` (no copy), valid until the set is launched again;
        otherwise they are assembled copies.  A caller that keeps a frame past the set's next
        launch clones it first (wait_slot orders that launch after the gather only, not after
        the caller's reads)."""
        import torch

        out = {}
        for kind, buf in self.bufsets[slot].items():
            if self.whole:  # the frames themselves (views of the output set)
                out[kind] = {f: buf[i] for i, f in enumerate(self.frame_ids)}
                continue
            got = gather_tiles(buf if self.backend == "nccl" else buf.cpu(), self.rank, self.world, self.dist,
                               collective=self.collective)
            if self.rank == 0:
                data = (got[0] if len(got) == 1 else torch.cat(got)).to(self.device).reshape(-1, 4)
                imgs = data[self.asm_idx]  # (frames, H, W, 4)
                out[kind] = {f: imgs[i] for i, f in enumerate(self.frame_ids)}
        return out if self.rank == 0 else None

    def wait_slot(self, stream, slot):
        """Order `stream` (a torch stream) after the gather that last read buffer set `slot`: the
        launch that writes the set next must not overwrite tiles still being gathered."""
        if self.done[slot] is not None:
            stream.wait_event(self.done[slot])

    def gather_async(self, slot, after):
        """gather(slot) on the gather stream, after everything queued so far on `after` (the
        stream of the set's launch); records the set's done event.  Returns what gather returns:
        rank 0's images are valid once the gather stream is synchronised (done event)."""
        import torch

        if self.gather_stream is None:
            self.gather_stream = torch.cuda.Stream(device=self.device)
        g = self.gather_stream
        g.wait_stream(after)
        with torch.cuda.stream(g):
            out = self.gather(slot)
            ev = torch.cuda.Event()
            ev.record(g)
        self.done[slot] = ev
        return out
