"""Multi-GPU tile sharding + gather (webgputracer_amd.dist), exercised on CPU with the
gloo backend at world size 2 (the GPU path uses the same code with RCCL)."""
import os
import socket

import numpy as np
import pytest


def pixel_fn(frame, x, y):
    """Stand-in for a rendered pixel: any deterministic function of (frame, x, y)."""
    v = (x.astype(np.uint32) * 73856093) ^ (y.astype(np.uint32) * 19349663) ^ np.uint32(frame * 83492791)
    return np.stack([(v >> s) & 0xFF for s in (0, 8, 16, 24)], axis=-1).astype(np.uint8)


def render_tiles(tiles, T):
    out = np.zeros((len(tiles), T, T, 4), np.uint8)
    yy, xx = np.meshgrid(np.arange(T), np.arange(T), indexing="ij")
    for k, t in enumerate(tiles):
        out[k] = pixel_fn(int(t["frame"]), xx + t["x0"], yy + t["y0"])
    return out


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shards_cover_every_tile_once(wgt, world):
    from webgputracer_amd import dist as wd

    W, H, T = 70, 45, 16
    frames = [(j, 100 + j) for j in range(world)]
    n_tiles = len(wd.frame_tiles(W, H, T))
    seen = {}
    per_rank = []
    for r in range(world):
        t = wd.shard_tiles(W, H, T, frames, r, world)
        per_rank.append(len(t))
        for x0, y0, seed, f in t.tolist():
            key = (f, x0, y0)
            assert key not in seen
            seen[key] = seed
            assert seed == 100 + f
    assert len(seen) == n_tiles * world
    assert max(per_rank) - min(per_rank) <= world  # round-robin balance
    assert wd.max_tiles_per_rank(W, H, T, world, world) == max(per_rank)


def test_assemble_single_rank(wgt):
    from webgputracer_amd import dist as wd

    W, H, T = 70, 45, 16
    tiles = wd.shard_tiles(W, H, T, [(5, 5)], 0, 1)
    frames = wd.assemble(tiles, render_tiles(tiles, T), W, H, T, [5])
    yy, xx = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    assert np.array_equal(frames[5], pixel_fn(5, xx, yy))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, result_path, strong=False):
    import torch
    import torch.distributed as dist

    from webgputracer_amd import dist as wd

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    W, H, T = 70, 45, 16
    # weak scaling: one frame per rank; strong: one frame split over the ranks (bench.py --scaling)
    frames = [(0, 0)] if strong else [(j, j) for j in range(world)]
    tiles = wd.shard_tiles(W, H, T, frames, rank, world)
    n_max = wd.max_tiles_per_rank(W, H, T, len(frames), world)
    local = np.zeros((n_max, T, T, 4), np.uint8)
    local[:len(tiles)] = render_tiles(tiles, T)
    bufs = wd.gather_tiles(torch.from_numpy(local), rank, world, dist)
    if rank == 0:
        all_tiles = np.concatenate([wd.pad_tiles(wd.shard_tiles(W, H, T, frames, r, world), n_max)
                                    for r in range(world)])
        imgs = wd.assemble(all_tiles, torch.cat(bufs).numpy(), W, H, T, [f for f, _ in frames])
        yy, xx = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
        ok = all(np.array_equal(imgs[f], pixel_fn(f, xx, yy)) for f, _ in frames)
        with open(result_path, "w") as fh:
            fh.write("ok" if ok else "mismatch")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("strong", [False, True])
def test_gloo_world2_gather_assembles_frames(tmp_path, strong):
    import torch.multiprocessing as mp

    result = tmp_path / "result.txt"
    mp.start_processes(_worker, args=(2, _free_port(), str(result), strong), nprocs=2, join=True,
                       start_method="spawn")
    assert result.read_text() == "ok"


def test_assemble_index_matches_assemble():
    """The one-op gather index used by bench.py equals the tile-by-tile assembly."""
    import numpy as np

    from webgputracer_amd import dist as wdist

    W, H, T, world = 70, 45, 16, 3
    frames = [(j, 100 + j) for j in range(world)]
    n_max = wdist.max_tiles_per_rank(W, H, T, world, world)
    layout = np.concatenate([wdist.pad_tiles(wdist.shard_tiles(W, H, T, frames, r, world), n_max)
                             for r in range(world)])
    rng = np.random.default_rng(0)
    data = rng.integers(0, 255, (len(layout), T, T, 4), dtype=np.uint8)
    ref = wdist.assemble(layout, data, W, H, T, [f for f, _ in frames])
    idx = wdist.assemble_index(layout, W, H, T, [f for f, _ in frames])
    got = data.reshape(-1, 4)[idx]
    for i, (f, _) in enumerate(frames):
        assert np.array_equal(got[i], ref[f])
