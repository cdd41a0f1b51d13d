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


@pytest.mark.parametrize("world", [2, 3, 8])
def test_curve_dealing_gives_each_rank_one_tile_per_run(wgt, world):
    """Every run of `world` consecutive Morton-curve positions holds one tile of each rank (in every
    frame of the batch), so neighbouring tiles, whose costs are alike, spread over the ranks."""
    from webgputracer_amd import dist as wd

    W, H, T = 1920, 1080, 32
    pos = wd.curve_positions(W, H, T)
    assert sorted(pos.tolist()) == list(range(len(pos)))
    xy = wd.frame_tiles(W, H, T)
    for j in range(2):
        owner = np.empty(len(pos), np.int64)
        for r in range(world):
            t = wd.shard_tiles(W, H, T, [(j, j)] * 1, r, world)
            idx = [int(np.nonzero((xy[:, 0] == x) & (xy[:, 1] == y))[0][0]) for x, y in zip(t["x0"], t["y0"])]
            owner[pos[idx]] = r
        full = len(pos) // world * world  # (the last, partial run: at most one tile per rank)
        runs = owner[:full].reshape(-1, world)
        assert all(sorted(run.tolist()) == list(range(world)) for run in runs)


@pytest.mark.parametrize("world", [3, 4, 8])
@pytest.mark.parametrize("field", ["arcades4", "arcades8", "bands", "iid"])
def test_curve_dealing_balances_a_structured_cost_field(wgt, field, world):
    """Tile cost fields at 1080p in 32x32 tiles: expensive tile columns every 4 or 8 (arcades; row-
    major dealing, t % N with 60 tiles per row, gives such a column to one rank), smooth bands with
    a bright centre, and independent lognormal tile costs.  The curve dealing keeps every rank's
    summed cost within 3% of the mean where costs repeat or vary smoothly, and within 8% for
    independent costs (the spread of a sum of ~2040/N random tiles)."""
    from webgputracer_amd import dist as wd

    W, H, T = 1920, 1080, 32
    xy = wd.frame_tiles(W, H, T)
    col, row = xy[:, 0] // T, xy[:, 1] // T
    cx, cy = xy[:, 0] / W, xy[:, 1] / H
    if field.startswith("arcades"):
        cost = 1.0 + 2.0 * (col % int(field[-1]) == 0) + 0.5 * (row % 2)
    elif field == "bands":
        cost = 1.0 + 0.8 * (np.sin(cx * 2 * np.pi * 3.3) > 0) + 2.0 * np.exp(-((cx - 0.5) ** 2 + (cy - 0.5) ** 2) * 8)
    else:
        cost = np.random.default_rng(0).lognormal(0.0, 0.5, len(xy))
    ranks = wd.tile_ranks(W, H, T, 0, world)
    per_rank = np.array([cost[ranks == r].sum() for r in range(world)])
    assert per_rank.max() / per_rank.mean() < (1.08 if field == "iid" else 1.03)
    if field == "arcades4" and world in (4, 8):
        rowmajor = np.array([cost[np.arange(len(cost)) % world == r].sum() for r in range(world)])
        assert rowmajor.max() / rowmajor.mean() > 1.2


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
