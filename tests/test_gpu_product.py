"""GPU parity of the product's user-visible paths against the CPU oracle:

  * C5 (BASELINE configs[4]) at its size: whole 1920x1080/64 spp bunny frames
    through the multi-frame launcher (webgputracer_amd/frames.py, one
    wgt_render_frames launch), checked tile by tile against the oracle;
  * the CLI's NNN.png files (wgt_tracer --frame s e, render.cpp:437-439 and
    493-500, save_texture.h:10-87), decoded and compared with the oracle's rgba8;
    and the Python frame launcher writing the same file set with equal bytes;
  * the N>1 chain (webgputracer_amd/dist.py ShardedFrames, bench.py's path):
    two fresh processes on cuda:0, gloo, shard -> render -> gather -> assemble,
    the assembled frames compared with the oracle bit for bit.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "webgputracer_amd", "wgt_tracer")


def _png(path):
    from PIL import Image

    return np.asarray(Image.open(path).convert("RGBA"))


@pytest.fixture(scope="module")
def bunny_full(wgt, oracle):
    L, Q, S, T = wgt.mesh_scene("bunny")
    osc = oracle.OracleScene(L, Q, S, T)
    yield (L, Q, S, T), osc
    osc.close()


def test_c5_frames_at_size_vs_oracle(ctx, wgt, oracle, bunny_full):
    """C5: bunny stand-in, 1920x1080, 64 spp, frames 0 and 1 (seed = frame index) in
    one launch.  Five 8x8 tiles per frame (centre, mesh, walls, light, frame edge)
    equal the oracle's rgba8 at the same global pixels and seed, and the whole frame
    equals a single-frame render_tile of the same seed."""
    from webgputracer_amd.frames import FrameRenderer

    (L, Q, S, T), osc = bunny_full
    ctx.upload_scene(L, Q, S, T)
    W, H, spp = 1920, 1080, 64
    imgs = FrameRenderer(ctx, W, H, spp).render([0, 1])
    for f in (0, 1):
        cam_o = oracle.camera_param(W / H, spp, f)
        for (x0, y0) in [(956, 536), (700, 860), (120, 400), (960, 40), (1912, 1072)]:
            r = osc.render(cam_o, W, H, x0, y0, 8, 8, want=("u8",))
            assert np.array_equal(imgs[f][y0:y0 + 8, x0:x0 + 8], r["u8"]), (f, x0, y0)
        single = ctx.render_tile(wgt.camera_param(W / H, spp, f), W, H, want=("u8",))["u8"]
        assert np.array_equal(imgs[f], single), f
    # the launcher's pipelined path (frames.py main): batches [1], [0, 1] and [0] on the two
    # pipeline streams, each frame equal to the batched render
    seen = []
    for b, got in FrameRenderer(ctx, W, H, spp).stream([[1], [0, 1], [0]]):
        for f in b:
            assert np.array_equal(got[f], imgs[f]), (b, f)
            seen.append(f)
    assert seen == [1, 0, 1, 0]


@pytest.mark.parametrize("scene", ["cornell", "mesh2k"])
def test_cli_png_vs_oracle(tmp_path, wgt, oracle, scene):
    """wgt_tracer --frame 1 2 --fixed-seed writes 000.png (seed 0) and 001.png
    (seed 1) (render.cpp:437 loops i = start-1 .. end-1, render.cpp:494-497 names
    the file %03d of i); decoded, they equal the oracle's rgba8 of those seeds.
    mesh2k: a 2k-triangle mesh written as OBJ and loaded by the CLI's Scene::LoadObj
    (scene.cpp:56-131), the oracle rendering load_obj of the same file."""
    W, H, spp = 64, 64, 4
    args = [EXE, "--frame", "1", "2", "--width", str(W), "--height", str(H), "--spp", str(spp), "--fixed-seed",
            "--out", str(tmp_path)]
    if scene == "cornell":
        L, Q, S = wgt.cornell_scene()
        osc = oracle.OracleScene(L, Q, S)
        args += ["--scene", "cornell"]
    else:
        obj = tmp_path / "mesh.obj"
        wgt.write_obj(str(obj), wgt.procedural_mesh("bunny", 2000))
        L, Q, S, T = wgt.mesh_scene("bunny", obj_path=str(obj))
        osc = oracle.OracleScene(L, Q, S, T)
        args += ["--scene", f"obj:{obj}"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert sorted(p.name for p in tmp_path.glob("*.png")) == ["000.png", "001.png"]
    for f in (0, 1):
        ref = osc.render(oracle.camera_param(W / H, spp, f), W, H, want=("u8",))["u8"]
        assert np.array_equal(_png(tmp_path / f"{f:03d}.png"), ref), f
    osc.close()


def test_frames_launcher_and_cli_write_same_files(tmp_path, wgt):
    """`python -m webgputracer_amd.frames --frame 1 5` and `wgt_tracer --frame 1 5
    --fixed-seed` produce the same file set (000.png .. 004.png) with equal bytes,
    batched or not."""
    common = ["--frame", "1", "5", "--width", "40", "--height", "24", "--spp", "4", "--scene", "bunny"]
    runs = {
        "py_b2": [sys.executable, "-m", "webgputracer_amd.frames", *common, "--batch", "2"],
        "cli_b1": [EXE, *common, "--fixed-seed", "--batch", "1"],
        "cli_b3": [EXE, *common, "--fixed-seed", "--batch", "3"],
    }
    files = {}
    for name, cmd in runs.items():
        d = tmp_path / name
        d.mkdir()
        r = subprocess.run(cmd + ["--out", str(d)], capture_output=True, text=True, timeout=300, cwd=ROOT)
        assert r.returncode == 0, r.stdout + r.stderr
        files[name] = {p.name: p.read_bytes() for p in sorted(d.glob("*.png"))}
    assert list(files["py_b2"]) == [f"{i:03d}.png" for i in range(5)]
    for name in ("cli_b1", "cli_b3"):
        assert files[name] == files["py_b2"], name


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dist_worker(rank, world, port, out_path, scene, scaling, W, H, T, spp):
    """One rank of bench.py's N>1 step (dist.ShardedFrames), both ranks on cuda:0."""
    import torch
    import torch.distributed as dist

    import webgputracer_amd as w
    from webgputracer_amd import dist as wd

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ctx = w.Context(0)
    if scene == "cornell":
        ctx.upload_scene(*w.cornell_scene())
    else:
        ctx.upload_scene(*w.mesh_scene("bunny", target_tris=2000))
    frames = [(j, 10 + j) for j in range(world)] if scaling == "weak" else [(0, 10)]
    cam = w.camera_param(W / H, spp, 0)
    shard = wd.ShardedFrames(ctx, cam, W, H, T, frames, rank, world, dist, dev, backend="gloo",
                             want=("u8", "f32"))
    stream = torch.cuda.Stream(device=dev)
    shard.launch(stream.cuda_stream)
    stream.synchronize()
    got = shard.gather()
    if rank == 0:
        np.savez(out_path, **{f"{k}_{f}": v.cpu().numpy() for k, d in got.items() for f, v in d.items()})
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("scene,scaling", [("mesh2k", "weak"), ("mesh2k", "strong"), ("cornell", "weak")])
def test_dist_two_ranks_vs_oracle(tmp_path, wgt, oracle, scene, scaling):
    """The real N>1 chain in two spawned processes (gloo; both ranks share cuda:0):
    shard_tiles -> render_tiles_async -> gather_tiles -> assemble_index.  The
    assembled frames (rgba8 and radiance) equal the oracle's frames of the same seeds
    bit for bit.  16x16 tiles over a 100x60 frame leave ragged edge tiles."""
    import torch.multiprocessing as mp

    W, H, T, spp = 100, 60, 16, 4
    out = tmp_path / "frames.npz"
    mp.start_processes(_dist_worker, args=(2, _free_port(), str(out), scene, scaling, W, H, T, spp), nprocs=2,
                       join=True, start_method="spawn")
    got = np.load(out)
    if scene == "cornell":
        osc = oracle.OracleScene(*wgt.cornell_scene())
    else:
        osc = oracle.OracleScene(*wgt.mesh_scene("bunny", target_tris=2000))
    frames = [(0, 10), (1, 11)] if scaling == "weak" else [(0, 10)]
    for f, seed in frames:
        ref = osc.render(oracle.camera_param(W / H, spp, seed), W, H)
        assert np.array_equal(got[f"u8_{f}"], ref["u8"]), f
        assert np.array_equal(got[f"f32_{f}"].view(np.uint32), ref["f32"].view(np.uint32)), f
    osc.close()


def test_pipelined_launches_vs_oracle(ctx, wgt, oracle):
    """bench.py's pipelined steps: launches alternate over the context's two pipeline
    streams (own hardware queues) and workspace slots, so consecutive launches run
    concurrently.  Four launches with seeds 10..13 into four buffers, issued back to
    back, each equal the oracle's frame of its seed bit for bit; a scene re-upload then
    waits for all of them (wgt_upload_scene drains every slot)."""
    import torch

    L, Q, S, T = wgt.mesh_scene("bunny", target_tris=2000)
    ctx.upload_scene(L, Q, S, T)
    W, H, TS, spp = 100, 60, 16, 16
    dev = torch.device("cuda", 0)
    streams = [ctx.pipeline_stream(i) for i in range(2)]
    assert streams[0] and streams[1] and streams[0] != streams[1]
    assert ctx.pipeline_stream(0) == streams[0]  # created once
    cam = wgt.camera_param(W / H, spp, 0)
    outs, tls = [], []
    for k in range(4):
        tiles = wgt.tile_grid(W, H, TS, seed=10 + k)
        d_t = torch.from_numpy(tiles.view(np.uint8).copy()).to(dev)
        out = torch.zeros((len(tiles), TS, TS, 4), dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        tls.append((tiles, d_t))
        outs.append(out)
    for k in range(4):
        tiles, d_t = tls[k]
        ctx.render_tiles_async(cam, W, H, TS, TS, d_t.data_ptr(), len(tiles), d_f32=outs[k].data_ptr(),
                               stream=streams[k % 2])
    ctx.upload_scene(L, Q, S, T)  # must wait for the four launches before freeing the scene
    torch.cuda.synchronize()
    from webgputracer_amd.dist import assemble

    osc = oracle.OracleScene(L, Q, S, T)
    for k in range(4):
        tiles, _ = tls[k]
        img = assemble(tiles, outs[k].cpu().numpy(), W, H, TS, [0])[0]
        ref = osc.render(oracle.camera_param(W / H, spp, 10 + k), W, H, want=("f32",))["f32"]
        assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), k
    osc.close()
    with pytest.raises(Exception):
        ctx.pipeline_stream(4)


def test_frames_launcher_two_ranks_union(tmp_path, wgt):
    """C5's replica launcher with two ranks (settings/run.py:11-24 splits a frame range
    over machines; here RANK/WORLD_SIZE deal frames round-robin, frames.py
    frames_of_rank): two fresh processes on cuda:0 write disjoint file sets whose
    union is 000.png .. 005.png (render.cpp:437-439, 494-497), each file byte-equal to
    a single-process run's."""
    common = [sys.executable, "-m", "webgputracer_amd.frames", "--frame", "1", "6", "--width", "64", "--height", "36",
              "--spp", "4", "--scene", "bunny", "--batch", "2"]
    single = tmp_path / "single"
    single.mkdir()
    r = subprocess.run(common + ["--out", str(single)], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr
    procs, dirs = [], []
    for rank in range(2):
        d = tmp_path / f"rank{rank}"
        d.mkdir()
        dirs.append(d)
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank))
        procs.append(subprocess.Popen(common + ["--out", str(d)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True, cwd=ROOT, env=env))
    for p in procs:
        out, _ = p.communicate(timeout=300)
        assert p.returncode == 0, out
    sets = [{p.name: p.read_bytes() for p in sorted(d.glob("*.png"))} for d in dirs]
    assert not set(sets[0]) & set(sets[1]), "ranks rendered a frame twice"
    assert sorted(sets[0]) == ["000.png", "002.png", "004.png"]  # i = start-1 .. end-1, dealt round-robin
    union = {**sets[0], **sets[1]}
    ref = {p.name: p.read_bytes() for p in sorted(single.glob("*.png"))}
    assert sorted(union) == [f"{i:03d}.png" for i in range(6)] == sorted(ref)
    assert union == ref


def test_bench_two_ranks_self_checks(tmp_path):
    """bench.py at N = 2 (torch.distributed.run, gloo, both ranks on cuda:0) runs its
    untimed check step without being asked: the line carries check_frames_bit_exact =
    true, i.e. the frames gathered over the collective equal single-launch renders."""
    import json

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--dist-backend", "gloo", "--scene", "bunny", "--width", "96", "--height", "64", "--spp", "4",
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--stats-reps", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["check_frames_bit_exact"] is True
    assert line["check"]["world_size"] == 2 and line["check"]["frames"] == 2
    # where the step's time goes at N > 1: each rank's launch and gather time
    pr = line["per_rank"]
    assert len(pr["kernel_ms"]) == 2 and len(pr["gather_ms"]) == 2 and len(pr["isolated_launch_ms"]) == 2
    assert all(x > 0 for x in pr["kernel_ms"]) and all(x >= 0 for x in pr["gather_ms"])
    assert pr["kernel_ms_min_max"] == [min(pr["kernel_ms"]), max(pr["kernel_ms"])]
    assert pr["gather_ms_min_max"] == [min(pr["gather_ms"]), max(pr["gather_ms"])]


def test_bench_four_ranks_full_line(tmp_path):
    """bench.py at N = 4 (torch.distributed.run, gloo, all ranks on cuda:0) at 1080p with a reduced
    spp: the line the driver's scaling run reads carries every field of the N = 1 line — the
    self-check (check_frames_bit_exact), the roofline with traffic from rank 0's live rocprofv3
    --pmc passes, the CPU baseline timed once on rank 0 — plus per_rank: each rank's launch and
    gather times and its own roofline fraction from its own counts (reference analogue: the
    multi-machine launcher, settings/run.py:10-24)."""
    import json

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "4",
           "--dist-backend", "gloo", "--scene", "bunny", "--spp", "4", "--steps", "2", "--warmup", "1",
           "--cpu-rows", "2", "--stats-reps", "1", "--pmc", "on"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    (tmp_path / "n4.json").write_text(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "build_id", "per_rank"):
        assert k in line, k
    assert line["n_gpus"] == 4 and line["check_frames_bit_exact"] is True and line["check"]["frames"] == 4
    assert line["config"]["workload"] == "bunny-1920x1080-4spp"
    rf = line["roofline"]
    assert rf["traffic_source"] == "live" and rf["traffic"] > 0 and rf["traffic_build_id"] == line["build_id"]
    assert rf["valu_busy"] is not None and rf["bound"] in ("hbm", "valu", "latency")
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port" and cb["sample"]
    pr = line["per_rank"]
    for k in ("kernel_ms", "gather_ms", "isolated_launch_ms", "roofline_frac", "traced_rays", "algorithmic_bytes"):
        assert len(pr[k]) == 4, k
    # rank 0's own fraction is the line's (the same bytes over the same launch time)
    assert abs(pr["roofline_frac"][0] - rf["frac"]) <= 1e-4 * max(rf["frac"], 1e-9) + 1e-5
    assert all(f > 0 for f in pr["roofline_frac"]) and all(t > 0 for t in pr["traced_rays"])
    # weak scaling: the ranks' rays sum to the value's numerator
    assert sum(pr["traced_rays"]) * line["steps"] / (line["ms_per_step"] * line["steps"] * 1e-3) / 1e6 == \
        pytest.approx(line["value"], rel=2e-3)


def test_bench_line_contract(tmp_path):
    """bench.py at N = 1 on a small workload prints one JSON line with every field of the driver's
    contract: throughput, timing, roofline (bound, achieved, peak, frac, traffic measured by the
    run's own rocprofv3 --pmc passes) and the CPU baseline (value, unit, cores, kind, sample),
    plus the build id."""
    import json

    cmd = [sys.executable, "bench.py", "--scene", "bunny", "--width", "96", "--height", "64", "--spp", "4",
           "--steps", "2", "--warmup", "1", "--cpu-rows", "2", "--stats-reps", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "build_id"):
        assert k in line, k
    assert line["n_gpus"] == 1 and line["steps"] == 2 and line["warmup"] == 1 and line["value"] > 0
    assert line["unit"] == "Mrays/s" and line["higher_is_better"] is True and line["dtype"] == "f32"
    assert line["config"]["workload"] == "bunny-96x64-4spp"
    rf = line["roofline"]
    assert rf["unit"] == "GB/s" and rf["peak"] > 0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    # the same algorithmic bytes over one launch alone (pipeline 2: a launch on an idle device)
    iso = line["timing"]["isolated_launch_ms"]
    assert abs(rf["frac_isolated"] - rf["frac"] * line["kernel_ms"] / iso) < 1e-3
    # what bounds the kernel, from the run's own measurements (bench.limiter): the measured HBM
    # traffic's share of the peak, the VALU-busy fraction and the wave-cycle split
    assert abs(rf["hbm_frac"] - rf["traffic"] / (line["kernel_ms"] * 1e-3) / 1e9 / rf["peak"]) < 1e-3
    assert 0.0 < rf["valu_busy"] < 1.5 and rf["write_bytes_per_launch"] >= 0
    ws = rf["wave_split"]
    assert abs(ws["issuing"] + ws["waiting"] + ws["issue_stalled"] - 1.0) < 0.05
    sys.path.insert(0, ROOT)
    import bench

    assert rf["bound"] == bench.limiter(rf["hbm_frac"], {"valu_busy": rf["valu_busy"]})
    # the per-launch time of pipelined frames cannot undercount the wall time per step at small K
    # (the first-to-last completion interval did: two frames in flight complete in pairs)
    assert line["kernel_ms"] <= line["ms_per_step"] * 1.001
    # measured live by the run's own rocprofv3 --pmc passes (no profile entry exists for this workload)
    assert rf["traffic_source"] == "live" and rf["traffic"] > 0 and rf["traffic_build_id"] == line["build_id"]
    assert rf["l2"]["requests_per_launch"] > 0 and 0.0 <= rf["l2"]["hit_rate"] <= 1.0
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port" and cb["sample"]


_RCCL_ONE_RANK = r"""
import os, sys, json
import numpy as np, torch, torch.distributed as dist
sys.path.insert(0, os.environ["WGT_ROOT"])
import webgputracer_amd as w
from webgputracer_amd import dist as wdist
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)  # RCCL on ROCm
ctx = w.Context(0)
ctx.upload_scene(*w.mesh_scene("bunny", target_tris=2000))
W, H, T = 96, 64, 32
cam = w.camera_param(W / H, 4, 0)
sh = wdist.ShardedFrames(ctx, cam, W, H, T, [(0, 0)], 0, 1, dist, dev, backend="nccl")
sh.launch(torch.cuda.current_stream().cuda_stream)
buf = sh.bufs["u8"]
# the collectives bench.py issues at N > 1, over RCCL: the tile gather to rank 0 and the
# all_gather of the per-rank timing vector
got = [torch.empty_like(buf)]
dist.gather(buf, gather_list=got, dst=0)
tv = torch.arange(7, dtype=torch.float64, device=dev)
allv = [torch.zeros_like(tv)]
dist.all_gather(allv, tv)
torch.cuda.synchronize()
img = sh.gather()["u8"][0].cpu().numpy()
ref = ctx.render_tile(cam, W, H)["u8"]
print(json.dumps({"backend": dist.get_backend(), "gather_equal": bool(torch.equal(got[0], buf)),
                  "all_gather_equal": bool(torch.equal(allv[0], tv)),
                  "frame_equal": bool(np.array_equal(img, ref))}))
ctx.close()
dist.destroy_process_group()
"""


_RCCL_PIPELINE = r"""
import os, sys, json
import numpy as np, torch, torch.distributed as dist
sys.path.insert(0, os.environ["WGT_ROOT"])
import webgputracer_amd as w
from webgputracer_amd import dist as wdist
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)  # RCCL on ROCm
ctx = w.Context(0)
ctx.upload_scene(*w.mesh_scene("bunny", target_tris=2000))
W, H, T, P, D = 160, 96, 32, 2, 4
cam = w.camera_param(W / H, 4, 0)
frames = [(7, 11), (8, 12)]
# bench.py's step loop: launches on the context's two pipeline streams into output set k % D, each
# set's gather + assembly on the gather stream through the process group's gather (collective=True:
# RCCL with one rank), waited for only by the launch that next writes the set
sh = wdist.ShardedFrames(ctx, cam, W, H, T, frames, 0, 1, dist, dev, backend="nccl", depth=D, collective=True)
streams = [torch.cuda.ExternalStream(ctx.pipeline_stream(i), device=dev) for i in range(P)]
outs = []
for k in range(9):
    s, slot = streams[k % P], k % D
    with torch.cuda.stream(s):
        sh.wait_slot(s, slot)
        sh.launch(s.cuda_stream, slot=slot)
    got = sh.gather_async(slot, s)
    outs.append(got["u8"])
torch.cuda.synchronize()
refs = ctx.render_frames(cam, W, H, np.array([sd for _, sd in frames], np.uint32))
ok = all(np.array_equal(o[fid].cpu().numpy(), refs[i]) for o in outs for i, (fid, _) in enumerate(frames))
print(json.dumps({"backend": dist.get_backend(), "steps": len(outs), "frames_equal": bool(ok)}))
ctx.close()
dist.destroy_process_group()
"""


def test_rccl_pipelined_gather_one_rank(tmp_path):
    """bench.py's N > 1 step loop at one rank through the real RCCL gather (not the one-rank
    short cut): launches alternate over two pipeline streams into four output sets, each set's
    gather and assembly run on the shard's gather stream, and a launch waits only for the gather
    that last read its set (dist.ShardedFrames.wait_slot / gather_async).  Every gathered frame of
    9 steps equals the single-launch render of its seed."""
    import json

    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), WGT_ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", _RCCL_PIPELINE], capture_output=True, text=True, timeout=240,
                       cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line == {"backend": "nccl", "steps": 9, "frames_equal": True}, line


def test_rccl_backend_one_rank(tmp_path):
    """The RCCL ("nccl") backend initialises and runs bench.py's two collectives (the tile gather
    to rank 0 and the all_gather of the timing vector) on this box's GPU, with one rank (RCCL
    refuses two ranks on one device); the gathered tiles assemble to the single-launch frame.
    The N > 1 RCCL runs themselves are the driver's (settings/run.py:11-24 is the reference's
    multi-node analogue)."""
    import json

    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), WGT_ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", _RCCL_ONE_RANK], capture_output=True, text=True, timeout=240,
                       cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line == {"backend": "nccl", "gather_equal": True, "all_gather_equal": True, "frame_equal": True}, line
