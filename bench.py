"""bench.py — BASELINE.json metric: Mrays/sec at 1080p/256spp (+ achieved GB/s vs HBM peak).

Workload (BASELINE configs[3], C4 — the config the metric's "1/2/4/8 MI355X" is quoted
on, and the one north_star's roofline target names): Sponza-sized procedural stand-in
(268,944 triangles; the asset is absent and there is no network) inside the reference
Cornell box + light, 1920x1080, 256 spp.  `--scene bunny` runs configs[2] (C3).  A
"step" renders one 1080p/256spp frame per GPU: the step's N frames are cut into 32x32
tiles dealt over the N ranks along a Morton curve (one process per GPU), then the tiles are
gathered to rank 0 (RCCL over xGMI) and assembled — weak scaling, per-GPU work fixed.
Steps are issued two deep (--pipeline 2): step k runs on the context's pipeline stream
k % 2 into output set k % 2, so each frame starts in the previous frame's end-of-launch
drain; every frame is still rendered whole.

value = closest-hit queries actually traced (non-NaN rays, counted on the device by
an instrumented pass over the same tiles) summed over ranks x steps / max-over-ranks
wall time of the K timed steps.  Scene/BVH upload and tile lists are resident in HBM
before timing.  Each render call is launched on its step's stream, where HIP events
bracket it; with frames in flight the per-launch time (roofline.achieved) is the span
from the first timed launch's start to the last one's end divided by K (a launch's own
event pair would also count the time it waits for the previous frame's CUs), with
--pipeline 1 the mean event pair: the 1-spp cost pre-pass + LPT ordering (~1 % of the
call at 256 spp) and the main kernel k_render_ps (the rocprof kernel trace under
profiles/ lists them separately).  At N > 1 every rank reports the same figures for its
own tiles (per_rank: launch ms, gather ms, roofline frac), rank 0 times the CPU baseline
and runs the live PMC passes on its own GPU (a frame of the per-GPU workload alone).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--scene sponza|bunny|cornell]
  torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrays/sec at 1080p/256spp + achieved HBM GB/s vs peak, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)
# algorithmic bytes per unit: a BVH4 node visit reads 7 x 16 B (6 SoA
# box rows + child refs) of its 128-B line, or with compact nodes 4 x 16 B of its
# 64-B node + its 16-B ref record; a triangle test all 4 x 16 B of its 64-B record
# (the padded box with the Moller-Trumbore inputs), a traced
# ray 32 B of per-triangle shading data
NODE_BYTES, CNODE_BYTES, TRI_BYTES, SHADE_BYTES = 112, 80, 64, 32
# SURVEY §8(d)'s format-independent figure: 32 B per BVH node visit, 48 B per triangle
# test, 32 B of shading record per traced ray (the same at any node encoding)
SURVEY_NODE_BYTES, SURVEY_TRI_BYTES = 32, 48
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md §L2: ~34.5 TB/s aggregate over the 8 XCDs
L2_CALIB_JSON = os.path.join(ROOT, "profiles", "l2_calibration.json")


def dominant_kernel(form: int, waves: int, tris: bool = True, park: bool = True) -> str:
    """The timed k_render_ps instantiation <STATS, COST, node form (0 = 128-B, 1 = 80-B compact),
    waves per SIMD, triangles, parked traversal state> (a scene without triangles runs the 8-wave
    instantiation without traversal)."""
    if not tris:
        return "wgt::k_render_ps<false, false, 0, 8, false, false>"
    return f"wgt::k_render_ps<false, false, {int(form)}, {waves}, true, {'true' if park else 'false'}>"


def node_form(info) -> int:
    """The node form k_render_ps reads for the reference camera (wgt_kernels.hip node_form, reported
    by the library as scene_info node_form): 0 = 128-B nodes, 1 = 80-B compact records."""
    return int(info["node_form"])


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--scene", default="sponza", choices=["sponza", "bunny", "cornell"])
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--spp", type=int, default=256)
    p.add_argument("--tile", type=int, default=32)
    p.add_argument("--cpu-rows", type=int, default=0, help="rows in the CPU-baseline sample (0 = auto)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl = RCCL over xGMI (default); gloo only to rehearse N ranks on fewer GPUs")
    p.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                   help="weak: one frame per GPU per step (default); strong: one frame split over the GPUs")
    p.add_argument("--stats-reps", type=int, default=2,
                   help="instrumented counting passes (node/triangle counts vary slightly between schedules)")
    p.add_argument("--pipeline", type=int, default=2,
                   help="frames in flight: step k runs on the context's pipeline stream k %% P, so the next "
                        "frame fills the CUs the previous frame's end-of-launch drain leaves idle (1 = serial)")
    p.add_argument("--pmc", default="auto", choices=["auto", "on", "off"],
                   help="after the timed region, measure the dominant kernel's HBM traffic and L2 requests with "
                        "separate rocprofv3 --pmc passes of one frame of this workload (child runs of this script); "
                        "auto: at N = 1 when rocprofv3 is on PATH.  Failing that, the build-id-keyed profile entry")
    p.add_argument("--check", default="auto", choices=["auto", "on", "off"],
                   help="one untimed step before timing whose gathered frames rank 0 compares bit for bit with "
                        "single-launch renders of the same seeds (auto: on when N > 1)")
    return p.parse_args()


PMC_PASSES = (("FETCH_SIZE",), ("WRITE_SIZE",), ("TCC_HIT_sum", "TCC_MISS_sum"),
              ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
               "SQ_INSTS_VALU"))
PMC_BUDGET_S = 180.0  # all live passes together (each also under its own kill timeout)
N_SIMDS = 256 * 4     # MI355X: 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)
VALU_ISSUE_CYCLES = 2  # cycles of a wave64 f32 VALU instruction on a SIMD-32 (MI355X_MICROARCH.md)


def sq_fields(agg, calls, grid_waves=None):
    """VALU-busy fraction and the wave-cycle split of the kernel from the SQ pass: waves are
    issuing (SQ_ACTIVE_INST_ANY), parked in s_waitcnt (SQ_WAIT_ANY) or ready but not issued
    (SQ_WAIT_INST_ANY); the three are disjoint and sum to SQ_WAVE_CYCLES (MI355X_MICROARCH.md
    §rocprofv3).  A persistent launch keeps its waves for the whole launch, so the launch
    lasts ~4 x SQ_WAVE_CYCLES / waves cycles (SQ_WAVE_CYCLES counts quad-cycles) and the
    VALU pipes are busy SQ_INSTS_VALU x 2 cycles / (SIMDs x that).  waves = the launch's grid
    (grid_waves, known to the caller) when given: SQ_WAVES read twice the grid on bunny's
    one-dispatch pass in round 5 (12,288 for 6,144 waves; sponza's pass counted 6,144) while
    SQ_WAVE_CYCLES matched the grid, so it is kept in `raw` only."""
    wc = agg.get("SQ_WAVE_CYCLES", 0.0)
    sq_waves = agg.get("SQ_WAVES", 0.0)
    waves = float(grid_waves) * calls if grid_waves else sq_waves
    if wc <= 0 or waves <= 0:
        return None
    launch_cycles = 4.0 * wc / waves
    valu = agg.get("SQ_INSTS_VALU", 0.0) / calls
    return {"valu_busy": round(valu * VALU_ISSUE_CYCLES / (N_SIMDS * launch_cycles), 4),
            "valu_insts_per_launch": valu,
            # the raw figures (per launch), for auditing the two ratios
            "raw": {"SQ_WAVES": sq_waves / calls, "grid_waves": waves / calls, "SQ_WAVE_CYCLES": wc / calls,
                    "SQ_INSTS_VALU": valu, "dispatches": calls},
            "wave_split": {"issuing": round(agg.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, 4),
                           "waiting": round(agg.get("SQ_WAIT_ANY", 0.0) / wc, 4),
                           "issue_stalled": round(agg.get("SQ_WAIT_INST_ANY", 0.0) / wc, 4)}}


def limiter(hbm_frac, sq):
    """What bounds the kernel, from the measurements: HBM bandwidth when the measured traffic
    runs at >= 70 % of the peak, the VALU when its pipes are busy >= 70 % of the time, else the
    latency of dependent memory round trips (waves parked in s_waitcnt) and VALU issue."""
    if hbm_frac is not None and hbm_frac >= 0.7:
        return "hbm"
    if sq is not None and sq["valu_busy"] >= 0.7:
        return "valu"
    if sq is None:
        return "unmeasured"
    return "latency"


def live_pmc(args, kernel, grid_waves=None, local=0):
    """HBM bytes and L2 requests per launch of `kernel`, measured now on this device and binary:
    one rocprofv3 --pmc pass per counter group (never combined with traces; each pass within the
    per-block counter limits, under its own kill timeout) over a child run of this script that
    renders one frame of the same workload alone.  HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) x
    1 KiB (FETCH_SIZE counts half the bytes of 16-B-per-lane reads on gfx950, MI355X_MICROARCH.md
    §HBM).  At N > 1 the child runs on this rank's GPU (`local`) as a one-rank job.  Returns
    (result dict, note); the dict is None when a pass fails."""
    import csv
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not on PATH"
    child = [sys.executable, os.path.abspath(__file__), "--scene", args.scene, "--width", str(args.width),
             "--height", str(args.height), "--spp", str(args.spp), "--tile", str(args.tile), "--steps", "1",
             "--warmup", "0", "--pipeline", "1", "--no-cpu-baseline", "--check", "off", "--pmc", "off",
             "--stats-reps", "1"]
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK=str(local), LOCAL_WORLD_SIZE="1")
    agg, calls = {}, 0
    t_end = time.monotonic() + PMC_BUDGET_S
    for ctrs in PMC_PASSES:
        d = tempfile.mkdtemp(prefix="wgt_pmc_")
        # a pass takes ~10-20 s (child start, scene build, one frame); a stuck one is killed, the
        # passes together stay within PMC_BUDGET_S, and the first failure ends the measurement
        # (the remaining passes are not tried)
        left = int(min(150.0, t_end - time.monotonic()))
        if left < 20:
            return None, f"live PMC passes exceeded their {PMC_BUDGET_S:.0f} s budget"
        cmd = ["timeout", "-s", "KILL", str(left), prof, "--pmc", *ctrs, "-d", d, "-o", "run", "--output-format",
               "csv", "--", *child]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=left + 30, cwd=ROOT, env=env)
            rows = []
            for root, _, files in os.walk(d):
                for fn in files:
                    if fn.endswith("counter_collection.csv"):
                        with open(os.path.join(root, fn)) as f:
                            rows += list(csv.DictReader(f))
            if r.returncode != 0 or not rows:
                return None, f"rocprofv3 --pmc {' '.join(ctrs)} failed (exit {r.returncode})"
            disp = set()
            for row in rows:
                if kernel in row["Kernel_Name"]:
                    agg[row["Counter_Name"]] = agg.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                    disp.add(row["Dispatch_Id"])
            if not disp:
                return None, f"no dispatch of {kernel} in the --pmc {' '.join(ctrs)} pass"
            calls = len(disp)
        except (OSError, subprocess.SubprocessError, KeyError, ValueError) as e:
            return None, f"rocprofv3 pass failed: {e}"
        finally:
            shutil.rmtree(d, ignore_errors=True)
    hbm = (2.0 * agg.get("FETCH_SIZE", 0.0) + agg.get("WRITE_SIZE", 0.0)) * 1024.0 / calls
    req = (agg.get("TCC_HIT_sum", 0.0) + agg.get("TCC_MISS_sum", 0.0)) / calls
    hit = agg.get("TCC_HIT_sum", 0.0) / max(agg.get("TCC_HIT_sum", 0.0) + agg.get("TCC_MISS_sum", 0.0), 1.0)
    return {"hbm_bytes_per_launch": hbm, "tcc_requests_per_launch": req, "tcc_hit_rate": round(hit, 4),
            "write_bytes_per_launch": agg.get("WRITE_SIZE", 0.0) * 1024.0 / calls,
            "sq": sq_fields(agg, calls, grid_waves)}, \
        f"live: {len(PMC_PASSES)} rocprofv3 --pmc passes of one frame of this workload alone, this run"


def build_scene(w, kind):
    if kind == "cornell":
        L, Q, S = w.cornell_scene()
        return L, Q, S, None
    return w.mesh_scene(kind)


def baseline_threads():
    """Threads for the CPU baseline: the CPUs this process may run on, capped by
    OMP_NUM_THREADS where the launcher sets it (the GPU box sets it to the box's CPU
    share, 16, and asks that worker pools stay within it)."""
    n = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(n, omp) if omp > 0 else n), n


def cpu_baseline(args, scene, rank, world):
    """The oracle (CPU port, OpenMP) on a bounded row sample of the same workload,
    timed with its x86-64-v3 build (oracle/Makefile: liboracle_v3.so), which is first
    checked bit for bit against the reference build liboracle.so on a small tile."""
    if rank != 0 or args.no_cpu_baseline:
        return None
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po

    L, Q, S, T = scene
    cores, affinity = baseline_threads()
    cam = po.camera_param(args.width / args.height, args.spp, 0)
    check = {}
    for build in ("liboracle.so", "liboracle_v3.so"):
        po.use_build(build)
        osc = po.OracleScene(L, Q, S, T)
        check[build] = osc.render(po.camera_param(args.width / args.height, 4, 0), args.width, args.height,
                                  args.width // 2, args.height // 2, 16, 8, nthreads=cores, want=("f32",))["f32"]
        osc.close()
    same = bool(np.array_equal(check["liboracle.so"].view(np.uint32), check["liboracle_v3.so"].view(np.uint32)))
    po.use_build("liboracle_v3.so" if same else "liboracle.so")
    osc = po.OracleScene(L, Q, S, T)

    def run(rows):
        # rows spread evenly over the frame, full width, same spp/seed as the GPU frame
        ys = np.linspace(0, args.height - 1, rows).astype(int)
        t0 = time.perf_counter()
        traced = 0
        for y in ys:
            r = osc.render(cam, args.width, args.height, 0, int(y), args.width, 1, nthreads=cores, want=())
            traced += int(r["counters"][po.CNT_TRACED])
        return traced, time.perf_counter() - t0

    rows = args.cpu_rows
    if not rows:  # calibrate on 2 rows, then size the sample to ~15 s of CPU work
        tr, dt = run(2)
        rows = int(min(args.height, max(2, 2 * 15.0 / max(dt, 1e-3))))
    traced, dt = run(rows)
    osc.close()
    build = "liboracle_v3.so (x86-64-v3, bit-identical to liboracle.so on a check tile)" if same else \
        "liboracle.so (the x86-64-v3 build differed on the check tile)"
    return {"value": traced / dt / 1e6, "unit": "Mrays/s", "cores": cores, "kind": "port",
            "sample": f"oracle/wgt_oracle.c as {build}, OpenMP {cores} threads (affinity {affinity} CPUs, "
                      f"OMP_NUM_THREADS {os.environ.get('OMP_NUM_THREADS', 'unset')}), on {rows} full-width rows "
                      f"of the same {args.width}x{args.height}/{args.spp}spp frame (seed 0): {traced} traced "
                      f"rays in {dt:.1f} s"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import webgputracer_amd as w
    from webgputracer_amd import dist as wdist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # one process per GPU; rehearsals with more ranks than GPUs share devices (gloo only)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    def barrier():
        if world > 1:
            dist.barrier()

    W, H, T, spp = args.width, args.height, args.tile, args.spp
    scene = build_scene(w, args.scene)
    ctx = w.Context(local)
    ctx.upload_scene(*scene)
    info = ctx.scene_info()

    # this step's frames (frame id, seed): one per GPU (weak scaling) or one in all (strong)
    frames = [(j, j) for j in range(world)] if args.scaling == "weak" else [(0, 0)]
    dev = torch.device("cuda", local)
    cam = w.camera_param(W / H, spp, 0)  # per-tile seeds override cam.seed
    # the rank's tiles, its compact output buffer and (rank 0) the assembly index, all resident
    P = max(1, min(args.pipeline, 4))
    # output sets: twice the frames in flight, so that a set's gather (on the shard's gather stream,
    # decoupled from the render streams) has a whole step to finish before the set is written again
    D = 2 * P
    shard = wdist.ShardedFrames(ctx, cam, W, H, T, frames, rank, world, dist, dev, backend=args.dist_backend,
                                depth=D)

    # instrumented passes (untimed): exact ray/sample counts for this rank's tiles.  The
    # node / triangle counts depend slightly on the schedule (which lanes run the
    # speculative second leaf of a step), so the spread over the passes is reported
    sts = [shard.stats() for _ in range(max(args.stats_reps, 1))]
    st = sts[0]

    # real (non-NULL) streams: a step's launch, its events and its gather are ordered on
    # one of them.  P > 1: the context's pipeline streams (each on a hardware queue of its
    # own), step k on stream k % P into output set k % P, so consecutive frames overlap
    if P == 1:
        streams = [torch.cuda.Stream(device=dev)]
    else:
        streams = [torch.cuda.ExternalStream(ctx.pipeline_stream(i), device=dev) for i in range(P)]
    torch.cuda.set_stream(streams[0])

    def step(k, ev):
        # step k: render on stream k % P into output set k % D (after the gather that last read the
        # set), then gather + assemble on the gather stream, which no render launch waits for: a
        # launch never queues behind a collective whose kernels wait for CUs
        s, slot = streams[k % P], k % D
        with torch.cuda.stream(s):
            shard.wait_slot(s, slot)
            if ev is not None:
                ev[0].record(s)
            shard.launch(s.cuda_stream, slot=slot)
            if ev is not None:
                ev[1].record(s)
        got = shard.gather_async(slot, s)
        if ev is not None:
            ev[2].record(shard.gather_stream)
        return got["u8"] if got is not None else None

    for k in range(args.warmup):
        step(k, None)
    # untimed check step (default with N > 1): the frames rank 0 gathered over the
    # collective equal single-launch renders of the same seeds on rank 0's GPU
    check = None
    if args.check == "on" or (args.check == "auto" and world > 1):
        got = step(0, None)
        torch.cuda.synchronize()
        if rank == 0:
            seeds = np.array([seed for _, seed in frames], np.uint32)
            refs = ctx.render_frames(w.camera_param(W / H, spp, 0), W, H, seeds)
            check = all(bool(np.array_equal(got[fid].cpu().numpy(), refs[i])) for i, (fid, _) in enumerate(frames))
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    # per step: launch start, launch end, gather end (the gather's time includes its wait for the
    # slowest rank's tiles: where a multi-GPU step's efficiency goes)
    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    img = None
    for k in range(args.steps):
        img = step(k, evs[k])
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # per-launch time: serial steps, the event pair around each launch; pipelined, the span
    # from the first launch's start (on an idle device: the region starts synchronised) to the
    # last launch's end over K launches.  An event pair would also count the time a launch
    # waits for the CUs its predecessor holds, and the interval between the first and last
    # completions is biased at small K: two frames in flight share the device and complete
    # in pairs (3 steps: 158 ms "per launch" against 301 ms per step).  The span includes
    # one fill and one drain, so it errs high (slower), by about 6% / K.
    spans = [a.elapsed_time(b) for a, b, _ in evs]
    gather_ms = float(np.mean([b.elapsed_time(c) for _, b, c in evs])) if args.steps else 0.0
    if P > 1 and args.steps > 1:
        kern_ms = evs[0][0].elapsed_time(evs[-1][1]) / args.steps
    else:
        kern_ms = float(np.mean(spans)) if args.steps else 0.0
    # one more launch alone on an idle device (untimed): the single-frame latency
    iso = None
    if P > 1:
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(streams[0]):
            shard.wait_slot(streams[0], 0)
            e0.record(streams[0])
            shard.launch(streams[0].cuda_stream, slot=0)
            e1.record(streams[0])
        torch.cuda.synchronize()
        iso = e0.elapsed_time(e1)

    mine = np.array([elapsed, st["traced_rays"], st["queries"], st["samples"], st["node_visits"],
                     st["tri_tests"], kern_ms, gather_ms, iso if iso is not None else kern_ms], np.float64)
    simt = {"path_loop": st["loop_lane_iters"] / max(64 * st["loop_wave_iters"], 1),
            "bvh_loop": st["trav_lane_steps"] / max(64 * st["trav_wave_steps"], 1)}
    if world > 1:
        tm = torch.tensor(mine, device=dev if args.dist_backend == "nccl" else "cpu")
        allv = [torch.zeros_like(tm) for _ in range(world)]
        dist.all_gather(allv, tm)
        allv = np.stack([a.cpu().numpy() for a in allv])
    else:
        allv = mine[None]
    max_t = float(allv[:, 0].max())
    traced = float(allv[:, 1].sum()) * args.steps
    queries = float(allv[:, 2].sum()) * args.steps
    samples = float(allv[:, 3].sum()) * args.steps
    value = traced / max_t / 1e6

    base = cpu_baseline(args, scene, rank, world)
    if rank == 0:
        # dominant kernel = k_render_ps; algorithmic bytes of rank 0's launch
        form = node_form(info)
        kernel = dominant_kernel(form, int(info.get("ps_waves", 5)), info["n_tris"] > 0,
                                 bool(info.get("ps_park", 0)))
        node_b = (NODE_BYTES, CNODE_BYTES)[form]
        bytes_launch = (mine[4] * node_b + mine[5] * TRI_BYTES + mine[1] * SHADE_BYTES)
        achieved = bytes_launch / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
        survey_bytes = mine[4] * SURVEY_NODE_BYTES + mine[5] * SURVEY_TRI_BYTES + mine[1] * SHADE_BYTES
        # PMC-derived figures (traffic, L2 requests) come from a profile of this exact binary
        # only: the entry must carry the running library's build id (a hash of the kernel
        # sources and flags, wgt_build_id), else they are null with the reason
        build_id = w.build_id()
        traffic, l2, tj_id, sq, write_b = None, None, None, None, None
        traffic_note = "no profile entry for this workload"
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            tj = tj.get(f"{args.scene}-{W}x{H}-{spp}spp", {})  # one entry per workload
            tj_id = tj.get("build_id")
            if tj and tj_id != build_id:
                traffic_note = f"profile entry is of build {tj_id}, not the running {build_id}: not applicable"
            elif tj and (tj.get("n_gpus", 1) != 1 or world != 1):
                traffic_note = "profiled on 1 GPU; not applicable at N > 1"
            elif tj and tj.get("kernel") != kernel:
                traffic_note = f"profile entry is of {tj.get('kernel')}, not the timed {kernel}"
            if tj and tj_id == build_id and tj.get("n_gpus", 1) == 1 and world == 1 and tj.get("kernel") == kernel:
                traffic_note = f"PMC passes of build {build_id} ({tj.get('source')})"
                traffic = tj.get("hbm_bytes_per_launch")
                sq, write_b = tj.get("sq"), tj.get("write_bytes_per_launch")
                req = tj.get("tcc_requests_per_launch")
                with open(L2_CALIB_JSON) as f:
                    bpr = json.load(f)["bytes_per_request"]
                if req and kern_ms > 0:
                    l2_gbs = req * bpr / (kern_ms * 1e-3) / 1e9
                    l2 = {"requests_per_launch": req, "bytes_per_request": bpr, "achieved": round(l2_gbs, 1),
                          "peak": L2_PEAK_GBS, "unit": "GB/s", "frac": round(l2_gbs / L2_PEAK_GBS, 4),
                          "hit_rate": tj.get("tcc_hit_rate"), "source": tj.get("source"),
                          "calibration": os.path.relpath(L2_CALIB_JSON, ROOT)}
        except (OSError, ValueError, KeyError):
            pass
        # live PMC passes of this binary on this device (N = 1), in place of the profile entry
        traffic_source = "profile" if traffic is not None else None
        if args.pmc == "on" or (args.pmc == "auto" and args.steps > 0):
            # the child renders one whole W x H frame at N = 1: its persistent grid is the device's
            # resident capacity or one wave per 8x8 pixel block, whichever is smaller
            res = int(info.get("ps_resident", 0))
            grid = min(((W + 7) // 8) * ((H + 7) // 8), res) if res else None
            live, note = live_pmc(args, kernel, grid, local)
            if live is not None and world > 1:
                note += f" (rank 0's GPU, after the {world}-rank timed region)"
            if live is not None:
                traffic, tj_id, traffic_note, traffic_source = live["hbm_bytes_per_launch"], build_id, note, "live"
                sq, write_b = live["sq"], live["write_bytes_per_launch"]
                req = live["tcc_requests_per_launch"]
                with open(L2_CALIB_JSON) as f:
                    bpr = json.load(f)["bytes_per_request"]
                if req and kern_ms > 0:
                    l2_gbs = req * bpr / (kern_ms * 1e-3) / 1e9
                    l2 = {"requests_per_launch": req, "bytes_per_request": bpr, "achieved": round(l2_gbs, 1),
                          "peak": L2_PEAK_GBS, "unit": "GB/s", "frac": round(l2_gbs / L2_PEAK_GBS, 4),
                          "hit_rate": live["tcc_hit_rate"], "source": "live rocprofv3 --pmc passes",
                          "calibration": os.path.relpath(L2_CALIB_JSON, ROOT)}
            else:
                traffic_note = f"{note}; {traffic_note}"
        hbm_frac = round(traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if traffic and kern_ms > 0 else None
        nodes = [int(x["node_visits"]) for x in sts]
        tris = [int(x["tri_tests"]) for x in sts]
        n_tris = info["n_tris"]
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(max_t / max(args.steps, 1) * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: procedural {args.scene} stand-in ({n_tris} tris) in the reference Cornell box"
                    if args.scene != "cornell" else "synthetic: reference Cornell box",
            "config": {"workload": f"{args.scene}-{W}x{H}-{spp}spp", "width": W, "height": H, "spp": spp,
                       "triangles": n_tris, "bvh_nodes": info["bvh_nodes"], "tile": T if world > 1 else f"{W}x{H} (one tile per frame)",
                       "frames_per_step": len(frames),
                       "parallelism": "1 GPU, no collective" if world == 1 else
                       f"tiles{world}+{'rccl' if args.dist_backend == 'nccl' else 'gloo'}-gather"},
            "samples_per_s": round(samples / max_t, 1),
            "reference_queries_per_s": round(queries / max_t, 1),
            "kernel_ms": round(kern_ms, 3),
            "persistent_grid_waves": int(info.get("ps_resident", 0)),
            "timing": {"pipeline": P,
                       "launch_ms": round(kern_ms, 3),
                       "launch_ms_is": "event pair around each launch" if P == 1 or args.steps < 2 else
                       "span from the first launch's start to the last launch's end / K (HIP events; "
                       f"{P} frames in flight on the context's pipeline streams)",
                       "isolated_launch_ms": round(iso, 3) if iso is not None else round(kern_ms, 3)},
            "simt_utilisation": {k: round(v, 4) for k, v in simt.items()},
            "per_launch": {"traced_rays": int(mine[1]), "node_visits": int(mine[4]), "tri_tests": int(mine[5]),
                           "algorithmic_bytes": int(survey_bytes), "loaded_bytes": int(bytes_launch),
                           "kernel": kernel, "bvh_nodes": ("128 B", "compact 80-B records")[form]},
            # achieved = SURVEY 8(d)'s algorithmic bytes (32 B per node visit, 48 B per triangle test, 32 B
            # per traced ray: independent of the node encoding) / the launch time.  The roofline priced is
            # HBM's; `bound` is what the measurements show bounds the kernel (limiter())
            "roofline": {"bound": limiter(hbm_frac, sq), "achieved": round(survey_bytes / (kern_ms * 1e-3) / 1e9, 2) if kern_ms > 0
                         else 0.0, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(survey_bytes / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5) if kern_ms > 0
                         else 0.0,
                         # the same bytes over one launch alone on an idle device (its ramp-up and drain
                         # included, no overlap with a neighbouring frame): the per-dispatch figure
                         "frac_isolated": round(survey_bytes / (iso * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                         if iso else None,
                         "traffic": traffic, "traffic_build_id": tj_id if traffic is not None else None,
                         "traffic_source": traffic_source, "traffic_note": traffic_note,
                         # measured HBM traffic / launch time / peak: the DRAM side of the roofline
                         "hbm_frac": hbm_frac, "write_bytes_per_launch": write_b,
                         # SQ pass: VALU pipes busy, and wave cycles issuing / in s_waitcnt / ready
                         # but not issued (sq_fields)
                         "valu_busy": sq["valu_busy"] if sq else None,
                         "wave_split": sq["wave_split"] if sq else None,
                         "sq_raw": sq.get("raw") if sq else None,
                         "bytes_per_unit": {"node": SURVEY_NODE_BYTES, "tri": SURVEY_TRI_BYTES,
                                            "shade_per_ray": SHADE_BYTES},
                         # the bytes this implementation's encodings load per launch (80-B compact or 112-B
                         # node reads, 64-B triangle records), mostly served by L2 and the Infinity Cache:
                         # their rate can exceed the HBM peak
                         "loaded": {"bytes_per_launch": int(bytes_launch), "achieved": round(achieved, 2),
                                    "frac": round(achieved / HBM_PEAK_GBS, 5),
                                    "bytes_per_unit": {"node": node_b, "tri": TRI_BYTES, "shade_per_ray": SHADE_BYTES}},
                         # L2 request traffic of the timed kernel (PMC pass, calibrated request size)
                         "l2": l2,
                         # node/triangle counts come from instrumented passes of the same tiles, whose
                         # schedule differs from the timed launch's: their spread over the passes
                         "count_spread": {"passes": len(sts), "node_visits": [min(nodes), max(nodes)],
                                          "tri_tests": [min(tris), max(tris)]}},
            "cpu_baseline": base,
            "build_id": build_id,
        }
        if world > 1:
            # where a multi-GPU step's time goes: each rank's launch time and its gather (which
            # waits for the slowest rank's tiles), per step; and each rank's roofline fraction from
            # its own counts (SURVEY 8(d) bytes of its tiles) over its own launch time
            rk_bytes = allv[:, 4] * SURVEY_NODE_BYTES + allv[:, 5] * SURVEY_TRI_BYTES + allv[:, 1] * SHADE_BYTES
            rk_frac = [round(float(b / (t * 1e-3) / 1e9 / HBM_PEAK_GBS), 5) if t > 0 else 0.0
                       for b, t in zip(rk_bytes, allv[:, 6])]
            line["per_rank"] = {"roofline_frac": rk_frac,
                                "traced_rays": [int(x) for x in allv[:, 1]],
                                "algorithmic_bytes": [int(x) for x in rk_bytes],"kernel_ms": [round(float(x), 3) for x in allv[:, 6]],
                                "gather_ms": [round(float(x), 3) for x in allv[:, 7]],
                                "isolated_launch_ms": [round(float(x), 3) for x in allv[:, 8]],
                                "kernel_ms_min_max": [round(float(allv[:, 6].min()), 3),
                                                      round(float(allv[:, 6].max()), 3)],
                                "gather_ms_min_max": [round(float(allv[:, 7].min()), 3),
                                                      round(float(allv[:, 7].max()), 3)]}
        if check is not None:
            line["check_frames_bit_exact"] = check
            line["check"] = {"frames": len(frames), "world_size": world,
                             "collective": "rccl" if args.dist_backend == "nccl" else "gloo",
                             "against": "ctx.render_frames of the same seeds on rank 0 (one launch)"}
        print(json.dumps(line), flush=True)
    # teardown: the process group and torch's buffers may still refer to the context's
    # pipeline streams, so they go first; the context (which destroys its streams) last
    torch.cuda.synchronize()
    if world > 1:
        dist.destroy_process_group()
    del shard
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
    ctx.close()


if __name__ == "__main__":
    main()
