"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bar (BASELINE.json north_star): radiance within 1e-4 relative per pixel, hit
triangle/primitive IDs bit-exact.  The kernels are built to reproduce the oracle's
fp32 evaluation exactly, so these tests demand bit equality of the float32
radiance (the 1e-4 relative check is asserted too, as the contractual bar).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL_TOL = 1e-4  # north_star: "output radiance matches ... within 1e-4 relative per pixel"


def assert_radiance(g, r):
    gf, rf = g[..., :3].astype(np.float64), r[..., :3].astype(np.float64)
    rel = np.abs(gf - rf) / np.maximum(np.abs(rf), 1e-30)
    rel[(gf == rf)] = 0.0
    assert rel.max() <= REL_TOL, f"max rel err {rel.max()}"
    assert np.array_equal(g.view(np.uint32), r.view(np.uint32)), \
        f"{np.count_nonzero(g.view(np.uint32) != r.view(np.uint32))} float words differ"


def check_counters(stats, cnt, oracle):
    assert stats["traced_rays"] == int(cnt[oracle.CNT_TRACED])
    assert stats["queries"] == int(cnt[oracle.CNT_QUERIES])
    assert stats["samples"] == int(cnt[oracle.CNT_SAMPLES])
    assert stats["nan_rays"] == int(cnt[oracle.CNT_NAN_RAYS])
    # the parked kernel's global stack never runs out (park_fix's overflow exit would end a
    # traversal early: a wrong pixel)
    assert stats["stack_overflows"] == 0


@pytest.fixture(scope="module")
def cornell(wgt, oracle):
    L, Q, S = wgt.cornell_scene()
    return (L, Q, S), oracle.OracleScene(L, Q, S)


@pytest.mark.parametrize("W,H,spp,seed", [(64, 64, 1, 0), (64, 64, 1, 1), (64, 64, 1, 2), (40, 24, 16, 5),
                                          (33, 17, 4, 123456789)])
def test_cornell_parity(ctx, wgt, oracle, cornell, W, H, spp, seed):
    (L, Q, S), osc = cornell
    ctx.upload_scene(L, Q, S)
    g = ctx.render_tile(wgt.camera_param(W / H, spp, seed), W, H, stats=True)
    r = osc.render(oracle.camera_param(W / H, spp, seed), W, H)
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["u8"], r["u8"])
    assert np.array_equal(g["hit"], r["hit"])
    check_counters(g["stats"], r["counters"], oracle)


def test_cornell_c1_full_frame(ctx, wgt, oracle, cornell):
    """BASELINE config 1 (Cornell 256x256, 1 spp), seeds 0..2, whole frame."""
    (L, Q, S), osc = cornell
    ctx.upload_scene(L, Q, S)
    for seed in (0, 1, 2):
        g = ctx.render_tile(wgt.camera_param(1.0, 1, seed), 256, 256, stats=True)
        r = osc.render(oracle.camera_param(1.0, 1, seed), 256, 256)
        assert_radiance(g["f32"], r["f32"])
        assert np.array_equal(g["hit"], r["hit"])
        check_counters(g["stats"], r["counters"], oracle)


def test_cornell_c2_subsample(ctx, wgt, oracle, cornell):
    """BASELINE config 2 (1024x1024, 64 spp): oracle on a strided pixel subsample."""
    (L, Q, S), osc = cornell
    ctx.upload_scene(L, Q, S)
    cam_g, cam_o = wgt.camera_param(1.0, 64, 9), oracle.camera_param(1.0, 64, 9)
    g = ctx.render_tile(cam_g, 1024, 1024)
    for (x0, y0) in [(0, 0), (512, 300), (1016, 1016), (250, 700)]:
        r = osc.render(cam_o, 1024, 1024, x0, y0, 8, 8)
        assert_radiance(g["f32"][y0:y0 + 8, x0:x0 + 8], r["f32"])
        assert np.array_equal(g["hit"][y0:y0 + 8, x0:x0 + 8], r["hit"])


def test_tiles_reassemble_full_frame(ctx, wgt, cornell):
    """Any tiling (global pixel coords + full-frame seed) reproduces the frame."""
    (L, Q, S), _ = cornell
    ctx.upload_scene(L, Q, S)
    W, H = 70, 45
    cam = wgt.camera_param(W / H, 4, 77)
    full = ctx.render_tile(cam, W, H)["f32"]
    out = np.zeros_like(full)
    for (x0, y0, tw, th) in [(0, 0, 33, 20), (33, 0, 37, 20), (0, 20, 70, 13), (0, 33, 50, 12), (50, 33, 20, 12)]:
        out[y0:y0 + th, x0:x0 + tw] = ctx.render_tile(cam, W, H, x0, y0, tw, th)["f32"]
    assert np.array_equal(out.view(np.uint32), full.view(np.uint32))


def test_tile_past_frame_edge(ctx, wgt, oracle, cornell):
    (L, Q, S), osc = cornell
    ctx.upload_scene(L, Q, S)
    cam = wgt.camera_param(1.0, 1, 4)
    g = ctx.render_tile(cam, 50, 50, 40, 40, 16, 16)
    r = osc.render(oracle.camera_param(1.0, 1, 4), 50, 50, 40, 40, 10, 10)
    assert_radiance(g["f32"][:10, :10], r["f32"])
    assert np.all(g["f32"][10:] == 0) and np.all(g["hit"][10:] == 0xFFFFFFFF)


@pytest.mark.parametrize("spp", [0, 2, 1000])
def test_spp_edge_cases(ctx, wgt, oracle, cornell, spp):
    """spp=0 -> black; spp not a perfect square -> u32(sqrt)^2 samples / spp (path_tracer.wgsl:380,393)."""
    (L, Q, S), osc = cornell
    ctx.upload_scene(L, Q, S)
    W, H = (8, 8) if spp == 1000 else (24, 16)
    g = ctx.render_tile(wgt.camera_param(W / H, spp, 1), W, H, stats=True)
    r = osc.render(oracle.camera_param(W / H, spp, 1), W, H)
    assert_radiance(g["f32"], r["f32"])
    check_counters(g["stats"], r["counters"], oracle)
    if spp == 0:
        assert np.all(g["f32"][..., :3] == 0)


def test_emissive_last_sphere_no_skip(ctx, wgt, oracle, cornell):
    """NaN rays hit the last sphere; if it is emissive the skip-ahead must not apply."""
    (L, Q, S), _ = cornell
    S2 = np.concatenate([S, S])
    S2[1]["center"] = (278.0, 100.0, 278.0)
    S2[1]["radius"] = 60.0
    S2[1]["col"] = (2.0, 1.0, 0.5)
    S2[1]["emissive"] = 1.0
    ctx.upload_scene(L, Q, S2)
    g = ctx.render_tile(wgt.camera_param(16 / 9, 4, 2), 48, 27, stats=True)
    r = oracle.OracleScene(L, Q, S2).render(oracle.camera_param(16 / 9, 4, 2), 48, 27)
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["hit"], r["hit"])
    check_counters(g["stats"], r["counters"], oracle)


def test_scene_without_quads(ctx, wgt, oracle, cornell):
    (L, Q, S), _ = cornell
    tris = wgt.procedural_mesh("bunny", 500)
    ctx.upload_scene(L, Q[:0], S, tris)
    g = ctx.render_tile(wgt.camera_param(1.0, 4, 3), 24, 24)
    r = oracle.OracleScene(L, Q[:0], S, tris).render(oracle.camera_param(1.0, 4, 3), 24, 24)
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["hit"], r["hit"])


def test_single_triangle_scene(ctx, wgt, oracle, cornell):
    (L, Q, S), _ = cornell
    tri = wgt.make_triangles(np.array([[[100, 0, 100], [450, 0, 100], [278, 400, 500]]], np.float32))
    ctx.upload_scene(L, Q[:5], S, tri)
    info = ctx.scene_info()
    assert info["n_tris"] == 1 and info["bvh_nodes"] == 1
    g = ctx.render_tile(wgt.camera_param(1.0, 4, 8), 32, 32)
    r = oracle.OracleScene(L, Q[:5], S, tri).render(oracle.camera_param(1.0, 4, 8), 32, 32)
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["hit"], r["hit"])


@pytest.fixture(scope="module")
def bunny(wgt, oracle):
    L, Q, S, T = wgt.mesh_scene("bunny")
    return (L, Q, S, T), oracle.OracleScene(L, Q, S, T)


def _random_rays(n, rng, inside=True):
    o = rng.uniform(5, 550, size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o, d.astype(np.float32)


def test_trace_rays_vs_oracle_bvh(ctx, wgt, oracle, bunny):
    """Closest-hit query (sample_hit) on 200k random rays: prim id + distance bit-exact."""
    (L, Q, S, T), osc = bunny
    ctx.upload_scene(L, Q, S, T)
    rng = np.random.default_rng(0)
    o, d = _random_rays(200_000, rng)
    gp, gd = ctx.trace_rays(o, d)
    rp, rd = osc.trace(o, d)
    assert np.array_equal(gp, rp)
    assert np.array_equal(gd.view(np.uint32), rd.view(np.uint32))
    n_tri_hits = np.count_nonzero((gp >= len(L) + len(Q)) & (gp < len(L) + len(Q) + len(T)))
    assert n_tri_hits > 10_000  # the test really exercises the BVH


def test_trace_rays_vs_bruteforce_spec(ctx, wgt, oracle, bunny):
    """The triangle SPEC is a linear scan (min (t, index)); BVH must match it exactly."""
    (L, Q, S, T), osc = bunny
    ctx.upload_scene(L, Q, S, T)
    rng = np.random.default_rng(1)
    # aim at triangle centroids so most rays hit the mesh
    idx = rng.integers(0, len(T), 3000)
    c = T["v0"][idx, :3] + (T["e1"][idx, :3] + T["e2"][idx, :3]) / 3.0
    o = rng.uniform(5, 550, size=(3000, 3)).astype(np.float32)
    d = (c - o).astype(np.float32)
    gp, gd = ctx.trace_rays(o, d)
    rp, rd = osc.trace(o, d, brute=True)
    assert np.array_equal(gp, rp)
    assert np.array_equal(gd.view(np.uint32), rd.view(np.uint32))


def test_trace_rays_nan_and_degenerate(ctx, wgt, oracle, bunny):
    (L, Q, S, T), osc = bunny
    ctx.upload_scene(L, Q, S, T)
    o = np.array([[278, 278, -800], [np.nan, 1, 1], [278, 100, 278], [278, 100, 278], [0, 0, 0]], np.float32)
    d = np.array([[0, 0, 1], [0, 0, 1], [np.nan, 0, 0], [0, 0, 0], [1e-38, 1e-38, 1]], np.float32)
    gp, gd = ctx.trace_rays(o, d)
    rp, rd = osc.trace(o, d)
    assert np.array_equal(gp, rp)
    assert np.array_equal(gd.view(np.uint32), rd.view(np.uint32))


@pytest.mark.parametrize("W,H,spp,seed", [(96, 54, 4, 0), (64, 36, 16, 11)])
def test_bunny_render_parity(ctx, wgt, oracle, bunny, W, H, spp, seed):
    (L, Q, S, T), osc = bunny
    ctx.upload_scene(L, Q, S, T)
    g = ctx.render_tile(wgt.camera_param(16 / 9, spp, seed), W, H, stats=True)
    r = osc.render(oracle.camera_param(16 / 9, spp, seed), W, H)
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["hit"], r["hit"])
    check_counters(g["stats"], r["counters"], oracle)


@pytest.mark.parametrize("W,H", [(1, 1), (1, 9), (9, 1), (7, 5), (65, 3)])
def test_tiny_and_ragged_mesh_frames(ctx, wgt, oracle, bunny, W, H):
    """Frames smaller than one 8x8 pixel block, or one block wide and ragged, through the
    persistent mesh kernel (a grid of one or a few waves, most lanes without a pixel, the
    cost pre-pass and LPT order over 1-9 blocks) against the oracle."""
    (L, Q, S, T), osc = bunny
    ctx.upload_scene(L, Q, S, T)
    g = ctx.render_tile(wgt.camera_param(W / H, 9, 4), W, H, stats=True)
    r = osc.render(oracle.camera_param(W / H, 9, 4), W, H)
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["hit"], r["hit"])
    check_counters(g["stats"], r["counters"], oracle)


def test_bunny_1080p_256spp_subsample(ctx, wgt, oracle, bunny):
    """BASELINE config 3 at full size: GPU tiles of the 1920x1080/256spp frame vs the
    oracle on the same global pixels."""
    (L, Q, S, T), osc = bunny
    ctx.upload_scene(L, Q, S, T)
    cam_g, cam_o = wgt.camera_param(16 / 9, 256, 1), oracle.camera_param(16 / 9, 256, 1)
    for (x0, y0) in [(960, 540), (700, 900), (1200, 300)]:
        g = ctx.render_tile(cam_g, 1920, 1080, x0, y0, 8, 4)
        r = osc.render(cam_o, 1920, 1080, x0, y0, 8, 4)
        assert_radiance(g["f32"], r["f32"])
        assert np.array_equal(g["hit"], r["hit"])


_SPONZA = {}


def _sponza(wgt, oracle):
    """The sponza stand-in and the oracle's 80x45 / 4 spp render of it (built once)."""
    if not _SPONZA:
        L, Q, S, T = wgt.mesh_scene("sponza")
        osc = oracle.OracleScene(L, Q, S, T)
        _SPONZA["scene"] = (L, Q, S, T)
        _SPONZA["r"] = osc.render(oracle.camera_param(16 / 9, 4, 5), 80, 45)
        osc.close()
    return _SPONZA["scene"]


@pytest.mark.parametrize("cnode", ["2", "0", "1"])
def test_sponza_render_parity(ctx, wgt, oracle, cnode, monkeypatch):
    """Sponza stand-in: the persistent kernel reads the 80-B compact records by default (1) and by
    the size rule (2: the 128-B tree exceeds one XCD's L2); 0 forces the 128-B nodes."""
    monkeypatch.setenv("WGT_CNODE", cnode)
    L, Q, S, T = _sponza(wgt, oracle)
    ctx.upload_scene(L, Q, S, T)
    g = ctx.render_tile(wgt.camera_param(16 / 9, 4, 5), 80, 45, stats=True)
    r = _SPONZA["r"]
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["hit"], r["hit"])
    check_counters(g["stats"], r["counters"], oracle)
    info = ctx.scene_info()
    assert info["n_tris"] == len(T) and info["bvh_max_depth"] <= 94
    assert info["bvh_compact"] == 1
    assert info["node_form"] == {"2": 1, "0": 0, "1": 1}[cnode]


_FULL = {}


@pytest.mark.parametrize("kind,spp,env", [("sponza", 4, {}), ("sponza", 4, {"WGT_CNODE": "0"}),
                                          ("sponza", 4, {"WGT_PARK": "1"}), ("bunny", 1, {}),
                                          ("bunny", 1, {"WGT_CNODE": "0"})])
def test_full_frame_1080p_bit_exact(ctx, wgt, oracle, kind, spp, env, monkeypatch):
    """Every pixel of a full 1920x1080 frame at the bench's resolution, GPU vs the
    oracle (OpenMP), through the default kernel of each scene: both on the 80-B compact
    records (round 6; until then bunny read the 128-B nodes), at 6 waves/SIMD with 3-byte stack entries; and each
    on the other node form, and sponza with parked traversal state (WGT_PARK=1, an 18-entry LDS
    stack)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    L, Q, S, T = wgt.mesh_scene(kind)
    ctx.upload_scene(L, Q, S, T)
    info = ctx.scene_info()
    if not any(os.environ.get(k) for k in ("WGT_CNODE", "WGT_PS_WAVES", "WGT_STACK_LIMIT", "WGT_PARK")):
        assert (info["bvh_compact"], info["ps_waves"]) == ((1, 6) if kind == "sponza" else (0, 6))
        assert info["ps_park"] == 0 and info["ps_stack"] == info["bvh_stack"] + 1
        assert info["node_form"] == 1
    g = ctx.render_tile(wgt.camera_param(16 / 9, spp, 3), 1920, 1080, stats=True)
    if kind not in _FULL:
        osc = oracle.OracleScene(L, Q, S, T)
        _FULL[kind] = osc.render(oracle.camera_param(16 / 9, spp, 3), 1920, 1080)
        osc.close()
    r = _FULL[kind]
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["hit"], r["hit"])
    check_counters(g["stats"], r["counters"], oracle)


def test_sponza_1080p_256spp_subsample_compact(ctx, wgt, oracle):
    """BASELINE config 4 (the bench workload) at full size through the compact nodes:
    GPU tiles of the 1920x1080/256spp frame vs the oracle on the same global pixels."""
    L, Q, S, T = _sponza(wgt, oracle)
    ctx.upload_scene(L, Q, S, T)
    osc = oracle.OracleScene(L, Q, S, T)
    cam_g, cam_o = wgt.camera_param(16 / 9, 256, 0), oracle.camera_param(16 / 9, 256, 0)
    for (x0, y0) in [(960, 540), (300, 800)]:
        g = ctx.render_tile(cam_g, 1920, 1080, x0, y0, 8, 2)
        r = osc.render(cam_o, 1920, 1080, x0, y0, 8, 2)
        assert_radiance(g["f32"], r["f32"])
        assert np.array_equal(g["hit"], r["hit"])


@pytest.mark.parametrize("kernel", ["1", "2"])
def test_kernel_families_agree_with_oracle(ctx, wgt, oracle, bunny, kernel, monkeypatch):
    """The simple megakernel (1) and the persistent phase-split one (2) are both
    bit-exact against the oracle (the tuning knobs change speed only)."""
    (L, Q, S, T), osc = bunny
    monkeypatch.setenv("WGT_KERNEL", kernel)
    ctx.upload_scene(L, Q, S, T)
    g = ctx.render_tile(wgt.camera_param(16 / 9, 4, 21), 72, 40, stats=True)
    r = osc.render(oracle.camera_param(16 / 9, 4, 21), 72, 40)
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["hit"], r["hit"])
    check_counters(g["stats"], r["counters"], oracle)


_SCHED_REF = {}


@pytest.mark.parametrize("env", [{"WGT_PQ_LPT": "0"}, {"WGT_PQ_LPT": "1"}, {"WGT_PQ_REFILL": "1"},
                                 {"WGT_PQ_REFILL": "64"}, {"WGT_PS_TO_TRAV": "1", "WGT_PS_TO_SERVICE": "63"},
                                 {"WGT_PQ_LPT": "2"}, {"WGT_PQ_LPT_ALL": "0"}, {"WGT_PS_SVC_FRAC": "0"},
                                 {"WGT_PS_SVC_FRAC": "1"},
                                 # the cost pre-pass's path depth (default 6): its shortest and the full path
                                 {"WGT_PQ_DEPTH": "1"}, {"WGT_PQ_DEPTH": "50"},
                                 {"WGT_CNODE": "0"}, {"WGT_CNODE": "0", "WGT_PQ_LPT": "0"}, {"WGT_PS_WAVES": "5"},
                                 {"WGT_PS_WAVES": "5", "WGT_CNODE": "0"}, {"WGT_NARROW": "1"},
                                 {"WGT_STACK_LIMIT": "20"},
                                 # parked traversal state (WGT_PARK=1): the default LDS stack, the
                                 # smallest (every node step near the top spills to the global stack),
                                 # per node form and wave budget
                                 {"WGT_PARK": "1"}, {"WGT_PARK": "1", "WGT_CNODE": "0"},
                                 {"WGT_PARK": "1", "WGT_PS_CAP": "8"}, {"WGT_PARK": "1", "WGT_PS_CAP": "8", "WGT_CNODE": "0"},
                                 {"WGT_PARK": "1", "WGT_PS_CAP": "8", "WGT_PS_WAVES": "5"},
                                 {"WGT_PARK": "1", "WGT_PS_CAP": "9", "WGT_PQ_LPT": "0"},
                                 # triangle steps as soon as one lane has a leaf open (1), or node steps
                                 # while any lane has a node (the most second leaves parked on the stack)
                                 {"WGT_TRI_RATIO": "1"}, {"WGT_TRI_RATIO": "1000000"},
                                 {"WGT_TRI_RATIO": "1", "WGT_CNODE": "0"},
                                 ])
def test_ps_schedule_invariance(ctx, wgt, oracle, bunny, env, monkeypatch):
    """The persistent phase-split kernel's scheduling knobs (queue order: LPT from the
    cost pre-pass (1 or 4 spp) or block order; refill threshold; phase thresholds and
    their sparse-wave scaling; the node form: 128-B nodes forced on the bunny; the
    wave budget: 6 waves per SIMD with 3-byte stack entries or, with WGT_PS_WAVES=5, 5
    with 4-byte ones; the narrow 25-entry tree, WGT_NARROW=1; a 20-entry bound, which moves
    the 3-byte stack's byte array; the parked traversal state with small LDS stacks,
    WGT_PARK=1 with LDS stacks down to WGT_PS_CAP=8)
    change which lane renders which pixel and when, never a bit of the result.  100x60
    leaves ragged 8x8 blocks at the frame edge.  The test runs after the kernel-family
    tests on the same context, the sequence that exposed a workspace-reuse bug (each
    pixel rendered twice in the stats pass) when the workspace came from
    hipMallocAsync."""
    (L, Q, S, T), osc = bunny
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ctx.upload_scene(L, Q, S, T)
    g = ctx.render_tile(wgt.camera_param(5 / 3, 9, 3), 100, 60, stats=True)
    if "r" not in _SCHED_REF:
        _SCHED_REF["r"] = osc.render(oracle.camera_param(5 / 3, 9, 3), 100, 60)
    r = _SCHED_REF["r"]
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["hit"], r["hit"])
    check_counters(g["stats"], r["counters"], oracle)


@pytest.mark.parametrize("cap,cnode", [("8", "2"), ("8", "1"), ("11", "2")])
def test_stack_overflow_spill_and_refill(ctx, wgt, oracle, bunny, cap, cnode, monkeypatch):
    """The parked kernel's LDS stack bounded at 8 (or 11) entries (WGT_PS_CAP; the builder's
    bound is 31, a node step may start only from a top <= 4 = 8 - 4, the 4-entry bound
    round 3's review asked for): node steps that leave fewer than 4 free entries park the lane, whose
    service pass moves the bottom of its stack to the global stack, and a lane whose LDS
    part runs empty refills from it (park_fix).  Both paths must
    run (the counters) and the frame stay bit-exact against the oracle."""
    (L, Q, S, T), osc = bunny
    monkeypatch.setenv("WGT_PARK", "1")
    monkeypatch.setenv("WGT_PS_CAP", cap)
    monkeypatch.setenv("WGT_CNODE", cnode)
    ctx.upload_scene(L, Q, S, T)
    info = ctx.scene_info()
    assert info["ps_park"] == 1 and info["ps_stack"] == int(cap) < info["bvh_stack"]
    g = ctx.render_tile(wgt.camera_param(5 / 3, 9, 3), 100, 60, stats=True)
    if "r" not in _SCHED_REF:
        _SCHED_REF["r"] = osc.render(oracle.camera_param(5 / 3, 9, 3), 100, 60)
    r = _SCHED_REF["r"]
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["hit"], r["hit"])
    check_counters(g["stats"], r["counters"], oracle)
    assert g["stats"]["stack_spills"] > 0 and g["stats"]["stack_refills"] > 0


def test_mesh_tiles_reassemble_full_frame(ctx, wgt, bunny):
    """Ragged tiles (not multiples of the 8x8 pixel blocks) through the persistent
    kernel reproduce the full frame bit for bit."""
    (L, Q, S, T), _ = bunny
    ctx.upload_scene(L, Q, S, T)
    W, H = 61, 43
    cam = wgt.camera_param(W / H, 4, 8)
    full = ctx.render_tile(cam, W, H)["f32"]
    out = np.zeros_like(full)
    for y0 in range(0, H, 12):
        for x0 in range(0, W, 12):
            tw, th = min(12, W - x0), min(12, H - y0)
            out[y0:y0 + th, x0:x0 + tw] = ctx.render_tile(cam, W, H, x0, y0, tw, th)["f32"]
    assert np.array_equal(out.view(np.uint32), full.view(np.uint32))


def test_triangle_tie_rule_on_gpu(ctx, wgt, oracle):
    """tests/test_oracle_kats.py::test_triangle_tie_rule_is_min_t_then_index through
    the kernel: equal ray_dist, different t -> the smaller t (index 1) wins."""
    from test_oracle_kats import TIE_D, TIE_O, tie_triangles

    L, Q, S = wgt.cornell_scene()
    T = tie_triangles(wgt)
    ctx.upload_scene(L, Q[:0], S, T)
    prim, dist = ctx.trace_rays(TIE_O, TIE_D)
    rp, rd = oracle.OracleScene(L, Q[:0], S, T).trace(TIE_O, TIE_D)
    assert prim[0] == rp[0] == len(L) + 1
    assert dist.view(np.uint32)[0] == rd.view(np.uint32)[0]
