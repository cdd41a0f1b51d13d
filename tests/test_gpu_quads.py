"""GPU parity of the quad scan without per-quad distances (wgt_device.h quad_scan_fast, DESIGN.md
§3.2 "quad distance") where it matters: rays whose two nearest quads tie, or almost tie, in the
rounded distance the reference compares (path_tracer.wgsl:314-338).  The scene doubles the back
wall one ulp nearer the camera (later in scan order), so every ray that reaches the back wall
sees two valid quads at t one ulp apart: the reference keeps the earlier one when their rounded
distances are equal, the nearer one otherwise.  The kernels' tie test must send those rays to
the reference scan (counted: wgt_stats.quad_ref_scans) and every frame stay bit-exact."""
import numpy as np
import pytest

from test_gpu_parity import assert_radiance, check_counters
from test_quad_scan import double_back_wall, edge_rays

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kernel,tris", [("2", False), ("2", True), ("1", False)])
def test_double_wall_render_parity(ctx, wgt, oracle, kernel, tris, monkeypatch):
    """The persistent kernel (with and without triangles) and the simple one, vs the oracle."""
    monkeypatch.setenv("WGT_KERNEL", kernel)
    L, Q, S = wgt.cornell_scene()
    quads = double_back_wall(Q)
    T = wgt.procedural_mesh("bunny", 2000) if tris else None
    ctx.upload_scene(L, quads, S, T)
    cam_g, cam_o = wgt.camera_param(1.0, 4, 7), oracle.camera_param(1.0, 4, 7)
    g = ctx.render_tile(cam_g, 64, 64, stats=True)
    r = oracle.OracleScene(L, quads, S, T).render(cam_o, 64, 64)
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["hit"], r["hit"])
    check_counters(g["stats"], r["counters"], oracle)
    # the back wall's primary rays (distances ~1,400, one ulp 1.2e-4) tie with the copy 3e-5 nearer:
    # the reference keeps the earlier wall, and the persistent kernel's tie test sends them to the
    # reference scan
    assert np.count_nonzero(r["hit"] == len(L) + 4) > 500
    if kernel == "2":
        assert g["stats"]["quad_ref_scans"] > 100


@pytest.mark.parametrize("kind", ["double_wall", "edges"])
def test_quad_ties_trace_rays(ctx, wgt, oracle, kind):
    """wgt_trace_rays (k_trace, the IEEE quad distance t) on rays aimed at the doubled back wall or
    at the lines where two walls meet (exactly and a few ulps off): prim ids and distances
    bit-exact against the oracle's reference scan."""
    L, Q, S = wgt.cornell_scene()
    rng = np.random.default_rng(11)
    if kind == "double_wall":
        quads = double_back_wall(Q)
        n = 50_000
        tgt = np.stack([rng.uniform(0, 555, n), rng.uniform(0, 555, n), np.full(n, 555.0)], 1).astype(np.float32)
        o = rng.uniform(5, 550, (n, 3)).astype(np.float32)
        o[: n // 4] = (278, 278, -800)
        d = (tgt - o).astype(np.float32)
    else:
        quads = Q[:5].copy()
        o, d = edge_rays(np.concatenate([L, quads]), 50_000, rng)
    ctx.upload_scene(L, quads, S)
    gp, gd = ctx.trace_rays(o, d)
    osc = oracle.OracleScene(L, quads, S)
    rp, rd = osc.trace(o, d)
    osc.close()
    assert np.array_equal(gp, rp)
    assert np.array_equal(gd.view(np.uint32), rd.view(np.uint32))


def test_traversal_level_counters(ctx, wgt):
    """The instrumented pass's traversal-by-level counters (round 6, wgt_stats top_node_visits,
    cyc_node_steps, cyc_top_steps, cyc_tri_steps; scripts/level_stats.py): levels 1-2 hold at most 20
    of a BVH4's nodes, visits of them are a part of all node visits, and the cycles of steps whose
    lanes are all at those levels are a part of the node steps' cycles."""
    L, Q, S, T = wgt.mesh_scene("bunny", 20000)
    ctx.upload_scene(L, Q, S, T)
    st = ctx.render_tile(wgt.camera_param(16 / 9, 4, 3), 96, 54, want=("u8",), stats=True)["stats"]
    assert 0 < st["top_node_visits"] < st["node_visits"]
    assert 0 <= st["cyc_top_steps"] <= st["cyc_node_steps"] and st["cyc_node_steps"] > 0
    assert st["cyc_tri_steps"] > 0
    assert st["cyc_node_steps"] + st["cyc_tri_steps"] <= st["cyc_trav"]
    assert st["quad_ref_scans"] <= st["traced_rays"]
