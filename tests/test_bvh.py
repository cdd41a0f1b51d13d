"""Host BVH builder invariants (CPU only, through the C-ABI wgt_bvh_build).

The kernels' traversal is exact (returns the brute-force closest triangle of the
geometry spec) only if the exported tree satisfies:
  * every triangle appears in exactly one leaf, leaves hold <= 8 triangles;
  * every child box contains, bit for bit, the padded boxes of all triangles
    below it (the slab test is then conservative: rounding is monotone);
  * the per-triangle padded box stored in the record equals tri_box of the spec;
  * the LDS stack (DevScene::stack entries) is >= the worst-case push depth.
These are checked here against an independent numpy walk of the exported nodes.
"""
import numpy as np
import pytest

import webgputracer_amd as w

f32 = np.float32
STACK_MAX = 31  # kStackMax (wgt_internal.h)
EMPTY = f32(3e38)  # kEmptySlotCoord (wgt_geom.h)


def tri_box_np(v0, e1, e2):
    """tri_box (wgt_geom.h) restated in numpy fp32: bounds of v0, v0+e1, v0+e2 padded by
    ((hi-lo)*1e-4 + (|lo|+|hi|)*1e-5) + 1e-6 per axis."""
    a, b, d = v0, v0 + e1, v0 + e2
    mn = np.where(a < b, a, b)
    mn = np.where(mn < d, mn, d)
    mx = np.where(a > b, a, b)
    mx = np.where(mx > d, mx, d)
    pad = ((mx - mn) * f32(1e-4) + (np.abs(mn) + np.abs(mx)) * f32(1e-5)) + f32(1e-6)
    return mn - pad, mx + pad


def random_soup(n, seed, spread=500.0, size=20.0):
    rng = np.random.default_rng(seed)
    v0 = rng.uniform(0, spread, (n, 3)).astype(f32)
    v = np.stack([v0, v0 + rng.normal(0, size, (n, 3)).astype(f32), v0 + rng.normal(0, size, (n, 3)).astype(f32)], 1)
    return w.make_triangles(v)


def check_tree(tris):
    info, nodes, recs = w.bvh_build(tris)
    n = len(tris)
    assert info["bvh_width"] == 4
    assert info["bvh_max_leaf"] <= 8
    assert 1 <= info["bvh_stack"] <= STACK_MAX
    assert info["bvh2_depth"] <= 24

    # records: v0/e1/e2 of the original triangle, index bits, padded box == spec
    idx = recs[:, 0, 3].view(np.uint32)
    assert sorted(idx.tolist()) == list(range(n))
    v0, e1, e2 = recs[:, 0, :3], recs[:, 1, :3], recs[:, 2, :3]
    np.testing.assert_array_equal(v0, tris["v0"][idx][:, :3])
    np.testing.assert_array_equal(e1, tris["e1"][idx][:, :3])
    np.testing.assert_array_equal(e2, tris["e2"][idx][:, :3])
    lo = np.stack([recs[:, 1, 3], recs[:, 2, 3], recs[:, 3, 0]], 1)
    hi = recs[:, 3, 1:4]
    elo, ehi = tri_box_np(v0, e1, e2)
    np.testing.assert_array_equal(lo, elo)
    np.testing.assert_array_equal(hi, ehi)

    # walk: child boxes contain their subtree's triangle boxes; leaves partition the triangles
    seen = np.zeros(n, np.int32)
    refs = nodes[:, 6, :].view(np.int32)

    def walk(node):
        """-> (lo, hi, stack_need) of the subtree under BVH4 node `node`."""
        sub_lo, sub_hi = np.full(3, np.inf, f32), np.full(3, -np.inf, f32)
        need_children, live = 0, 0
        for s in range(4):
            box_lo = nodes[node, [0, 2, 4], s]
            box_hi = nodes[node, [1, 3, 5], s]
            if (box_lo == EMPTY).all():  # empty slot: far point box, never entered
                assert (box_hi == EMPTY).all()
                continue
            live += 1
            r = int(refs[node, s])
            if r >= 0:
                assert r > node  # preorder: children after the parent
                clo, chi, need = walk(r)
                need_children = max(need_children, need)
            else:
                u = (~r) & 0xFFFFFFFF
                first, count = u >> 3, (u & 7) + 1
                seen[first:first + count] += 1
                clo, chi = lo[first:first + count].min(0), hi[first:first + count].max(0)
            assert (box_lo <= clo).all() and (box_hi >= chi).all(), f"node {node} slot {s} does not contain its subtree"
            sub_lo, sub_hi = np.minimum(sub_lo, box_lo), np.maximum(sub_hi, box_hi)
        assert live >= 1
        return sub_lo, sub_hi, (live - 1) + need_children

    import sys
    old = sys.getrecursionlimit()
    sys.setrecursionlimit(max(old, 10000))
    try:
        _, _, need = walk(0)
    finally:
        sys.setrecursionlimit(old)
    assert (seen == 1).all(), "every triangle in exactly one leaf"
    assert max(need, 1) == info["bvh_stack"], (need, info["bvh_stack"])  # >= 1 entry allocated
    return info


@pytest.mark.parametrize("n,seed", [(1, 0), (2, 1), (7, 2), (9, 3), (1000, 4), (5000, 5)])
def test_bvh_random_soup(n, seed):
    check_tree(random_soup(n, seed))


def test_bvh_coincident_centroids():
    # 300 copies of one triangle: no SAH split exists, median splits must still terminate
    v = np.tile(np.array([[[0, 0, 0], [10, 0, 0], [0, 10, 0]]], f32), (300, 1, 1))
    check_tree(w.make_triangles(v))


def test_bvh_procedural_bunny():
    info = check_tree(w.procedural_mesh("bunny", 20000))
    assert info["bvh_max_depth"] < info["bvh2_depth"]  # the collapse shortens paths


def test_bvh_full_size_meshes_stack_bound():
    # the BASELINE mesh configs at full size: only the counts (the walk is the small cases' job)
    for kind in ("bunny", "sponza"):
        info, _, _ = w.bvh_build(w.procedural_mesh(kind))
        assert 1 <= info["bvh_stack"] <= STACK_MAX
        assert info["bvh2_depth"] <= 24 and info["bvh_max_leaf"] <= 8


@pytest.mark.parametrize("limit", [24, 20, 16])
def test_bvh_stack_budget(monkeypatch, limit):
    """The budgeted collapse meets any stack bound >= the BVH2 height by narrowing
    only stack-heavy nodes (WGT_STACK_LIMIT lowers kStackMax for the build): the
    walk's exact need equals the reported one and stays within the bound."""
    monkeypatch.setenv("WGT_STACK_LIMIT", str(limit))
    tris = random_soup(5000, 11)
    info = check_tree(tris)
    assert info["bvh_stack"] <= limit
    assert info["bvh2_depth"] <= limit  # feasibility: the BVH2 height fits


def test_bvh_stack_budget_below_height_fails(monkeypatch):
    """A bound below the BVH2 height cannot be met: the build fails loudly."""
    monkeypatch.setenv("WGT_STACK_LIMIT", "3")
    with pytest.raises(RuntimeError, match="stack limit"):
        w.bvh_build(random_soup(5000, 11))


def check_compact(tris):
    """The compact node form (wgt_geom.h) of the same tree.  The kernel's fused slab step
    fma(h, s/d, fma(org/s, s/d, ot)) rounds differently from the exact fma(b, 1/d, ot), so
    every live child plane org' + h*s (org' = stored org/s times s) keeps the margin
    G = 2^-21 M from the 128-B child bound (lo planes <= lo - G, hi planes >= hi + G),
    with M = max(4 x the triangles' extent, 2 x every node coordinate) (BuildBvh's
    origin_bound for the host export); each code is the tightest such binary16 value,
    org' is the largest value of its form <= the union's lower bound - G, empty slots
    have +inf codes on every plane (never entered), and refs are the 128-B node's refs."""
    info, nodes, _ = w.bvh_build(tris)
    cn, cr, step = w.bvh_build_compact(tris)
    step = f32(step)
    assert step > 0 and np.log2(step) == np.round(np.log2(step))  # a power of two
    assert cn.shape == (info["bvh_nodes"], 16)
    np.testing.assert_array_equal(cr, nodes[:, 6, :].view(np.int32))
    live = ~((nodes[:, 0, :] == EMPTY) & (nodes[:, 1, :] == EMPTY))  # (n, 4)
    assert (cn[:, 3] == 0).all()  # reserved
    v0 = tris["v0"][:, :3].astype(np.float64)
    v = np.concatenate([v0, v0 + tris["e1"][:, :3].astype(np.float64), v0 + tris["e2"][:, :3].astype(np.float64)])
    coords = nodes[:, :6, :].astype(np.float64)[np.broadcast_to(live[:, None, :], (len(nodes), 6, 4))]
    M = max(4.0 * np.abs(v).max(), 2.0 * np.abs(coords).max(), 2.0 ** -60)
    G = np.ldexp(M, -21)
    orgs = cn[:, 0:3].view(np.float32)
    org = orgs.astype(np.float64) * np.float64(step)  # exact

    def codes(words):  # (n, 2) words -> (n, 4) half bit patterns, children 0..3
        return np.stack([words[:, 0] & 0xFFFF, words[:, 0] >> 16, words[:, 1] & 0xFFFF, words[:, 1] >> 16], 1)

    def dec(h, o):  # the plane org' + h*s, exact in float64 (+inf codes: inf)
        with np.errstate(invalid="ignore", over="ignore"):
            return h.astype(np.uint16).view(np.float16).astype(np.float64) * np.float64(step) + o[:, None]

    for a in range(3):
        lo_h, hi_h = codes(cn[:, 4 + 4 * a:6 + 4 * a]), codes(cn[:, 6 + 4 * a:8 + 4 * a])
        # live: finite, non-negative halves; empty: +inf
        assert (lo_h[live] <= 0x7BFF).all() and (hi_h[live] <= 0x7BFF).all()
        assert (lo_h[~live] == 0x7C00).all() and (hi_h[~live] == 0x7C00).all()
        blo = nodes[:, 2 * a, :].astype(np.float64) - G
        bhi = nodes[:, 2 * a + 1, :].astype(np.float64) + G
        dlo, dhi = dec(lo_h, org[:, a]), dec(hi_h, org[:, a])
        assert (dlo[live] <= blo[live]).all() and (dhi[live] >= bhi[live]).all()
        # tightest: the next code outward would no longer keep the margin
        up = live & (lo_h < 0x7BFF)
        assert (dec(lo_h + 1, org[:, a])[up] > blo[up]).all()
        down = live & (hi_h > 0)
        assert (dec(hi_h - 1, org[:, a])[down] < bhi[down]).all()
        # org' <= the union's lower bound - G, and the next float of org/s would exceed it
        target = np.where(live, blo, np.inf).min(1)
        assert (org[:, a] <= target).all()
        nxt = np.nextafter(orgs[:, a], np.float32(np.inf)).astype(np.float64) * np.float64(step)
        assert (nxt > target).all()
    return info


@pytest.mark.parametrize("n,seed", [(1, 0), (9, 3), (5000, 5)])
def test_compact_nodes_random_soup(n, seed):
    check_compact(random_soup(n, seed))


def test_compact_nodes_wide_and_tiny_extents():
    # a 1e6-wide scene (step > 1) with millimetre triangles (subnormal-range codes)
    rng = np.random.default_rng(7)
    v0 = rng.uniform(-5e5, 5e5, (2000, 3)).astype(f32)
    v = np.stack([v0, v0 + rng.normal(0, 1e-3, (2000, 3)).astype(f32), v0 + rng.normal(0, 1e-3, (2000, 3)).astype(f32)], 1)
    check_compact(w.make_triangles(v))


def test_compact_nodes_full_size_meshes():
    """The size rule (scene_info bvh_compact; WGT_CNODE=2 reads the node form by it): the bunny
    stand-in's 128-B tree (2.3 MB) fits one XCD's 4 MB L2, sponza's (8.5 MB) does not.  The
    default (WGT_CNODE=1) reads the compact form for both."""
    for kind, compact in (("bunny", 0), ("sponza", 1)):
        tris = w.procedural_mesh(kind)
        assert check_compact(tris)["bvh_compact"] == compact


def test_wave_budget_and_narrow_tree(monkeypatch):
    """The persistent kernel runs 6 waves per SIMD with 3-byte stack entries whenever
    every ref of the tree fits them (< 2^16 nodes, < 2^20 triangles): both stand-ins, on
    their wide trees (the 31-entry bound).  WGT_NARROW=1 builds the 25-entry tree when
    its SAH cost is within 3% of the wide one's (bunny stand-in: SAH-optimal trees of cost
    22.77 at 25 entries vs 22.63 at 31; sponza's would cost 5% more and stays wide);
    WGT_PS_WAVES=5 selects 5 waves with 4-byte entries."""
    for kind in ("bunny", "sponza"):
        info, _, _ = w.bvh_build(w.procedural_mesh(kind))
        assert info["ps_waves"] == 6 and info["bvh_nodes"] < 1 << 16
        assert 25 < info["bvh_stack"] <= 31
        # by default the whole stack in LDS
        assert info["ps_park"] == 0 and info["ps_stack"] == info["bvh_stack"] + 1
    # the parked kernel (WGT_PARK=1) keeps 18 of the 32 entries in LDS at 6 waves (3 B each beside
    # 11 parked words: 6,400 B per wave, kPsLdsPerCu)
    monkeypatch.setenv("WGT_PARK", "1")
    info, _, _ = w.bvh_build(w.procedural_mesh("sponza"))
    assert info["ps_park"] == 1 and info["ps_stack"] == 18
    monkeypatch.setenv("WGT_PS_WAVES", "7")  # no longer a wave budget (round 6): 6 as without it
    info, _, _ = w.bvh_build(w.procedural_mesh("sponza"))
    assert info["ps_waves"] == 6 and info["ps_park"] == 1 and info["ps_stack"] == 18
    monkeypatch.delenv("WGT_PS_WAVES")
    monkeypatch.setenv("WGT_PS_CAP", "11")
    info, _, _ = w.bvh_build(w.procedural_mesh("bunny"))
    assert info["ps_stack"] == 11
    monkeypatch.setenv("WGT_PS_CAP", "2")  # clamped to kMinPsCap
    info, _, _ = w.bvh_build(w.procedural_mesh("bunny"))
    assert info["ps_stack"] == 8
    monkeypatch.setenv("WGT_PARK", "0")
    info, _, _ = w.bvh_build(w.procedural_mesh("bunny"))
    assert info["ps_park"] == 0 and info["ps_stack"] == info["bvh_stack"] + 1
    monkeypatch.delenv("WGT_PARK")
    monkeypatch.delenv("WGT_PS_CAP")
    monkeypatch.setenv("WGT_NARROW", "1")
    bunny = w.procedural_mesh("bunny", 20000)
    info = check_tree(bunny)  # the exported (= uploaded) tree passes the full walk
    assert info["ps_waves"] == 6 and info["bvh_stack"] <= 25
    for kind, stack in (("bunny", 25), ("sponza", 31)):
        info, _, _ = w.bvh_build(w.procedural_mesh(kind))
        assert info["ps_waves"] == 6 and info["bvh_stack"] <= stack
    monkeypatch.setenv("WGT_PS_WAVES", "5")
    monkeypatch.delenv("WGT_NARROW")
    info, _, _ = w.bvh_build(w.procedural_mesh("bunny"))
    assert info["ps_waves"] == 5 and info["bvh_stack"] == 31


def stack24_roundtrip(v):
    """Stack24 (wgt_device.h): a ref stored as its low 16 bits and its bits 16..23 as a signed byte,
    read back as (int8 << 16) | uint16."""
    v = np.asarray(v, np.int64)
    lo = (v & 0xFFFF).astype(np.uint16)
    hi = ((v >> 16) & 0xFF).astype(np.uint8).view(np.int8)
    return (hi.astype(np.int64) << 16) | lo.astype(np.int64)


@pytest.mark.parametrize("kind", ["bunny", "sponza"])
def test_stack24_holds_every_ref(kind):
    """Every ref the 6-wave kernel can push survives the 3-byte stack entry: internal refs as the
    device's byte offsets into either node form (x 128 for 128-B nodes, x 80 for compact records)
    and leaf refs as they are (wgt_runtime.cpp converts the device copies)."""
    tris = w.procedural_mesh(kind)
    info, nodes, _ = w.bvh_build(tris)
    assert info["ps_waves"] == 6
    refs = nodes.reshape(-1, 8, 4)[:, 6, :].view(np.int32).ravel().astype(np.int64)
    for stride in (128, 80):
        dev = np.where(refs >= 0, refs * stride, refs)
        assert np.array_equal(stack24_roundtrip(dev), dev)
    edge = np.array([0, 1, (1 << 23) - 1, -1, -(1 << 23), 65535, 65536, -65536, -65537])
    assert np.array_equal(stack24_roundtrip(edge), edge)


def test_stack24_fit_rule():
    """6 waves per SIMD need every ref in a 3-byte stack entry: a tree of 2^20 triangles (leaf refs
    below -2^23) and > 2^16 nodes (128-B node offsets >= 2^23) falls back to 5 waves and 4-byte
    entries (wgt_runtime.cpp ps_waves_for, wgt_internal.h kStack24Nodes / kStack24Tris)."""
    info, _, _ = w.bvh_build(random_soup(1 << 20, 7))
    assert info["n_tris"] == 1 << 20 and info["bvh_nodes"] >= 1 << 16
    assert info["ps_waves"] == 5


def bvh4_sah(nodes):
    """SAH cost of an exported BVH4 (root-relative): the root plus every internal child's box
    area (node visits), and count x area of every leaf child (triangle tests)."""
    N = nodes.reshape(-1, 8, 4).astype(np.float64)
    refs = nodes.reshape(-1, 8, 4)[:, 6, :].view(np.int32)
    lx, hx, ly, hy, lz, hz = (N[:, i, :] for i in range(6))
    live = ~((lx == np.float64(EMPTY)) & (hx == np.float64(EMPTY)))
    dx, dy, dz = np.maximum(hx - lx, 0), np.maximum(hy - ly, 0), np.maximum(hz - lz, 0)
    area = 2 * (dx * dy + dy * dz + dz * dx) * live
    r = live[0]
    ext = [hx[0][r].max() - lx[0][r].min(), hy[0][r].max() - ly[0][r].min(), hz[0][r].max() - lz[0][r].min()]
    ra = 2 * (ext[0] * ext[1] + ext[1] * ext[2] + ext[2] * ext[0])
    inner, leaf = (refs >= 0) & live, (refs < 0) & live
    cnt = ((~refs) & 7) + 1
    return 1.0 + area[inner].sum() / ra, (area[leaf] * cnt[leaf]).sum() / ra


@pytest.mark.parametrize("leaf", ["0", "8"])
def test_optimal_collapse_vs_greedy(monkeypatch, leaf):
    """The SAH-optimal collapse (default, WGT_COLLAPSE=dp) exports a tree that passes the full
    walk (containment, leaf partition, exact stack need), and at the same stack bound its
    node-visit SAH is never above the greedy collapse's (WGT_COLLAPSE=greedy); with leaf
    merging off (WGT_DP_LEAF=0) the leaves are the same, so the triangle SAH is equal."""
    monkeypatch.setenv("WGT_PS_WAVES", "5")  # both at the 31-entry bound
    monkeypatch.setenv("WGT_DP_LEAF", leaf)
    for tris in (random_soup(3000, 5), w.procedural_mesh("bunny", 20000)):
        monkeypatch.setenv("WGT_COLLAPSE", "greedy")
        g_info, g_nodes, _ = w.bvh_build(tris)
        monkeypatch.setenv("WGT_COLLAPSE", "dp")
        d_info = check_tree(tris)
        _, d_nodes, _ = w.bvh_build(tris)
        gn, gt = bvh4_sah(g_nodes)
        dn, dt = bvh4_sah(d_nodes)
        if leaf == "0":
            assert dn <= gn * (1 + 1e-6), (dn, gn)
            assert abs(dt - gt) <= 1e-6 * gt
        else:
            assert dn + dt <= (gn + gt) * (1 + 1e-6), (dn + dt, gn + gt)
        assert d_info["bvh_stack"] <= STACK_MAX
