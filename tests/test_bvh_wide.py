"""The wide BVH form (wgt_geom.h kW8*), CPU only, through the host
export wgt_bvh_build_wide.

The persistent kernel's wide traversal (wgt_device.h node_step_w8 / tri_step_w8 / w8_resolve)
returns the brute-force closest triangle of the geometry spec only if:
  * every triangle sits in exactly one leaf slot's record positions 4(8g + s) + i, the unused
    positions of a group hold degenerate triangles (e1 = e2 = 0: every ray rejects them), and
    each record equals the spec's (v0, e1, e2, index bits, padded box);
  * the record of group g's slot s is 8g + s; internal slots come first (W[5] = ni); W[4]'s
    nibble s holds leaf slot s's triangles as contiguous low bits, internal nibbles are 0;
  * every live slot's decoded box keeps the fused step's margin G around its subtree's
    triangle boxes (the same codes and margin as the compact BVH4 records, §3.4);
  * the LDS stack (2 entries per level) covers every root-to-node path.
The second half restates the traversal's control flow in Python (groups on the stack, the
nearest internal child first, one open triangle group, a second one pushed) with exact per-
triangle results and float64 slab tests, under random schedules of node and triangle steps,
and checks the closest hit against brute force and the stack depth against the bound.
"""
import numpy as np
import pytest

import webgputracer_amd as w

from test_bvh import random_soup, tri_box_np

f32 = np.float32
K_RAY_MIN, K_RAY_MAX = 0.001, 1e20
# word offsets of a wide record (wgt_geom.h kW8*): header, meta, the lo / hi code rows per axis
HEAD, META = 0, 28
LO_ROW, HI_ROW = (8, 16, 4), (12, 24, 20)


def decode(recs, step):
    """-> org (n, 3) f64, lo/hi (n, 8, 3) f64 planes (inf for +inf codes), live (n, 8)."""
    orgs = recs[:, HEAD:HEAD + 3].view(np.float32).astype(np.float64) * np.float64(step)
    lo = np.zeros((len(recs), 8, 3))
    hi = np.zeros((len(recs), 8, 3))
    codes_lo = np.zeros((len(recs), 8, 3), np.uint32)
    for a in range(3):
        for kind, base in (("lo", LO_ROW[a]), ("hi", HI_ROW[a])):
            words = recs[:, base:base + 4]
            h = np.stack([words & 0xFFFF, words >> 16], 2).reshape(len(recs), 8)
            with np.errstate(invalid="ignore", over="ignore"):
                v = h.astype(np.uint16).view(np.float16).astype(np.float64) * np.float64(step) + orgs[:, a:a + 1]
            if kind == "lo":
                lo[:, :, a] = v
                codes_lo[:, :, a] = h
            else:
                hi[:, :, a] = v
    live = (codes_lo != 0x7C00).all(2)
    return orgs, lo, hi, live


def check_wide(tris):
    info, recs, trec = w.bvh_build_wide(tris)
    n = len(tris)
    step = f32(info["w8_step"])
    assert step > 0 and np.log2(step) == np.round(np.log2(step))
    assert info["w8_stack"] == 2 * info["w8_depth"] and info["w8_depth"] <= 16
    _, lo, hi, live = decode(recs, step)
    g = recs[:, HEAD + 3]
    L = recs[:, META]
    ni = recs[:, META + 1]
    imask = recs[:, META + 2]
    assert (recs[:, META + 3] == 0).all()
    for a in range(3):  # an axis's lo and hi rows differ in address bit 4 + a
        assert (HI_ROW[a] - LO_ROW[a]) * 4 == 16 << a
    nrec = len(recs)
    assert live[0].any(), "record 0 is the root"
    # the triangle records: v0, e1, e2, index bits, padded box = the spec; the rest degenerate
    idx = trec[:, 0, 3].view(np.uint32)
    v0, e1, e2 = trec[:, 0, :3], trec[:, 1, :3], trec[:, 2, :3]
    seen = np.zeros(n, np.int32)
    M = max(4.0 * np.abs(np.concatenate([tris["v0"][:, :3], tris["v0"][:, :3] + tris["e1"][:, :3],
                                         tris["v0"][:, :3] + tris["e2"][:, :3]])).max(), 2.0 ** -60)
    M = max(M, float(info["w8_bound"]))
    G = np.ldexp(float(info["w8_bound"]), -21)

    groups = set()
    depth_max = 0

    def visit(k, depth):
        """-> (lo, hi) of the triangle boxes under record k (float64)."""
        nonlocal depth_max
        depth_max = max(depth_max, depth)
        gi = int(g[k])
        assert gi >= 1 and gi not in groups
        groups.add(gi)
        nl = int(live[k].sum())
        # live slots first, internal ones first of them
        assert live[k, :nl].all() and not live[k, nl:].any(), "live slots first"
        assert 0 <= ni[k] <= nl and imask[k] == (1 << int(ni[k])) - 1
        assert (int(imask[k]) & ~sum(1 << s for s in range(8) if live[k, s])) == 0
        sub_lo, sub_hi = np.full(3, np.inf), np.full(3, -np.inf)
        for s in range(8):
            if not live[k, s]:
                assert (int(L[k]) >> (4 * s)) & 0xF == 0
                continue
            nib = (int(L[k]) >> (4 * s)) & 0xF
            child = gi * 8 + s
            if (int(imask[k]) >> s) & 1:
                assert nib == 0
                clo, chi = visit(child, depth + 1)
            else:
                assert nib in (1, 3, 7, 15), "a leaf's triangles are its low record positions"
                cnt = bin(nib).count("1")
                pos = np.arange(4 * child, 4 * child + cnt)
                seen[idx[pos]] += 1
                blo, bhi = tri_box_np(v0[pos], e1[pos], e2[pos])
                np.testing.assert_array_equal(np.stack([trec[pos, 1, 3], trec[pos, 2, 3], trec[pos, 3, 0]], 1), blo)
                np.testing.assert_array_equal(trec[pos, 3, 1:4], bhi)
                np.testing.assert_array_equal(v0[pos], tris["v0"][idx[pos]][:, :3])
                np.testing.assert_array_equal(e1[pos], tris["e1"][idx[pos]][:, :3])
                np.testing.assert_array_equal(e2[pos], tris["e2"][idx[pos]][:, :3])
                rest = np.arange(4 * child + cnt, 4 * child + 4)
                assert (trec[rest, 1, :3] == 0).all() and (trec[rest, 2, :3] == 0).all()
                clo, chi = blo.astype(np.float64).min(0), bhi.astype(np.float64).max(0)
            # the decoded slot keeps the margin G around every triangle box below it
            assert (lo[k, s] <= clo - G).all() and (hi[k, s] >= chi + G).all(), (k, s)
            sub_lo, sub_hi = np.minimum(sub_lo, clo), np.maximum(sub_hi, chi)
        return sub_lo, sub_hi

    import sys
    old = sys.getrecursionlimit()
    sys.setrecursionlimit(max(old, 10000))
    try:
        visit(0, 1)
    finally:
        sys.setrecursionlimit(old)
    assert (seen == 1).all(), "every triangle in exactly one leaf slot"
    assert depth_max == info["w8_depth"]
    assert len(groups) == info["w8_groups"] and max(groups) == info["w8_groups"]
    assert nrec == 8 * (info["w8_groups"] + 1)
    return info, recs, trec


@pytest.mark.parametrize("n,seed", [(1, 0), (2, 1), (5, 2), (9, 3), (1000, 4), (5000, 5)])
def test_wide_random_soup(n, seed):
    check_wide(random_soup(n, seed))


def test_wide_coincident_centroids():
    v = np.tile(np.array([[[0, 0, 0], [10, 0, 0], [0, 10, 0]]], f32), (300, 1, 1))
    check_wide(w.make_triangles(v))


def test_wide_procedural_bunny():
    info, _, _ = check_wide(w.procedural_mesh("bunny", 20000))
    assert info["w8_groups"] < (1 << 15)  # Stack24 group indices (6 waves per SIMD)


def test_wide_full_size_meshes():
    for kind in ("bunny", "sponza"):
        _, _, _, T = w.mesh_scene(kind)
        info, _, _ = w.bvh_build_wide(T)
        assert info["w8_depth"] <= 16 and info["w8_stack"] == 2 * info["w8_depth"]
        assert info["w8_groups"] < (1 << 15), "the 6-wave kernel's 3-byte stack entries hold the group"
        avg = (info["w8_nodes"] - 1 + info["w8_leaves"]) / info["w8_nodes"]
        assert avg > 4.0, f"{kind}: {avg:.2f} slots per node"


@pytest.mark.parametrize("w8,cnode,built", [(None, None, 0), (None, "4", 1), (None, "2", 0), ("1", None, 1),
                                             ("0", "4", 0)])
def test_wide_built_on_request(monkeypatch, w8, cnode, built):
    """The wide form is opt-in at the build (host/bvh.cpp WideWanted): with WGT_CNODE=4 or WGT_W8=1,
    never with WGT_W8=0; the explicit export (wgt_bvh_build_wide) builds it whatever the environment."""
    for k, v in (("WGT_W8", w8), ("WGT_CNODE", cnode)):
        if v is None:
            monkeypatch.delenv(k, raising=False)
        else:
            monkeypatch.setenv(k, v)
    tris = random_soup(100, 1)
    info, _, _ = w.bvh_build(tris)
    assert info["bvh_w8"] == built
    winfo, recs, _ = w.bvh_build_wide(tris)
    assert winfo["bvh_w8"] == 1 and len(recs) == winfo["w8_records"]


# ---------------------------------------------------------------------------------------------
# The traversal's control flow, restated (wgt_device.h node_step_w8, tri_step_w8, w8_resolve)

def spread4(m):
    return sum(0xF << (4 * k) for k in range(8) if (m >> k) & 1)


def tri_hits(o, d, v0, e1, e2, blo, bhi):
    """The spec per triangle (Moller-Trumbore + the padded-box slab check) in float64: t or inf."""
    pvec = np.cross(d, e2)
    det = (e1 * pvec).sum(1)
    ok = np.abs(det) >= 1e-12
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / det
        tvec = o - v0
        u = (tvec * pvec).sum(1) * inv
        qvec = np.cross(tvec, e1)
        v = (d * qvec).sum(1) * inv
        t = (e2 * qvec).sum(1) * inv
        ok &= (u >= 0) & (u <= 1) & (v >= 0) & (u + v <= 1) & (t >= K_RAY_MIN) & (t <= K_RAY_MAX)
        sinv = 1.0 / np.where(np.abs(d) < 1e-30, np.copysign(1e-30, d), d)
        t0, t1 = (blo - o) * sinv, (bhi - o) * sinv
        bn, bf = np.minimum(t0, t1).max(1), np.maximum(t0, t1).min(1)
    ok &= (bn <= t) & (t <= bf)
    return np.where(ok, t, np.inf)


def trace_wide(o, d, info, recs, trec, lo, hi, stack_max, rng):
    """-> (t, index) of the closest triangle, by the wide traversal under a random schedule."""
    inv = 1.0 / np.where(np.abs(d) < 1e-30, np.copysign(1e-30, d), d)
    # a popped triangle group's records: its slots' nibbles of the owning record's L (w8leaf)
    live_rec = recs[:, HEAD + 3] != 0
    leaf_of = dict(zip(recs[live_rec, HEAD + 3].tolist(), recs[live_rec, META].tolist()))
    tri_t = {}

    def tt(pos):
        if pos not in tri_t:
            r = trec[pos]
            blo = np.array([r[1, 3], r[2, 3], r[3, 0]], np.float64)
            tri_t[pos] = tri_hits(o, d, r[0, :3][None].astype(np.float64), r[1, :3][None].astype(np.float64),
                                  r[2, :3][None].astype(np.float64), blo[None], r[3, 1:4][None].astype(np.float64))[0]
        return tri_t[pos]

    bt, bi = K_RAY_MAX, 0xFFFFFFFF
    stack = []
    ref, T = 0, None  # record index; (group, mask of record positions)

    def resolve():
        nonlocal ref, T
        for _ in range(2):
            if not stack:
                break
            kind, g, m = stack[-1]
            if kind == "node":
                j = (m & -m).bit_length() - 1
                m2 = m & (m - 1)
                if m2 == 0:
                    stack.pop()
                else:
                    stack[-1] = ("node", g, m2)
                ref = 8 * g + j
                return
            if T is not None:
                break
            stack.pop()
            T = (g, spread4(m) & leaf_of[g])
        ref = None

    while True:
        can_node, can_tri = ref is not None, T is not None
        if not can_node and not can_tri:
            assert not stack
            return bt, bi
        if can_node and (not can_tri or rng.random() < 0.5):
            k = ref
            t0 = (lo[k] - o) * inv
            t1 = (hi[k] - o) * inv
            with np.errstate(invalid="ignore"):
                nn = np.maximum(np.where(inv < 0, t1, t0).max(1), K_RAY_MIN)
                ff = np.minimum(np.where(inv < 0, t0, t1).min(1), bt)
            hit = nn <= ff  # inf planes (empty slots) never hit
            im, g, L = int(recs[k, META + 2]), int(recs[k, HEAD + 3]), int(recs[k, META])
            hits = sum(1 << s for s in range(8) if hit[s])
            internal = [s for s in range(8) if hit[s] and (im >> s) & 1]
            near = min(internal, key=lambda s: nn[s]) if internal else None
            sib = hits & im & ~((1 << near) if near is not None else 0)
            lh = hits & ~im
            if sib:
                stack.append(("node", g, sib))
            if lh:
                if T is None:
                    T = (g, spread4(lh) & L)
                else:
                    stack.append(("tri", g, lh))
            assert len(stack) <= stack_max
            if near is not None:
                ref = 8 * g + near
            else:
                resolve()
            if T is not None and T[1] == 0:
                T = None
        else:
            g, m = T
            for _ in range(2):
                if m == 0:
                    break
                i = (m & -m).bit_length() - 1
                m &= m - 1
                pos = 32 * g + i
                t = tt(pos)
                idx = int(trec[pos, 0, 3].view(np.uint32))
                if t < bt or (t == bt and idx < bi):
                    bt, bi = t, idx
            T = (g, m) if m else None
            if T is None and ref is None:
                resolve()


@pytest.mark.parametrize("n,seed", [(40, 7), (3000, 8)])
def test_wide_traversal_matches_brute_force(n, seed):
    tris = random_soup(n, seed, spread=200.0, size=15.0)
    info, recs, trec = check_wide(tris)
    _, lo, hi, live = decode(recs, f32(info["w8_step"]))
    lo = np.where(live[:, :, None], lo, np.inf)
    hi = np.where(live[:, :, None], hi, np.inf)
    rng = np.random.default_rng(seed)
    v0 = tris["v0"][:, :3].astype(np.float64)
    e1 = tris["e1"][:, :3].astype(np.float64)
    e2 = tris["e2"][:, :3].astype(np.float64)
    blo, bhi = tri_box_np(tris["v0"][:, :3], tris["e1"][:, :3], tris["e2"][:, :3])
    for r in range(150):
        if r % 3 == 0:  # from outside toward the scene
            o = rng.uniform(-300, 500, 3)
            d = rng.uniform(0, 200, 3) - o
        else:
            o = rng.uniform(0, 200, 3)
            d = rng.normal(0, 1, 3)
        if r % 25 == 0:
            d[rng.integers(3)] = 0.0  # axis-parallel
        t_all = tri_hits(o[None], d[None], v0, e1, e2, blo.astype(np.float64), bhi.astype(np.float64))
        want_t = t_all.min()
        want_i = int(np.argmin(t_all)) if np.isfinite(want_t) else 0xFFFFFFFF
        got_t, got_i = trace_wide(o, d, info, recs, trec, lo, hi, info["w8_stack"], rng)
        if np.isfinite(want_t):
            assert (got_t, got_i) == (want_t, want_i), r
        else:
            assert got_i == 0xFFFFFFFF, r
