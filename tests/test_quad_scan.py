"""The persistent kernel's quad scan without per-quad distances (wgt_device.h quad_scan_fast,
DESIGN.md §3.2 "quad distance"), restated in numpy float32 and checked on the CPU against the
oracle's reference scan (path_tracer.wgsl:314-338 over every quad, oracle/wgt_oracle.c) on rays
built to make distance ties: a second back wall one ulp in front of the first (its rays hit both
planes at t one ulp apart, so their rounded distances often tie and the reference keeps the
earlier quad) and rays aimed at the lines where two walls meet.

The restatement follows the kernel's operations (the same fp32 roundings; div_rn is the IEEE
quotient where it is used, tests/test_gpu_numerics.py) and its fallback test; without the
fallback it disagrees with the oracle on these rays, so the test can tell.
TEST INFRASTRUCTURE ONLY (the oracle is the checker)."""
import numpy as np
import pytest

from numpy_restatement import cross, dot, f32, kRayMax, kRayMin

NO_HIT = np.uint32(0xFFFFFFFF)


def v3(a):
    return (a[:, 0].astype(f32), a[:, 1].astype(f32), a[:, 2].astype(f32))


def quad_scan_fast(o, d, quads):
    """(prim, t, exact) per ray: the smallest-t valid quad (first on equal t), and whether the
    kernel's tie test lets it stand (else the kernel runs the reference scan)."""
    n = len(o[0])
    prim = np.full(n, NO_HIT, np.uint32)
    qt = np.full(n, np.inf, f32)
    prev = np.full(n, np.inf, f32)
    with np.errstate(all="ignore"):
        for k, q in enumerate(quads):
            qn = tuple(f32(x) for x in q["norm"][:3])
            denom = dot(qn, d)
            num = f32(q["d"]) - dot(qn, o)
            t = (num / denom).astype(f32)
            ok = ~(np.abs(denom) < kRayMin) & ~((t < kRayMin) | (kRayMax < t)) & ~(t >= qt)
            pos = (o[0] + t * d[0], o[1] + t * d[1], o[2] + t * d[2])
            hv = (pos[0] - f32(q["pos"][0]), pos[1] - f32(q["pos"][1]), pos[2] - f32(q["pos"][2]))
            w = tuple(f32(x) for x in q["w"])
            a = dot(w, cross(hv, tuple(f32(x) for x in q["up"][:3])))
            b = dot(w, cross(tuple(f32(x) for x in q["right"][:3]), hv))
            # (a < 0) || (1 < a) || (b < 0) || (1 < b) with NaN false (fminf / fmaxf of the kernel)
            out = (np.fmin(a, b) < 0) | (1 < np.fmax(a, b))
            ok &= ~out
            prev = np.where(ok, qt, prev)
            qt = np.where(ok, t, qt)
            prim = np.where(ok, np.uint32(k), prim)
        D = np.maximum(np.maximum(np.abs(d[0]), np.abs(d[1])), np.abs(d[2]))
        L = np.maximum(np.maximum(np.abs(o[0]), np.abs(o[1])), np.abs(o[2]))
        exact = (qt * D < f32(2.0 ** 64))
        g = (prev - qt) - f32(2.0 ** -19) * (prev + qt)
        tie_free = (g * D > f32(2.0 ** -18) * L) & (prev * D >= f32(2.0 ** -49))
        exact &= np.where(prev != np.inf, tie_free, True)
        exact = np.where(prim != NO_HIT, exact, True)
    return prim, qt, exact


def far_sphere(S):
    S = S.copy()
    S["center"][:] = (1e6, 1e6, 1e6)
    S["radius"][:] = 1.0
    return S


def double_back_wall(Q):
    """The Cornell walls plus a copy of the back wall (z = 555) one ulp nearer the camera, later
    in scan order."""
    walls = Q[:5].copy()
    k = int(np.argmax(walls["pos"][:, 2] * (np.abs(walls["norm"][:, 2]) == 1)))
    extra = walls[k:k + 1].copy()
    z = np.nextafter(f32(extra["pos"][0, 2]), f32(0))
    extra["pos"][0, 2] = z
    n = extra["norm"][0, :3].astype(f32)
    p = extra["pos"][0, :3].astype(f32)
    extra["d"][0] = (n[0] * p[0] + n[1] * p[1]) + n[2] * p[2]
    return np.concatenate([walls, extra])


def edge_rays(quads, n, rng):
    """Rays from points inside the box (and the reference camera) at points on the quads' edges,
    some exactly and some nudged by a few ulps."""
    ends = []
    for q in quads:
        p, r, u = (q[f][:3].astype(np.float64) for f in ("pos", "right", "up"))
        for a, b in ((p, p + r), (p, p + u), (p + r, p + r + u), (p + u, p + r + u)):
            ends.append((a, b))
    ends = np.array(ends)
    e = ends[rng.integers(0, len(ends), n)]
    s = rng.uniform(0, 1, (n, 1))
    target = (e[:, 0] + s * (e[:, 1] - e[:, 0])).astype(f32)
    o = rng.uniform(5, 550, (n, 3)).astype(f32)
    o[: n // 8] = (278, 278, -800)
    d = (target - o).astype(f32)
    nudge = rng.integers(-3, 4, (n, 3)).astype(np.int32)
    nudge[: n // 3] = 0
    d = (d.view(np.int32) + nudge).view(f32)
    return o, d


@pytest.fixture(scope="module")
def scenes(oracle):
    L, Q, S = oracle.cornell_scene()
    return L, Q, far_sphere(S)


@pytest.mark.parametrize("kind", ["double_wall", "edges"])
def test_fast_quad_scan_equals_reference_on_ties(oracle, scenes, kind):
    L, Q, S = scenes
    rng = np.random.default_rng(5 if kind == "edges" else 6)
    if kind == "double_wall":
        quads = double_back_wall(Q)
        n = 60_000
        tgt = np.stack([rng.uniform(0, 555, n), rng.uniform(0, 555, n), np.full(n, 555.0)], 1).astype(f32)
        o = rng.uniform(5, 550, (n, 3)).astype(f32)
        o[: n // 4] = (278, 278, -800)
        d = (tgt - o).astype(f32)
    else:
        quads = Q[:5].copy()
        o, d = edge_rays(np.concatenate([L, quads]), 60_000, rng)
    osc = oracle.OracleScene(L, quads, S)
    rp, rd = osc.trace(o, d)
    osc.close()
    allq = np.concatenate([L, quads])
    prim, qt, exact = quad_scan_fast(v3(o), v3(d), allq)
    quad_hit = rp < len(allq)
    assert np.all(rp[~quad_hit] == NO_HIT)  # the far sphere is never hit
    # where the tie test passes, the smallest-t quad is the reference's
    assert np.array_equal(prim[exact], rp[exact])
    # the test must bite: some rays need the fallback, and on some of them the smallest-t quad is
    # not the reference's answer (an earlier quad ties in rounded distance)
    assert (~exact).sum() > 50
    if kind == "double_wall":
        assert np.count_nonzero(prim[~exact] != rp[~exact]) > 10
        assert np.count_nonzero(rp == len(allq) - 1) > 1000  # the nearer copy does win where no tie


def test_fast_quad_scan_fallback_is_rare(oracle, scenes):
    """On the reference walls and rays not built to tie, the tie test almost never sends a ray to
    the reference scan, and the smallest-t quad is the reference's answer wherever it passes."""
    L, Q, S = scenes
    rng = np.random.default_rng(9)
    o = rng.uniform(5, 550, (100_000, 3)).astype(f32)
    d = rng.normal(size=(100_000, 3)).astype(f32)
    quads = Q[:5].copy()
    allq = np.concatenate([L, quads])
    prim, _, exact = quad_scan_fast(v3(o), v3(d), allq)
    assert exact.mean() > 0.999
    osc = oracle.OracleScene(L, quads, S)
    rp, _ = osc.trace(o, d)
    osc.close()
    assert np.array_equal(prim[exact], rp[exact])
