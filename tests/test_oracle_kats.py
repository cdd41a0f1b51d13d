"""Known-answer tests pinning the CPU oracle (oracle/wgt_oracle.c).

The reference has no tests or golden vectors: parity with it is
UNPINNED.  These KATs pin the oracle with values derived independently of it —
closed-form geometry, an integer restatement of the PCG hash, float64 math, and
SURVEY Appendix B (computed by a separate throwaway restatement).
"""
import math

import numpy as np
import pytest

K_RAY_MAX = np.float32(1e20)


def py_rand_seq(seed, n):
    """Integer restatement of rand() (path_tracer.wgsl:90-95) with Python ints."""
    scale = np.frombuffer(np.uint32(0x2F800004).tobytes(), np.float32)[0]
    out = []
    for _ in range(n):
        seed = (seed * 747796405 + 2891336453) & 0xFFFFFFFF
        word = (((seed >> ((seed >> 28) + 4)) ^ seed) * 277803737) & 0xFFFFFFFF
        out.append(np.float32(np.float32((word >> 22) ^ word) * scale))
    return np.array(out, np.float32), seed


def test_rand_kat_survey_appendix_b(oracle):
    r, _ = oracle.rand_seq(0, 6)
    expect = [0.030200012028217316, 0.13560055196285248, 0.23423591256141663, 0.3405679762363434,
              0.5272876024246216, 0.20467491447925568]
    assert np.array_equal(r, np.array(expect, np.float32))


@pytest.mark.parametrize("seed", [0, 1, 12345, 0xFFFFFFFF, 2891336453])
def test_rand_matches_integer_restatement(oracle, seed):
    r, fin = oracle.rand_seq(seed, 1000)
    p, pfin = py_rand_seq(seed, 1000)
    assert np.array_equal(r.view(np.uint32), p.view(np.uint32)) and fin == pfin


def test_rand_can_reach_one():
    """bitcast 0x2f800004 is slightly above 2^-32: rand() >= 1 iff word >= 0xFFFFF780 (App. B)."""
    scale = np.frombuffer(np.uint32(0x2F800004).tobytes(), np.float32)[0]
    words = np.array([0xFFFFF77F, 0xFFFFF780, 0xFFFFFFFF], np.uint32)
    vals = words.astype(np.float32) * scale
    assert vals[0] < 1.0 <= vals[1] and vals[2] == np.float32(1.0000004768371582)


@pytest.mark.parametrize("fn,ref", [("o_sin", math.sin), ("o_cos", math.cos)])
def test_sin_cos_accuracy(oracle, fn, ref):
    f = getattr(oracle.lib(), fn)
    xs = np.linspace(0.0, 2 * math.pi * 1.0000005, 20001, dtype=np.float32)
    got = np.array([f(float(x)) for x in xs], np.float32)
    exact = np.array([ref(float(x)) for x in xs])
    ulp = np.spacing(np.abs(exact).astype(np.float32) + np.float32(1e-30))
    err = np.abs(got.astype(np.float64) - exact)
    assert np.all(err <= 4 * ulp + 2e-8)


def test_tan_and_radians(oracle):
    L = oracle.lib()
    theta = L.o_radians(40.0)
    assert abs(theta - math.radians(40.0)) < 1e-7
    h = L.o_tan(theta * 0.5)
    assert abs(h - math.tan(math.radians(20.0))) < 1e-6


def cornell(oracle):
    L, Q, S = oracle.cornell_scene()
    return L, Q, S, oracle.OracleScene(L, Q, S)


def test_cornell_scene_structure(oracle):
    L, Q, S, _ = cornell(oracle)
    assert len(L) == 1 and len(Q) == 17 and len(S) == 1
    # light: norm = normalize(cross((130,0,0),(0,0,105))) = (0,-1,0), d = -554, w = n/|n|^2
    assert np.array_equal(L[0]["norm"], np.float32([0, -1, 0, 1]))
    assert L[0]["d"] == np.float32(-554.0)
    assert L[0]["w"][1] == np.float32(-13650.0) / np.float32(13650.0 * 13650.0)
    assert L[0]["emissive"] == 1.0 and np.all(L[0]["col"] == np.float32(15))
    # walls (cornell_box.cpp:6-10): green x=555 facing -x, red x=0 facing +x, ...
    assert np.array_equal(Q[0]["norm"][:3], np.float32([-1, 0, 0])) and Q[0]["d"] == -555
    assert np.allclose(Q[1]["norm"][:3], [1, 0, 0]) and Q[1]["d"] == 0
    assert np.array_equal(Q[4]["norm"][:3], np.float32([0, 0, -1])) and Q[4]["d"] == -555
    assert np.array_equal(Q[0]["col"], np.float32([.12, .45, .15]))
    # box1 front face rotated by 15 degrees about y (box.cpp:14, quad.cpp:15-25)
    n = Q[5]["norm"][:3]
    assert abs(n[0] - math.sin(math.radians(15))) < 1e-6 and abs(n[2] - math.cos(math.radians(15))) < 1e-6
    # box2 translated by (130,0,65): its 4th face starts at the translated origin
    assert np.array_equal(Q[14]["pos"][:3], np.float32([130, 0, 65]))
    assert S[0]["radius"] == 0 and S[0]["emissive"] == 0


def test_analytic_intersections(oracle):
    L, Q, S, sc = cornell(oracle)
    o = np.float32([[100, 500, -800], [278, 400, 278], [278, 278, -800], [np.nan, 0, 0]])
    d = np.float32([[0, 0, 1], [0, 1, 0], [0, 0, -1], [0, 0, 1]])
    pid, dist = sc.trace(o, d)
    assert pid[0] == 1 + 4 and dist[0] == np.float32(1355.0)   # back wall (z = 555)
    assert pid[1] == 0 and dist[1] == np.float32(154.0)        # the light (y = 554)
    assert pid[2] == oracle.NO_HIT and dist[2] == K_RAY_MAX    # behind the camera: miss
    assert pid[3] == 1 + 17 + 0 and np.isnan(dist[3])          # NaN ray: last primitive (dummy sphere) wins


def test_sphere_and_triangle_intersections(oracle):
    L, Q, S, _ = cornell(oracle)
    S2 = np.concatenate([S, S])
    S2[1]["center"] = (400, 400, 278)
    S2[1]["radius"] = 50
    tri = oracle.make_triangles(np.float32([[0, 0, 100]]), np.float32([[600, 0, 100]]),
                                np.float32([[0, 600, 100]]), np.float32([0.5, 0.5, 0.5]))
    sc = oracle.OracleScene(L, Q[:5], S2, tri)
    o = np.float32([[400, 400, -800], [50, 50, -800]])  # x + y > 600 misses the triangle
    d = np.float32([[0, 0, 1], [0, 0, 1]])
    pid, dist = sc.trace(o, d)
    assert pid[0] == 1 + 5 + 1 + 1 and dist[0] == np.float32(1028.0)  # sphere: 1078 - 50
    assert pid[1] == 1 + 5 + 0 and dist[1] == np.float32(900.0)       # triangle plane z = 100
    tid, t = sc.trace_tris(o, d, brute=True)
    assert tid[1] == 0 and t[1] == np.float32(900.0) and tid[0] == oracle.NO_HIT


def test_triangle_ctor(oracle):
    t = oracle.make_triangles(np.float32([[1, 2, 3]]), np.float32([[4, 2, 3]]), np.float32([[1, 6, 3]]),
                              np.float32([1, 0, 0]), emissive=True)[0]
    assert np.array_equal(t["e1"], np.float32([3, 0, 0, 1])) and np.array_equal(t["e2"], np.float32([0, 4, 0, 1]))
    assert np.array_equal(t["fn"], np.float32([0, 0, 1, 1])) and t["emissive"] == 1.0


def test_sqrt_spp_table(oracle):
    """u32(sqrt(f32(spp))) (path_tracer.wgsl:380): 1->1, 64->8, 256->16, 1000->31 (App. B)."""
    for spp, n in [(1, 1), (64, 8), (256, 16), (1000, 31)]:
        assert int(np.sqrt(np.float32(spp))) == n


def test_cornell_statistics_regression(oracle):
    """SURVEY App. B sizing (fp64 throwaway restatement, 96^2, 1 spp): ~9.5 queries/path,
    primary miss ~9 %, NaN-absorbed queries ~68 %.  The fp32 oracle must be close."""
    L, Q, S, sc = cornell(oracle)
    r = sc.render(oracle.camera_param(1.0, 1, 0), 96, 96)
    c = r["counters"]
    q_per_path = c[oracle.CNT_QUERIES] / c[oracle.CNT_SAMPLES]
    assert 9.0 < q_per_path < 10.0
    assert 0.07 < np.mean(r["hit"] == oracle.NO_HIT) < 0.11
    assert 0.62 < c[oracle.CNT_NAN_RAYS] / c[oracle.CNT_QUERIES] < 0.72
    assert c[oracle.CNT_QUERIES] == c[oracle.CNT_TRACED] + c[oracle.CNT_NAN_RAYS]


def test_oracle_bvh_equals_bruteforce(oracle, wgt):
    """The oracle's own BVH returns exactly the linear-scan triangle spec."""
    tris = wgt.procedural_mesh("bunny", 3000)
    L, Q, S = oracle.cornell_scene()
    sc = oracle.OracleScene(L, Q[:5], S, tris)
    rng = np.random.default_rng(3)
    o = rng.uniform(5, 550, (4000, 3)).astype(np.float32)
    idx = rng.integers(0, len(tris), 4000)
    c = tris["v0"][idx, :3] + (tris["e1"][idx, :3] + tris["e2"][idx, :3]) / np.float32(3)
    d = (c - o).astype(np.float32)
    a = sc.trace_tris(o, d, brute=False)
    b = sc.trace_tris(o, d, brute=True)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))
    assert np.mean(a[0] != oracle.NO_HIT) > 0.5


# Two triangles whose hits round to the same ray_dist at different t (found by a
# search with the oracle): A = tri index 0 at z = 0.5000009 (t = 5.351351), B = tri
# index 1 at z = 0.500001 (t = 5.3513503), ray from (0.3, 0.3, 20.3) along -3.7 z.
TIE_O = np.array([[0.3, 0.3, 20.3]], np.float32)
TIE_D = np.array([[0.0, 0.0, -3.7]], np.float32)


def tie_triangles(wgt):
    z = [np.float32(0.5000009), np.float32(0.500001)]
    return np.concatenate([wgt.make_triangles(np.array([[[-1, -1, zz], [3, -1, zz], [-1, 3, zz]]], np.float32))
                           for zz in z])


def test_triangle_tie_rule_is_min_t_then_index(oracle, wgt):
    """The closest triangle is the minimum of (t, index), a
    deliberate departure from the reference's sequential scan rule for quads and
    spheres (`ray_dist >= closest.dist` rejects, path_tracer.wgsl:320-325), which
    would keep the FIRST of two hits with equal rounded ray_dist.  Here the two
    hits have the same ray_dist but B (index 1) has the smaller t, so B wins; a
    future change to the rule fails this test."""
    L, Q, S = wgt.cornell_scene()
    A, B = tie_triangles(wgt)
    dist = [oracle.OracleScene(L, Q[:0], S, T[None]).trace(TIE_O, TIE_D)[1][0] for T in (A, B)]
    t = [oracle.OracleScene(L, Q[:0], S, T[None]).trace_tris(TIE_O, TIE_D)[1][0] for T in (A, B)]
    assert dist[0] == dist[1] and t[1] < t[0]
    osc = oracle.OracleScene(L, Q[:0], S, tie_triangles(wgt))
    for brute in (True, False):
        prim, d = osc.trace(TIE_O, TIE_D, brute=brute)
        assert prim[0] == len(L) + 1 and d[0] == dist[1]  # triangle B, not the first-scanned A
