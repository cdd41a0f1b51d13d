"""The render kernels' axis-aligned quad path (wgt_device.h isect_quad_axis)
against the reference's intersect_quad arithmetic (path_tracer.wgsl:314-338), in numpy float32 on
the CPU: for the light and every wall of the reference Cornell box (axis-aligned) and 200k rays
(camera rays, rays from inside the box, from far outside, along the axes, grazing the planes), the
short forms give the same bits wherever the reference's decision reads them:

  * denom = s d_K and num = D - s o_K equal dot(n, d) and D - dot(n, o) (up to the sign of a zero,
    which the |denom| < kRayMin and t < kRayMin tests cannot see);
  * the sign pre-rejection (num, denom of opposite signs, or num = +-0) only rejects rays the
    reference rejects at t < kRayMin;
  * t, the hit point and ray_dist follow (same operands), and a = (h_ia v_m) W, b = (u_n h_ib) W
    equal dot(w, cross(hit_vec, up)) and dot(w, cross(right, hit_vec)) bit for bit (zeros: any
    sign).

The code of each record is derived here by the rule of wgt_runtime.cpp quad_axis_code; the GPU
parity tests check the product's codes through whole images.
"""
import numpy as np

import webgputracer_amd as w

f32 = np.float32
RAY_MIN = f32(0.001)  # kRayMin (path_tracer.wgsl)


def axis_code(rec):
    """(K, s, swap, W, u_n, v_m) of a wgt_quad record, or None (wgt_runtime.cpp quad_axis_code)."""
    def axis_of(v):
        nz = [c for c in range(3) if v[c] != 0]
        return (nz[0], v[nz[0]]) if len(nz) == 1 and np.all(np.isfinite(v[:3])) else (-1, None)
    k, s = axis_of(rec["norm"])
    if k < 0 or s not in (1.0, -1.0):
        return None
    kw, wk = axis_of(rec["w"])
    if kw != k:
        return None
    m, v = axis_of(rec["up"])
    n, u = axis_of(rec["right"])
    if m < 0 or n < 0 or k in (m, n) or m == n:
        return None
    swap = m == (k + 1) % 3
    return k, f32(s), swap, f32(-wk if swap else wk), f32(u), f32(v)


def dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def rays(n, rng):
    o = np.empty((n, 3), f32)
    d = np.empty((n, 3), f32)
    k = n // 5
    o[:k] = (278, 278, -800)  # camera rays through the box
    d[:k] = (rng.uniform(0, 556, (k, 3)) - o[:k]).astype(f32)
    o[k:2 * k] = rng.uniform(1, 554, (k, 3))  # bounces inside the box, unit directions
    dd = rng.normal(size=(k, 3))
    d[k:2 * k] = dd / np.linalg.norm(dd, axis=1, keepdims=True)
    o[2 * k:3 * k] = rng.uniform(-3e4, 3e4, (k, 3))  # far outside
    d[2 * k:3 * k] = rng.normal(size=(k, 3))
    o[3 * k:4 * k] = rng.uniform(0, 555, (k, 3))  # axis-aligned directions (exact zeros)
    ax = rng.integers(0, 3, k)
    d[3 * k:4 * k] = 0
    d[3 * k + np.arange(k), ax] = rng.choice([-1.0, 1.0, 1e-3, -1e-3], k)
    r = n - 4 * k  # grazing: origins on a wall plane, directions nearly in it
    o[4 * k:] = rng.uniform(0, 555, (r, 3))
    o[4 * k:, 1] = rng.choice([0.0, 555.0, 554.0], r)
    d[4 * k:] = rng.normal(size=(r, 3))
    d[4 * k:, 1] = rng.choice([0.0, 1e-4, -1e-4, 1e-7], r)
    return o.astype(f32), d.astype(f32)


def test_axis_path_matches_reference_arithmetic():
    L, Q, S = w.cornell_scene()
    recs = np.concatenate([L, Q])
    rng = np.random.default_rng(11)
    o, d = rays(200_000, rng)
    O, Dv = (o[:, 0], o[:, 1], o[:, 2]), (d[:, 0], d[:, 1], d[:, 2])
    n_axis = 0
    with np.errstate(all="ignore"):
        for rec in recs:
            code = axis_code(rec)
            if code is None:
                continue
            n_axis += 1
            k, s, swap, W, u_n, v_m = code
            qn = tuple(f32(x) for x in rec["norm"][:3])
            wv = tuple(f32(x) for x in rec["w"][:3])
            Qp = tuple(f32(x) for x in rec["pos"][:3])
            up = tuple(f32(x) for x in rec["up"][:3])
            rt = tuple(f32(x) for x in rec["right"][:3])
            D = f32(rec["d"])
            # reference
            denom = dot(qn, Dv)
            num = D - dot(qn, O)
            # short forms
            denom_s = s * Dv[k]
            num_s = D - s * O[k]
            live = ~(np.abs(denom) < RAY_MIN)
            assert np.array_equal(live, ~(np.abs(denom_s) < RAY_MIN))
            nz = live & (denom != 0)
            assert np.array_equal(denom[nz], denom_s[nz])
            t = num / np.where(live, denom, f32(1))
            t_s = num_s / np.where(live, denom_s, f32(1))
            # the num values equal, zeros aside (which give t = +-0, rejected either way)
            assert np.array_equal(num[live & (num != 0)], num_s[live & (num != 0)])
            acc = live & ~(t < RAY_MIN)
            assert np.array_equal(acc, live & ~(t_s < RAY_MIN))
            assert np.array_equal(t[acc], t_s[acc])
            # the pre-rejection only drops rays the reference drops
            pre = ((num_s.view(np.uint32) ^ denom_s.view(np.uint32)) >> 31 != 0) | (num_s == 0)
            assert not np.any(acc & pre)
            # edge coordinates at the hit point
            tt = np.where(acc, t, f32(0))
            pos = (O[0] + tt * Dv[0], O[1] + tt * Dv[1], O[2] + tt * Dv[2])
            hv = (pos[0] - Qp[0], pos[1] - Qp[1], pos[2] - Qp[2])
            a = dot(wv, cross(hv, up))
            b = dot(wv, cross(rt, hv))
            h1, h2 = hv[(k + 1) % 3], hv[(k + 2) % 3]
            a_s = ((h2 if swap else h1) * v_m) * W
            b_s = (u_n * (h1 if swap else h2)) * W
            for ref, short in ((a, a_s), (b, b_s)):
                same = (ref == short) & ((ref != 0) <= (ref.view(np.uint32) == short.view(np.uint32)))
                assert np.all(same[acc]), (k, swap)
            inside = acc & ~((np.minimum(a, b) < 0) | (1 < np.maximum(a, b)))
            inside_s = acc & ~((np.minimum(a_s, b_s) < 0) | (1 < np.maximum(a_s, b_s)))
            assert np.array_equal(inside, inside_s)
            assert inside.sum() > 0
    # the light and the five walls (the two boxes' faces have rotated edges: the general path)
    assert n_axis == 6 and len(recs) == 18
