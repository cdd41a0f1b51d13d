"""A second, independent restatement of resources/shader/path_tracer.wgsl in numpy
float32 (vectorised over pixels), written from the WGSL rather than from the C
oracle.  Two restatements agreeing bit for bit pins the oracle's reading of the
shader (the reference itself cannot run here: parity with it is unpinned).
TEST INFRASTRUCTURE ONLY.  Quads + spheres (the reference scene); no triangles.
"""
import numpy as np

f32 = np.float32
U32 = np.uint32
kPI = f32(3.14159265359)
k_1_PI = f32(0.318309886184)
kRayMin = f32(0.001)
kRayMax = f32(1e20)
kRayDepth = 50
RAND_SCALE = np.frombuffer(np.uint32(0x2F800004).tobytes(), np.float32)[0]
NO_HIT = U32(0xFFFFFFFF)

# numerics contract: Cody-Waite by pi/2, fdlibm-style polynomials
_TWO_OVER_PI = f32(0.636619772367581343)
_PIO2_HI = np.frombuffer(np.uint32(0x3FC90F80).tobytes(), np.float32)[0]
_PIO2_LO = np.frombuffer(np.uint32(0x37354443).tobytes(), np.float32)[0]
_S = [f32(-1.6666667163e-01), f32(8.3333337680e-03), f32(-1.9841270114e-04), f32(2.7557314297e-06)]
_C = [f32(4.1666667908e-02), f32(-1.3888889225e-03), f32(2.4801587642e-05), f32(-2.7557314297e-07)]


def _reduce(x):
    k = np.floor(x * _TWO_OVER_PI + f32(0.5))
    q = k - f32(4) * np.floor(k * f32(0.25))
    return (x - k * _PIO2_HI) - k * _PIO2_LO, q


def _ksin(r):
    z = r * r
    return r + (r * z) * (_S[0] + z * (_S[1] + z * (_S[2] + z * _S[3])))


def _kcos(r):
    z = r * r
    return (f32(1) - f32(0.5) * z) + (z * z) * (_C[0] + z * (_C[1] + z * (_C[2] + z * _C[3])))


def wsin(x):
    r, q = _reduce(x)
    s, c = _ksin(r), _kcos(r)
    return np.where(q == 0, s, np.where(q == 1, c, np.where(q == 2, -s, -c)))


def wcos(x):
    r, q = _reduce(x)
    s, c = _ksin(r), _kcos(r)
    return np.where(q == 0, c, np.where(q == 1, -s, np.where(q == 2, -c, s)))


# vec3 = tuple of three float32 arrays
def add(a, b): return (a[0] + b[0], a[1] + b[1], a[2] + b[2])
def sub(a, b): return (a[0] - b[0], a[1] - b[1], a[2] - b[2])
def mul(a, b): return (a[0] * b[0], a[1] * b[1], a[2] * b[2])
def scl(s, a): return (s * a[0], s * a[1], s * a[2])
def dvs(a, s): return (a[0] / s, a[1] / s, a[2] / s)
def neg(a): return (-a[0], -a[1], -a[2])
def dot(a, b): return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]
def cross(a, b): return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])
def length(a): return np.sqrt(dot(a, a))
def normalize(a): return dvs(a, length(a))
def sel(c, t, f): return tuple(np.where(c, ti, fi) for ti, fi in zip(t, f))
def full(n, v): return tuple(np.full(n, f32(x), f32) for x in v)


class RNG:
    def __init__(self, seed):
        self.s = seed.astype(U32)

    def rand(self, m):
        """rand() for the lanes in mask m (path_tracer.wgsl:91-95)."""
        s = self.s * U32(747796405) + U32(2891336453)
        self.s = np.where(m, s, self.s)
        word = ((s >> ((s >> U32(28)) + U32(4))) ^ s) * U32(277803737)
        return ((word >> U32(22)) ^ word).astype(f32) * RAND_SCALE


def intersect_quad(o, d, q, qid, hit):
    n = tuple(f32(v) for v in q["norm"][:3])
    denom = dot(d, n)
    ok = ~(np.where(denom < 0, -denom, denom) < kRayMin)
    t = (f32(q["d"]) - dot(o, n)) / denom
    ok &= ~((t < kRayMin) | (kRayMax < t))
    pos = add(o, scl(t, d))
    ray_dist = length(sub(pos, o))
    ok &= ~(ray_dist >= hit["dist"])
    hv = sub(pos, tuple(f32(v) for v in q["pos"][:3]))
    w = tuple(f32(v) for v in q["w"])
    a = dot(w, cross(hv, tuple(f32(v) for v in q["up"][:3])))
    b = dot(w, cross(tuple(f32(v) for v in q["right"][:3]), hv))
    ok &= ~((a < 0) | (1 < a) | (b < 0) | (1 < b))
    ff = dot(d, n) < 0
    _store(hit, ok, ray_dist, q["emissive"] > 0, ff, pos, sel(ff, n, neg(n)), q["col"], qid)


def intersect_sphere(o, d, s, sid, hit):
    c = tuple(f32(v) for v in s["center"])
    oc = sub(o, c)
    a = dot(d, d)
    half_b = dot(oc, d)
    cc = dot(oc, oc) - f32(s["radius"]) * f32(s["radius"])
    disc = half_b * half_b - a * cc
    ok = ~(disc < 0)
    sq = np.sqrt(disc)
    root = (-half_b - sq) / a
    bad = (root < kRayMin) | (kRayMax < root)
    root = np.where(bad, (-half_b + sq) / a, root)
    ok &= ~(bad & ((root < kRayMin) | (kRayMax < root)))
    pos = add(o, scl(root, d))
    ray_dist = length(sub(pos, o))
    ok &= ~(ray_dist >= hit["dist"])
    sn = dvs(sub(pos, c), f32(s["radius"]))
    ff = dot(d, sn) < 0
    _store(hit, ok, ray_dist, s["emissive"] > 0, ff, pos, sel(ff, sn, neg(sn)), s["col"], sid)


def _store(hit, ok, dist, emissive, ff, pos, norm, col, pid):
    hit["dist"] = np.where(ok, dist, hit["dist"])
    hit["emissive"] = np.where(ok, bool(emissive), hit["emissive"])
    hit["ff"] = np.where(ok, ff, hit["ff"])
    hit["pos"] = sel(ok, pos, hit["pos"])
    hit["norm"] = sel(ok, norm, hit["norm"])
    hit["col"] = sel(ok, tuple(np.full_like(pos[0], f32(c)) for c in col), hit["col"])
    hit["prim"] = np.where(ok, U32(pid), hit["prim"])


def sample_hit(o, d, lights, quads, spheres):
    n = len(o[0])
    hit = {"dist": np.full(n, kRayMax, f32), "emissive": np.zeros(n, bool), "ff": np.zeros(n, bool),
           "pos": full(n, (0, 0, 0)), "norm": full(n, (0, 0, 0)), "col": full(n, (0, 0, 0)),
           "prim": np.full(n, NO_HIT, U32)}
    pid = 0
    for q in lights:
        intersect_quad(o, d, q, pid, hit)
        pid += 1
    for q in quads:
        intersect_quad(o, d, q, pid, hit)
        pid += 1
    for s in spheres:
        intersect_sphere(o, d, s, pid, hit)
        pid += 1
    return hit


def build_onb_from_w(w):
    ww = normalize(w)
    sgn = np.where(ww[0] > 0, f32(1), np.where(ww[0] < 0, f32(-1), f32(0)))
    a = sel((sgn * ww[0]) > f32(0.9), full(len(w[0]), (0, 1, 0)), full(len(w[0]), (1, 0, 0)))
    v = normalize(cross(ww, a))
    u = cross(ww, v)
    return u, v, ww


def render(lights, quads, spheres, cam, W, H):
    """compute_sample over the whole W x H frame; returns (H, W, 4) float32 and primary hit ids."""
    with np.errstate(all="ignore"):
        ys, xs = np.meshgrid(np.arange(H, dtype=U32), np.arange(W, dtype=U32), indexing="ij")
        xs, ys = xs.ravel(), ys.ravel()
        n = len(xs)
        seed = xs + ys * U32(W) + U32(cam["seed"]) * U32(W) * U32(H)
        rng = RNG(seed)
        spp = U32(cam["spp"])
        sqrt_spp = int(np.sqrt(f32(spp)))
        col = full(n, (0, 0, 0))
        L0 = lights[0]
        lpos, lright, lup = (tuple(f32(v) for v in L0[k][:3]) for k in ("pos", "right", "up"))
        hit0 = np.full(n, NO_HIT, U32)
        # setup_camera_ray frame terms (path_tracer.wgsl:240-257), evaluated as written
        origin = tuple(f32(v) for v in cam["origin"])
        end = tuple(f32(v) for v in cam["target"])
        theta = f32(cam["fovy"]) * f32(0.017453292519943295)
        focal = length(sub(origin, end))
        h = wsin(theta * f32(0.5)) / wcos(theta * f32(0.5))
        vh = f32(2.0) * h * focal
        vw = vh * f32(cam["aspect"])
        w = normalize(sub(origin, end))
        u = normalize(cross((f32(0), f32(1), f32(0)), w))
        v = cross(w, u)
        vu = scl(vw, u)
        vv = scl(vh, neg(v))
        du = dvs(vu, f32(W))
        dv = dvs(vv, f32(H))
        vul = sub(sub(sub(origin, scl(focal, w)), scl(f32(0.5), vu)), scl(f32(0.5), vv))
        po = add(vul, scl(f32(0.5), add(du, dv)))
        pc = add(add(po, scl(xs.astype(f32), du)), scl(ys.astype(f32), dv))
        recip = f32(1.0) / np.sqrt(f32(spp))
        everyone = np.ones(n, bool)
        for s_j in range(sqrt_spp):
            for s_i in range(sqrt_spp):
                px = f32(-0.5) + recip * (f32(s_i) + rng.rand(everyone))
                py = f32(-0.5) + recip * (f32(s_j) + rng.rand(everyone))
                sample = add(pc, add(scl(px, du), scl(py, dv)))
                o = tuple(np.full(n, c, f32) for c in origin)
                d = sub(sample, origin)
                pcol = full(n, (1, 1, 1))
                alive = np.ones(n, bool)
                for i in range(kRayDepth):
                    hit = sample_hit(o, d, lights, quads, spheres)
                    if s_i == 0 and s_j == 0 and i == 0:
                        hit0 = hit["prim"].copy()
                    em = alive & hit["emissive"]
                    ff = hit["ff"].astype(f32)
                    em_col = hit["col"] if i == 0 else mul(scl(ff, hit["col"]), pcol)
                    ne = alive & ~hit["emissive"]
                    # sample_direction: 3 rand() for non-emissive lanes
                    r0 = rng.rand(ne)
                    use_cos = r0 > f32(0.5)
                    cu, cv, cw = build_onb_from_w(hit["norm"])
                    r1 = rng.rand(ne)
                    r2 = rng.rand(ne)
                    z = np.sqrt(f32(1) - r2)
                    phi = f32(2.0) * kPI * r1
                    cdir = add(add(scl(wcos(phi) * np.sqrt(r2), cu), scl(wsin(phi) * np.sqrt(r2), cv)), scl(z, cw))
                    lp = add(add(lpos, scl(r1, lright)), scl(r2, lup))
                    ldir = sub(lp, hit["pos"])
                    sdir = sel(use_cos, cdir, ldir)
                    # mixture_pdf
                    cpd = dot(normalize(sdir), cw)
                    cpdf = np.where(cpd <= 0, f32(0), cpd * k_1_PI)
                    area = length(cross(lright, lup))
                    dsq = length(sdir) * length(sdir)
                    lc = normalize(sdir)[1]
                    lc = np.where(lc < 0, -lc, lc) + kRayMin
                    lpdf = dsq / (lc * area)
                    pdf = f32(0.5) * cpdf + f32(0.5) * lpdf
                    ndir = normalize(sdir)
                    sc = dot(hit["norm"], normalize(ndir))
                    spdf = np.where(sc < 0, f32(0), sc * k_1_PI)
                    new_col = dvs(scl(spdf, mul(pcol, hit["col"])), pdf)
                    pcol = sel(em, em_col, sel(ne, new_col, pcol))
                    o = sel(ne, hit["pos"], o)
                    d = sel(ne, ndir, d)
                    alive = ne
                    if not alive.any():
                        break
                fs = f32(spp)
                col = add(col, tuple(np.where(c > 0, c, f32(0)) / fs for c in pcol))
        img = np.stack([col[0], col[1], col[2], np.ones(n, f32)], axis=1).reshape(H, W, 4)
        return img, hit0.reshape(H, W)
