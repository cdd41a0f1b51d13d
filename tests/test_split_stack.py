"""CPU model of the parked persistent kernel's split traversal stack.

k_render_ps keeps DevScene::ps_cap stack entries per lane in LDS and moves the rest to a
per-lane global stack in its service passes (wgt_device.h park_fix): a lane leaves its
traversal phase when a node step leaves it fewer than 4 free LDS entries, or when its LDS
part runs empty while the global part still holds entries.  This restates that control flow
per ray, in Python over the tree wgt_bvh_build exports (the uploaded tree), and checks on the
CPU what the GPU parity tests can only check by their images:

  * every LDS write lands below ps_cap and the global part never exceeds the builder's
    bound (DevScene::stack = the exported bvh_stack + 1), the size of the global stack;
  * the closest hit equals a brute-force scan for every LDS size down to kMinPsCap = 8,
    whatever order the steps take (the kernel's wave-uniform step modes are modelled by a
    random choice between a node and a triangle step);
  * both fix-ups (spill, refill) run at small LDS sizes.

The box and triangle arithmetic is float64 here (the padded boxes contain their triangles, so
the culling stays conservative): the model checks the stack logic, not the kernels' fp32 bits,
which the -m gpu parity tests pin against the oracle.
"""
import numpy as np
import pytest

import webgputracer_amd as w

NOREF = 0x7FFFFFFF
MISS = np.inf
RAY_MIN, RAY_MAX = 0.001, 1e10  # kRayMin, kRayMax (wgt_math.h; the exact values do not matter here)
TRI_PER_STEP = 2


def leaf_first(ref):
    return (~ref & 0xFFFFFFFF) >> 3


def leaf_count(ref):
    return ((~ref & 0xFFFFFFFF) & 7) + 1


class Tree:
    def __init__(self, tris):
        info, nodes, recs = w.bvh_build(tris)
        self.stack = info["bvh_stack"] + 1  # DevScene::stack (+ the parking entry)
        n = nodes.reshape(-1, 32)
        self.lo = np.stack([n[:, 0:4], n[:, 8:12], n[:, 16:20]], -1).astype(np.float64)   # (nodes, 4, 3)
        self.hi = np.stack([n[:, 4:8], n[:, 12:16], n[:, 20:24]], -1).astype(np.float64)
        self.refs = n[:, 24:28].copy().view(np.int32)
        r = recs.reshape(-1, 16)
        self.v0 = r[:, 0:3].astype(np.float64)
        self.e1 = r[:, 4:7].astype(np.float64)
        self.e2 = r[:, 8:11].astype(np.float64)
        self.idx = r[:, 3].copy().view(np.uint32)


def mt(o, d, v0, e1, e2):
    """Two-sided Moller-Trumbore in float64; t or None."""
    p = np.cross(d, e2)
    det = float(np.dot(e1, p))
    if abs(det) < 1e-12:
        return None
    inv = 1.0 / det
    tv = o - v0
    u = float(np.dot(tv, p)) * inv
    if u < 0.0 or u > 1.0:
        return None
    q = np.cross(tv, e1)
    v = float(np.dot(d, q)) * inv
    if v < 0.0 or u + v > 1.0:
        return None
    t = float(np.dot(e2, q)) * inv
    return t if RAY_MIN <= t <= RAY_MAX else None


class Lane:
    """One lane's traversal: the kernel's Trav (ref, open leaf [lf, le), LDS top sp, best (bt,
    bi)) plus the LDS part (cap entries) and the global part of its stack."""

    def __init__(self, tree, cap, o, d, rng):
        self.T, self.cap, self.o, self.d, self.rng = tree, cap, o, d, rng
        with np.errstate(divide="ignore"):
            self.inv = np.where(np.abs(d) < 1e-30, np.copysign(1e30, d), 1.0 / d)
        self.lds = [None] * cap
        self.glob = []
        self.sp = 0
        self.ref, self.lf, self.le = 0, 0, 0
        self.bt, self.bi = RAY_MAX, 0xFFFFFFFF
        # no bound when the LDS holds the whole stack (k_render_ps top_max)
        self.top_max = cap - 4 if cap < tree.stack else 1 << 30
        self.spills = self.refills = 0

    # -- the stack (Stack24 ld/st), with the bounds the kernel relies on
    def st(self, i, v):
        assert 0 <= i < self.cap, (i, self.cap)
        self.lds[i] = v

    def ld(self, i):
        assert 0 <= i < self.cap
        return self.lds[i]

    def depth(self):
        return self.sp + len(self.glob)

    # -- wgt_device.h trav_resolve
    def resolve(self, cand):
        for _ in range(3):
            if cand == NOREF:
                if self.sp == 0:
                    break
                self.sp -= 1
                cand = self.ld(self.sp)
            if cand >= 0:
                self.ref = cand
                return
            if self.lf >= self.le:
                self.lf = leaf_first(cand)
                self.le = self.lf + leaf_count(cand)
                cand = NOREF
                continue
            self.st(self.sp, cand)
            self.sp += 1
            break
        self.ref = NOREF

    def done(self):
        return self.ref == NOREF and self.lf >= self.le and self.sp == 0

    # -- node_step: keys, the 3 compare-exchanges, pushes (a missed child's write lands at sp)
    def node_step(self):
        T, r = self.T, self.ref
        t0 = (T.lo[r] - self.o) * self.inv
        t1 = (T.hi[r] - self.o) * self.inv
        near = np.maximum(np.minimum(t0, t1).max(1), RAY_MIN)
        far = np.minimum(np.maximum(t0, t1).min(1), self.bt)
        keys = [float(near[c]) if near[c] <= far[c] else MISS for c in range(4)]
        refs = [int(x) for x in T.refs[r]]
        kr = list(zip(keys, refs))

        def cas(a, b):
            if kr[b][0] < kr[a][0]:
                kr[a], kr[b] = kr[b], kr[a]
        cas(0, 1)
        cas(2, 3)
        cas(0, 2)
        for c in (3, 2, 1):
            self.st(self.sp, kr[c][1])
            self.sp += 1 if kr[c][0] != MISS else 0
        self.resolve(kr[0][1] if kr[0][0] != MISS else NOREF)
        assert self.depth() <= self.T.stack

    def tri_step(self):
        T = self.T
        n = min(TRI_PER_STEP, self.le - self.lf)
        best = None
        for j in range(n):
            k = self.lf + j
            t = mt(self.o, self.d, T.v0[k], T.e1[k], T.e2[k])
            if t is None:
                continue
            i = int(T.idx[k])
            if t < self.bt or (t == self.bt and i < self.bi):
                if best is None or t < best[0] or (t == best[0] and i < best[1]):
                    best = (t, i)
        if best is not None:
            self.bt, self.bi = best
        self.lf += n
        if self.lf >= self.le and self.ref == NOREF:
            self.resolve(NOREF)

    # -- park_fix: the service-phase move between the LDS and the global part
    def fix(self):
        cap = self.cap
        if self.sp + 4 > cap:
            keep = (cap - 3) // 2
            m = self.sp - keep
            assert 1 <= keep <= cap - 4 and m >= 1
            assert len(self.glob) + m <= self.T.stack
            self.glob += [self.ld(i) for i in range(m)]
            for i in range(keep):
                self.st(i, self.ld(i + m))
            self.sp = keep
            self.spills += 1
            return
        assert self.sp == 0 and self.ref == NOREF and self.lf >= self.le and self.glob
        half = (cap - 3) // 2 + 1
        m = min(len(self.glob), half)
        for i in range(m):
            self.st(i, self.glob[len(self.glob) - m + i])
        del self.glob[len(self.glob) - m:]
        self.sp = m
        self.resolve(NOREF)
        assert not self.done()
        self.refills += 1

    def run(self):
        # root step in the service pass: it pushes at most 4, so with an LDS stack of >= 8 the
        # ray starts its traversal within the bound
        self.node_step()
        assert self.sp <= self.top_max
        steps = 0
        while True:
            steps += 1
            assert steps < 100000
            can_node, can_tri = self.ref != NOREF, self.lf < self.le
            if not can_node and not can_tri:
                if self.sp == 0 and not self.glob:
                    return self.bt, self.bi  # finished: finalise
                self.fix()  # the LDS part ran empty: refill (the lane left as if done)
                continue
            if can_tri and (not can_node or self.rng.random() < 0.5):
                self.tri_step()
            else:
                assert self.sp <= self.top_max  # a node step may push 3 + park 1 above the top
                self.node_step()
                if self.sp > self.top_max:
                    self.fix()  # the lane parked on its LDS bound: its service pass spills


def brute(tree, o, d):
    best = (RAY_MAX, 0xFFFFFFFF)
    for k in range(len(tree.idx)):
        t = mt(o, d, tree.v0[k], tree.e1[k], tree.e2[k])
        if t is None:
            continue
        i = int(tree.idx[k])
        if t < best[0] or (t == best[0] and i < best[1]):
            best = (t, i)
    return best


def rays_into(tree, n, seed):
    rng = np.random.default_rng(seed)
    lo = tree.v0.min(0)
    hi = tree.v0.max(0)
    c, ext = (lo + hi) / 2, (hi - lo).max()
    o = c + rng.normal(0, 1, (n, 3)) * ext
    tgt = c + (rng.uniform(-0.5, 0.5, (n, 3)) * (hi - lo))
    return o, tgt - o


@pytest.mark.parametrize("cap", [8, 9, 12, 20, None])
def test_split_stack_finds_brute_force_hit(cap):
    """The split stack (any LDS size >= kMinPsCap = 8; None = the whole stack in LDS) returns the
    brute-force closest hit on a 3k-triangle bunny, with every LDS write below the LDS size
    and the global part within the builder's bound."""
    tree = Tree(w.procedural_mesh("bunny", 3000))
    c = tree.stack if cap is None else cap
    o, d = rays_into(tree, 150, 7)
    rng = np.random.default_rng(1)
    spills = refills = 0
    for k in range(len(o)):
        lane = Lane(tree, c, o[k], d[k], rng)
        got = lane.run()
        assert got == brute(tree, o[k], d[k]), k
        spills += lane.spills
        refills += lane.refills
    if c <= 9:
        assert spills > 0 and refills > 0
    if cap is None:
        assert spills == 0 and refills == 0


def test_split_stack_bound_on_full_size_sponza():
    """The full-size sponza stand-in's tree (the bench scene; a 31-entry bound, 32 with the
    parking entry) at the default LDS size of 20 and at 8: the depth never exceeds the bound
    the global stack is sized to, and the closest hit equals a traversal with the whole stack
    in LDS."""
    tree = Tree(w.procedural_mesh("sponza"))
    assert tree.stack == 32
    o, d = rays_into(tree, 120, 3)
    rng = np.random.default_rng(2)
    for k in range(len(o)):
        ref = Lane(tree, tree.stack, o[k], d[k], rng).run()
        for cap in (20, 8):
            assert Lane(tree, cap, o[k], d[k], rng).run() == ref, (k, cap)
