"""GPU parity on random scenes (round 5): the HIP path against the CPU oracle on scenes no fixed
test covers — random lights, quads (any orientation, some emissive), spheres (the last one emissive
or not), triangle soups and cameras placed anywhere in and around the Cornell box's extent.

Each scene is rendered by the persistent kernel (its default schedule, then the 128-B node form
and block order) and by the simple kernel; every radiance word, hit ID and exact counter must equal
the oracle's.  The records' derived fields (quad normal, w, d; triangle edges and face normal) are
computed in numpy fp32: parity compares the two implementations on the same input bytes, whatever
those are, so they need only be plausible and inside the render limits (wgt_api.h)."""
import numpy as np
import pytest

from test_gpu_parity import assert_radiance, check_counters
from webgputracer_amd._lib import QUAD_DTYPE, SPHERE_DTYPE

pytestmark = pytest.mark.gpu

f32 = np.float32


def _quads(wgt, rng, n, emissive_frac):
    q = np.zeros(n, QUAD_DTYPE)
    for i in range(n):
        pos = rng.uniform(-50, 600, 3).astype(f32)
        right = rng.normal(0, 150, 3).astype(f32)
        up = rng.normal(0, 150, 3).astype(f32)
        nrm = np.cross(right, up).astype(f32)
        nn = f32(np.dot(nrm, nrm))
        norm = (nrm / np.sqrt(nn)).astype(f32)
        q[i]["pos"][:3], q[i]["right"][:3], q[i]["up"][:3], q[i]["norm"][:3] = pos, right, up, norm
        q[i]["w"] = (nrm / nn).astype(f32)
        q[i]["d"] = f32(np.dot(norm, pos))
        q[i]["col"] = rng.uniform(0.05, 0.95, 3).astype(f32)
        q[i]["emissive"] = f32(1.0) if rng.random() < emissive_frac else f32(0.0)
        if q[i]["emissive"]:
            q[i]["col"] *= f32(15.0)
    return q


def _spheres(wgt, rng, n, last_emissive):
    s = np.zeros(n, SPHERE_DTYPE)
    s["center"] = rng.uniform(0, 555, (n, 3)).astype(f32)
    s["radius"] = rng.uniform(5, 120, n).astype(f32)
    s["col"] = rng.uniform(0.1, 0.9, (n, 3)).astype(f32)
    s["emissive"] = 0.0
    if last_emissive:
        s[-1]["emissive"] = 1.0
        s[-1]["col"] = (4.0, 3.0, 2.0)
    return s


def _soup(wgt, rng, n):
    c = rng.uniform(0, 555, (n, 1, 3))
    v = (c + rng.normal(0, rng.choice([3.0, 20.0, 80.0]), (n, 3, 3))).astype(f32)
    col = tuple(float(x) for x in rng.uniform(0.2, 0.9, 3))
    return wgt.make_triangles(v, col=col, emissive=bool(rng.random() < 0.1))


def _camera(wgt, oracle, rng, W, H, spp, seed):
    g = wgt.camera_param(W / H, spp, seed, fovy=float(rng.uniform(20, 90)))
    g["origin"] = rng.uniform(-200, 750, 3).astype(f32)
    g["target"] = rng.uniform(50, 500, 3).astype(f32)
    o = oracle.camera_param(W / H, spp, seed)
    assert o.dtype.itemsize == g.dtype.itemsize
    o.view(np.uint8)[:] = g.view(np.uint8)  # the same 48 bytes
    return g, o


@pytest.mark.parametrize("seed", range(24))
def test_random_scene_parity(ctx, wgt, oracle, seed, monkeypatch):
    rng = np.random.default_rng(1000 + seed)
    L = _quads(wgt, rng, 1 + int(rng.integers(0, 2)), 1.0)
    Q = _quads(wgt, rng, int(rng.integers(0, 9)), 0.2)
    S = _spheres(wgt, rng, 1 + int(rng.integers(0, 3)), bool(seed % 2))
    T = _soup(wgt, rng, int(rng.choice([1, 7, 60, 900, 4000])))
    W, H = 40, 24
    cam_g, cam_o = _camera(wgt, oracle, rng, W, H, int(rng.choice([1, 4, 9])), int(rng.integers(0, 2**32)))
    osc = oracle.OracleScene(L, Q, S, T)
    r = osc.render(cam_o, W, H)
    osc.close()
    for env in ({}, {"WGT_CNODE": "0", "WGT_PQ_LPT": "0"}, {"WGT_KERNEL": "1"}):
        for k in ("WGT_CNODE", "WGT_PQ_LPT", "WGT_KERNEL"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        ctx.upload_scene(L, Q, S, T)
        g = ctx.render_tile(cam_g, W, H, stats=True)
        assert_radiance(g["f32"], r["f32"])
        assert np.array_equal(g["u8"], r["u8"])
        assert np.array_equal(g["hit"], r["hit"])
        check_counters(g["stats"], r["counters"], oracle)


def test_random_scene_parity_larger(ctx, wgt, oracle):
    """A larger random scene and frame (20,000 triangles of mixed sizes, 96 x 64 at 16 spp): long
    traversals, many refills of the pixel queue, every wave through several phase switches."""
    rng = np.random.default_rng(77)
    L = _quads(wgt, rng, 1, 1.0)
    Q = _quads(wgt, rng, 5, 0.0)
    S = _spheres(wgt, rng, 2, False)
    T = np.concatenate([_soup(wgt, rng, 10000), _soup(wgt, rng, 10000)])
    W, H = 96, 64
    cam_g, cam_o = _camera(wgt, oracle, rng, W, H, 16, 12345)
    osc = oracle.OracleScene(L, Q, S, T)
    r = osc.render(cam_o, W, H)
    osc.close()
    ctx.upload_scene(L, Q, S, T)
    g = ctx.render_tile(cam_g, W, H, stats=True)
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["hit"], r["hit"])
    check_counters(g["stats"], r["counters"], oracle)
