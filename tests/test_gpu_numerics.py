"""GPU parity outside the usual scene scale, and the ABI's guards.

The kernels' short correctly-rounded sqrt / division sequences (wgt_math.h
sqrt_rn, div_rn) drop the IEEE input scaling and fix-ups of the compiler's
lowering.  These tests render scenes scaled by powers of two far from the
Cornell box's (squared lengths below 2^-96, where the dropped scaling matters,
and large ones) and require bit parity with the oracle's IEEE arithmetic: the
product must never silently diverge.  Also: the spp bound, and a scene
re-upload racing an asynchronous render on a caller stream (advisor finding).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from test_gpu_parity import assert_radiance, check_counters  # noqa: E402


def scale_quads(Q, s):
    """A quad scaled by s about the origin: pos, right, up, d scale by s; the normal
    stays; w = n/(n.n) with n = cross(right, up) scales by 1/s^2.  Powers of two
    keep every field exact (no rounding, no underflow at these scales)."""
    Q = Q.copy()
    with np.errstate(over="ignore", invalid="ignore"):  # 2^-70: w overflows to inf, as in fp32
        for f in ("pos", "right", "up"):
            Q[f][:, :3] *= np.float32(s)
        Q["w"] *= np.float32(min(1.0 / (s * s), 1e300))
        Q["d"] *= np.float32(s)
    return Q


def scale_scene(wgt, s, tris=None):
    L, Q, S = wgt.cornell_scene()
    L, Q = scale_quads(L, s), scale_quads(Q, s)
    S = S.copy()
    S["center"] *= np.float32(s)
    S["radius"] *= np.float32(s)
    if tris is not None:
        tris = tris.copy()
        for f in ("v0", "e1", "e2"):
            tris[f][:, :3] *= np.float32(s)
        return L, Q[:5].copy(), S, tris
    return L, Q, S, None


def scaled_camera(mod, aspect, spp, seed, s):
    cam = mod.camera_param(aspect, spp, seed)
    cam["origin"] *= np.float32(s)
    cam["target"] *= np.float32(s)
    return cam


@pytest.mark.parametrize("log2s", [-70, -60, -12, -4, 8, 20])
def test_scaled_cornell_vs_oracle(ctx, wgt, oracle, log2s):
    """Cornell box and camera scaled by 2^log2s.  From 2^-12 to 2^20 the frame is a
    normal render (80% lit pixels, bounces traced); at 2^-60 / 2^-70 the primary
    directions fall below kRayMin's reach and squared lengths below 2^-96 (w
    overflows to inf at 2^-70).  Bit parity with the oracle's IEEE arithmetic at
    every scale within the render limits (2^20 is the largest power of two whose
    primary directions stay within 2^32)."""
    s = 2.0 ** log2s
    L, Q, S, _ = scale_scene(wgt, s)
    ctx.upload_scene(L, Q, S)
    W, H, spp, seed = 40, 40, 4, 9
    g = ctx.render_tile(scaled_camera(wgt, 1.0, spp, seed, s), W, H, stats=True)
    r = oracle.OracleScene(L, Q, S).render(scaled_camera(oracle, 1.0, spp, seed, s), W, H)
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["u8"], r["u8"])
    assert np.array_equal(g["hit"], r["hit"])
    check_counters(g["stats"], r["counters"], oracle)


@pytest.mark.parametrize("cnode", ["2", "1"])
@pytest.mark.parametrize("log2s", [-60, -8, 20])
def test_scaled_mesh_vs_oracle(ctx, wgt, oracle, log2s, cnode, monkeypatch):
    """The BVH path (a 2k-triangle mesh in the Cornell walls) at the same scales, on the
    size rule's node form (WGT_CNODE=2: 128-B nodes for this small tree) and on the compact nodes,
    whose fused slab step relies on the builder's code margin."""
    monkeypatch.setenv("WGT_CNODE", cnode)
    s = 2.0 ** log2s
    L, Q, S, T = scale_scene(wgt, s, wgt.procedural_mesh("bunny", 2000))
    ctx.upload_scene(L, Q, S, T)
    W, H, spp, seed = 48, 27, 4, 2
    g = ctx.render_tile(scaled_camera(wgt, 16 / 9, spp, seed, s), W, H, stats=True)
    r = oracle.OracleScene(L, Q, S, T).render(scaled_camera(oracle, 16 / 9, spp, seed, s), W, H)
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["hit"], r["hit"])
    check_counters(g["stats"], r["counters"], oracle)


def test_render_limits_fail_cleanly(ctx, wgt):
    """Outside the numeric limits that keep the quad distance's short division exact
    (scene coordinates and camera within 2^40, quad normals within 2 or NaN, triangle
    edges within 2^30, primary directions within 2^32; wgt_runtime.cpp
    check_scene_limits / check_render_args)
    the calls return WGT_E_INVALID instead of rendering."""
    from webgputracer_amd._lib import WGT_E_INVALID, WgtError

    def invalid(fn):
        with pytest.raises(WgtError) as e:
            fn()
        assert e.value.code == WGT_E_INVALID, e.value

    L, Q, S = wgt.cornell_scene()
    big = scale_scene(wgt, 2.0 ** 40)
    invalid(lambda: ctx.upload_scene(*big[:3]))  # coordinates beyond 2^40
    Qn = Q.copy()
    Qn["norm"][3, :3] = (0.0, 3.0, 0.0)  # not a unit normal
    invalid(lambda: ctx.upload_scene(L, Qn, S))
    Qnan = Q.copy()
    Qnan["pos"][2, 0] = np.nan
    invalid(lambda: ctx.upload_scene(L, Qnan, S))
    T = wgt.procedural_mesh("bunny", 500)
    T["v0"][7, 1] = np.inf
    invalid(lambda: ctx.upload_scene(L, Q[:5], S, T))
    T = wgt.procedural_mesh("bunny", 500)
    T["e2"][3, 2] = 2.0 ** 31  # an edge beyond 2^30 (Moller-Trumbore's short 1/det)
    invalid(lambda: ctx.upload_scene(L, Q[:5], S, T))
    Qd = Q.copy()
    Qd["norm"][4, :3] = np.nan  # a degenerate quad's NaN normal is accepted
    ctx.upload_scene(L, Qd, S)
    ctx.upload_scene(L, Q, S)
    invalid(lambda: ctx.render_tile(scaled_camera(wgt, 1.0, 1, 0, 2.0 ** 24), 8, 8))  # directions > 2^32
    cam = wgt.camera_param(1.0, 1, 0)
    cam["origin"][0, 0] = np.nan
    invalid(lambda: ctx.render_tile(cam, 8, 8))
    # round 6: a pixel's coordinates are the 16-bit halves of one register (frames up to 65,535 on a
    # side), a pending quad's index + 1 fits 26 bits
    cam = wgt.camera_param(1.0, 1, 0)
    invalid(lambda: ctx.render_tile(cam, 65536, 4, 0, 0, 8, 4))
    from webgputracer_amd._lib import ptr

    # the count is refused before any quad is read: a one-quad buffer with a count of 2^26 - 2
    invalid(lambda: ctx._check(ctx._L.wgt_upload_scene(ctx.h, ptr(L), len(L), ptr(Q), (1 << 26) - 2, ptr(S),
                                                       len(S), None, 0)))
    ctx.upload_scene(L, Q, S)


@pytest.mark.parametrize("seed", [1, 2])
def test_selftest_math_sequences_are_exact(ctx, seed):
    """sqrt_rn equals correctly rounded sqrt on all 2^32 inputs, sqrt_fast on every
    input of its domain; div_rn gives the IEEE accept decision and accepted bits on
    16M quad-distance operand pairs under the render limits (zeros, denormals and
    every exponent of the numerator included; denominators up to 2^35, the bound
    2*sqrt(3)*2^32 of |qn . d|), and the IEEE bits of 1/det on 16M determinants over
    Moller-Trumbore's range 2^-40 <= |det| < 2^95 under the limits; since round 6 also the
    short reciprocal of the traversal's 1/d on every bit pattern 1e-30 <= |x| <= 2^34 (render rays'
    direction components after safe_inv's clamp), DESIGN.md §3.2."""
    c = ctx.selftest_math(1 << 24, seed)
    print("selftest", c)
    lo = int(np.float32(1e-30).view(np.uint32))
    hi = int(np.float32(2.0 ** 34).view(np.uint32))
    # div_tests: 2^24 quad-distance quotients + 2^24 Moller-Trumbore reciprocals 1/det + every
    # traversal reciprocal pattern (both signs)
    assert c["sqrt_tests"] == 1 << 32 and c["div_tests"] == (2 << 24) + 2 * (hi - lo + 1)
    assert c["sqrt_fast_tests"] > 3 << 30
    assert c["sqrt_rn_bad"] == 0 and c["sqrt_fast_bad"] == 0 and c["div_rn_bad"] == 0, c


@pytest.mark.parametrize("spp", [0xFFFFFFFF, 0xFFFFFF80])
def test_spp_beyond_sample_index_range_rejected(ctx, wgt, spp):
    """u32(sqrt(f32(spp))) > 65535 would overflow the kernels' 16-bit sample indices
    (and sqrt_spp^2 in u32): the call fails cleanly with WGT_E_INVALID, no launch."""
    from webgputracer_amd._lib import WGT_E_INVALID, WgtError

    ctx.upload_scene(*wgt.cornell_scene())
    with pytest.raises(WgtError) as e:
        ctx.render_tile(wgt.camera_param(1.0, spp, 0), 8, 8)
    assert e.value.code == WGT_E_INVALID


def test_upload_waits_for_async_render_on_caller_stream(ctx, wgt, oracle):
    """An asynchronous render on a caller's stream, then a scene re-upload with no
    synchronisation in between: the upload must wait for the render before it frees
    the scene (the render sees the first scene, bit for bit)."""
    import torch

    from webgputracer_amd._lib import TILE_DTYPE

    L, Q, S = wgt.cornell_scene()
    T = wgt.procedural_mesh("sponza", 60000)
    ctx.upload_scene(L, Q[:5], S, T)
    W, H, spp, seed = 64, 48, 64, 5
    dev = torch.device("cuda", 0)
    tiles = np.zeros(1, TILE_DTYPE)
    tiles["seed"] = seed
    d_tiles = torch.from_numpy(tiles.view(np.uint8).copy()).to(dev)
    out = torch.zeros((H, W, 4), dtype=torch.float32, device=dev)
    stream = torch.cuda.Stream(device=dev)
    ctx.render_tiles_async(wgt.camera_param(W / H, spp, 0), W, H, W, H, d_tiles.data_ptr(), 1,
                           d_f32=out.data_ptr(), stream=stream.cuda_stream)
    ctx.upload_scene(L, Q, S)  # no sync: must not free the mesh scene under the render
    stream.synchronize()
    r = oracle.OracleScene(L, Q[:5], S, T).render(oracle.camera_param(W / H, spp, seed), W, H)
    assert_radiance(out.cpu().numpy(), r["f32"])


@pytest.mark.parametrize("offset,cam_z", [((65536.0, -32768.0, 16384.0), None), ((0.0, 0.0, 0.0), -1.0e6)])
def test_compact_nodes_far_origins_vs_oracle(ctx, wgt, oracle, offset, cam_z, monkeypatch):
    """Compact nodes forced (WGT_CNODE=1) where their code margin matters most:
    (1) scene and camera translated far from the origin (coordinates ~2^16 against a
    box of 555: the fused slab step's rounding grows with |org| and |ray origin|, and
    the margin with them); (2) a camera 10^6 away, beyond the bound the codes were
    built for, which makes the frame read the 128-B nodes instead.  Bit parity with
    the oracle either way."""
    monkeypatch.setenv("WGT_CNODE", "1")
    L, Q, S, T = wgt.mesh_scene("bunny", target_tris=2000)
    off = np.array(offset, np.float32)
    L, Q, S, T = L.copy(), Q.copy(), S.copy(), T.copy()
    for arr in (L, Q):  # translated quads: the plane offset D = dot(normal, Q) follows (quad.cpp)
        arr["pos"][:, :3] += off
        n, p = arr["norm"][:, :3], arr["pos"][:, :3]
        arr["d"] = (n[:, 0] * p[:, 0] + n[:, 1] * p[:, 1]) + n[:, 2] * p[:, 2]
    S["center"][:, :3] += off
    T["v0"][:, :3] += off
    ctx.upload_scene(L, Q, S, T)
    W, H, spp, seed = 48, 27, 4, 6

    def cam(mod):
        c = mod.camera_param(16 / 9, spp, seed)
        c["origin"] += off
        c["target"] += off
        if cam_z is not None:
            c["origin"][..., 2] = np.float32(cam_z)
        return c

    g = ctx.render_tile(cam(wgt), W, H, stats=True)
    r = oracle.OracleScene(L, Q, S, T).render(cam(oracle), W, H)
    assert_radiance(g["f32"], r["f32"])
    assert np.array_equal(g["hit"], r["hit"])
    check_counters(g["stats"], r["counters"], oracle)
