"""Host-side logic of the product (no GPU): scene construction and packing in the
reference byte layouts, triangle construction, OBJ reading, procedural stand-ins,
PNG output and the CLI error path."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cornell_bytes_equal_oracle(wgt, oracle):
    """Product C++ Scene::Scene (include/wgt, csrc/host) == independent C restatement."""
    L, Q, S = wgt.cornell_scene()
    oL, oQ, oS = oracle.cornell_scene()
    assert L.tobytes() == oL.tobytes()
    assert Q.tobytes() == oQ.tobytes()
    assert S.tobytes() == oS.tobytes()


def test_triangle_packing_equal_oracle(wgt, oracle):
    rng = np.random.default_rng(0)
    v = (rng.random((500, 3, 3)) * 300).astype(np.float32)
    tr = np.float32([12.5, -3.0, 7.25])
    col = np.float32([0.3, 0.6, 0.9])
    p = wgt.make_triangles(v, col=col, emissive=True, translation=tr)
    o = oracle.make_triangles(v[:, 0] + tr, v[:, 1] + tr, v[:, 2] + tr, col, emissive=True)
    assert p.tobytes() == o.tobytes()


OBJ_TEXT = """# test mesh
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0 0 1
vt 0.5 0.25
vn 0 0 1
o quad
f 1/1/1 2/1/1 3/1/1 4/1/1
g tri
f -5//1 -3//1 -1//1
f 1 2 5
"""


def test_obj_reader_fan_triangulation(wgt, oracle, tmp_path):
    p = tmp_path / "t.obj"
    p.write_text(OBJ_TEXT)
    tris = wgt.load_obj(p, col=(1, 0, 0), translation=(10, 0, 0))
    # quad -> (1,2,3), (1,3,4); then (1,3,5); then (1,2,5)
    verts = np.float32([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [0, 0, 1]]) + np.float32([10, 0, 0])
    faces = [(0, 1, 2), (0, 2, 3), (0, 2, 4), (0, 1, 4)]
    ref = oracle.make_triangles(verts[[f[0] for f in faces]], verts[[f[1] for f in faces]],
                                verts[[f[2] for f in faces]], np.float32([1, 0, 0]))
    assert len(tris) == 4
    assert tris.tobytes() == ref.tobytes()


def test_obj_reader_nonplanar_quad_is_a_fan_from_vertex_0(wgt, oracle, tmp_path):
    """Polygons are split as a fan from their first vertex, (0,1,2), (0,2,3), ...:
    an assumption about tinyobjloader's default triangulation (its submodule is
    empty in the reference, so the rule is unpinned).  On this
    non-planar quad the shorter-diagonal rule some tinyobjloader versions use would
    split along 1-3 instead, giving different triangles; switching rules must be a
    visible choice."""
    p = tmp_path / "q.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 1 1 1\nv 0 1 0\nf 1 2 3 4\n")
    tris = wgt.load_obj(p)
    verts = np.float32([[0, 0, 0], [1, 0, 0], [1, 1, 1], [0, 1, 0]])
    white = np.float32([0.73, 0.73, 0.73])  # color_util.h:8, load_obj's default
    fan = oracle.make_triangles(verts[[0, 0]], verts[[1, 2]], verts[[2, 3]], white)
    assert tris.tobytes() == fan.tobytes()
    shorter = oracle.make_triangles(verts[[0, 1]], verts[[1, 2]], verts[[3, 3]], white)
    assert tris.tobytes() != shorter.tobytes()


def test_obj_reader_errors(wgt, tmp_path):
    p = tmp_path / "bad.obj"
    p.write_text("v 0 0 0\nf 1 2 3\n")
    with pytest.raises(RuntimeError):
        wgt.load_obj(p)


def test_obj_roundtrip(wgt, tmp_path):
    tris = wgt.procedural_mesh("bunny", 800)
    p = tmp_path / "m.obj"
    wgt.write_obj(p, tris)
    back = wgt.load_obj(p)
    assert len(back) == len(tris)
    assert np.array_equal(back["v0"], tris["v0"])
    assert np.allclose(back["e1"], tris["e1"], atol=1e-3) and np.allclose(back["e2"], tris["e2"], atol=1e-3)


@pytest.mark.parametrize("kind,target", [("bunny", 69451), ("sponza", 262267), ("bunny", 1000)])
def test_procedural_meshes(wgt, kind, target):
    a = wgt.procedural_mesh(kind, target)
    b = wgt.procedural_mesh(kind, target)
    assert a.tobytes() == b.tobytes()  # deterministic
    assert abs(len(a) - target) / target < 0.05
    pts = np.concatenate([a["v0"][:, :3], a["v0"][:, :3] + a["e1"][:, :3], a["v0"][:, :3] + a["e2"][:, :3]])
    assert np.all(np.isfinite(pts))
    assert pts.min() >= -1 and pts.max() <= 556  # inside the Cornell box (cornell_box.cpp:6-10)


def test_mesh_scene_composition(wgt):
    L, Q, S, T = wgt.mesh_scene("bunny", 500)
    cL, cQ, cS = wgt.cornell_scene()
    assert L.tobytes() == cL.tobytes() and Q.tobytes() == cQ[:5].tobytes() and S.tobytes() == cS.tobytes()
    assert len(T) > 0


def test_png_writer(wgt, tmp_path):
    from PIL import Image

    img = (np.arange(7 * 5 * 4) % 251).astype(np.uint8).reshape(5, 7, 4)
    p = tmp_path / "000.png"
    wgt.write_png(p, img)
    back = np.asarray(Image.open(p).convert("RGBA"))
    assert np.array_equal(back, img)


def test_cli_without_gpu_fails_cleanly():
    exe = os.path.join(ROOT, "webgputracer_amd", "wgt_tracer")
    from webgputracer_amd import device_count

    if device_count() > 0:
        pytest.skip("GPU present")
    r = subprocess.run([exe, "--frame", "1", "1", "--width", "8", "--height", "8", "--spp", "1", "--no-png"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "Something went wrong" in r.stderr
