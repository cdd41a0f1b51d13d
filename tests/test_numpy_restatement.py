"""Two independent restatements of path_tracer.wgsl — the C oracle and a numpy
float32 one (tests/numpy_restatement.py) — must agree bit for bit."""
import numpy as np
import pytest

import numpy_restatement as nr


@pytest.mark.parametrize("W,H,spp,seed", [(16, 16, 1, 0), (12, 9, 4, 3), (20, 12, 1, 77)])
def test_numpy_restatement_matches_oracle(oracle, W, H, spp, seed):
    L, Q, S = oracle.cornell_scene()
    cam = oracle.camera_param(W / H, spp, seed)
    ref = oracle.OracleScene(L, Q, S).render(cam, W, H)
    img, hit0 = nr.render(L, Q, S, cam[0], W, H)
    assert np.array_equal(hit0, ref["hit"])
    assert np.array_equal(img.view(np.uint32), ref["f32"].view(np.uint32))


def test_numpy_sincos_matches_oracle(oracle):
    xs = np.linspace(0, 6.3, 5001, dtype=np.float32)
    L = oracle.lib()
    assert np.array_equal(nr.wsin(xs), np.array([L.o_sin(float(x)) for x in xs], np.float32))
    assert np.array_equal(nr.wcos(xs), np.array([L.o_cos(float(x)) for x in xs], np.float32))
