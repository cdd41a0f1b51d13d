"""The product's host code (BVH builder, OBJ parser, procedural meshes, host C-ABI) built
with AddressSanitizer + UBSan and run over random, degenerate and malformed inputs
(tests/host_sanitize/host_fuzz.cpp).  CPU only: GPU sanitizers are not available on the
GPU pool, and the device code is covered by the -m gpu parity suite instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "webgputracer_amd", "csrc", "host")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_host_code_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_fuzz")
    srcs = [os.path.join(ROOT, "tests", "host_sanitize", "host_fuzz.cpp")] + [
        os.path.join(HOST, f) for f in ("bvh.cpp", "obj_loader.cpp", "procedural.cpp", "host_api.cpp", "scene.cpp",
                                        "objects.cpp")]
    # host-only compile: each sanitizer flag directly after -Xarch_host
    cmd = [HIPCC, "-x", "c++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-D__HIP_PLATFORM_AMD__",
           "-I/opt/rocm/include", "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=all"] + srcs + ["-o", exe, "-lz"]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "host_fuzz: ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
