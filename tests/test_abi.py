"""The C-ABI library loads and exports every symbol include/wgt_api.h declares.
No compute calls here (CPU container): only host-side entry points and error paths."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "wgt_api.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(wgt_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for required in ("wgt_create", "wgt_upload_scene", "wgt_render_tile", "wgt_last_error", "wgt_destroy"):
        assert required in names


def test_library_exports_every_declared_symbol(wgt):
    from webgputracer_amd import _lib

    L = _lib.lib()
    names = declared_functions()
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\bT (wgt_\w+)", out.stdout))
    assert set(names) <= exported
    assert set(_lib.EXPORTS) == set(names), "python binding and header disagree"


def test_struct_sizes_match_reference_layouts(wgt):
    from webgputracer_amd import _lib

    assert _lib.QUAD_DTYPE.itemsize == 96      # scene.h:46 quad_stride_
    assert _lib.SPHERE_DTYPE.itemsize == 32    # scene.h:47 sphere_stride_
    assert _lib.TRI_DTYPE.itemsize == 80       # scene.h:45 tri_stride_
    assert _lib.CAMERA_DTYPE.itemsize == 48    # camera.h:19-31
    # + stack_spills, stack_refills (round 4), stack_overflows (5), the four by-level traversal figures and quad_ref_scans (6)
    assert ctypes.sizeof(_lib.WgtStats) == 232


def test_ctypes_structs_match_the_header(tmp_path):
    """The ctypes mirrors of wgt_stats and wgt_scene_info have the C header's size and field
    offsets (a C program built from include/wgt_api.h with gcc prints them)."""
    import subprocess

    from webgputracer_amd import _lib

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lines = []
    for cname, cls in (("wgt_stats", _lib.WgtStats), ("wgt_scene_info", _lib.WgtSceneInfo)):
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    src = tmp_path / "sizes.c"
    src.write_text("#include <stdio.h>\n#include <stddef.h>\n#include \"wgt_api.h\"\nint main(void) {\n" +
                   "\n".join(lines) + "\nreturn 0;\n}\n")
    exe = tmp_path / "sizes"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(ln.split() for ln in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines())
    for cname, cls in (("wgt_stats", _lib.WgtStats), ("wgt_scene_info", _lib.WgtSceneInfo)):
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(cls, f).offset, (cname, f)


def test_version(wgt):
    from webgputracer_amd import _lib

    # 2 since round 6 (the 64-B and wide node forms' scene-info fields removed); the wrapper refuses
    # a library of another version (its structs mirror this header)
    assert _lib.lib().wgt_version() == _lib.API_VERSION == 2


def test_build_id_names_the_kernel_sources(wgt):
    """wgt_build_id = the Makefile's hash of the HIP sources, their headers and the flags
    (bench.py keys the PMC traffic of profiles/pmc_traffic.json by it)."""
    bid = wgt.build_id()
    assert re.fullmatch(r"[0-9a-f]{16}", bid)
    gen = open(os.path.join(ROOT, "webgputracer_amd", "build", "build_id.cpp")).read()
    assert f'"{bid}"' in gen


def test_no_device_fails_loudly(wgt):
    """Without a GPU the product refuses to run (no CPU fallback exists)."""
    if wgt.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(RuntimeError, match="no HIP device"):
        wgt.Context(0)


def test_null_and_invalid_arguments(wgt):
    from webgputracer_amd import _lib

    L = _lib.lib()
    assert L.wgt_create(0, None) == _lib.WGT_E_INVALID
    assert L.wgt_upload_scene(None, None, 0, None, 0, None, 0, None, 0) == _lib.WGT_E_INVALID
    assert b"null context" in L.wgt_last_error(None)
    assert L.wgt_render_tile(None, None, 1, 1, 0, 0, 1, 1, None, None, None, None) == _lib.WGT_E_INVALID
    assert L.wgt_trace_rays(None, None, 0, None, None) == _lib.WGT_E_INVALID
    assert L.wgt_sync(None) == _lib.WGT_E_INVALID
    L.wgt_destroy(None)  # idempotent for NULL
    n = ctypes.c_uint32(0)
    assert L.wgt_procedural_mesh(7, 10, 0, None, ctypes.byref(n)) == _lib.WGT_E_INVALID
    assert L.wgt_write_png(b"/nonexistent/dir/x.png", np.zeros(4, np.uint8).ctypes.data_as(ctypes.c_void_p),
                           1, 1) == _lib.WGT_E_IO
    assert L.wgt_load_obj(b"/nonexistent.obj", np.zeros(3, np.float32).ctypes.data_as(ctypes.c_void_p), None, 0,
                          None, ctypes.byref(n)) == _lib.WGT_E_IO


def test_cli_binary_built():
    exe = os.path.join(ROOT, "webgputracer_amd", "wgt_tracer")
    assert os.access(exe, os.X_OK)
    r = subprocess.run([exe, "--bogus"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "unknown option" in r.stderr
