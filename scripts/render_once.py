"""One render of a mesh scene at 1080p (profiling child): python scripts/render_once.py SCENE SPP"""
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, ROOT)
import webgputracer_amd as w  # noqa: E402

ctx = w.Context(0)
L, Q, S, T = w.mesh_scene(sys.argv[1])
ctx.upload_scene(L, Q, S, T)
ctx.render_tile(w.camera_param(16 / 9, int(sys.argv[2]), 1), 1920, 1080)
print("done", flush=True)
