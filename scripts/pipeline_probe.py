"""Frames issued back to back on one stream vs alternated over S streams (the
context's workspace slots let consecutive launches on different streams overlap:
the next frame's pre-pass and first waves fill the CUs the previous frame's drain
leaves idle).  Prints one JSON line per mode: wall ms per frame over K frames.
  python scripts/pipeline_probe.py [scene] [W H spp] [K]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import webgputracer_amd as w  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "sponza"
W, H, spp = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1920, 1080, 256)
K = int(sys.argv[5]) if len(sys.argv) > 5 else 6
T = 32
dev = torch.device("cuda", 0)
ctx = w.Context(0)
ctx.upload_scene(*w.mesh_scene(scene))
cam = w.camera_param(W / H, spp, 0)
tiles = w.tile_grid(W, H, T, seed=0)
d_tiles = torch.from_numpy(tiles.view(np.uint8).copy()).to(dev)
nt = len(tiles)
outs = [torch.zeros((nt, T, T, 4), dtype=torch.uint8, device=dev) for _ in range(4)]
ref = None
import ctypes  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def hip_streams(n):  # streams created by HIP directly (not torch's pool), non-blocking
    out = []
    for _ in range(n):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
        out.append(s.value)
    return out


def cumask_streams(n):  # a CU-masked stream (all CUs) gets a hardware queue of its own
    cus = ctypes.c_int()
    assert hip.hipDeviceGetAttribute(ctypes.byref(cus), 63, 0) == 0  # hipDeviceAttributeMultiprocessorCount
    words = (cus.value + 31) // 32
    mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
    out = []
    for _ in range(n):
        s = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
        assert rc == 0, rc
        out.append(s.value)
    return out


def prio_streams(n):  # alternate priorities: high / normal
    lo, hi = ctypes.c_int(), ctypes.c_int()
    hip.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi))
    out = []
    for i in range(n):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreateWithPriority(ctypes.byref(s), 1, hi if i % 2 == 0 else lo) == 0
        out.append(s.value)
    return out


class Raw:
    def __init__(self, v):
        self.cuda_stream = v


modes = [(m, S) for _ in range(int(os.environ.get("PROBE_REPS", "2")))
         for m, S in (("seq", 1), ("pipe2-hip", 2), ("pipe2-cumask", 2), ("pipe2-prio", 2))]
for mode, S in modes:
    if mode.endswith("-hip"):
        streams = [Raw(v) for v in hip_streams(S)]
    elif mode.endswith("-cumask"):
        streams = [Raw(v) for v in cumask_streams(S)]
    elif mode.endswith("-prio"):
        streams = [Raw(v) for v in prio_streams(S)]
    else:
        streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    for o in outs:
        o.zero_()
    # warm-up frame on each stream
    for s in streams:
        ctx.render_tiles_async(cam, W, H, T, T, d_tiles.data_ptr(), nt, d_u8=outs[0].data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        s = streams[k % S]
        ctx.render_tiles_async(cam, W, H, T, T, d_tiles.data_ptr(), nt, d_u8=outs[k % S].data_ptr(),
                               stream=s.cuda_stream)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    same = True
    for j in range(min(S, K)):
        img = outs[j].cpu().numpy()
        ref = img if ref is None else ref
        same &= bool(np.array_equal(img, ref))
    print(json.dumps({"scene": scene, "W": W, "H": H, "spp": spp, "mode": mode, "streams": S, "frames": K,
                      "ms_per_frame": round(dt / K * 1e3, 2), "identical": same}), flush=True)
ctx.close()
