"""Debug (GVRT_TRACE build): per-ray crossing / composite trace of chosen pixels of the bicycle stand-in,
FAST and LITERAL, saved to gpurun_out/trace_rays.npz.  Run with GVRT_LIB_PATH=.../build/trace/libgvrt.so."""
import ctypes as C
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gv = importlib.import_module("3dgvrt_lightfield_amd")
L = gv.lib()
L.gvrt_debug_trace_set.argtypes = [C.c_ulonglong]
L.gvrt_debug_trace_get.argtypes = [C.c_void_p, C.c_int]
W, H = 1920, 1080
splats = gv.scene.mipnerf_standin(1_000_000, seed=1)
vi, pi = gv.scene.mipnerf_camera(W, H)
out = {}
with gv.Renderer(0) as r:
    r.prepare(splats)
    for ray in map(int, sys.argv[1:]):
        for mode, name in ((gv.MODE_FAST, "fast"), (gv.MODE_LITERAL, "lit")):
            L.gvrt_debug_trace_set(ray)
            img = r.render(vi, pi, W, H, mode=mode)["rgba32f"].reshape(-1, 4)[ray]
            buf = np.zeros((8192, 8), np.float32)
            n = L.gvrt_debug_trace_get(buf.ctypes.data, 8192)
            out[f"{name}_{ray}"] = buf[:min(n, 8192)]
            out[f"{name}_{ray}_px"] = img
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/trace_rays.npz", **out)
print("saved", list(out)[:4])
