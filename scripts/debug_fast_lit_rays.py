"""Debug: rays where FAST and LITERAL differ on the bicycle stand-in (1080p).  Saves, for each such ray,
FAST at several k-buffer depths, LITERAL, and the accepted-hit counts to gpurun_out/fastlit_rays.npz."""
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gv = importlib.import_module("3dgvrt_lightfield_amd")
W, H = 1920, 1080
splats = gv.scene.mipnerf_standin(1_000_000, seed=1)
vi, pi = gv.scene.mipnerf_camera(W, H)
out = {}
with gv.Renderer(0) as r:
    r.prepare(splats)
    fast = r.render(vi, pi, W, H, hit_counts=True)
    lit = r.render(vi, pi, W, H, mode=gv.MODE_LITERAL, hit_counts=True)
    fa, fb = fast["rgba32f"].reshape(-1, 4), lit["rgba32f"].reshape(-1, 4)
    d = np.abs(fa[:, :3] - fb[:, :3]).max(axis=1)
    rays = np.nonzero((d > 1e-4) | (fa[:, 3] != fb[:, 3]))[0]
    out["rays"] = rays
    out["fast"] = fa[rays]
    out["lit"] = fb[rays]
    out["hc_fast"] = fast["hit_counts"].reshape(-1)[rays]
    out["hc_lit"] = lit["hit_counts"].reshape(-1)[rays]
    for k in (8, 16, 32):
        out[f"fast_k{k}"] = r.render(vi, pi, W, H, kbuffer_depth=k)["rgba32f"].reshape(-1, 4)[rays]
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/fastlit_rays.npz", **out)
print(len(rays), "rays saved")
