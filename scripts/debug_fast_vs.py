"""Debug: FAST and LITERAL renders of the bicycle stand-in saved to gpurun_out/<tag>.npz (run once per
library build via GVRT_LIB_PATH, then diff the files)."""
import sys, os, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib
gv = importlib.import_module("3dgvrt_lightfield_amd")
tag = sys.argv[1]
W, H = 1920, 1080
splats = gv.scene.mipnerf_standin(1_000_000, seed=1)
vi, pi = gv.scene.mipnerf_camera(W, H)
with gv.Renderer(0) as r:
    r.prepare(splats)
    fast = r.render(vi, pi, W, H)
    lit = r.render(vi, pi, W, H, mode=gv.MODE_LITERAL)
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed(f"gpurun_out/{tag}.npz", fast=fast["rgba32f"], lit=lit["rgba32f"],
                    fast8=fast["rgba8"], lit8=lit["rgba8"])
print(tag, "saved")
