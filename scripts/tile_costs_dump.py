"""Per-tile cost classes of a bench frame (gvrt_read_tile_costs after a cost-ordered launch), saved with the
camera for offline analysis of first-frame order estimators: python scripts/tile_costs_dump.py OUT.npz cfg..."""
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gv = importlib.import_module("3dgvrt_lightfield_amd")
out = {}
for cfg in sys.argv[2:]:
    gen, W, H, _ = gv.scene.CONFIGS[cfg]
    s = gv.scene.make(**gen)
    vi, pi = gv.scene.mipnerf_camera(W, H)
    with gv.Renderer(0) as r:
        r.prepare(s, builder=2, collapse=1)
        for _ in range(3):
            r.render(vi, pi, W, H, rgba32f=False)
        out[cfg + "_classes"] = r.tile_costs(W, H)
        out[cfg + "_ms"] = np.float64(r.render_ms())
    out[cfg + "_vi"], out[cfg + "_pi"] = np.asarray(vi), np.asarray(pi)
    print(cfg, W, H, out[cfg + "_classes"].shape, float(out[cfg + "_ms"]), flush=True)
np.savez(sys.argv[1], **out)
