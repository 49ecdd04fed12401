"""Per-tile cost classes along the orbit camera path (moving-camera dispatch order):
    python scripts/orbit_costs_dump.py OUT.npz cfg [step_deg ...]          (GPU)
For each step D: the ordered (second-launch) classes of the frames at azimuth 30 and 30 + D, plus a repeated static
frame at azimuth 30 (the measurement noise of the classes).  scripts/orbit_order_model.py scores predictors of the
moved frame's costs from the previous frame's (list scheduling over 4096 wave slots)."""
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gv = importlib.import_module("3dgvrt_lightfield_amd")


def classes(r, az, W, H):
    vi, pi = gv.scene.mipnerf_camera(W, H, azimuth_deg=az)
    for _ in range(3):
        r.render(vi, pi, W, H, rgba32f=False, rgba8=False)
    return r.tile_costs(W, H)[0], r.render_ms()


def main():
    out = {}
    cfg = sys.argv[2]
    steps = [float(x) for x in sys.argv[3:]] or [0.5, 2.0]
    gen, W, H, _ = gv.scene.CONFIGS[cfg]
    s = gv.scene.make(**gen)
    with gv.Renderer(0) as r:
        r.prepare(s, **gv.QUALITY_BUILD)
        c0, ms0 = classes(r, 30.0, W, H)
        c0b, _ = classes(r, 30.0, W, H)
        out["static"], out["static_repeat"], out["static_ms"] = c0, c0b, ms0
        for d in steps:
            c1, ms1 = classes(r, 30.0 + d, W, H)
            out[f"moved_{d:g}"], out[f"moved_{d:g}_ms"] = c1, ms1
            print(cfg, d, ms0, ms1, flush=True)
    np.savez(sys.argv[1], **out)


if __name__ == "__main__":
    main()
