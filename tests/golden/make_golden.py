"""Regenerate tests/golden/*.npz from the CPU oracle (oracle/gvrt_oracle.cpp).

The reference itself cannot run here (GLSL + Vulkan RT, no SPIR-V compiler or Vulkan device; SURVEY
§8c), so these vectors are the oracle's restatement on seeded inputs.  They pin the oracle against
regressions; the oracle in turn is pinned by the analytic known-answer tests in
tests/test_oracle_kat.py.  The camera matrices stored with them (view_inv / proj_inv) are the
reference's own: camera.py is bit-identical to base/camera.hpp + vendored glm compiled from the
reference sources (tests/test_camera_reference.py).  Run:  python tests/golden/make_golden.py
"""
import importlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
gv = importlib.import_module("3dgvrt_lightfield_amd")
import oracle as O  # noqa: E402


def main():
    s = gv.scene.config1()
    e = O.enclose(s)
    W = H = 64
    vi, pi = gv.scene.config1_camera(W, H)
    tri = O.render(e, vi, pi, W, H, proxy_mode=0)
    ana = O.render(e, vi, pi, W, H, proxy_mode=1)
    rt = O.render(e, vi, pi, W, H, proxy_mode=0, pixel_offset=0.5, alpha_init=1.0)
    np.savez_compressed(
        os.path.join(HERE, "config1_64.npz"),
        m=np.array([e["m"]]), src_index=e["src_index"], density_head=e["density"][: 12 * 256],
        sh_head=e["sh"][: 48 * 256], verts_head=e["verts"][: 36 * 256], tris_head=e["tris"][: 60 * 256],
        view_inv=vi, proj_inv=pi,
        rgba_tri=tri["rgba32f"], stats_tri=tri["stats"], rgba_analytic=ana["rgba32f"], stats_analytic=ana["stats"],
        margin_analytic=ana["margin"], rgba_rt=rt["rgba32f"])
    # light-field ring rig (raygenGaussianLightField.rgen), 4 x 24 x 24, rayDirs layout [cam][x][y]
    vl, pl = gv.camera.lightfield_ring_rig(s["positions"], 4, 24, 24)
    lf = O.render(e, vl, pl, 24, 24, ncams=4, proxy_mode=0, pixel_offset=0.5, alpha_init=1.0, ray_dirs=True,
                  ray_dirs_layout=1)
    np.savez_compressed(os.path.join(HERE, "lightfield_ring_24.npz"), view_inv=vl, proj_inv=pl,
                        rgba=lf["rgba32f"], ray_dirs=lf["ray_dirs"], stats=lf["stats"])
    print("m", e["m"], "written to", HERE)


if __name__ == "__main__":
    main()
