"""Debug: chosen rays of a bench configuration, GPU (FAST, LITERAL, with hit counts) next to the oracle (its
per-crossing trace, margins and flip bound).  python tests/tools/debug_rays.py <config> <ray index>...  (quality
build, the bench camera); prints one JSON record per ray."""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
gv = importlib.import_module("3dgvrt_lightfield_amd")
import oracle as O  # noqa: E402  (checker)

cfg = sys.argv[1]
rays = [int(x) for x in sys.argv[2:]]
gen, W, H, _ = gv.scene.CONFIGS[cfg]
s = gv.scene.make(**gen)
vi, pi = gv.scene.mipnerf_camera(W, H)
with gv.Renderer(0) as r:
    r.prepare(s, builder=2, collapse=1)
    fast = r.render(vi, pi, W, H, hit_counts=True)
    lit = r.render(vi, pi, W, H, mode=gv.MODE_LITERAL, hit_counts=True)
e = O.enclose(s)
sc = O.Scene(e)
sub = np.asarray(rays, np.uint64)
ref = sc.render(vi, pi, W, H, subset=sub, margin=True)
for k, ray in enumerate(rays):
    tr = sc.trace(vi, pi, W, H, ray)
    rec = {"ray": ray,
           "fast": fast["rgba32f"].reshape(-1, 4)[ray].tolist(), "fast_hits": int(fast["hit_counts"].reshape(-1)[ray]),
           "literal": lit["rgba32f"].reshape(-1, 4)[ray].tolist(), "lit_hits": int(lit["hit_counts"].reshape(-1)[ray]),
           "oracle": ref["rgba32f"][k].tolist(), "oracle_stats": ref["stats"][k].tolist(),
           "margin": ref["margin"][k].tolist(),
           "trace": [[float(x) for x in row] for row in tr]}  # id, t, gres, galpha, T after, accepted, round
    print(json.dumps(rec), flush=True)
