"""Diagnostics (GPU box): rays the oracle does not flag that the GPU renders more than 1e-4 away from it, on one
configuration at full frame.  Writes their indices, both values, the margins and each ray's explain() result to
gpurun_out/r06/unflagged_<cfg>.json for analysis on the CPU (oracle trace of those rays)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import importlib  # noqa: E402

gv = importlib.import_module("3dgvrt_lightfield_amd")
import oracle as O  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "trained"
gen, W, H, _ = gv.scene.CONFIGS[cfg]
splats = gv.scene.make(**gen)
vi, pi = gv.scene.mipnerf_camera(W, H)
with gv.Renderer(0) as r:
    r.prepare(splats, builder=2, collapse=1)
    fast = r.render(vi, pi, W, H)["rgba32f"].reshape(-1, 4)
    lit = r.render(vi, pi, W, H, mode=gv.MODE_LITERAL)["rgba32f"].reshape(-1, 4)
e = O.enclose(splats)
sc = O.Scene(e)
ref = sc.render(vi, pi, W, H, margin=True)
b = ref["rgba32f"].reshape(-1, 4)
amb = O.ambiguous(ref["margin"])
out = {"config": cfg, "rays": int(len(b)), "flagged": int(amb.sum())}
for name, g in (("fast", fast), ("literal", lit)):
    d = np.abs(g[:, :3] - b[:, :3]).max(axis=1)
    bad = np.nonzero(~amb & (d > 1e-4))[0]
    ex = sc.explain(vi, pi, W, H, bad.astype(np.uint64), g[bad], tol=1e-4)
    out[name] = [{"ray": int(i), "gpu": [float(x) for x in g[i]], "oracle": [float(x) for x in b[i]],
                  "margin": [float(x) for x in ref["margin"].reshape(-1, 4)[i]], "d": float(d[i]),
                  "explain_dist": float(ex["dist"][k]), "explain_kind": int(ex["kind"][k])}
                 for k, i in enumerate(bad[:200])]
    out[name + "_count"] = int(len(bad))
sc.close()
os.makedirs(os.path.join(ROOT, "gpurun_out", "r06"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "r06", f"unflagged_{cfg}.json"), "w") as f:
    json.dump(out, f, indent=1)
print({k: v for k, v in out.items() if not isinstance(v, list)})
