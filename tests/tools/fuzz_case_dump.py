"""Test infrastructure (GPU box): one case of tests/test_gpu_fuzz.py rendered on the GPU and by the CPU oracle; the
rays that differ by more than 1e-4 are written with both values, hit counts and margins to
gpurun_out/r06/fuzz_case_<seed>.json for analysis on the CPU.  usage: python tests/tools/fuzz_case_dump.py SEED"""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
gv = importlib.import_module("3dgvrt_lightfield_amd")
import oracle as O  # noqa: E402
import test_gpu_fuzz as F  # noqa: E402

seed = int(sys.argv[1])
c = F._case(gv, seed)
W, H, vi, pi = c["W"], c["H"], c["vi"], c["pi"]
with gv.Renderer(0) as r:
    m = r.prepare(c["splats"], **c["build"], **c["enc"])
    kw = dict(c["variant"])
    if not c["literal"]:
        kw["kbuffer_depth"] = c["depth"]
    mode = gv.MODE_LITERAL if c["literal"] else gv.MODE_FAST
    out = r.render(vi, pi, W, H, mode=mode, hit_counts=True, **kw)
    other = {}
    for k in (8, 16, 24, 32):  # the same frame at every FAST depth
        other[k] = r.render(vi, pi, W, H, hit_counts=True, kbuffer_depth=k, **c["variant"])
e = O.enclose(c["splats"], **c["enc"])
sc = O.Scene(e, **c["enc"])
ref = sc.render(vi, pi, W, H, margin=True, **c["variant"])
b = ref["rgba32f"].reshape(-1, 4)
g = out["rgba32f"].reshape(-1, 4)
d = np.abs(g[:, :3] - b[:, :3]).max(axis=1)
amb = O.ambiguous(ref["margin"].reshape(-1, 4))
bad = np.nonzero(d > 1e-4)[0]
rows = []
for i in bad:
    rows.append({"ray": int(i), "flagged": bool(amb[i]), "d": float(d[i]), "gpu": [float(x) for x in g[i]],
                 "oracle": [float(x) for x in b[i]], "gpu_hits": int(out["hit_counts"].reshape(-1)[i]),
                 "oracle_stats": [int(x) for x in ref["stats"].reshape(-1, 3)[i]],
                 "margin": [float(x) for x in ref["margin"].reshape(-1, 4)[i]],
                 "gpu_by_depth": {k: [float(x) for x in v["rgba32f"].reshape(-1, 4)[i]] for k, v in other.items()}})
sc.close()
os.makedirs(os.path.join(ROOT, "gpurun_out", "r06"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "r06", f"fuzz_case_{seed}.json"), "w") as f:
    json.dump({"seed": seed, "m": m, "rows": rows}, f, indent=1)
print(json.dumps([r for r in rows if not r["flagged"]], indent=1))
