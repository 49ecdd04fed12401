"""Same-box timing of render variants: python scripts/ab_time.py <config> <variant>...

A variant is 'default' (the in-tree libgvrt.so), a build name ('3dgvrt_lightfield_amd/build/<name>/libgvrt.so'),
or 'name:key=v,key2=w' (the in-tree library with handle options, gvrt_set_option by name, e.g. tile_order=0,
or environment settings such as AB_K=16 for the k-buffer depth, AB_SPLIT=10 for split_cells, AB_SPAN=3 for split_min_span; 'lib@name:key=v' both).  One child process
per variant; FAST mode, median kernel ms of 15 renders; each frame is compared with the first variant's
(max |d rgba| and the count of pixels differing by more than 1e-4)."""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3dgvrt_lightfield_amd"))
from _lib import OPTIONS  # noqa: E402  (option names only; the library is loaded in the children)

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import importlib, json, os, sys
import numpy as np
sys.path.insert(0, %r)
gv = importlib.import_module("3dgvrt_lightfield_amd")
cfg, outp, opts = sys.argv[1], sys.argv[2], json.loads(sys.argv[3])
gen, W, H, _ = gv.scene.CONFIGS[cfg]
s = gv.scene.make(**gen)
vi, pi = gv.scene.mipnerf_camera(W, H) if cfg != "config1" else gv.scene.config1_camera(W, H)
k = int(os.environ.get("AB_K", "0"))
with gv.Renderer(0) as r:
    for name, val in opts.items():
        r.set_option(name, val)
    r.prepare(s, builder=2, collapse=1, split_cells=int(os.environ.get("AB_SPLIT", "0")),
              split_min_span=int(os.environ.get("AB_SPAN", "0")))
    img = r.render(vi, pi, W, H, kbuffer_depth=k, rgba8=False)["rgba32f"]
    np.save(outp, img)
    r.set_stats(True)
    r.render(vi, pi, W, H, kbuffer_depth=k, rgba8=False, rgba32f=False)
    st = r.stats()
    r.set_stats(False)
    ms = []
    for i in range(18):
        r.render(vi, pi, W, H, kbuffer_depth=k, rgba8=False, rgba32f=False)
        if i >= 3:
            ms.append(r.stats()["render_ms"])
    ms.sort()
    waves = (W + 7) // 8 * ((H + 7) // 8)
    print(json.dumps({"ms": round(ms[len(ms) // 2], 4), "min": round(ms[0], 4),
                      "nodes/wave": round(st["wave_node_visits"] / waves, 1),
                      "leaves/wave": round(st["wave_leaf_visits"] / waves, 1),
                      "rounds/wave": round(st["wave_rounds"] / waves, 3),
                      "flushes/wave": round(st.get("wave_flushes", 0) / waves, 2),
                      "leaf_lane_util": round(st["lane_leaf_tests"] / max(64 * st["wave_leaf_visits"], 1), 3),
                      "dead_node_frac": round(st["wave_dead_visits"] / max(st["wave_node_visits"], 1), 3)}))
''' % ROOT

cfg = sys.argv[1]
ref = None
for v in sys.argv[2:]:
    env = dict(os.environ)
    lib, _, envs = v.partition(":")
    if "@" in lib:
        lib = lib.split("@")[0]
    if lib not in ("default", "") and envs == "" or "@" in v:
        env["GVRT_LIB_PATH"] = os.path.join(ROOT, "3dgvrt_lightfield_amd", "build", lib, "libgvrt.so")
    opts = {}
    for kv in filter(None, envs.split(",")):
        k, _, val = kv.partition("=")
        if k in OPTIONS:
            opts[k] = int(val)
        else:
            env[k] = val
    outp = f"/tmp/ab_{cfg}_{abs(hash(v))}.npy"
    out = subprocess.run([sys.executable, "-c", CHILD, cfg, outp, json.dumps(opts)], env=env, capture_output=True,
                         text=True, timeout=300)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    if not line:
        print(cfg, v, "FAILED", out.stderr[-600:], flush=True)
        continue
    res = json.loads(line[-1])
    img = np.load(outp)
    if ref is None:
        ref = img
    else:
        d = np.abs(img - ref).reshape(-1, 4).max(axis=1)
        res["max_d"] = float(d.max())
        res["px>1e-4"] = int((d > 1e-4).sum())
    print(cfg, v, json.dumps(res), flush=True)
