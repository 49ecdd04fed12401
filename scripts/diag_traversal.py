"""Traversal diagnostics of the render kernel on a bench scene (stats-enabled renders).

python scripts/diag_traversal.py [config] [kbuffer depths...]
DIAG_OPTS="octant_nodes=0,tile_order=0" sets handle options (gvrt_set_option) first.
"""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gv = importlib.import_module("3dgvrt_lightfield_amd")
cfg = sys.argv[1] if len(sys.argv) > 1 else "bicycle"
depths = [int(x) for x in sys.argv[2:]] or [16]
gen, W, H, _ = gv.scene.CONFIGS[cfg]
s = gv.scene.make(**gen)
vi, pi = (gv.scene.mipnerf_camera(W, H) if cfg != "config1" else gv.scene.config1_camera(W, H))
waves = (W + 7) // 8 * ((H + 7) // 8)
rays = W * H
out = {}
with gv.Renderer(0) as r:
    for kv in filter(None, os.environ.get("DIAG_OPTS", "").split(",")):
        name, _, val = kv.partition("=")
        r.set_option(name, int(val))
    bkw = {} if os.environ.get("GVRT_BUILD") == "fast" else dict(builder=2, collapse=1)  # bench default
    r.prepare(s, split_cells=int(os.environ.get("DIAG_SPLIT", "0")), **bkw)
    runs = [("literal", gv.MODE_LITERAL, 0)] + [(f"fast_k{k}", gv.MODE_FAST, k) for k in depths]
    for name, mode, k in runs:
        kw = dict(mode=mode, kbuffer_depth=k, rgba8=False, rgba32f=False)
        r.render(vi, pi, W, H, **kw)  # warm
        r.set_stats(True)
        r.render(vi, pi, W, H, **kw)
        st = r.stats()
        r.set_stats(False)
        ms = []
        for _ in range(5):
            r.render(vi, pi, W, H, **kw)
            ms.append(r.stats()["render_ms"])
        ms = sorted(ms)[len(ms) // 2]
        out[name] = {"ms": round(ms, 3), "Mrays/s": round(rays / ms / 1e3, 1),
                     "crossings/ray": round(st["crossings"] / rays, 3),
                     "accepted/ray": round(st["accepted"] / rays, 3), "rounds/ray": round(st["rounds"] / rays, 3),
                     "node_visits/wave": round(st["wave_node_visits"] / waves, 1),
                     "leaf_visits/wave": round(st["wave_leaf_visits"] / waves, 1),
                     "dead_visits/wave": round((st["wave_dead_visits"] & 0xFFFFFFFF) / waves, 1),
                     "pruned_pops/wave": round((st["wave_dead_visits"] >> 32) / waves, 1),
                     "rounds/wave": round(st["wave_rounds"] / waves, 3),
                     "late_node_visits/wave": round(st["wave_late_node_visits"] / waves, 1),
                     "lane_leaf_tests/ray": round(st["lane_leaf_tests"] / rays, 2), "bvh_depth": st["bvh_depth"], "bvh_nodes": st["bvh_nodes"], "bvh_leaves": st["bvh_leaves"], "accel_ms": round(st["accel_ms"], 2)}
        pc = st["phase_cycles"]
        if pc[3]:
            out[name]["phase_frac"] = {"node": round(pc[0] / pc[3], 3), "leaf+insert": round(pc[1] / pc[3], 3),
                                       "composite": round(pc[2] / pc[3], 3),
                                       "cycles/wave": round(pc[3] / waves),
                                       "node_cycles/wave": round(pc[0] / waves), "leaf_cycles/wave": round(pc[1] / waves),
                                       "composite_cycles/wave": round(pc[2] / waves)}
print(json.dumps(out, indent=1))
