"""Per-tile cost map (GVRT_EXP_TILECOST build: hit_counts = the tile's wave cycles) and a list-scheduling
model of the dispatch order: python scripts/tile_cost.py <config> [slots]"""
import importlib, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gv = importlib.import_module("3dgvrt_lightfield_amd")
cfg = sys.argv[1]
slots = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
gen, W, H, _ = gv.scene.CONFIGS[cfg]
s = gv.scene.make(**gen)
vi, pi = gv.scene.mipnerf_camera(W, H)
with gv.Renderer(0) as r:
    r.prepare(s, builder=2, collapse=1)
    for _ in range(3):
        out = r.render(vi, pi, W, H, hit_counts=True, rgba8=False, rgba32f=False)
    ms = r.stats()["render_ms"]
hc = out["hit_counts"].reshape(H, W)
tx, ty = (W + 7) // 8, (H + 7) // 8
cost = np.zeros((ty, tx))
for j in range(ty):
    for i in range(tx):
        cost[j, i] = hc[j * 8, i * 8]
np.save(f"gpurun_out/tilecost_{cfg}.npy", cost)
c = cost.reshape(-1)
print(cfg, "kernel ms", round(ms, 3), "tiles", c.size, "mean cycles", int(c.mean()), "p50", int(np.median(c)),
      "p99", int(np.percentile(c, 99)), "max", int(c.max()), "sum/slots", int(c.sum() / slots))
import heapq
def makespan(order):
    h = [0.0] * slots
    heapq.heapify(h)
    for t in order:
        f = heapq.heappop(h)
        heapq.heappush(h, f + c[t])
    return max(h)
def st_order(sw, sh):
    o = []
    for sy in range(0, ty, sh):
        for sx in range(0, tx, sw):
            for j in range(sy, min(sy + sh, ty)):
                for i in range(sx, min(sx + sw, tx)):
                    o.append(j * tx + i)
    return o
lb = c.sum() / slots
for name, order in (("rowmajor", list(range(c.size))), ("st8x4", st_order(8, 4)), ("st8x4_rev", st_order(8, 4)[::-1]),
                    ("LPT", list(np.argsort(-c))), ("SPT", list(np.argsort(c)))):
    m = makespan(order)
    print(f"  {name:10s} makespan {m / 1e6:.3f} Mcyc  ({m / lb:.3f} x lower bound)")
