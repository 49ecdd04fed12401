"""Offline model of two-launch first frames (a strided probe launch, then the rest ordered by the probe's costs) and
static orders, over the measured tile costs of scripts/tile_costs_dump.py: python scripts/first_frame_model.py."""
import heapq, numpy as np
d = np.load(__import__("sys").argv[1] if len(__import__("sys").argv) > 1 else "gpurun_out/tile_costs.npz")
SLOTS = 4096
def makespan(c):
    h = [0.0] * SLOTS
    for x in c:
        t = heapq.heappop(h); heapq.heappush(h, t + x)
    return max(h)
def supertile(tx_n, ty_n, mask=None, W=8, H=4):
    out = []
    for sy in range(0, ty_n, H):
        for sx in range(0, tx_n, W):
            for ty in range(sy, min(sy + H, ty_n)):
                for tx in range(sx, min(sx + W, tx_n)):
                    if mask is None or mask[ty, tx]:
                        out.append(ty * tx_n + tx)
    return np.array(out)
from scipy.ndimage import maximum_filter, uniform_filter
for cfg in ["bicycle", "garden", "dense", "truck"]:
    cls = d[cfg + "_classes"][0].astype(np.float64); ty_n, tx_n = cls.shape
    cost2 = np.exp2(cls / 4); cost = cost2.reshape(-1); bound = cost.sum() / SLOTS
    full = makespan(cost[supertile(tx_n, ty_n)]) / bound
    res = {"one launch, supertile": round(full, 3)}
    for step in (2, 3, 4):
        yy, xx = np.mgrid[0:ty_n, 0:tx_n]
        A = (yy % step == 0) & (xx % step == 0)
        oa = supertile(tx_n, ty_n, A)
        ma = makespan(cost[oa])
        # estimate B from the sampled tiles: nearest sample (block replicate), then a max filter of radius 1
        samp = cost2[::step, ::step]
        est = np.kron(samp, np.ones((step, step)))[:ty_n, :tx_n]
        for name, e in (("nearest", est), ("max3", maximum_filter(est, size=3))):
            B = ~A
            ob = np.flatnonzero(B.reshape(-1))
            ob = ob[np.argsort(-e.reshape(-1)[ob], kind="stable")]
            mb = makespan(cost[ob])
            res[f"1/{step*step} probe + {name}"] = round((ma + mb) / bound, 3)
    print(cfg, res)
