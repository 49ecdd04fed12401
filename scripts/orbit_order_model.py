"""Offline model of moving-camera dispatch orders: python scripts/orbit_order_model.py costs.npz
(scripts/orbit_costs_dump.py).  The moved frame's measured costs (2^(class/4)) are list-scheduled over 4096 wave slots
in the order of each predictor built from the PREVIOUS frame's classes; prints makespan / balanced bound and the
Spearman correlation of the predictor with the moved frame's cost."""
import heapq
import sys

import numpy as np
from scipy.ndimage import maximum_filter, uniform_filter

SLOTS = 4096


def makespan(costs):
    h = [0.0] * SLOTS
    heapq.heapify(h)
    for c in costs:
        heapq.heappush(h, heapq.heappop(h) + c)
    return max(h)


def rank(x):
    r = np.empty(len(x))
    r[np.argsort(x, kind="stable")] = np.arange(len(x))
    return r


def score(cost, proxy):
    proxy = proxy.reshape(-1)
    order = np.argsort(-proxy, kind="stable")
    bound = max(cost.sum() / SLOTS, cost.max())
    return round(float(np.corrcoef(rank(proxy), rank(cost))[0, 1]), 3), round(makespan(cost[order]) / bound, 4)


d = np.load(sys.argv[1])
prev = d["static"].astype(np.float64)
w = np.exp2(prev / 4.0)
print("static repeat", score(np.exp2(d["static_repeat"] / 4.0).reshape(-1), w))
for k in [k for k in d.files if k.startswith("moved_") and not k.endswith("_ms")]:
    cost = np.exp2(d[k] / 4.0).reshape(-1)
    print(k, "true", score(cost, cost), "prev", score(cost, w))
    for r in (1, 2, 3, 5):
        print("   max", r, score(cost, maximum_filter(w, size=2 * r + 1)), " mean", r,
              score(cost, uniform_filter(w, size=2 * r + 1)), " max+mean", r,
              score(cost, maximum_filter(w, size=2 * r + 1) + uniform_filter(w, size=2 * r + 1)))
    for b in (2, 4, 8):  # coarse blocks: the block's largest cost for every tile in it
        ty, tx = w.shape
        pad = np.zeros(((ty + b - 1) // b * b, (tx + b - 1) // b * b))
        pad[:ty, :tx] = w
        blk = pad.reshape(pad.shape[0] // b, b, pad.shape[1] // b, b).max(axis=(1, 3))
        up = np.repeat(np.repeat(blk, b, 0), b, 1)[:ty, :tx]
        print("   block max", b, score(cost, up))
