"""Offline model of the dynamic seed-and-offer tile order (DESIGN.md §4 round-4 experiments; built, measured and
removed): python scripts/dyn_order_model.py profiles/r04/orbit_costs_bicycle.npz ...

Measured per-tile costs (2^(class/4), scripts/orbit_costs_dump.py) are list-scheduled over 4096 wave slots.  Seeds
(odd tile column and row) start first in supertile order; a finished seed offers its 8 neighbours at its own cost,
and a free slot takes the costliest offer not yet taken, else the next free tile in supertile order.  Printed:
makespan / balanced bound for the static frame and for the moved frames (prev-order scores: orbit_order_model.py)."""
import heapq
import sys

import numpy as np

SLOTS = 4096


def supertile_order(tx, ty):
    out = []
    for sy in range(0, ty, 4):
        for sx in range(0, tx, 8):
            for y in range(sy, min(sy + 4, ty)):
                for x in range(sx, min(sx + 8, tx)):
                    out.append(y * tx + x)
    return out


def dynamic_makespan(c2d):
    ty, tx = c2d.shape
    c = c2d.reshape(-1)
    n = len(c)
    seed = np.zeros((ty, tx), bool)
    seed[1::2, 1::2] = True
    order = supertile_order(tx, ty)
    seeds = [t for t in order if seed.flat[t]]
    rest = [t for t in order if not seed.flat[t]]
    users = {}
    for s in seeds:
        y, x = divmod(s, tx)
        users[s] = [(y + dy) * tx + x + dx for dy in (-1, 0, 1) for dx in (-1, 0, 1)
                    if (dx or dy) and 0 <= y + dy < ty and 0 <= x + dx < tx]
    claimed = np.zeros(n, bool)
    offers, busy = [], []
    q1, fb, idle, now, started, t_end = list(reversed(seeds)), 0, SLOTS, 0.0, 0, 0.0
    while started < n or busy:
        while idle > 0 and started < n:
            t = None
            if q1:
                t = q1.pop()
            else:
                while offers:
                    _, cand = heapq.heappop(offers)
                    if not claimed[cand]:
                        t = cand
                        break
                if t is None:
                    while claimed[rest[fb]]:
                        fb += 1
                    t = rest[fb]
            claimed[t] = True
            heapq.heappush(busy, (now + c[t], t))
            idle -= 1
            started += 1
        fin, t = heapq.heappop(busy)
        now, idle, t_end = fin, idle + 1, max(t_end, fin)
        for u in users.get(t, []):
            if not claimed[u]:
                heapq.heappush(offers, (-c[t], u))
    return round(t_end / max(c.sum() / SLOTS, c.max()), 4)


for f in sys.argv[1:]:
    d = np.load(f)
    print(f, "static", dynamic_makespan(np.exp2(d["static"].astype(float) / 4)))
    for k in [k for k in d.files if k.startswith("moved_") and not k.endswith("_ms")]:
        print("  ", k, dynamic_makespan(np.exp2(d[k].astype(float) / 4)))
