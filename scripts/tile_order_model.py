"""Offline model of first-frame dispatch orders: python scripts/tile_order_model.py tile_costs.npz
(from scripts/tile_costs_dump.py).  Measured per-tile costs (2^(class/4)) are list-scheduled over 4096 wave slots
in supertile order, in true-cost order, and in the order of a footprint estimate (each Gaussian's bounding
sphere rasterised into tile counts by a 2D difference array); prints makespans over the balanced bound and the
Spearman correlation of the estimate with the measured cost."""
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gv = importlib.import_module("3dgvrt_lightfield_amd")
d = np.load(sys.argv[1])
SLOTS = 4096

def makespan(costs_in_order):
    # list scheduling: each tile to the earliest-free slot, in the given order
    h = [0.0] * SLOTS
    heapq.heapify(h)
    for c in costs_in_order:
        t = heapq.heappop(h); heapq.heappush(h, t + c)
    return max(h)

def supertile_order(tx_n, ty_n):
    out = []
    for sy in range(0, ty_n, 4):
        for sx in range(0, tx_n, 8):
            for ty in range(sy, min(sy + 4, ty_n)):
                for tx in range(sx, min(sx + 8, tx_n)):
                    out.append(ty * tx_n + tx)
    return np.array(out)

for cfg in [k[:-8] for k in d.files if k.endswith("_classes")]:
    cls = d[cfg + "_classes"][0].astype(np.float64)
    ty_n, tx_n = cls.shape
    cost = np.exp2(cls / 4.0).reshape(-1)
    gen, W, H, _ = gv.scene.CONFIGS[cfg]
    s = gv.scene.make(**gen)
    p = s["positions"].reshape(-1, 3).astype(np.float64)
    sc = np.exp(s["scale"].reshape(-1, 3).astype(np.float64)).max(axis=1)
    op = 1 / (1 + np.exp(-s["opacity"].reshape(-1).astype(np.float64)))
    vi = d[cfg + "_vi"].reshape(4, 4).T  # column-major -> matrix
    pi = d[cfg + "_pi"].reshape(4, 4).T
    PIm = pi
    V = np.linalg.inv(vi)
    c = np.c_[p, np.ones(len(p))] @ V.T
    z = -c[:, 2]
    ok = z > 0.05
    ax, ay = PIm[0, 0], PIm[1, 1]
    nx = c[:, 0] / np.maximum(z, 1e-3) / ax
    ny = c[:, 1] / np.maximum(z, 1e-3) / ay
    cx = (nx + 1) / 2 * W; cy = (ny + 1) / 2 * H
    R = 3.0 * sc * 1.26
    rx = R / np.maximum(z, 1e-3) / abs(ax) * W / 2
    ry = R / np.maximum(z, 1e-3) / abs(ay) * H / 2
    rpx = np.maximum(rx, ry)
    est = {}
    for name, wgt in (("count", np.ones(len(p))), ("opacity", op)):
        grid = np.zeros((ty_n + 1, tx_n + 1))
        x0 = np.clip(np.floor((cx - rpx) / 8), 0, tx_n).astype(int); x1 = np.clip(np.floor((cx + rpx) / 8) + 1, 0, tx_n).astype(int)
        y0 = np.clip(np.floor((cy - rpx) / 8), 0, ty_n).astype(int); y1 = np.clip(np.floor((cy + rpx) / 8) + 1, 0, ty_n).astype(int)
        m = ok & (x1 > x0) & (y1 > y0)
        np.add.at(grid, (y0[m], x0[m]), wgt[m]); np.add.at(grid, (y0[m], x1[m]), -wgt[m])
        np.add.at(grid, (y1[m], x0[m]), -wgt[m]); np.add.at(grid, (y1[m], x1[m]), wgt[m])
        g = grid.cumsum(0).cumsum(1)[:ty_n, :tx_n].reshape(-1)
        est[name] = g
    ideal = cost.sum() / SLOTS
    st = supertile_order(tx_n, ty_n)
    print(cfg, "tiles", cost.size, "bound", round(ideal, 1))
    print("  supertile", round(makespan(cost[st]) / ideal, 3))
    print("  true-cost LPT", round(makespan(np.sort(cost)[::-1]) / ideal, 3))
    from scipy.stats import spearmanr
    for name, g in est.items():
        order = np.argsort(-g, kind="stable")
        print(f"  est {name}: spearman {spearmanr(g, cost).correlation:.3f} makespan {makespan(cost[order]) / ideal:.3f}")
        # blend: classes of estimate quantised like the kernel's classes (4 per octave)
        q = np.floor(4 * np.log2(g + 1))
        order = np.lexsort((np.arange(len(q)), -q))
        print(f"  est {name} quantised: makespan {makespan(cost[order]) / ideal:.3f}")
