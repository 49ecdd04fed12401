"""First-frame dispatch order: how well does a sparse probe of the frame predict the per-tile cost?

    python scripts/first_frame_probe.py OUT.json cfg...        (GPU)

Per config: the measured per-tile cost classes of the static frame (gvrt_read_tile_costs of an ordered launch), the
FAST hit counts of every pixel, and the same for a 2-degree-moved camera (the orbit step).  Candidate proxies of a
tile's cost: the accepted-hit count of its centre ray (a 1-ray-per-tile pre-pass would measure it), the mean / max of
its 4 corner-and-centre rays, the mean over all its 64 rays, and the previous (moved) frame's class spread by the
motion radius, and a low-resolution probe render (one ray per tile centre: what a pre-pass would measure, with its
kernel time).  Each is scored by its Spearman correlation with the measured cost and by the list-scheduling makespan
(measured costs dispatched in the proxy's order over 4096 wave slots) over the balanced bound.  Round 4 also built the
probe pre-pass into the library (an option, since removed): profiles/r04/first_frame_probe.json "first_frames"."""
import heapq
import importlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gv = importlib.import_module("3dgvrt_lightfield_amd")
SLOTS = 4096


def makespan(costs_in_order):
    h = [0.0] * SLOTS
    heapq.heapify(h)
    for c in costs_in_order:
        t = heapq.heappop(h)
        heapq.heappush(h, t + c)
    return max(h)


def supertile_order(tx_n, ty_n):
    out = []
    for sy in range(0, ty_n, 4):
        for sx in range(0, tx_n, 8):
            for ty in range(sy, min(sy + 4, ty_n)):
                for tx in range(sx, min(sx + 8, tx_n)):
                    out.append(ty * tx_n + tx)
    return np.array(out)


def rank(x):
    r = np.empty(len(x))
    r[np.argsort(x, kind="stable")] = np.arange(len(x))
    return r


def spearman(a, b):
    return float(np.corrcoef(rank(a), rank(b))[0, 1])


def score(cost, proxy):
    order = np.argsort(-proxy, kind="stable")
    bound = max(cost.sum() / SLOTS, cost.max())
    return {"spearman": round(spearman(proxy, cost), 3), "makespan_over_bound": round(makespan(cost[order]) / bound, 4)}


def main():
    out = {}
    for cfg in sys.argv[2:]:
        gen, W, H, _ = gv.scene.CONFIGS[cfg]
        s = gv.scene.make(**gen)
        tx_n, ty_n = (W + 7) // 8, (H + 7) // 8
        res = {}
        with gv.Renderer(0) as r:
            r.prepare(s, builder=2, collapse=1)
            for az, tag in ((30.0, "static"), (32.0, "moved2")):
                vi, pi = gv.scene.mipnerf_camera(W, H, azimuth_deg=az)
                for _ in range(3):
                    img = r.render(vi, pi, W, H, rgba32f=False, hit_counts=True)
                res[tag + "_classes"] = r.tile_costs(W, H)[0].astype(np.float64)
                res[tag + "_hits"] = img["hit_counts"].reshape(H, W).astype(np.float64)
                res[tag + "_ms"] = r.render_ms()
            # a low-resolution probe: one ray per 8x8 tile through its centre (pixel_offset 0.5 at W/8 x H/8: the
            # same NDC as full-resolution pixel 8i + 4), its accepted-hit counts as the tile cost proxy; its kernel
            # time is what a probe pass would cost (first launch unordered, then ordered)
            vi, pi = gv.scene.mipnerf_camera(W, H)
            probe_ms = []
            for _ in range(3):
                lo = r.render(vi, pi, tx_n, ty_n, rgba32f=False, hit_counts=True, pixel_offset=0.5)
                probe_ms.append(r.render_ms())
            res["probe_hits"] = lo["hit_counts"].reshape(ty_n, tx_n).astype(np.float64)
            res["probe_ms"] = probe_ms
            # the first frame of the static camera (no previous costs): supertile order
            r.set_option("tile_order", 0)
            vi, pi = gv.scene.mipnerf_camera(W, H)
            for _ in range(2):
                r.render(vi, pi, W, H, rgba32f=False, rgba8=False)
            first_ms = r.render_ms()
        cost = np.exp2(res["static_classes"] / 4.0).reshape(-1)
        hits = res["static_hits"]
        hp = np.zeros((ty_n * 8, tx_n * 8))
        hp[:H, :W] = hits
        t = hp.reshape(ty_n, 8, tx_n, 8)
        centre = t[:, 4, :, 4].reshape(-1)
        five = np.stack([t[:, 0, :, 0], t[:, 0, :, 7], t[:, 7, :, 0], t[:, 7, :, 7], t[:, 4, :, 4]], -1)
        prev = np.exp2(res["moved2_classes"] / 4.0)
        rec = {"kernel_ms_ordered": res["static_ms"], "kernel_ms_first_frame": first_ms,
               "supertile": score(cost, -np.argsort(supertile_order(tx_n, ty_n)).astype(np.float64)),
               "true_cost": score(cost, cost),
               "centre_hits": score(cost, centre),
               "five_mean_hits": score(cost, five.mean(-1).reshape(-1)),
               "five_max_hits": score(cost, five.max(-1).reshape(-1)),
               "tile_mean_hits": score(cost, t.mean(axis=(1, 3)).reshape(-1)),
               "prev_2deg_classes": score(cost, prev.reshape(-1)),
               "probe_hits": score(cost, res["probe_hits"].reshape(-1)),
               "probe_kernel_ms": res["probe_ms"]}
        from scipy.ndimage import maximum_filter, uniform_filter
        ph = res["probe_hits"]
        rec["probe_hits_max3"] = score(cost, maximum_filter(ph, size=3).reshape(-1))
        rec["probe_hits_mean3"] = score(cost, uniform_filter(ph, size=3).reshape(-1))
        rec["probe_hits_plus_max3"] = score(cost, (ph + maximum_filter(ph, size=3)).reshape(-1))
        # the supertile order as a proxy: position p gets proxy -p
        st = supertile_order(tx_n, ty_n)
        prox = np.empty(len(st))
        prox[st] = -np.arange(len(st), dtype=np.float64)
        rec["supertile"] = score(cost, prox)
        for rad in (1, 2, 3):
            from scipy.ndimage import maximum_filter
            rec[f"prev_2deg_dilated_{rad}"] = score(cost, maximum_filter(prev, size=2 * rad + 1).reshape(-1))
        out[cfg] = rec
        print(cfg, json.dumps(rec), flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(sys.argv[1])), exist_ok=True)
    with open(sys.argv[1], "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
