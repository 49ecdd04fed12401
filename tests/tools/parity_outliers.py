"""Diagnose the off-threshold parity outliers (VERDICT r03 "what's next" #1): rays the oracle does not flag whose
GPU colour differs from the oracle's by more than 1e-4.

    python tests/tools/parity_outliers.py <config> [stride] [offset]     (config: bicycle, dense, lightfield, garden)

Renders the bench view (FAST and LITERAL, hit counts, ray directions) on the GPU, runs the oracle with margins on
every stride-th ray, and for each unflagged ray beyond 1e-4 prints one JSON record: the two colours, the accepted
counts, whether the GPU's ray direction equals the oracle's bit for bit, and per composited crossing of the oracle's
trace its response evaluated three ways — the oracle's float32 value, float64 from the same float32 inputs, and a
float32 emulation of the kernel's arithmetic (kernel_org / kernel_dir with fmaf, the GPU ray direction) — with its
relative distance to the thresholds and the conditioning estimate kappa = 4 |ln gres| |ok| / |ok x g| 2^-24 (the
relative change of gres per ulp of ray direction or kernel-frame origin).  Writes gpurun_out/outliers_<config>.json.
"""
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
gv = importlib.import_module("3dgvrt_lightfield_amd")
import oracle as O  # noqa: E402  (checker)

S_K = -0.0555555555556
HITMIN, AMIN = 0.0113, 0.0039215686275
U = 2.0 ** -24


def quat_mat(q):  # utils.glsl:13-34 (GLSL columns), float64
    w, x, y, z = [float(v) for v in q]
    c0 = [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)]
    c1 = [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)]
    c2 = [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]
    return np.array([c0, c1, c2], np.float64)  # rows = GLSL columns


def resp64(rec, o, d):
    """processHit's response in float64 from the float32 record and ray (gaussianfunctions.glsl:186-200)."""
    C = quat_mat(rec[4:8])
    p = rec[0:3].astype(np.float64)
    isc = 1.0 / rec[8:11].astype(np.float64)
    e = o.astype(np.float64) - p
    # mul(R, v) = c0 v.x + c1 v.y + c2 v.z
    ok = isc * (C[0] * e[0] + C[1] * e[1] + C[2] * e[2])
    dk = isc * (C[0] * d[0] + C[1] * d[1] + C[2] * d[2])
    g = dk / np.linalg.norm(dk)
    c = np.cross(g, ok)
    gd = float(c @ c)
    gres = np.exp(S_K * gd * gd)
    return gres, min(0.99, gres * float(rec[3])), float(np.linalg.norm(ok)), float(np.sqrt(gd))


def f32(x):
    return np.float32(x)


def fma32(a, b, c):
    return f32(np.float64(a) * np.float64(b) + np.float64(c))


def resp_gpu32(rec, o, d):
    """float32 emulation of the kernel's particle_alpha(kernel_frame(...)) (gvrt_render.hip kernel_org / kernel_dir /
    particle_alpha; v_rsq and v_exp taken as correctly rounded)."""
    w, x, y, z = [f32(v) for v in rec[4:8]]
    # RenderRec columns as gvrt_enclose.hip stores them: quaternionWXYZToMatrix in float32
    two = f32(2.0)
    c0 = [f32(1) - two * (y * y + z * z), two * (x * y - w * z), two * (x * z + w * y)]
    c1 = [two * (x * y + w * z), f32(1) - two * (x * x + z * z), two * (y * z - w * x)]
    c2 = [two * (x * z - w * y), two * (y * z + w * x), f32(1) - two * (x * x + y * y)]
    isc = [f32(1) / f32(s) for s in rec[8:11]]
    ex, ey, ez = f32(o[0]) - f32(rec[0]), f32(o[1]) - f32(rec[1]), f32(o[2]) - f32(rec[2])
    ok = [fma32(c2[i], ez, fma32(c1[i], ey, c0[i] * ex)) * isc[i] for i in range(3)]
    dk = [fma32(c2[i], f32(d[2]), fma32(c1[i], f32(d[1]), c0[i] * f32(d[0]))) * isc[i] for i in range(3)]
    l2 = fma32(dk[2], dk[2], fma32(dk[1], dk[1], dk[0] * dk[0]))
    rl = f32(1.0 / np.sqrt(np.float64(l2)))
    gx, gy, gz = dk[0] * rl, dk[1] * rl, dk[2] * rl
    cx = fma32(gy, ok[2], -(gz * ok[1]))
    cy = fma32(gz, ok[0], -(gx * ok[2]))
    cz = fma32(gx, ok[1], -(gy * ok[0]))
    gd = fma32(cz, cz, fma32(cy, cy, cx * cx))
    gres = f32(np.exp(np.float64(f32(f32(S_K) * gd) * gd)))
    return float(gres), float(min(f32(0.99), gres * f32(rec[3])))


def main():
    cfg = sys.argv[1]
    stride = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    offset = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    gen, W, H, ncams = gv.scene.CONFIGS[cfg]
    s = gv.scene.make(**gen)
    kw = {}
    if cfg == "lightfield":
        vi, pi = gv.camera.lightfield_grid_rig(gv.camera.orbit_eye(4.0, 20.0, 90.0), (0.0, 0.0, 0.0), nx=4, ny=4,
                                               spacing=0.1, aspect=gv.camera.aspect_ratio(W, H))
    else:
        vi, pi = gv.scene.mipnerf_camera(W, H)
        ncams = 1
    t0 = time.time()
    with gv.Renderer(0) as r:
        r.prepare(s, builder=2, collapse=1)
        fast = r.render(vi, pi, W, H, ncams=ncams, hit_counts=True, ray_dirs=True, rgba8=False)
        lit = r.render(vi, pi, W, H, ncams=ncams, mode=gv.MODE_LITERAL, hit_counts=True, rgba8=False)
    print(f"[gpu] {time.time() - t0:.1f} s", flush=True)
    e = O.enclose(s)
    sc = O.Scene(e)
    sub = np.arange(offset, W * H * ncams, stride, dtype=np.uint64)
    t0 = time.time()
    ref = sc.render(vi, pi, W, H, ncams=ncams, subset=sub, margin=True)
    print(f"[oracle] {len(sub)} rays {time.time() - t0:.1f} s", flush=True)
    idx = sub.astype(np.int64)
    fa = fast["rgba32f"].reshape(-1, 4)[idx].astype(np.float64)
    la = lit["rgba32f"].reshape(-1, 4)[idx].astype(np.float64)
    rb = ref["rgba32f"].astype(np.float64)
    amb = O.ambiguous(ref["margin"])
    dF = np.abs(fa[:, :3] - rb[:, :3]).max(axis=1)
    dL = np.abs(la[:, :3] - rb[:, :3]).max(axis=1)
    out_idx = np.nonzero(((dF > 1e-4) | (dL > 1e-4)) & ~amb)[0]
    print(f"[cmp] flagged {int(amb.sum())}, unflagged beyond 1e-4: FAST {int(((dF > 1e-4) & ~amb).sum())} "
          f"LITERAL {int(((dL > 1e-4) & ~amb).sum())}; max unflagged FAST {dF[~amb].max():.3g}", flush=True)
    # off-threshold distribution of |d| (how far the 1e-4 tail reaches)
    hist = {f"gt_{t:g}": int((dF[~amb] > t).sum()) for t in (1e-6, 1e-5, 3e-5, 1e-4, 3e-4, 1e-3)}
    dirs_gpu = fast["ray_dirs"].reshape(-1, 4)
    dens = e["density"].reshape(-1, 12)
    recs = []
    for k in out_idx[:40]:
        ray = int(idx[k])
        cam = ray // (W * H)
        o = vi.reshape(-1, 16)[cam][12:15].astype(np.float32)
        rd = O.render(e, vi, pi, W, H, ncams=ncams, proxy_mode=1, subset=np.array([ray], np.uint64), ray_dirs=True)
        d_or = rd["ray_dirs"][0, :3].astype(np.float32)
        d_gpu = dirs_gpu[ray, :3].astype(np.float32)
        tr = sc.trace(vi, pi, W, H, ray, ncams=ncams)
        rows = []
        for (pid, t, gres, galpha, T, acc, rnd) in tr:
            rec = dens[int(pid)]
            g64, a64, okn, cn = resp64(rec, o, d_or)
            gg, ga = resp_gpu32(rec, o, d_gpu)
            kappa = 4.0 * abs(np.log(max(g64, 1e-30))) * okn / max(cn, 1e-30) * U
            thr = min(abs(gres / HITMIN - 1), abs(galpha / AMIN - 1))
            acc_gpu = gg > HITMIN and ga > AMIN
            rows.append({"id": int(pid), "t": float(t), "round": int(rnd), "T": float(T), "acc": bool(acc),
                         "gres": float(gres), "galpha": float(galpha), "gres64_rel": float(gres / g64 - 1),
                         "gres_gpu_rel": float(gg / gres - 1) if gres > 0 else 0.0, "acc_gpu_emul": bool(acc_gpu),
                         "thr_rel": float(thr), "ok": okn, "line_dist": cn, "kappa": float(kappa)})
        flips = [x for x in rows if x["acc"] != x["acc_gpu_emul"]]
        worst = sorted(rows, key=lambda x: -(x["kappa"] / max(x["thr_rel"], 1e-12)))[:3]
        recs.append({"ray": ray, "d_fast": float(dF[k]), "d_lit": float(dL[k]), "fast": fa[k].tolist(),
                     "lit": la[k].tolist(), "oracle": rb[k].tolist(), "hits_fast": int(fast["hit_counts"].reshape(-1)[ray]),
                     "hits_lit": int(lit["hit_counts"].reshape(-1)[ray]), "hits_oracle": int(ref["stats"][k, 1]),
                     "dir_equal": bool((d_or == d_gpu).all()), "dir_ulps": (d_or.view(np.int32) - d_gpu.view(np.int32)).tolist(),
                     "margin": ref["margin"][k].tolist(), "n_crossings": len(rows),
                     "emulated_flips": flips, "worst_kappa_over_margin": worst,
                     "max_abs_gres_gpu_rel_accepted": max([abs(x["gres_gpu_rel"]) for x in rows if x["acc"]] or [0.0])})
        print(json.dumps({k2: v for k2, v in recs[-1].items() if k2 not in ("worst_kappa_over_margin",)}), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"outliers_{cfg}.json"), "w") as f:
        json.dump({"config": cfg, "stride": stride, "offset": offset, "rays": len(sub), "flagged": int(amb.sum()),
                   "offthreshold_hist": hist, "outliers": recs}, f, indent=1)
    sc.close()


if __name__ == "__main__":
    main()
