"""Synthetic splat sets (SplatSet layout) standing in for the reference's assets.

The reference's scenes (hotdog / bicycle / garden / truck PLYs) are not in the container
(SURVEY §7 'Real scenes are not in the container'); these generators are the stated
stand-ins of SURVEY §8d / BASELINE.md §4, deterministic in numpy's PCG64 for a given seed.

Arrays follow vk3DGRT::SplatSet (base/Vulkan3DGRTModel.h:16-28): positions 3N, f_dc 3N,
f_rest 45N coefficient-major RGB, opacity N (logit), scale 3N (log), rotation 4N (w,x,y,z).
"""
from __future__ import annotations

import math

import numpy as np

from . import camera as cam

CONFIG1_SEED = 20250824


def _band_sigma():
    # SH coefficient k = 1..15 -> band 1 (k<=3), 2 (k<=8), 3
    k = np.arange(1, 16)
    band = np.where(k <= 3, 1, np.where(k <= 8, 2, 3))
    return 0.08 / (1.0 + band)


def _finish(rng, n, pos, log_scale, opacity, f_dc, frac_filter=0.02):
    rot = rng.normal(0.0, 1.0, (n, 4))
    f_rest = rng.normal(0.0, 1.0, (n, 15, 3)) * _band_sigma()[None, :, None]
    # exercise the abnormal-particle filter (particlePrimitives.comp:137-140)
    nf = int(round(frac_filter * n))
    if nf:
        idx = rng.choice(n, size=2 * nf, replace=False)
        a, b = idx[:nf], idx[nf:]
        f_dc[a] = f_dc[a] / np.linalg.norm(f_dc[a], axis=1, keepdims=True) * 3.5  # |f_dc| > 3
        f_rest[b, 1, :] = 1e-7  # coefficient #2 tiny -> running-sum ratio > 150
    return {
        "positions": np.ascontiguousarray(pos, np.float32).reshape(-1),
        "f_dc": np.ascontiguousarray(f_dc, np.float32).reshape(-1),
        "f_rest": np.ascontiguousarray(f_rest, np.float32).reshape(-1),
        "opacity": np.ascontiguousarray(opacity, np.float32).reshape(-1),
        "scale": np.ascontiguousarray(log_scale, np.float32).reshape(-1),
        "rotation": np.ascontiguousarray(rot, np.float32).reshape(-1),
    }


def config1(n=10_000, seed=CONFIG1_SEED):
    """Config 1: N=10k, pos U[-1,1]^3, log-scale U[ln .01, ln .06]^3, rot N(0,1)^4,
    opacity logit U[-2,4], f_dc N(0,.6)^3 (+2% forced |f_dc|=3.5), f_rest N(0,.08/(1+band))
    (+2% with a tiny coefficient #2)."""
    rng = np.random.default_rng(seed)
    pos = rng.uniform(-1.0, 1.0, (n, 3))
    log_scale = rng.uniform(math.log(0.01), math.log(0.06), (n, 3))
    opacity = rng.uniform(-2.0, 4.0, n)
    f_dc = rng.normal(0.0, 0.6, (n, 3))
    return _finish(rng, n, pos, log_scale, opacity, f_dc)


def config1_camera(width=256, height=256):
    """eye (0,0,3) -> origin, up +y, fovy 39.6 deg (Define.h:33-35)."""
    return cam.pinhole((0.0, 0.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), cam.FOV_Y, cam.aspect_ratio(width, height))


def mipnerf_standin(n=1_000_000, seed=1, scale_mult=1.0, opacity_mean=1.0, opacity_std=2.0):
    """Configs 2-5 stand-in: 60% in an object ball (radius 1.5), 40% in a background
    shell r in [3, 15] with scale proportional to r; log-scale N(ln(0.008 * r_rel), 0.5) with
    r_rel = 1 in the object and r/1.5 in the shell; opacity logit N(1, 2); SH degree 3 as config 1;
    colour f_dc = 0.8 sin(2 pos) + N(0, 0.3) so views have structure; 1% of each filter case."""
    rng = np.random.default_rng(seed)
    n_obj = int(round(0.6 * n))
    n_bg = n - n_obj
    d = rng.normal(size=(n_obj, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = 1.5 * rng.uniform(0.0, 1.0, n_obj) ** (1.0 / 3.0)
    pos_o = d * r[:, None]
    d = rng.normal(size=(n_bg, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rb = rng.uniform(3.0, 15.0, n_bg)
    pos_b = d * rb[:, None]
    pos = np.concatenate([pos_o, pos_b])
    r_rel = np.concatenate([np.ones(n_obj), rb / 1.5])
    log_scale = rng.normal(np.log(0.008 * scale_mult * r_rel)[:, None], 0.5, (n, 3))
    opacity = rng.normal(opacity_mean, opacity_std, n)
    f_dc = 0.8 * np.sin(2.0 * pos) + rng.normal(0.0, 0.3, (n, 3))
    perm = rng.permutation(n)  # PLY order is not spatially sorted
    return _finish(rng, n, pos[perm], log_scale[perm], opacity[perm], f_dc[perm], frac_filter=0.01)


def dense_standin(n=1_000_000, seed=4, scale_mult=3.5, opacity_mean=-3.0):
    """Dense stand-in ("hundreds of crossings per ray"): the config-2 generator with
    scales x3.5 and opacity logit N(-3, 2), seed 4.  Oracle counters at 1920x1080 (every 2003rd ray):
    151.7 crossings, 78.7 accepted and 9.95 LITERAL rounds per ray (vs 22.1 / 17.7 / 1.85 for config 2)."""
    return mipnerf_standin(n, seed, scale_mult=scale_mult, opacity_mean=opacity_mean)


def _quat_mul(a, b):
    """Hamilton product of (w, x, y, z) quaternions, row-wise."""
    w1, x1, y1, z1 = a.T
    w2, x2, y2, z2 = b.T
    return np.stack([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2], axis=1)


def _surfel_quats(rng, normals):
    """(w, x, y, z) rotations taking local +z onto each normal (world = R local), then a random
    twist about it: the thin axis of a surfel lies along the surface normal, as in a trained 3DGRT scene."""
    n = normals / np.linalg.norm(normals, axis=1, keepdims=True)
    q = np.stack([1.0 + n[:, 2], -n[:, 1], n[:, 0], np.zeros(len(n))], axis=1)
    flip = q[:, 0] < 1e-6  # normal ~ -z: a half turn about x
    q[flip] = (0.0, 1.0, 0.0, 0.0)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    phi = rng.uniform(0.0, 2.0 * math.pi, len(n))
    twist = np.stack([np.cos(phi / 2), np.zeros(len(n)), np.zeros(len(n)), np.sin(phi / 2)], axis=1)
    return _quat_mul(q, twist)


def trained_standin(n=1_000_000, seed=5):
    """A stand-in shaped like a trained 3DGRT scene (the reference loads such PLYs,
    base/Vulkan3DGRTModel.cpp:7-125, Define.h:69-89), seed 5:
      * positions on noisy 2-D surfaces: 30 % a ground disk (y = -1, radius 8), 35 % four object spheres and a box,
        25 % a distant shell r in [12, 30] (scenery), 9.9 % volumetric floaters in a ball of radius 6 (log-scale
        N(ln 0.004, 1));
      * anisotropy: 70 % surfels (one axis x U[0.01, 0.05], along the surface normal), 15 % needles (two axes),
        15 % unchanged; floaters random;
      * heavy-tailed sizes: log-scale N(ln(s0 r_rel), 1.5) clipped at 3 sigma and at 0.3 units, s0 = 0.003, r_rel 1
        on the objects, 1 + r / 4 on the ground, sqrt(r / 1.5) in the scenery;
      * 0.1 % giant background Gaussians (scale 1-5 units) in a shell r in [10, 40];
      * bimodal opacity: 40 % logit N(-4.5, 1) (nearly clear), 60 % N(3.5, 1.2) (nearly opaque);
      * SH as config 1, colour f_dc from position; 0.5 % of each filter case."""
    rng = np.random.default_rng(seed)
    counts = [int(round(f * n)) for f in (0.30, 0.35, 0.25, 0.099)]
    counts.append(n - sum(counts))  # giants (0.1 %)
    ng, no, nb, nf, nz = counts
    pos, nrm, rrel = [], [], []
    # ground disk
    r = 8.0 * np.sqrt(rng.uniform(0.0, 1.0, ng))
    th = rng.uniform(0.0, 2.0 * math.pi, ng)
    p = np.stack([r * np.cos(th), -1.0 + rng.normal(0.0, 0.01, ng) * (1.0 + r / 4.0), r * np.sin(th)], axis=1)
    nr = np.tile([0.0, 1.0, 0.0], (ng, 1)) + rng.normal(0.0, 0.05, (ng, 3))
    pos.append(p), nrm.append(nr), rrel.append(1.0 + r / 4.0)
    # object surfaces: four spheres (centre, radius) and the faces of a cube
    spheres = [((0.0, 0.0, 0.0), 0.8), ((1.2, -0.4, 0.5), 0.5), ((-1.0, -0.5, -0.6), 0.45), ((0.2, 0.9, -0.3), 0.3)]
    n_cube = no // 5
    per = np.full(len(spheres), (no - n_cube) // len(spheres))
    per[: (no - n_cube) - per.sum()] += 1
    for (c, rad), k in zip(spheres, per):
        d = rng.normal(size=(k, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        pos.append(np.asarray(c) + d * (rad + rng.normal(0.0, 0.003, (k, 1)))), nrm.append(d), rrel.append(np.ones(k))
    face = rng.integers(0, 6, n_cube)
    ax, sg = face // 2, np.where(face % 2 == 0, -1.0, 1.0)
    p = rng.uniform(-0.35, 0.35, (n_cube, 3))
    p[np.arange(n_cube), ax] = sg * 0.35 + rng.normal(0.0, 0.003, n_cube)
    nr = np.zeros((n_cube, 3))
    nr[np.arange(n_cube), ax] = sg
    pos.append(p + (0.3, -0.6, -1.3)), nrm.append(nr), rrel.append(np.ones(n_cube))
    # distant scenery: a shell, upper half weighted, normals towards the centre
    d = rng.normal(size=(nb, 3))
    d[:, 1] = np.abs(d[:, 1]) * 0.6
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rb = rng.uniform(12.0, 30.0, nb)
    pos.append(d * rb[:, None]), nrm.append(-d), rrel.append(np.sqrt(rb / 1.5))
    # floaters and giants: no surface
    d = rng.normal(size=(nf, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    pos.append(d * 6.0 * rng.uniform(0.0, 1.0, (nf, 1)) ** (1.0 / 3.0)), nrm.append(rng.normal(size=(nf, 3)))
    rrel.append(np.ones(nf))
    d = rng.normal(size=(nz, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    pos.append(d * rng.uniform(10.0, 40.0, (nz, 1))), nrm.append(rng.normal(size=(nz, 3))), rrel.append(np.ones(nz))
    pos = np.concatenate(pos)
    nrm = np.concatenate(nrm)
    rrel = np.concatenate(rrel)
    surf = ng + no + nb
    z = rng.normal(0.0, 1.0, (n, 3)).clip(-3.0, 3.0)
    log_scale = np.log(0.003 * rrel)[:, None] + 1.5 * z[:, :1] + 0.3 * z  # one size per Gaussian, mild per-axis spread
    # floaters: small (the camera sits inside their ball; sigma 1.5 floaters put ~3 k proxies around it)
    log_scale[surf:surf + nf] = np.log(0.004) + 1.0 * z[surf:surf + nf, :1] + 0.3 * z[surf:surf + nf]
    kind = rng.uniform(0.0, 1.0, n)
    thin = np.log(rng.uniform(0.01, 0.05, (n, 2)))
    surfel = (kind < 0.70) & (np.arange(n) < surf)
    needle = (kind >= 0.70) & (kind < 0.85) & (np.arange(n) < surf)
    log_scale[surfel, 2] += thin[surfel, 0]
    log_scale[needle, 1] += thin[needle, 0]
    log_scale[needle, 2] += thin[needle, 1]
    np.minimum(log_scale, math.log(0.3), out=log_scale)  # the tail stops at 0.3 units: only the giants are larger
    log_scale[surf + nf:] = np.log(rng.uniform(1.0, 5.0, (nz, 1))) + rng.normal(0.0, 0.2, (nz, 3))
    opacity = np.where(rng.uniform(0.0, 1.0, n) < 0.4, rng.normal(-4.5, 1.0, n), rng.normal(3.5, 1.2, n))
    f_dc = 0.8 * np.sin(2.0 * pos + 0.5) + rng.normal(0.0, 0.3, (n, 3))
    rot = np.concatenate([_surfel_quats(rng, nrm[:surf]), rng.normal(0.0, 1.0, (n - surf, 4))])
    perm = rng.permutation(n)  # PLY order is not spatially sorted
    out = _finish(rng, n, pos[perm], log_scale[perm], opacity[perm], f_dc[perm], frac_filter=0.005)
    out["rotation"] = np.ascontiguousarray(rot[perm], np.float32).reshape(-1)
    return out


def morton_chain(levels=60, per=8, extent=2.0, seed=6):
    """A clustered scene whose Karras LBVH is a chain (a tree deeper than the traversal stack):
    cluster i (i < levels <= 63) has its quantised centroids' Morton code (63 bits, gvrt_lbvh.hip k_morton) zero above
    bit 62 - i and one at it, i.e. on axis k = i % 3 a coordinate in [h, 2h) with h = extent 2^-(i // 3 + 1), the axes
    before k in [0, h), the axes after k in [0, 2h).  The Karras hierarchy splits cluster i from the rest at every
    level, and the Gaussians of cluster i are larger than everything deeper (bulging boxes, size ~ 2^-i/3), so the
    greedy 4-wide collapse opens the cluster first and descends one chain level per 4-wide level: ~levels + 2
    4-wide levels, beyond the 42 the 128-entry stack allows.  Two anchors pin the Morton bounds to [0, extent]^3."""
    rng = np.random.default_rng(seed)
    pos, ls = [], []
    for i in range(levels):
        j, k = divmod(i, 3)
        h = extent * 2.0 ** -(j + 1)
        lo = np.zeros(3)
        hi = np.full(3, 2.0 * h)
        hi[:k] = h
        lo[k] = h
        p = lo + (hi - lo) * rng.uniform(0.1, 0.9, (per, 3))
        pos.append(p)
        ls.append(np.log(0.6 * extent * 2.0 ** (-i / 3.0)) + rng.normal(0.0, 0.1, (per, 3)))
    pos.append(np.array([[0.0, 0.0, 0.0], [extent, extent, extent]]))
    ls.append(np.full((2, 3), np.log(0.01 * extent * 2.0 ** -21)))
    pos = np.concatenate(pos)
    ls = np.concatenate(ls)
    n = len(pos)
    opacity = rng.normal(0.0, 1.0, n)
    f_dc = 0.8 * np.sin(3.0 * pos) + rng.normal(0.0, 0.2, (n, 3))
    return _finish(rng, n, pos, ls, opacity, f_dc, frac_filter=0.0)


def mipnerf_camera(width=1920, height=1080, azimuth_deg=30.0):
    """Orbit camera radius 4, elevation 20 deg, fovy 50 deg."""
    return cam.orbit_camera(4.0, 20.0, azimuth_deg, (0.0, 0.0, 0.0), 50.0, cam.aspect_ratio(width, height))


CONFIGS = {
    # name: (generator kwargs, width, height, ncams)
    "config1": (dict(kind="config1", n=10_000, seed=CONFIG1_SEED), 256, 256, 1),
    "bicycle": (dict(kind="mipnerf", n=1_000_000, seed=1), 1920, 1080, 1),
    "garden": (dict(kind="mipnerf", n=3_000_000, seed=2), 1920, 1080, 1),
    "truck": (dict(kind="mipnerf", n=2_000_000, seed=3), 3840, 2160, 1),
    "lightfield": (dict(kind="mipnerf", n=1_000_000, seed=1), 1920, 1080, 16),
    "dense": (dict(kind="dense", n=1_000_000, seed=4), 1920, 1080, 1),
    "trained": (dict(kind="trained", n=1_000_000, seed=5), 1920, 1080, 1),
}


def make(kind="config1", n=10_000, seed=CONFIG1_SEED):
    if kind == "config1":
        return config1(n, seed)
    if kind == "mipnerf":
        return mipnerf_standin(n, seed)
    if kind == "dense":
        return dense_standin(n, seed)
    if kind == "trained":
        return trained_standin(n, seed)
    raise ValueError(kind)


def subset(splats, idx):
    idx = np.asarray(idx)
    out = {}
    for k, m in (("positions", 3), ("f_dc", 3), ("f_rest", 45), ("opacity", 1), ("scale", 3), ("rotation", 4)):
        out[k] = np.ascontiguousarray(splats[k].reshape(-1, m)[idx].reshape(-1))
    return out
