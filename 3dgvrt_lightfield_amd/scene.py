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
}


def make(kind="config1", n=10_000, seed=CONFIG1_SEED):
    if kind == "config1":
        return config1(n, seed)
    if kind == "mipnerf":
        return mipnerf_standin(n, seed)
    if kind == "dense":
        return dense_standin(n, seed)
    raise ValueError(kind)


def subset(splats, idx):
    idx = np.asarray(idx)
    out = {}
    for k, m in (("positions", 3), ("f_dc", 3), ("f_rest", 45), ("opacity", 1), ("scale", 3), ("rotation", 4)):
        out[k] = np.ascontiguousarray(splats[k].reshape(-1, m)[idx].reshape(-1))
    return out
