"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / CPU baseline.  See gvrt_oracle.cpp for what it restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


class OracleParams(C.Structure):
    _fields_ = [("aabb", C.c_float * 6), ("min_transmittance", C.c_float), ("hit_min_gaussian_response", C.c_float),
                ("sph_eval_degree", C.c_uint32), ("alpha_min", C.c_float), ("pixel_offset", C.c_float),
                ("alpha_init", C.c_float), ("tmin_inclusive", C.c_uint32), ("proxy_mode", C.c_uint32),
                ("drop_rejected", C.c_uint32), ("max_rounds", C.c_uint32), ("ray_dirs_layout", C.c_uint32),
                ("kernel_min_response", C.c_float), ("kernel_opts", C.c_uint32), ("kernel_degree", C.c_float),
                ("perturb_ulps", C.c_uint32), ("flag_cond_ulps", C.c_float)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp = C.c_void_p
        L.oracle_enclose.argtypes = [vp] * 6 + [C.c_uint32, C.c_float, C.c_uint32, C.c_float] + [vp] * 6
        L.oracle_enclose.restype = C.c_int
        L.oracle_render.argtypes = [vp, vp, vp, vp, C.c_uint32, C.POINTER(OracleParams), vp, vp, C.c_uint32,
                                    C.c_uint32, C.c_uint32, vp, C.c_uint64, vp, vp, vp, vp, vp, C.c_int]
        L.oracle_render.restype = C.c_int
        L.oracle_scene_create.argtypes = [vp, vp, vp, vp, C.c_uint32, C.c_uint32, C.c_float, C.c_uint32, C.c_float]
        L.oracle_scene_create.restype = vp
        L.oracle_scene_destroy.argtypes = [vp]
        L.oracle_scene_render.argtypes = [vp, C.POINTER(OracleParams), vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, vp,
                                          C.c_uint64, vp, vp, vp, vp, vp, C.c_int]
        L.oracle_scene_render.restype = C.c_int
        L.oracle_scene_trace.argtypes = [vp, C.POINTER(OracleParams), vp, vp, C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.c_uint64, vp, C.c_int]
        L.oracle_scene_trace.restype = C.c_int
        L.oracle_scene_explain.argtypes = [vp, C.POINTER(OracleParams), vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, vp,
                                           C.c_uint64, vp, C.c_float, C.c_uint32, vp, vp, C.c_int]
        L.oracle_scene_explain.restype = C.c_int
        L.oracle_eval_response.argtypes = [vp] * 5
        L.oracle_kernel_scale.argtypes = [C.c_float, C.c_float, C.c_uint32, C.c_float]
        L.oracle_kernel_scale.restype = C.c_float
        L.oracle_radiance_from_sh.argtypes = [C.c_uint32, vp, vp, vp]
        L.oracle_flag_eps.argtypes = [vp]
        L.oracle_flag_eps.restype = None
        _lib = L
    return _lib


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def default_params(**kw):
    p = OracleParams()
    p.aabb[:] = [-100.0, -100.0, -100.0, 100.0, 100.0, 100.0]
    p.min_transmittance = 0.001
    p.hit_min_gaussian_response = 0.0113
    p.sph_eval_degree = 3
    p.alpha_min = 0.0039215686275
    p.pixel_offset = 0.0
    p.alpha_init = 0.0
    p.tmin_inclusive = 0
    p.proxy_mode = 0
    p.drop_rejected = 0
    p.max_rounds = 0
    p.ray_dirs_layout = 0
    p.kernel_min_response = 0.0113
    p.kernel_opts = 0
    p.kernel_degree = 4.0
    p.perturb_ulps = 0
    p.flag_cond_ulps = COND_ULPS
    for k, v in kw.items():
        if k == "aabb":
            p.aabb[:] = list(v)
        else:
            setattr(p, k, v)
    return p


def enclose(splats, kernel_min_response=0.0113, opts=0, degree=4.0):
    """particlePrimitives.comp restated; returns dict(verts, tris, density, sh, src_index, m)."""
    n = splats["positions"].size // 3
    a = {k: np.ascontiguousarray(splats[k], np.float32) for k in
         ("positions", "rotation", "scale", "opacity", "f_dc", "f_rest")}
    verts = np.zeros(36 * max(n, 1), np.float32)
    tris = np.zeros(60 * max(n, 1), np.uint32)
    dens = np.zeros(12 * max(n, 1), np.float32)
    sh = np.zeros(48 * max(n, 1), np.float32)
    src = np.zeros(max(n, 1), np.uint32)
    cnt = np.zeros(1, np.uint32)
    rc = lib().oracle_enclose(_p(a["positions"]), _p(a["rotation"]), _p(a["scale"]), _p(a["opacity"]), _p(a["f_dc"]),
                              _p(a["f_rest"]), n, kernel_min_response, opts, degree, _p(verts), _p(tris), _p(dens),
                              _p(sh), _p(cnt), _p(src))
    assert rc == 0
    m = int(cnt[0])
    return {"m": m, "verts": verts[:36 * m], "tris": tris[:60 * m], "density": dens[:12 * m], "sh": sh[:48 * m],
            "src_index": src[:m]}


def render(enc, view_inv, proj_inv, width, height, ncams=1, params=None, subset=None, threads=0, ray_dirs=False,
           **kw):
    """Per-ray ray-march restated; returns dict(rgba32f, depth, stats[X, A, rounds], ray_dirs)."""
    p = params if params is not None else default_params(**kw)
    vi = np.ascontiguousarray(view_inv, np.float32).reshape(-1)
    pi = np.ascontiguousarray(proj_inv, np.float32).reshape(16)
    nr = width * height * ncams if subset is None else len(subset)
    sub = None if subset is None else np.ascontiguousarray(subset, np.uint64)
    rgba = np.zeros((nr, 4), np.float32)
    depth = np.zeros(nr, np.float32)
    stats = np.zeros((nr, 3), np.uint32)
    margin = np.zeros((nr, 4), np.float32)
    dirs = np.zeros((nr if subset is not None else width * height * ncams, 4), np.float32) if ray_dirs else None
    rc = lib().oracle_render(_p(enc["verts"]), _p(enc["tris"]), _p(enc["density"]), _p(enc["sh"]), enc["m"],
                             C.byref(p), _p(vi), _p(pi), width, height, ncams, _p(sub), 0 if sub is None else len(sub),
                             _p(rgba), _p(depth), _p(dirs), _p(stats), _p(margin), int(threads))
    assert rc == 0
    out = {"rgba32f": rgba, "depth": depth, "stats": stats, "margin": margin}
    if ray_dirs:
        out["ray_dirs"] = dirs
    if subset is None:
        out["rgba32f"] = rgba.reshape(ncams, height, width, 4)
        out["stats"] = stats.reshape(ncams, height, width, 3)
        out["depth"] = depth.reshape(ncams, height, width)
        out["margin"] = margin.reshape(ncams, height, width, 4)
    return out


def eval_response(density_rec, o, d):
    g = np.zeros(1, np.float32)
    a = np.zeros(1, np.float32)
    rec = np.ascontiguousarray(density_rec, np.float32)
    oo = np.ascontiguousarray(o, np.float32)
    dd = np.ascontiguousarray(d, np.float32)
    lib().oracle_eval_response(_p(rec), _p(oo), _p(dd), _p(g), _p(a))
    return float(g[0]), float(a[0])


def kernel_scale(density, min_response=0.0113, opts=0, degree=4.0):
    return float(lib().oracle_kernel_scale(density, min_response, opts, degree))


def radiance_from_sh(deg, sh48, d):
    out = np.zeros(3, np.float32)
    c = np.ascontiguousarray(sh48, np.float32)
    dd = np.ascontiguousarray(d, np.float32)
    lib().oracle_radiance_from_sh(deg, _p(c), _p(dd), _p(out))
    return out


class Scene:
    """Persistent oracle scene (BVH built once); render() times only the per-ray ray-march."""

    def __init__(self, enc, proxy_mode=1, kernel_min_response=0.0113, opts=0, degree=4.0):
        self.enc = enc  # keep arrays alive
        self.proxy_mode = proxy_mode
        self.kw = dict(kernel_min_response=kernel_min_response, kernel_opts=opts, kernel_degree=degree)
        self.h = lib().oracle_scene_create(_p(enc["verts"]) if proxy_mode == 0 else None,
                                           _p(enc["tris"]) if proxy_mode == 0 else None, _p(enc["density"]),
                                           _p(enc["sh"]), enc["m"], proxy_mode, kernel_min_response, opts, degree)
        assert self.h

    def close(self):
        if self.h:
            lib().oracle_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def render(self, view_inv, proj_inv, width, height, ncams=1, subset=None, threads=0, margin=False, **kw):
        p = default_params(proxy_mode=self.proxy_mode, **self.kw, **kw)
        vi = np.ascontiguousarray(view_inv, np.float32).reshape(-1)
        pi = np.ascontiguousarray(proj_inv, np.float32).reshape(16)
        nr = width * height * ncams if subset is None else len(subset)
        sub = None if subset is None else np.ascontiguousarray(subset, np.uint64)
        rgba = np.zeros((nr, 4), np.float32)
        stats = np.zeros((nr, 3), np.uint32)
        marg = np.zeros((nr, 4), np.float32) if margin else None
        rc = lib().oracle_scene_render(self.h, C.byref(p), _p(vi), _p(pi), width, height, ncams, _p(sub),
                                       0 if sub is None else len(sub), _p(rgba), None, None, _p(stats), _p(marg),
                                       int(threads))
        assert rc == 0, rc
        out = {"rgba32f": rgba, "stats": stats}
        if margin:
            out["margin"] = marg
        return out


    def explain(self, view_inv, proj_inv, width, height, rays, target_rgb, tol=1e-4, max_pairs=4096, ncams=1,
                threads=0, **kw):
        """Each ray re-marched with its flagged decisions taken the other way (oracle_scene_explain): the base march,
        each single variant, then pairs of variants of two different decisions, until one is within tol of target_rgb
        (n x 3, e.g. the GPU's values; max |d rgb|); without such an exact alternative, the one closest to within tol
        plus its own value bound (FLAG_VALUE_EPS in gvrt_oracle.cpp).  Returns dict(dist, kind (0 base, 1 single
        flip, 2 pair), variants, decisions, vbound, alt_rgba): a ray is explained when dist <= tol + vbound, exactly
        when dist <= tol."""
        p = default_params(proxy_mode=self.proxy_mode, **self.kw, **kw)
        vi = np.ascontiguousarray(view_inv, np.float32).reshape(-1)
        pi = np.ascontiguousarray(proj_inv, np.float32).reshape(16)
        r = np.ascontiguousarray(rays, np.uint64).reshape(-1)
        if len(r) == 0:
            z = np.zeros(0, np.float32)
            return {"dist": z, "kind": z.astype(np.int32), "variants": z.astype(np.int32),
                    "decisions": z.astype(np.int32), "vbound": z, "alt_rgba": np.zeros((0, 4), np.float32)}
        tg = np.ascontiguousarray(np.asarray(target_rgb, np.float32).reshape(-1, 4)[:, :3]
                                  if np.asarray(target_rgb).reshape(len(r), -1).shape[1] == 4
                                  else np.asarray(target_rgb, np.float32).reshape(-1, 3))
        out = np.zeros((len(r), 5), np.float32)
        alt = np.zeros((len(r), 4), np.float32)
        if len(r):
            rc = lib().oracle_scene_explain(self.h, C.byref(p), _p(vi), _p(pi), width, height, ncams, _p(r), len(r),
                                            _p(tg), float(tol), int(max_pairs), _p(out), _p(alt), int(threads))
            assert rc == 0, rc
        return {"dist": out[:, 0], "kind": out[:, 1].astype(np.int32), "variants": out[:, 2].astype(np.int32),
                "decisions": out[:, 3].astype(np.int32), "vbound": out[:, 4], "alt_rgba": alt}

    def trace(self, view_inv, proj_inv, width, height, ray, ncams=1, maxn=4096, **kw):
        """Processed crossings of one ray (debugging): array of (id, t, gres, galpha, T after, accepted, round)."""
        p = default_params(proxy_mode=self.proxy_mode, **self.kw, **kw)
        vi = np.ascontiguousarray(view_inv, np.float32).reshape(-1)
        pi = np.ascontiguousarray(proj_inv, np.float32).reshape(16)
        out = np.zeros((maxn, 7), np.float32)
        n = lib().oracle_scene_trace(self.h, C.byref(p), _p(vi), _p(pi), width, height, ncams, int(ray), _p(out), maxn)
        assert n >= 0, n
        return out[:min(n, maxn)]


# Parity accounting (see out_margin in gvrt_oracle.cpp): a ray is "on a threshold" when one of its composite
# decisions lies within its float uncertainty of the threshold: the larger of a fixed relative epsilon -- THR_EPS for
# the hit / alpha / transmittance thresholds, PAIR_EPS between consecutive accepted crossings in t, BOUND_EPS for a
# crossing at a round / buffer / termination boundary against its neighbour (or a bitwise tie at the exclusive tmin)
# -- and COND_ULPS ulps of the decision's own conditioning (a response of a particle far away in kernel units, a face
# crossed at grazing incidence).  The C oracle stores each margin normalised to its fixed epsilon (distance x eps /
# max(eps, uncertainty)), so the comparisons below are unchanged.  Only such rays may decide differently under a
# few-ulp different float evaluation (the GPU's v_exp / v_rsq / v_rcp and FMA contraction); every other ray must
# match.
THR_EPS = 1e-4
PAIR_EPS = 2e-6
BOUND_EPS = 1e-5
COND_ULPS = 6.0


def _margin_rows(margin):
    m = np.asarray(margin, np.float32)
    cols = m.shape[-1] if m.ndim > 1 and m.shape[-1] in (3, 4) else 4
    return m.reshape(-1, cols)


def ambiguous(margin):
    """Boolean mask of rays whose result legitimately depends on ulp-level float differences (margin columns
    0..2; fixtures written before the flip bound have only those three)."""
    m = _margin_rows(margin)
    return (m[:, 0] < THR_EPS) | (m[:, 1] < PAIR_EPS) | (m[:, 2] < BOUND_EPS)


def flip_bound(margin):
    """Per ray, the bound on |d rgb| that its flagged decisions allow (margin column 3, gvrt_oracle.cpp): the sum over
    flagged decisions of T x alpha moved, plus minTransmittance, times the largest radiance channel on the ray."""
    m = _margin_rows(margin)
    if m.shape[1] < 4:
        raise ValueError("margin without the flip-bound column (regenerate the fixture)")
    return m[:, 3]


def flag_eps():
    """The C oracle's flag thresholds (must equal THR_EPS, PAIR_EPS, BOUND_EPS, COND_ULPS)."""
    out = np.zeros(4, np.float32)
    lib().oracle_flag_eps(_p(out))
    return out
