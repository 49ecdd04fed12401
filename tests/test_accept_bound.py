"""The acceptance-box bound behind GVRT_OPT_ACCEPT_BOXES (gvrt_render.hip k_accept_leaf), checked in float64.

FAST launches admit only accepted crossings.  A crossing of particle P is accepted when gres > m with
m = max(hitMinGaussianResponse, alphaMin / density) (gaussianfunctions.glsl:192-200, particleResponse of degree 4:
gres = exp(S d^4), d the line's distance from P's centre in the kernel frame), so the ray's line passes through the
ball E of radius r = (ln m / S)^(1/4).  The all-leaf nodes of the FAST node copy bound E instead of the
icosahedron proxy and widen the ray's t-range by D = s_max sqrt(Rc^2 - r^2) (Rc: the proxy's circumradius).  This
restates the geometry independently of the kernel: for every accepted particle the entry and exit crossings of the
icosahedron (the 10 slab pairs of the render kernel's ico_clip) lie within D of E's chord along the ray, and never-
accepted particles (density <= alphaMin) have no accepted ray.  No GPU: the render-side check is
tests/test_gpu_parity.py::test_tuning_options_change_no_pixel (the frame with the option off is bit-identical).
"""
import math

import numpy as np
import pytest

S = -0.0555555555556  # KERNEL_S, gaussianfunctions.glsl:31-35 (degree 4)
PHI = (1 + 5 ** 0.5) / 2
IPHI = PHI - 1
RC = 1.2584086  # icosahedron circumradius / inradius
# slab normals of ico_clip (each of norm sqrt(3), half-width sqrt(3) kS)
NORMALS = np.array([[1, 1, 1], [1, 1, -1], [1, -1, 1], [-1, 1, 1], [0, PHI, IPHI], [0, PHI, -IPHI],
                    [IPHI, 0, PHI], [-IPHI, 0, PHI], [PHI, IPHI, 0], [PHI, -IPHI, 0]], dtype=np.float64)


def kernel_scale(density, kmin, adaptive):
    """particlePrimitives.comp:81-105, degree 4 (gvrt_device.h kernel_scale)."""
    mr = np.minimum(kmin / (density if adaptive else 1.0), 0.97)
    return (np.log(mr) / S) ** 0.25


def quat_rows(q):
    q = q / np.linalg.norm(q, axis=1, keepdims=True)
    w, x, y, z = q.T
    r0 = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y + w * z), 2 * (x * z - w * y)], 1)
    r1 = np.stack([2 * (x * y - w * z), 1 - 2 * (x * x + z * z), 2 * (y * z + w * x)], 1)
    r2 = np.stack([2 * (x * z + w * y), 2 * (y * z - w * x), 1 - 2 * (x * x + y * y)], 1)
    return np.stack([r0, r1, r2], 2)  # R[:, i, j] = column j, component i (world = p + R diag(s) x_k)


@pytest.mark.parametrize("min_response,alpha_min,adaptive", [(0.0113, 1 / 255, False), (0.0113, 1 / 255, True),
                                                             (0.005, 1 / 255, False), (0.0113, 0.05, False)])
def test_admitted_crossings_lie_within_d_of_the_acceptance_chord(min_response, alpha_min, adaptive):
    rng = np.random.default_rng(7)
    n = 200_000
    R = quat_rows(rng.normal(size=(n, 4)))
    s = np.exp(rng.uniform(np.log(0.01), np.log(0.2), (n, 3)))
    rho = 1 / (1 + np.exp(-rng.normal(-1.0, 3.0, n)))
    # rays from points around the particle (centre at 0), aimed near it
    o = rng.normal(size=(n, 3))
    o *= (rng.uniform(0.5, 3.0, n) / np.linalg.norm(o, axis=1))[:, None]
    tgt = rng.normal(scale=0.25, size=(n, 3)) * s.max(axis=1, keepdims=True)
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    # kernel frame (kernel_org / kernel_dir): x_k = diag(1/s) R^T x
    ok = np.einsum("nji,nj->ni", R, o) / s
    dk = np.einsum("nji,nj->ni", R, d) / s
    g = dk / np.linalg.norm(dk, axis=1, keepdims=True)
    gd = (np.cross(g, ok) ** 2).sum(1)  # squared line distance
    gres = np.exp(S * gd * gd)
    acc = (gres > min_response) & (np.minimum(0.99, gres * rho) > alpha_min)
    assert acc.sum() > 5000
    assert not acc[rho <= alpha_min].any()  # dropped leaves: never accepted
    # ico_clip: slab |n . x| <= sqrt(3) kS
    ks = np.broadcast_to(kernel_scale(rho, 0.0113, adaptive), rho.shape)
    hk = math.sqrt(3) * ks
    sa = ok @ NORMALS.T
    sb = dk @ NORMALS.T
    with np.errstate(divide="ignore"):
        ib = 1 / sb
    lo = np.max(np.minimum((-sa - hk[:, None]) * ib, (-sa + hk[:, None]) * ib), axis=1)
    hi = np.min(np.maximum((-sa - hk[:, None]) * ib, (-sa + hk[:, None]) * ib), axis=1)
    hit = acc & (lo <= hi)
    assert hit.sum() > 5000
    # E's chord along the ray (t is world distance: |d| = 1)
    m = np.maximum(min_response, alpha_min / rho)
    r = (np.log(np.minimum(m, 1.0)) / S) ** 0.25  # m >= 1: never accepted, r = 0
    l2 = (dk * dk).sum(1)
    tstar = -(ok * dk).sum(1) / l2
    half = np.sqrt(np.maximum(r * r - gd, 0.0) / l2)
    e0, e1 = tstar - half, tstar + half
    D = s.max(axis=1) * np.sqrt(np.maximum((RC * ks) ** 2 - r * r, 0.0))
    for t in (lo, hi):
        gap = np.maximum(e0 - t, 0.0) + np.maximum(t - e1, 0.0)
        assert np.all(gap[hit] <= D[hit] * (1 + 1e-9) + 1e-12), float((gap - D)[hit].max())
    # the bound is not loose by orders of magnitude: some accepted crossing's gap exceeds half of its D
    gap_lo = np.maximum(e0 - lo, 0.0)
    assert np.any(gap_lo[hit] > 0.5 * D[hit])
