"""The robustness stand-ins of round 6, on the CPU: what they claim to be.

  * scene.trained_standin: surfel / needle anisotropy along surface normals, heavy-tailed sizes, 0.1 % giants,
    bimodal opacity (the shape of a trained 3DGRT scene, base/Vulkan3DGRTModel.cpp:7-125 loads such PLYs);
  * scene.morton_chain: a clustered scene whose Karras LBVH + greedy 4-wide collapse (the C-ABI's default build,
    csrc/gvrt_lbvh.hip) is deeper than the render kernel's 128-entry traversal stack allows (42 4-wide levels).
    Before round 6 gvrt_build_accel refused it (GVRT_ERR_UNSUPPORTED); the restatement below (the oracle's
    enclosing records -> proxy boxes as gvrt_enclose.hip pads them -> 63-bit Morton codes as k_morton -> the
    radix hierarchy of sorted (code, index) keys -> the greedy largest-area collapse of k_collapse_level) shows the
    depth the device build meets, and tests/test_gpu_deep.py checks that the library now rebuilds it with the
    depth-bounded SAH build and renders it.
"""
import math
import sys

import numpy as np


def test_trained_standin_shape(gv):
    s = gv.scene.trained_standin(n=200_000, seed=5)
    n = 200_000
    ls = s["scale"].reshape(n, 3)
    srt = np.sort(ls, axis=1)
    thin1 = srt[:, 1] - srt[:, 0] > math.log(10.0)  # one axis at least 10x below the others: surfel
    assert 0.45 < thin1.mean() < 0.85, thin1.mean()
    big = ls.max(axis=1) > math.log(0.5)  # the giants only (scale 1-5 units, per-axis noise)
    assert abs(big.sum() - 0.001 * n) <= 0.0002 * n, big.sum()
    assert ls[~big].max() <= math.log(0.3) + 1e-5  # (float32 of the clip)
    spread = ls[~big].max(axis=1)
    assert np.percentile(spread, 99) - np.percentile(spread, 1) > 6.0  # heavy-tailed: > e^6 between 1 % and 99 %
    op = s["opacity"]
    assert (op < -2.0).mean() > 0.3 and (op > 1.5).mean() > 0.5  # bimodal
    # deterministic in the seed
    t = gv.scene.trained_standin(n=200_000, seed=5)
    for k in s:
        np.testing.assert_array_equal(s[k], t[k])


def _morton_greedy_depths(gv, O):
    e = O.enclose(gv.scene.morton_chain())
    dens = e["density"].reshape(-1, 12).astype(np.float64)
    m = len(dens)
    pos, q, scl = dens[:, :3], dens[:, 4:8], dens[:, 8:11]
    w, x, y, z = q.T
    R = np.stack([np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)], -1),
                  np.stack([2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)], -1),
                  np.stack([2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1)], 1)
    rc = 2.997154714 * 0.6615845382 * math.sqrt(1 + 1.618033988749895 ** 2)  # kS x icosahedron circumradius
    ext = (np.abs(R) * scl[:, None, :]).sum(2) * rc
    pad = 2e-5 * ext + 1e-6 * np.abs(pos) + 2.0 ** -18 * np.abs(pos).max()
    lo, hi = pos - ext - pad, pos + ext + pad
    cen = 0.5 * (lo + hi)
    cl, ch = cen.min(0), cen.max(0)
    u = np.clip((cen - cl) / (ch - cl) * 2097152.0, 0, 2097151).astype(np.uint64)

    def expand(v):
        out = np.zeros_like(v)
        for b in range(21):
            out |= ((v >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b)
        return out

    code = (expand(u[:, 0]) << np.uint64(2)) | (expand(u[:, 1]) << np.uint64(1)) | expand(u[:, 2])
    order = np.lexsort((np.arange(m), code))
    keys = [(int(c) << 32) | i for i, c in enumerate(code[order])]
    lo, hi = lo[order], hi[order]
    sys.setrecursionlimit(20000)

    def build(i, j):  # radix hierarchy: split at the highest differing bit of the range's first and last key
        if i == j:
            return (i,)
        b = (keys[i] ^ keys[j]).bit_length() - 1
        k = i
        while k < j and ((keys[k + 1] >> b) & 1) == ((keys[i] >> b) & 1):
            k += 1
        return (build(i, k), build(k + 1, j))

    boxes = {}

    def box(n):
        if id(n) not in boxes:
            if len(n) == 1:
                boxes[id(n)] = (lo[n[0]], hi[n[0]])
            else:
                a, b = box(n[0]), box(n[1])
                boxes[id(n)] = (np.minimum(a[0], b[0]), np.maximum(a[1], b[1]))
        return boxes[id(n)]

    def area(n):
        e = box(n)[1] - box(n)[0]
        return e[0] * e[1] + e[1] * e[2] + e[2] * e[0]

    def depth2(n):
        return 1 if len(n) == 1 else 1 + max(depth2(n[0]), depth2(n[1]))

    def depth4(n):  # k_collapse_level: open the largest-area inner child until 4 children
        kids = [n[0], n[1]]
        while len(kids) < 4:
            inner = [j for j, c in enumerate(kids) if len(c) == 2]
            if not inner:
                break
            j = max(inner, key=lambda j: (area(kids[j]), -j))
            kids[j:j + 1] = [kids[j][0], kids[j][1]]
        return 1 + max([depth4(c) for c in kids if len(c) == 2], default=0)

    root = build(0, m - 1)
    return depth2(root), depth4(root)


def test_morton_chain_exceeds_the_stack(gv, O):
    d2, d4 = _morton_greedy_depths(gv, O)
    # 3 x 42 + 2 = 128 stack entries: a greedy 4-wide tree of more than 42 levels was refused before round 6
    assert d4 > 42 and d2 > 43, (d2, d4)
