"""SplitBLAS analogue (gvrt_accel_params.split_cells; SplitBLAS.cpp:91-186) on the GPU.

Splitting the proxies into grid-cell pieces changes the BVH, not the crossings: every crossing is
admitted by exactly one piece (the one whose cell holds the crossing point), so the image is the
unsplit image.  Tolerances: the k-buffer sees the same crossings in a different insertion order, so
only crossings whose t ties bitwise may composite in another order (float rounding of the sum) —
|d rgb| <= 1e-5 on all but 1e-4 of the pixels, accepted-hit counts equal on all but 1e-4.
"""
import numpy as np
import pytest

from test_gpu_parity import _cmp_images

pytestmark = pytest.mark.gpu


def _close(a, b, frac=1e-4):
    fa, fb = np.asarray(a).reshape(-1, 4), np.asarray(b).reshape(-1, 4)
    d = np.abs(fa[:, :3] - fb[:, :3]).max(axis=1)
    assert (d > 1e-5).mean() <= frac and d.max() <= 0.05, (int((d > 1e-5).sum()), float(d.max()))
    assert (fa[:, 3] != fb[:, 3]).mean() <= frac


@pytest.mark.parametrize("cells", [1, 3, 10, 40])
def test_split_config1_equals_unsplit(gv, O, config1, config1_enc, cells):
    W = H = 160
    vi, pi = gv.scene.config1_camera(W, H)
    with gv.Renderer(0) as r:
        m = r.prepare(config1)
        base = {mode: r.render(vi, pi, W, H, mode=mode, hit_counts=True) for mode in (0, 1)}
        r.set_stats(True)
        r.render(vi, pi, W, H, mode=gv.MODE_LITERAL)
        st0 = r.stats()
        r.build_accel(split_cells=cells)
        st = r.stats()
        assert st["bvh_leaves"] >= m and st["bvh_nodes"] > 0
        if cells >= 10:
            assert st["bvh_leaves"] > m  # some proxies straddle a cell boundary
        r.render(vi, pi, W, H, mode=gv.MODE_LITERAL)
        st1 = r.stats()
        r.set_stats(False)
        for mode in (0, 1):
            out = r.render(vi, pi, W, H, mode=mode, hit_counts=True)
            _close(out["rgba32f"], base[mode]["rgba32f"])
            assert (out["hit_counts"] != base[mode]["hit_counts"]).mean() <= 1e-4
    # each crossing found exactly once: the literal crossing / accepted counts are the unsplit ones
    for k in ("crossings", "accepted"):
        assert abs(int(st1[k]) - int(st0[k])) <= 1e-4 * st0[k] + 2, (k, st1[k], st0[k])
    ref = O.render(config1_enc, vi, pi, W, H, proxy_mode=1)
    _cmp_images(out["rgba32f"], ref)


@pytest.mark.parametrize("cells,span", [(40, 3), (40, 8), (10, 2)])
def test_split_min_span_equals_unsplit(gv, O, config1, config1_enc, cells, span):
    """Size-selective split (gvrt_accel_params.split_min_span): only proxies whose box overlaps at least `span` cells
    along one axis are split, the others stay one piece admitting every crossing -- fewer pieces than the
    reference's rule (span <= 2: every straddler, the same tree as split_min_span = 0), the same image."""
    W = H = 160
    vi, pi = gv.scene.config1_camera(W, H)
    with gv.Renderer(0) as r:
        m = r.prepare(config1)
        base = r.render(vi, pi, W, H, hit_counts=True)
        r.build_accel(split_cells=cells)
        every = r.stats()["bvh_leaves"]
        r.build_accel(split_cells=cells, split_min_span=span)
        some = r.stats()["bvh_leaves"]
        out = r.render(vi, pi, W, H, hit_counts=True)
        if span <= 2:
            assert some == every
        else:
            assert m < some < every
        _close(out["rgba32f"], base["rgba32f"])
        assert (out["hit_counts"] != base["hit_counts"]).mean() <= 1e-4
        with pytest.raises(gv.GvrtError):
            r.build_accel(split_cells=cells, split_min_span=1024)
    _cmp_images(out["rgba32f"], O.render(config1_enc, vi, pi, W, H, proxy_mode=1))


def test_split_without_pieces_is_the_unsplit_build(gv, config1):
    """A split that splits no proxy (split_min_span above every proxy's span) builds the unsplit tree: the same
    4-wide nodes word for word, no cell tests, the same frame."""
    W = H = 96
    vi, pi = gv.scene.config1_camera(W, H)
    with gv.Renderer(0) as r:
        m = r.prepare(config1, builder=2, collapse=1)
        tree = r.read_accel(1)
        img = r.render(vi, pi, W, H)["rgba32f"]
        r.build_accel(builder=2, collapse=1, split_cells=10, split_min_span=1023)
        assert r.stats()["bvh_leaves"] == m
        np.testing.assert_array_equal(r.read_accel(1), tree)
        np.testing.assert_array_equal(r.render(vi, pi, W, H)["rgba32f"], img)


def test_split_bicycle_vs_oracle(gv, O):
    splats = gv.scene.mipnerf_standin(1_000_000, seed=1)
    W, H = 1920, 1080
    vi, pi = gv.scene.mipnerf_camera(W, H)
    with gv.Renderer(0) as r:
        m = r.prepare(splats)
        base = r.render(vi, pi, W, H)
        r.build_accel(split_cells=10)  # NUMBER_OF_CELLS_PER_LONGEST_AXIS (base/Define.h:46)
        leaves = r.stats()["bvh_leaves"]
        out = r.render(vi, pi, W, H)
        again = r.render(vi, pi, W, H)
    assert m < leaves < 4 * m
    np.testing.assert_array_equal(out["rgba32f"], again["rgba32f"])
    diff = np.abs(out["rgba8"].astype(np.int32) - base["rgba8"].astype(np.int32))
    assert (diff.max(axis=-1) > 0).mean() <= 1e-4 and diff.max() <= 8, ((diff > 0).sum(), diff.max())
    e = O.enclose(splats)
    sub = np.arange(0, W * H, 997, dtype=np.uint64)
    ref = O.render(e, vi, pi, W, H, proxy_mode=1, subset=sub)
    _cmp_images(out["rgba32f"].reshape(-1, 4)[sub.astype(np.int64)], ref)


def test_split_tiny_scenes_and_limits(gv, O):
    W = H = 48
    vi, pi = gv.scene.config1_camera(W, H)
    with gv.Renderer(0) as r:
        for n in (2, 7, 64):
            r.prepare(gv.scene.config1(n=n, seed=n), split_cells=10)
            out = r.render(vi, pi, W, H)
            r.build_accel()
            _close(out["rgba32f"], r.render(vi, pi, W, H)["rgba32f"], frac=0.0)
        # one Gaussian = the whole scene: its proxy spans every cell (10 x 10 x 10 pieces); the
        # rays through its centre cross two pieces, each admitting one of the two crossings
        one = {"positions": np.zeros(3, np.float32), "f_dc": np.array([0.3, -0.2, 0.1], np.float32),
               "f_rest": np.zeros(45, np.float32), "opacity": np.array([0.5], np.float32),
               "scale": np.log(np.full(3, 0.2, np.float32)), "rotation": np.array([1, 0, 0, 0], np.float32)}
        assert r.prepare(one, split_cells=10) == 1
        assert 1000 <= r.stats()["bvh_leaves"] <= 1331
        vi1, pi1 = gv.camera.pinhole((0.0, 0.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 10.0, 1.0)
        a = r.render(vi1, pi1, 31, 31, pixel_offset=0.5)["rgba32f"]
        r.build_accel()
        b = r.render(vi1, pi1, 31, 31, pixel_offset=0.5)["rgba32f"]
        np.testing.assert_array_equal(a, b)
        assert a[0, 15, 15, 3] == 2.0
        # no survivors
        s = gv.scene.config1(n=8, seed=3)
        s["f_dc"][:] = 5.0
        assert r.prepare(s, split_cells=10) == 0
        assert (r.render(vi, pi, 16, 16)["rgba32f"] == 0).all()
        r.prepare(gv.scene.config1(n=16, seed=1))
        with pytest.raises(gv.GvrtError):
            r.build_accel(split_cells=1024)
        with pytest.raises(gv.GvrtError):
            r.build_accel(builder=4)


@pytest.mark.parametrize("split", [0, 10])
def test_sah_optimal_collapse_same_image(gv, O, config1, config1_enc, split):
    """gvrt_accel_params.collapse = 1 (surface-area-optimal 4-wide collapse) changes only the tree: the
    image and the literal crossing counts are those of the greedy collapse (same tolerances as above)."""
    W = H = 160
    vi, pi = gv.scene.config1_camera(W, H)
    with gv.Renderer(0) as r:
        r.prepare(config1, split_cells=split)
        base = {mode: r.render(vi, pi, W, H, mode=mode, hit_counts=True) for mode in (0, 1)}
        nodes0 = r.stats()["bvh_nodes"]
        r.set_stats(True)
        r.render(vi, pi, W, H, mode=gv.MODE_LITERAL)
        st0 = r.stats()
        r.build_accel(split_cells=split, collapse=1)
        st = r.stats()
        assert st["bvh_nodes"] > 0 and st["bvh_depth"] == st0["bvh_depth"]
        r.render(vi, pi, W, H, mode=gv.MODE_LITERAL)
        st1 = r.stats()
        r.set_stats(False)
        for mode in (0, 1):
            out = r.render(vi, pi, W, H, mode=mode, hit_counts=True)
            _close(out["rgba32f"], base[mode]["rgba32f"])
        with pytest.raises(RuntimeError):
            r.build_accel(collapse=2)
    for k in ("crossings", "accepted"):
        assert abs(int(st1[k]) - int(st0[k])) <= 1e-4 * st0[k] + 2, (k, st1[k], st0[k])
    assert nodes0 > 0


@pytest.mark.parametrize("split,collapse", [(0, 0), (0, 1), (10, 1)])
def test_sah_builder_same_image(gv, O, config1, config1_enc, split, collapse):
    """gvrt_accel_params.builder = 2 (host binned-SAH binary tree) changes only the tree: same image and
    literal counters as the LBVH build, and the same image vs the oracle; deterministic across builds."""
    W = H = 160
    vi, pi = gv.scene.config1_camera(W, H)
    with gv.Renderer(0) as r:
        r.prepare(config1, split_cells=split)
        base = {mode: r.render(vi, pi, W, H, mode=mode)["rgba32f"] for mode in (0, 1)}
        r.set_stats(True)
        r.render(vi, pi, W, H, mode=gv.MODE_LITERAL)
        st0 = r.stats()
        r.build_accel(split_cells=split, builder=2, collapse=collapse)
        r.render(vi, pi, W, H, mode=gv.MODE_LITERAL)
        st1 = r.stats()
        r.set_stats(False)
        outs = {mode: r.render(vi, pi, W, H, mode=mode)["rgba32f"] for mode in (0, 1)}
        r.build_accel(split_cells=split, builder=2, collapse=collapse)
        again = r.render(vi, pi, W, H)["rgba32f"]
    for mode in (0, 1):
        _close(outs[mode], base[mode])
    np.testing.assert_array_equal(again, outs[0])
    for k in ("crossings", "accepted"):
        assert abs(int(st1[k]) - int(st0[k])) <= 1e-4 * st0[k] + 2, (k, st1[k], st0[k])
    if split == 0:
        ref = O.render(config1_enc, vi, pi, W, H, proxy_mode=1)
        d = np.abs(outs[0].reshape(-1, 4)[:, :3] - ref["rgba32f"].reshape(-1, 4)[:, :3]).max(axis=1)
        assert (d > 2e-3).mean() <= 1e-3 and d.max() <= 0.05
