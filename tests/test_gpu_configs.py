"""Full-size SURVEY §8d configurations 3-5 and the dense stand-in on the GPU: size-independent properties plus
the oracle over every ray of the frame (garden 2.07 M rays, truck 4K 8.29 M, the 16-view light field 33.2 M; round 5,
VERDICT r04 #1) or, for the dense stand-in, every 2nd ray (1.04 M: its ~10 LITERAL rounds of ~150 crossings per ray
cost the oracle ~10 min per whole frame on the GPU box's 16 threads).  The oracle restates the reference's loop per
ray, so a strided sample is a valid sample.  Tolerances and the on-threshold accounting as in test_gpu_parity.py
(every unflagged ray within 1e-4, every flagged ray within its flip bound, and -- round 6, VERDICT r05 #1 -- every
flagged ray that differs by more than 1e-4 equal to the oracle's re-march of that ray with some of its flagged
decisions taken the other way, test_gpu_parity.explain_flagged); the on-threshold caps sit just above the
measured fractions (the flags are the CPU oracle's, so the fraction is the same on every box); tile / view splits are
checked bit for bit.

  * config 3 "garden": 3 M Gaussians, 1920x1080
  * config 4 "truck":  2 M Gaussians, 3840x2160, image split in 64x64 blocks over 8 simulated ranks
  * config 5 light field: 1 M Gaussians, 4x4 camera grid, 16 views of 1920x1080 in one call
"""
import numpy as np
import pytest

from test_gpu_parity import _cmp_images, assert_explained, explain_flagged, parity_figures, record_parity

pytestmark = pytest.mark.gpu


def _scene(gv, name):
    gen, W, H, ncams = gv.scene.CONFIGS[name]
    return gv.scene.make(**gen), W, H, ncams


def _oracle_subset(O, splats, vi, pi, W, H, ncams=1, stride=1, offset=0):
    """The oracle on every stride-th ray of the frame(s) from `offset` (stride 1: all of them); the scene stays open
    for explain_flagged (the caller closes it)."""
    e = O.enclose(splats)
    sub = np.arange(offset, W * H * ncams, stride, dtype=np.uint64)
    sc = O.Scene(e)
    ref = sc.render(vi, pi, W, H, ncams=ncams, subset=None if stride == 1 else sub, margin=True)
    if stride == 1:
        ref = {k: v.reshape(len(sub), -1) for k, v in ref.items()}
    return e["m"], sub, ref, sc


def test_garden_3m(gv, O):
    splats, W, H, _ = _scene(gv, "garden")
    vi, pi = gv.scene.mipnerf_camera(W, H)
    with gv.Renderer(0) as r:
        m = r.prepare(splats)
        a = r.render(vi, pi, W, H)
        b = r.render(vi, pi, W, H)
        st = r.stats()
    assert m > 2_700_000 and st["bvh_nodes"] > 0
    np.testing.assert_array_equal(a["rgba32f"], b["rgba32f"])  # deterministic
    assert (a["rgba32f"][..., 3] > 0).mean() > 0.5  # the object and the shell cover the frame
    m_ref, sub, ref, sc = _oracle_subset(O, splats, vi, pi, W, H)  # all 2 073 600 rays
    assert m_ref == m
    got = a["rgba32f"].reshape(-1, 4)[sub.astype(np.int64)]
    try:
        _cmp_images(got, ref, amb_max=0.0097)  # measured 0.924 % flagged
        ex = explain_flagged(O, sc, vi, pi, W, H, got, ref, rays=sub)
    finally:
        sc.close()
    record_parity("garden", **parity_figures(O, gv, got, ref), **ex)
    assert_explained(ex)


@pytest.mark.timeout(900)
def test_truck_4k_tile_split(gv, O):
    """Config 4 split over 8 simulated ranks in both layouts: the 64x64-block round-robin, and the cost bands the
    bench and SplitFrame ship (calibration renders, gvrt_read_tile_costs, dist.band_tiles over
    dist.cost_weights, each rank's part rendered tile-packed and unpacked): both assemble the full frame bit for
    bit."""
    torch = pytest.importorskip("torch")
    import importlib
    dist = importlib.import_module("3dgvrt_lightfield_amd.dist")
    splats, W, H, _ = _scene(gv, "truck")
    vi, pi = gv.scene.mipnerf_camera(W, H)
    world = 8
    with gv.Renderer(0) as r:
        r.prepare(splats)
        full = r.render(vi, pi, W, H)
        # the full frame's per-tile cost classes, from a second (cost-ordered) launch, as the bench calibrates
        full2 = r.render(vi, pi, W, H, rgba32f=False)
        classes = r.tile_costs(W, H)
        np.testing.assert_array_equal(full2["rgba8"], full["rgba8"])
        layouts = {"blocks": [gv.tiles_for_rank(W, H, 1, k, world, block=8) for k in range(world)],
                   "cost-bands": dist.band_tiles(W, H, world, costs=dist.cost_weights(classes))}
        for name, parts in layouts.items():
            frame = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
            covered = 0
            for t in parts:  # rendered rank by rank, as each rank would
                covered += len(t)
                part = r.render(vi, pi, W, H, tiles=t, packed=True, rgba32f=False)["rgba8"]
                dev = torch.from_numpy(part).cuda()
                r.unpack_tiles_rgba8(dev.data_ptr(), t, W, H, frame.data_ptr())
            torch.cuda.synchronize()
            assert covered == ((W + 7) // 8) * ((H + 7) // 8), name
            np.testing.assert_array_equal(frame.cpu().numpy(), full["rgba8"][0], err_msg=name)
        sizes = [len(t) for t in layouts["cost-bands"]]
        assert max(sizes) != min(sizes)  # cost bands: unequal tile counts (equal cost)
    _, sub, ref, sc = _oracle_subset(O, splats, vi, pi, W, H)  # all 8 294 400 rays
    got = full["rgba32f"].reshape(-1, 4)
    del full
    try:
        _cmp_images(got, ref, amb_max=0.0190)  # 1.595 % of the 8.29 M rays flagged (round 5), + ill-conditioned values
        ex = explain_flagged(O, sc, vi, pi, W, H, got, ref, rays=sub)
    finally:
        sc.close()
    record_parity("truck_4k", **parity_figures(O, gv, got, ref), **ex)
    assert_explained(ex)


@pytest.mark.timeout(900)
def test_lightfield_grid_16_views(gv, O):
    splats, W, H, ncams = _scene(gv, "lightfield")
    assert ncams == 16
    vi, pi = gv.camera.lightfield_grid_rig(gv.camera.orbit_eye(4.0, 20.0, 90.0), (0.0, 0.0, 0.0), nx=4, ny=4,
                                           spacing=0.1, aspect=gv.camera.aspect_ratio(W, H))
    with gv.Renderer(0) as r:
        r.prepare(splats)
        batch = r.render(vi, pi, W, H, ncams=ncams, ray_dirs=True, ray_dirs_layout=1, rgba8=False)
        singles = [r.render(vi[16 * c:16 * (c + 1)], pi, W, H, rgba8=False)["rgba32f"][0] for c in (0, 5, 15)]
    img = batch["rgba32f"]
    assert img.shape == (ncams, H, W, 4)
    for c, s in zip((0, 5, 15), singles):  # one batched launch == per-view launches, bit for bit
        np.testing.assert_array_equal(img[c], s)
    d = batch["ray_dirs"].reshape(ncams, W, H, 4)  # light-field layout [cam][x][y]
    np.testing.assert_allclose(np.linalg.norm(d[..., :3], axis=-1), 1.0, atol=2e-6)
    # neighbouring views see (slightly) different images
    assert np.abs(img[0] - img[15]).max() > 0.01
    del batch, singles, d
    _, sub, ref, sc = _oracle_subset(O, splats, vi, pi, W, H, ncams=ncams)  # all 33 177 600 rays
    got = img.reshape(-1, 4)
    try:
        _cmp_images(got, ref, amb_max=0.0195)  # 1.539 % of the 33.2 M rays flagged (round 5), + ill-conditioned values
        ex = explain_flagged(O, sc, vi, pi, W, H, got, ref, rays=sub, ncams=ncams)
    finally:
        sc.close()
    record_parity("lightfield_16", **parity_figures(O, gv, got, ref), **ex)
    assert_explained(ex)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("half", [0, 1])
def test_dense_standin(gv, O, half):
    """The dense stand-in (scene.dense_standin: ~150 crossings, ~79 accepted, ~10 LITERAL rounds per ray):
    FAST and LITERAL vs the oracle on every 2nd ray of the 1080p frame (1.04 M rays; the oracle's ~10 LITERAL
    rounds of ~150 crossings per ray make the whole frame take ~10 min on the GPU box's 16 threads, too long for
    one test), in two tests of every 4th ray (offsets 0 and 2, ~85 s each), FAST's accepted-hit counts vs the
    oracle's on every off-threshold ray."""
    splats, W, H, _ = _scene(gv, "dense")
    vi, pi = gv.scene.mipnerf_camera(W, H)
    with gv.Renderer(0) as r:
        m = r.prepare(splats, **gv.QUALITY_BUILD)  # the bench's build: its largest proxies split into cell pieces
        assert r.stats()["bvh_leaves"] > m
        fast = r.render(vi, pi, W, H, hit_counts=True)
        lit = r.render(vi, pi, W, H, mode=gv.MODE_LITERAL)
    m_ref, sub, ref, sc = _oracle_subset(O, splats, vi, pi, W, H, stride=4, offset=2 * half)
    assert m_ref == m
    st = ref["stats"].reshape(-1, 3)
    assert st[:, 0].mean() > 140, st.mean(axis=0)  # the workload is what it claims to be
    idx = sub.astype(np.int64)
    # ~150 crossings and ~10 round boundaries per ray: 7.8 % of the rays carry a decision within the
    # on-threshold margins (measured on a 1/64 sample); each of them is bounded by its flip bound,
    # every other ray must match as everywhere else
    try:
        _cmp_images(fast["rgba32f"].reshape(-1, 4)[idx], ref, amb_max=0.085)  # ~7.9 % of the sample flagged
        _cmp_images(lit["rgba32f"].reshape(-1, 4)[idx], ref, amb_max=0.085)
        amb = O.ambiguous(ref["margin"])
        assert (fast["hit_counts"].reshape(-1)[idx] != st[:, 1])[~amb].sum() == 0
        ex = explain_flagged(O, sc, vi, pi, W, H, fast["rgba32f"].reshape(-1, 4)[idx], ref, rays=sub)
        ex_lit = explain_flagged(O, sc, vi, pi, W, H, lit["rgba32f"].reshape(-1, 4)[idx], ref, rays=sub)
    finally:
        sc.close()
    record_parity("dense" if half == 0 else "dense_b", stride=4, offset=2 * half,
                  **parity_figures(O, gv, fast["rgba32f"].reshape(-1, 4)[idx], ref), **ex, literal=ex_lit)
    assert_explained(ex)
    assert_explained(ex_lit)
