"""C-ABI argument checking and the size limits of gvrt_render (include/gvrt.h), through libgvrt.so.

Error behaviour follows the reference's VK_CHECK_RESULT policy moved to the caller: every refused call
returns a status (GvrtError here) and leaves the handle usable.  Limits: 32768 pixels per side, 255
cameras per launch (tile words carry the camera in 8 bits).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cmp(a, b, frac_tol=1e-3, tol=2e-3, max_tol=0.05):
    a = np.asarray(a, np.float64).reshape(-1, 4)
    b = np.asarray(b, np.float64).reshape(-1, 4)
    d = np.abs(a[:, :3] - b[:, :3]).max(axis=1)
    assert (d > tol).mean() <= frac_tol and d.max() <= max_tol, (float((d > tol).mean()), float(d.max()))
    assert (a[:, 3] != b[:, 3]).mean() <= frac_tol


def test_refused_calls_leave_the_handle_usable(gv, config1):
    W = H = 16
    vi, pi = gv.scene.config1_camera(W, H)
    with gv.Renderer(0) as r:
        with pytest.raises(gv.GvrtError):  # no acceleration structure yet
            r.render(vi, pi, W, H)
        r.prepare(config1)
        good = r.render(vi, pi, W, H)["rgba32f"]
        bad = [
            dict(width=0),
            dict(width=32769),
            dict(height=40000),
            dict(kbuffer_depth=7),
            dict(mode=5),
            dict(tmin_inclusive=1),                                   # FAST mode
            dict(tmin_inclusive=1, mode=gv.MODE_LITERAL, max_rounds=0),  # would never terminate
        ]
        for kw in bad:
            w, h = kw.pop("width", W), kw.pop("height", H)
            with pytest.raises(gv.GvrtError):
                r.render(vi, pi, w, h, **kw)
        with pytest.raises(gv.GvrtError):  # tile outside the image
            r.render(vi, pi, W, H, tiles=[(0, 5, 0, 0)])
        with pytest.raises(gv.GvrtError):  # packed output without a tile list
            r.render(vi, pi, W, H, packed=True)
        with pytest.raises(gv.GvrtError):  # 256 cameras
            r.render(np.tile(np.asarray(vi, np.float32), 256), pi, 8, 8, ncams=256)
        np.testing.assert_array_equal(r.render(vi, pi, W, H)["rgba32f"], good)


def test_inclusive_tmin_with_round_cap_vs_oracle(renderer, gv, O, config1, config1_enc):
    """LITERAL + tmin_inclusive (+ the ITERATIONS cap it needs): the variant the reference gets when its
    tmin comparison is inclusive; the HIP path and the oracle agree on image and counters."""
    renderer.prepare(config1)
    W = H = 48
    vi, pi = gv.scene.config1_camera(W, H)
    kw = dict(tmin_inclusive=1, max_rounds=6)
    out = renderer.render(vi, pi, W, H, mode=gv.MODE_LITERAL, **kw)
    ref = O.render(config1_enc, vi, pi, W, H, proxy_mode=1, **kw)
    _cmp(out["rgba32f"], ref["rgba32f"])


def test_255_cameras_in_one_launch(renderer, gv, config1):
    """The largest batch: 255 ring cameras in one launch equal the same cameras rendered one by one."""
    renderer.prepare(config1)
    W = H = 8
    n = 255
    vi, pi = gv.camera.lightfield_ring_rig(config1["positions"], n, W, H)
    vi = np.asarray(vi, np.float32).reshape(n, 16)
    batch = renderer.render(vi, pi, W, H, ncams=n, pixel_offset=0.5, alpha_init=1.0)["rgba32f"]
    assert batch.shape[0] == n
    for c in (0, 1, 127, 200, 254):
        one = renderer.render(vi[c], pi, W, H, pixel_offset=0.5, alpha_init=1.0)["rgba32f"][0]
        np.testing.assert_array_equal(batch[c], one)


def test_widest_image_vs_oracle(renderer, gv, O, config1, config1_enc):
    """32768 x 8 (the width limit): ragged tiles at neither edge, a 4096-tile row; vs the oracle."""
    renderer.prepare(config1)
    W, H = 32768, 8
    vi, pi = gv.camera.pinhole((0.0, 0.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 2.0, W / H)
    out = renderer.render(vi, pi, W, H)
    ref = O.render(config1_enc, vi, pi, W, H, proxy_mode=1)
    _cmp(out["rgba32f"], ref["rgba32f"])
