"""C-ABI argument checking and the size limits of gvrt_render (include/gvrt.h), through libgvrt.so.

Error behaviour follows the reference's VK_CHECK_RESULT policy moved to the caller: every refused call
returns a status (GvrtError here) and leaves the handle usable.  Limits: 32768 pixels per side, 255
cameras per launch (tile words carry the camera in 8 bits).
"""
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


from test_gpu_parity import _cmp_images as _cmp  # noqa: E402  (on-threshold accounting, test_gpu_parity.py)


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
    _cmp(out["rgba32f"], ref)


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
    _cmp(out["rgba32f"], ref)


def test_device_properties_and_buffers(gv, config1):
    """gvrt_get_device_properties (vks::Benchmark's deviceName / driverVersion) and gvrt_get_device_buffers
    (Model::Attributes storage buffers + enclosing outputs)."""
    import torch
    p = gv.device_properties(0)
    assert p["device_name"] and p["compute_units"] > 0 and p["total_memory"] > 0 and p["arch_name"].startswith("gfx")
    n = config1["positions"].size // 3
    with gv.Renderer(0) as r:
        b = r.device_buffers()
        assert b["n"] == 0 and not b["positions"] and not b["particle_density"]
        r.load_splats(config1)
        b = r.device_buffers()
        assert b["n"] == n and all(b[k] for k in ("positions", "rotations", "scales", "densities", "features_albedo",
                                                   "features_specular"))
        assert b["m"] == 0 and not b["vertices"]
        m = r.build_enclosing(emit_triangles=1)
        b = r.device_buffers()
        assert b["m"] == m and b["vertices"] and b["indices"] and b["particle_density"] and b["particle_sph"]
        # the device copy of the positions is the SplatSet's (read through a torch view of the pointer)
        host = torch.empty(3 * n, dtype=torch.float32)
        dev = torch.empty(3 * n, dtype=torch.float32, device="cuda")
        import ctypes
        torch.cuda.synchronize()
        hip = ctypes.CDLL("libamdhip64.so")
        assert hip.hipMemcpy(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(b["positions"]),
                             ctypes.c_size_t(12 * n), 3) == 0  # hipMemcpyDeviceToDevice
        host.copy_(dev.cpu())
        np.testing.assert_array_equal(host.numpy(), config1["positions"])


def test_failed_load_leaves_no_half_loaded_scene(gv, config1):
    """an allocation failure inside gvrt_load_splats must not leave mixed-size buffers; the
    next build then reports GVRT_ERR_STATE instead of launching on them.  1.6e9 splats need ~380 GB
    (f_rest alone 288 GB), beyond one MI355X; the first five buffers (~90 GB) do get allocated."""
    import ctypes as C
    from importlib import import_module
    L = import_module("3dgvrt_lightfield_amd._lib")
    tiny = np.zeros(64, np.float32)
    p = L.fptr(tiny)
    s = L.Splats(1_600_000_000, p, p, p, p, p, p)
    with gv.Renderer(0) as r:
        r.prepare(config1)
        st = gv.lib().gvrt_load_splats(r.h, C.byref(s))
        assert st == -2, st  # GVRT_ERR_OOM, before any copy from the (tiny) host arrays
        m = C.c_uint64(0)
        assert gv.lib().gvrt_build_enclosing(r.h, None, C.byref(m)) == -4  # GVRT_ERR_STATE
        assert r.device_buffers()["n"] == 0
        assert r.prepare(config1) > 0  # the handle stays usable


def test_unpack_tiles_rejects_tiles_outside_the_frame(gv, config1):
    import torch
    W, H = 40, 24
    with gv.Renderer(0) as r:
        packed = torch.zeros((64, 4), dtype=torch.uint8, device="cuda")
        frame = torch.zeros((2, H, W, 4), dtype=torch.uint8, device="cuda")
        for bad in ((5, 0, 0), (0, 3, 0), (0, 0, 2), (4095, 0, 0)):
            with pytest.raises(gv.GvrtError):
                r.unpack_tiles_rgba8(packed.data_ptr(), [(bad[0], bad[1], bad[2], 0)], W, H, frame.data_ptr(), ncams=2)
        packed.fill_(7)
        r.unpack_tiles_rgba8(packed.data_ptr(), [(4, 2, 1, 0)], W, H, frame.data_ptr(), ncams=2)
        f = frame.cpu().numpy()
        assert (f[1, 16:24, 32:40] == 7).all() and f.sum() == 7 * 64 * 4
        with pytest.raises(ValueError):  # short camera arrays are refused on the host side
            vi, pi = gv.scene.config1_camera(W, H)
            r.render_device(vi, pi, W, H, ncams=2, rgba8_ptr=frame.data_ptr())


def test_cost_ordered_dispatch_changes_no_pixel(gv, config1):
    """Cost-ordered dispatch (gvrt_api.hip: each launch records its tiles' cost classes, the next launch of the
    same frame size takes the tiles costliest first): the first launch (default order), the ordered ones after
    it, launches after a frame-size change, a multi-camera launch, and a tile-list launch (which keeps the
    caller's order) all give the same pixels, rgba8, hit counts and ray directions."""
    W, H = 72, 40  # 9 x 5 tiles
    vi, pi = gv.scene.config1_camera(W, H)
    with gv.Renderer(0) as r:
        r.prepare(config1)
        kw = dict(hit_counts=True, ray_dirs=True)
        first = r.render(vi, pi, W, H, **kw)
        for _ in range(3):
            again = r.render(vi, pi, W, H, **kw)
            for k in ("rgba32f", "rgba8", "hit_counts", "ray_dirs"):
                np.testing.assert_array_equal(again[k], first[k])
        other = r.render(vi, pi, 33, 17)  # a new frame size restarts from the default order
        np.testing.assert_array_equal(r.render(vi, pi, 33, 17)["rgba32f"], other["rgba32f"])
        np.testing.assert_array_equal(r.render(vi, pi, W, H)["rgba32f"], first["rgba32f"])
        # three cameras in one launch vs each alone
        vi3, pi3 = gv.camera.lightfield_grid_rig((0.0, 0.0, 3.0), (0.0, 0.0, 0.0), nx=3, ny=1, spacing=0.2,
                                                  aspect=gv.camera.aspect_ratio(W, H))
        multi = [r.render(vi3, pi3, W, H, ncams=3)["rgba32f"] for _ in range(3)]
        np.testing.assert_array_equal(multi[1], multi[0])
        np.testing.assert_array_equal(multi[2], multi[0])
        for cam in range(3):
            single = r.render(vi3[16 * cam:16 * (cam + 1)], pi3, W, H)["rgba32f"]
            np.testing.assert_array_equal(single[0], multi[0][cam])
        # a tile list keeps the caller's order and covers only its tiles
        t = np.asarray([(2, 1, 0, 0), (0, 0, 0, 0), (8, 4, 0, 0)], np.uint16)
        part = r.render(vi, pi, W, H, tiles=t)["rgba32f"][0]
        for tx, ty, _, _ in t:
            np.testing.assert_array_equal(part[8 * ty:8 * ty + 8, 8 * tx:8 * tx + 8],
                                          first["rgba32f"][0][8 * ty:8 * ty + 8, 8 * tx:8 * tx + 8])


def test_duplicate_tile_list_then_moving_camera(gv, config1):
    """a caller's tile list with duplicates and at least as many entries as the frame has tiles
    must not leave cells of the dilation grid unwritten (the grid is cleared unless the list is the handle's own
    full-frame list; classes are clamped to TILE_BUCKETS - 1).  The frames of a moving camera after such a list
    equal a fresh handle's frames of the same cameras, bit for bit."""
    W, H = 72, 40  # 9 x 5 = 45 tiles
    eyes = [gv.camera.orbit_eye(3.0, 15.0, 30.0 + 2.0 * k) for k in range(4)]
    cams = [gv.camera.pinhole(e, (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 45.0, gv.camera.aspect_ratio(W, H)) for e in eyes]
    dup = [(0, 0, 0, 0)] * 20 + [(tx, ty, 0, 0) for ty in range(5) for tx in range(9)] + [(8, 4, 0, 0)] * 7
    t = np.asarray(dup, np.uint16)
    assert len(t) >= 45
    with gv.Renderer(0) as r, gv.Renderer(0) as fresh:
        r.prepare(config1)
        fresh.prepare(config1)
        vi0, pi0 = cams[0]
        full0 = r.render(vi0, pi0, W, H)["rgba32f"]
        part = r.render(vi0, pi0, W, H, tiles=t)["rgba32f"]
        np.testing.assert_array_equal(part, full0)  # every tile listed, some twice: the same pixels
        for vi, pi in cams[1:]:  # moving camera: each launch dilates the previous classes by its motion
            got = r.render(vi, pi, W, H, hit_counts=True)
            want = fresh.render(vi, pi, W, H, hit_counts=True)
            for k in ("rgba32f", "rgba8", "hit_counts"):
                np.testing.assert_array_equal(got[k], want[k])


def test_record_origin_prep_changes_no_pixel(gv, config1):
    """Single-origin FAST launches read each leaf's kernel-frame origin from its record (k_rec_origin writes it
    per launch in place of the position; other launches get the positions back, k_rec_restore).  Frames agree
    bit for bit with the same cameras rendered by a multi-origin launch (positions path), across mode
    switches, and for queued launches with different origins (each launch's records prepared in stream order)."""
    W, H = 64, 48
    vi3, pi3 = gv.camera.lightfield_grid_rig((0.0, 0.0, 3.0), (0.0, 0.0, 0.0), nx=3, ny=1, spacing=0.3,
                                              aspect=gv.camera.aspect_ratio(W, H))
    cams = [vi3[16 * k:16 * (k + 1)] for k in range(3)]
    with gv.Renderer(0) as r:
        r.prepare(config1)
        multi = r.render(vi3, pi3, W, H, ncams=3)["rgba32f"]          # three origins: positions
        single = [r.render(v, pi3, W, H)["rgba32f"][0] for v in cams]  # one origin each: prepared records
        for k in range(3):
            np.testing.assert_array_equal(single[k], multi[k])
        lit = r.render(cams[1], pi3, W, H, mode=gv.MODE_LITERAL)["rgba32f"]  # LITERAL: positions restored
        np.testing.assert_array_equal(r.render(cams[1], pi3, W, H)["rgba32f"][0], single[1])
        np.testing.assert_array_equal(r.render(cams[1], pi3, W, H, mode=gv.MODE_LITERAL)["rgba32f"], lit)
        # queued launches alternating between two origins, device outputs
        import torch
        outs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(4)]
        for i, o in enumerate(outs):
            r.render_device(cams[i % 2 * 2], pi3, W, H, rgba32f_ptr=o.data_ptr(), async_=True)
        r.sync()
        for i, o in enumerate(outs):
            np.testing.assert_array_equal(o.cpu().numpy(), single[i % 2 * 2])


def test_caller_stream_queued_split_frame(gv, config1):
    """The multi-GPU exchange's device-side pipeline on one GPU: renders queued (gvrt_render_async) on a
    caller stream (gvrt_set_stream), each rank part of a tile-split frame rendered tile-packed, then all parts
    unpacked behind the queued renders (gvrt_unpack_tiles_rgba8 with renders pending: queued, done by
    gvrt_sync), repeated with the same static tile lists (uploaded once, no host round trip) — the frame
    equals the synchronous full-frame render; back on the handle's own stream nothing changes."""
    import torch
    W, H = 200, 120
    vi, pi = gv.scene.config1_camera(W, H)
    world = 3
    parts = importlib.import_module("3dgvrt_lightfield_amd.dist").rank_tiles(W, H, 1, world, block=2)
    with gv.Renderer(0) as r:
        r.prepare(config1)
        ref = r.render(vi, pi, W, H)["rgba8"][0]
        s = torch.cuda.Stream()
        r.set_stream(s.cuda_stream)
        bufs = [torch.zeros((t.shape[0] * 64, 4), dtype=torch.uint8, device="cuda") for t in parts]
        frames = [torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda") for _ in range(2)]
        for it in range(4):
            frame = frames[it % 2]
            for b, t in zip(bufs, parts):
                r.render_device(vi, pi, W, H, tiles=t, rgba8_ptr=b.data_ptr(), packed=True, async_=True)
            for b, t in zip(bufs, parts):
                r.unpack_tiles_rgba8(b.data_ptr(), t, W, H, frame.data_ptr())
        r.sync()
        for frame in frames:
            np.testing.assert_array_equal(frame.cpu().numpy(), ref)
        r.set_stream(None)
        np.testing.assert_array_equal(r.render(vi, pi, W, H)["rgba8"][0], ref)
