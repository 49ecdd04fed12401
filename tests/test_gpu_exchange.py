"""bench.py's multi-GPU frame exchange on one GPU, with the real collective backend (RCCL, one rank): the
device-side ordering of dist.FrameExchange + gvrt_set_stream + gvrt_render_async.  Frames
alternate between two cameras, so a gather that ran ahead of its render, or a render into a buffer still
being gathered, would deliver the other camera's pixels: every gathered frame must equal the synchronous
render of its own camera, for the view split and for the tile split (parts assembled on rank 0 by
gvrt_unpack_tiles_rgba8 queued behind the renders)."""
import importlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    import torch
    import torch.distributed as dist
    d = importlib.import_module("3dgvrt_lightfield_amd.dist")
    if not dist.is_initialized():
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{d.free_port()}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
    yield dist, d
    dist.destroy_process_group()


@pytest.mark.parametrize("split", ["views", "tiles"])
def test_exchange_frames_match_their_cameras(gv, config1, pg, split):
    import torch
    dist, d = pg
    W, H = 160, 96
    ncam, nframes = 3, 7  # three cameras over two buffers: a buffer's stale content is another camera's
    vis, pi = gv.camera.lightfield_grid_rig((0.0, 0.0, 3.0), (0.0, 0.0, 0.0), nx=ncam, ny=1, spacing=0.6,
                                            aspect=gv.camera.aspect_ratio(W, H))
    cams = [np.ascontiguousarray(vis[16 * k:16 * (k + 1)]) for k in range(ncam)]
    dev = torch.device("cuda", 0)
    with gv.Renderer(0) as r:
        r.prepare(config1)
        ref = [r.render(c, pi, W, H)["rgba8"][0] for c in cams]
        assert not np.array_equal(ref[0], ref[1]) and not np.array_equal(ref[1], ref[2])
        packed = split == "tiles"
        if packed:
            tiles = d.rank_tiles(W, H, 1, 1, block=2)[0]
            part_sizes, item_shape = [tiles.shape[0] * 64], (4,)
        else:
            tiles, part_sizes, item_shape = None, [1], (H, W, 4)
        out = [torch.zeros((H, W, 4), dtype=torch.uint8, device=dev) for _ in range(nframes)]
        xs = torch.cuda.Stream(dev)
        torch.cuda.synchronize()
        prev = torch.cuda.current_stream(dev)
        torch.cuda.set_stream(xs)
        try:
            r.set_stream(xs.cuda_stream)

            def assemble(parts, f):  # on the exchange stream, after the gather (work.wait)
                if packed:
                    r.unpack_tiles_rgba8(parts[0].data_ptr(), tiles, W, H, out[f].data_ptr())
                else:
                    out[f].copy_(parts[0][0])

            ex = d.FrameExchange(dist, 0, 1, part_sizes, item_shape, torch.uint8, dev, nbuf=2, assemble=assemble)
            for f in range(nframes):
                cam = cams[f % ncam]
                ex.step(lambda buf, cam=cam: r.render_device(cam, pi, W, H, tiles=tiles, rgba8_ptr=buf.data_ptr(),
                                                             packed=packed, async_=True))
            ex.drain()
            r.sync()
            torch.cuda.synchronize()
        finally:
            torch.cuda.set_stream(prev)
            r.set_stream(None)
        for f in range(nframes):
            np.testing.assert_array_equal(out[f].cpu().numpy(), ref[f % ncam], err_msg=f"frame {f}")
