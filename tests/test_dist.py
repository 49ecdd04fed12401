"""Multi-rank frame split + RCCL-style gather, exercised with torch.distributed 'gloo' on CPU (world 2 and 3).

The renderer is replaced by a deterministic per-pixel pattern so the test checks what the N>1 path
owns: tile assignment (disjoint, complete), padding of unequal parts for the gather, the gather
itself and the tile unpack indexing (host mirror of k_unpack)."""
import importlib
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def pattern(width, height):
    y, x = np.mgrid[0:height, 0:width]
    return np.stack([x % 251, y % 253, (x * 7 + y * 3) % 255, np.full_like(x, 255)], -1).astype(np.uint8)


def _worker(rank, world, port, width, height, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    gv = importlib.import_module("3dgvrt_lightfield_amd")
    d = importlib.import_module("3dgvrt_lightfield_amd.dist")
    img = pattern(width, height)

    def fake_render(tiles):  # tile-packed rgba8 of this rank's tiles, 0 outside the image
        out = np.zeros((len(tiles) * 64, 4), np.uint8)
        lane = np.arange(64)
        for i, (tx, ty, cam, _) in enumerate(tiles.astype(np.int64)):
            px, py = tx * 8 + (lane & 7), ty * 8 + (lane >> 3)
            ok = (px < width) & (py < height)
            out[i * 64 + lane[ok]] = img[py[ok], px[ok]]
        return torch.from_numpy(out)

    frame = d.render_split_frame(dist, fake_render, width, height, rank, world, block=2)
    if rank == 0:
        q.put(frame.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,width,height", [(2, 100, 60), (3, 37, 29)])
def test_split_gather_assembles_frame(world, width, height):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, width, height, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=240)
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    np.testing.assert_array_equal(frame, pattern(width, height))


def test_tile_assignment_disjoint_and_complete(gv):
    d = importlib.import_module("3dgvrt_lightfield_amd.dist")
    for world in (1, 2, 4, 8):
        W, H, ncams = 1920, 1080, 2
        tl = d.rank_tiles(W, H, ncams, world)
        allt = np.concatenate(tl)
        keys = {tuple(t) for t in allt.tolist()}
        assert len(keys) == len(allt) == ((W + 7) // 8) * ((H + 7) // 8) * ncams
        sizes = [len(t) for t in tl]
        assert max(sizes) - min(sizes) <= 64  # one 64x64 block at most
