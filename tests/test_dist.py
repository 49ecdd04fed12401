"""Multi-rank frame split + RCCL-style gather, exercised with torch.distributed 'gloo' on CPU (world 2, 3 and 8:
the driver's 8-GPU node, config 5 with 16 views over 8 ranks).

The renderer is replaced by a deterministic per-pixel pattern so the test checks what the N>1 path
owns: tile assignment (disjoint, complete), the exact-size point-to-point exchange of unequal parts to
rank 0 (no padding since round 4), and the tile unpack indexing (host mirror of k_unpack)."""
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


# ---------------------------------------------------------------- the exchange bench.py runs (dist.FrameExchange)
def frame_pattern(k, width, height, views=1):
    y, x = np.mgrid[0:height, 0:width]
    return np.stack([np.stack([(x + 3 * k + 11 * v) % 251, (y + 5 * k) % 253, (x * 7 + y * 3 + v) % 255,
                               np.full_like(x, k % 256)], -1) for v in range(views)]).astype(np.uint8)


def _exchange_worker(rank, world, port, split, width, height, views, nframes, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = importlib.import_module("3dgvrt_lightfield_amd.dist")
    counter = [0]
    if split == "bands":
        # the cost-band layout bench.py and SplitFrame ship: contiguous runs of equal cost over a seeded class map
        # (rank 0's calibration broadcasts one; every rank cuts the same bands)
        ty_n, tx_n = (height + 7) // 8, (width + 7) // 8
        classes = np.random.default_rng(5).integers(0, 40, (1, ty_n, tx_n)).astype(np.uint8)
        all_tiles = d.band_tiles(width, height, world, costs=d.cost_weights(classes), block=2)
        sizes, item = [t.shape[0] * 64 for t in all_tiles], (4,)
        split = "tiles"
    elif split == "tiles":
        all_tiles = d.rank_tiles(width, height, 1, world, block=2)
        sizes, item = [t.shape[0] * 64 for t in all_tiles], (4,)
    else:
        all_views = d.rank_views(views, world)
        sizes, item = [len(v) for v in all_views], (height, width, 4)
    got = {}

    def render(buf):  # frame k's part of this rank, as the GPU renderer would write it
        k = counter[0]
        counter[0] += 1
        img = frame_pattern(k, width, height, views)
        if split == "tiles":
            lane = np.arange(64)
            out = np.zeros((buf.shape[0], 4), np.uint8)
            for i, (tx, ty, cam, _) in enumerate(all_tiles[rank].astype(np.int64)):
                px, py = tx * 8 + (lane & 7), ty * 8 + (lane >> 3)
                ok = (px < width) & (py < height)
                out[i * 64 + lane[ok]] = img[0, py[ok], px[ok]]
        else:
            out = img[all_views[rank]]
        buf.copy_(torch.from_numpy(out))

    def assemble(parts, k):
        if split == "tiles":
            frame = np.zeros((1, height, width, 4), np.uint8)
            for p, t in zip(parts, all_tiles):
                d.unpack_tiles_host(p.numpy(), t, width, height, 1, frame)
        else:
            frame = np.zeros((views, height, width, 4), np.uint8)
            for p, vs in zip(parts, all_views):
                frame[vs] = p.numpy()
        got[k] = frame

    ex = d.FrameExchange(dist, rank, world, sizes, item, torch.uint8, "cpu", nbuf=2, assemble=assemble)
    for _ in range(nframes):
        ex.step(render)
    ex.drain()
    # the strong-scaling record's per-phase probe: one more frame, one phase at a time, marks in order
    marks = []
    ex.probe(render, marks.append, barrier=dist.barrier)
    if rank == 0:
        q.put({"frames": {k: v.copy() for k, v in got.items()}, "marks": marks, "exchange_bytes": ex.exchange_bytes,
               "padded": ex.padded_gather_bytes, "sizes": sizes, "send_shape": tuple(ex.send[0].shape)})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,split,width,height,views", [(2, "tiles", 100, 60, 1), (3, "tiles", 37, 29, 1),
                                                             (2, "views", 24, 16, 5), (3, "views", 16, 8, 3),
                                                             (8, "tiles", 72, 40, 1), (8, "views", 16, 8, 16),
                                                             (8, "bands", 200, 120, 1)])
def test_frame_exchange_double_buffered(world, split, width, height, views):
    """bench.py's N-rank path on CPU: dist.FrameExchange with two send buffers in flight, unequal parts (tiles:
    ragged block counts; views: 5 views over 2 ranks) sent point to point at their exact sizes (no padding: every
    buffer has its own rank's part shape), rank-0 assembly per frame, then the strong-scaling record's one-frame
    probe.  Every frame arrives, in order, equal to the 1-rank frame."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    nframes = 5
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, split, width, height, views, nframes, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    got = res["frames"]
    assert sorted(got) == list(range(nframes + 1))
    for k in range(nframes + 1):
        np.testing.assert_array_equal(got[k], frame_pattern(k, width, height, views))
    assert res["marks"] == ["rendered", "posted", "exchanged", "assembled"]
    sizes = res["sizes"]
    item = 4 if split in ("tiles", "bands") else height * width * 4
    assert res["send_shape"][0] == sizes[0]
    assert res["exchange_bytes"] == sum(sizes[1:]) * item  # exact parts: no padding on the wire
    assert res["padded"] == (world - 1) * max(sizes) * item
    if len(set(sizes)) > 1:
        assert res["exchange_bytes"] < res["padded"]


def test_launch_ranks_gives_n_processes():
    """`script --gpus 2` started as ONE process comes back as 2 ranks (dist.launch_ranks, bench.py's launcher);
    a job whose WORLD_SIZE disagrees with --gpus is refused."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    probe = os.path.join(root, "tests", "dist_probe.py")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    for n in (1, 2, 3):
        r = subprocess.run([sys.executable, probe, "--gpus", str(n)], capture_output=True, text=True, timeout=240,
                           env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(line) == 1, r.stdout
        assert json.loads(line[0]) == {"n_gpus": n, "gpus_arg": n}
    r = subprocess.run([sys.executable, probe, "--gpus", "2"], capture_output=True, text=True, timeout=120,
                       env=dict(env, WORLD_SIZE="3", RANK="0"))
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


def test_balanced_views_equal_counts_and_lpt(gv):
    """dist.balanced_views: equal view counts per rank (floor / ceil), costliest views placed first on the least
    loaded rank with room, deterministic; never worse than round-robin on skewed costs."""
    from importlib import import_module
    d = import_module("3dgvrt_lightfield_amd.dist")
    rng = np.random.default_rng(3)
    for views, world in ((16, 8), (16, 4), (5, 3), (7, 7), (9, 2)):
        c = rng.uniform(1.0, 2.5, views)
        g = d.balanced_views(c, world)
        assert sorted(v for x in g for v in x) == list(range(views))
        assert sorted(len(x) for x in g) == sorted(views // world + (1 if r < views % world else 0) for r in range(world))
        assert g == d.balanced_views(list(c), world)
        bal = max(sum(c[v] for v in x) for x in g)
        rr = max(sum(c[v] for v in x) for x in d.rank_views(views, world))
        assert bal <= rr + 1e-12
    assert d.balanced_views([3.0, 1.0, 2.0, 2.0], 2) == [[0, 1], [2, 3]]


@pytest.mark.parametrize("W,H,world", [(3840, 2160, 8), (1920, 1080, 3), (100, 60, 2), (8, 8, 4)])
def test_band_tiles_cover_the_frame_in_contiguous_parts(gv, W, H, world):
    """dist.band_tiles: every tile exactly once, each rank a contiguous run of rank_tiles' block order (world 1:
    rank_tiles' own list), equal counts without costs and (near) equal summed cost with them."""
    dist = importlib.import_module("3dgvrt_lightfield_amd.dist")
    tx_n, ty_n = (W + 7) // 8, (H + 7) // 8
    order = dist.rank_tiles(W, H, 1, 1)[0].astype(np.int64)
    order = order[:, 1] * tx_n + order[:, 0]
    np.testing.assert_array_equal(dist.band_tiles(W, H, 1)[0], dist.rank_tiles(W, H, 1, 1)[0])
    for costs in (None, np.random.default_rng(world).random((1, ty_n, tx_n)) * 3 + 0.1):
        parts = dist.band_tiles(W, H, world, costs=costs)
        assert len(parts) == world
        lin = [p[:, 1].astype(np.int64) * tx_n + p[:, 0] for p in parts]
        allt = np.concatenate(lin)
        np.testing.assert_array_equal(allt, order)  # the block order, cut in runs: each tile once
        w = np.ones(tx_n * ty_n) if costs is None else costs.reshape(-1)
        sums = [w[l].sum() for l in lin]
        if tx_n * ty_n >= 100 * world:
            assert max(sums) <= (1.0 + 0.01) * np.mean(sums) + w.max()


@pytest.mark.parametrize("layout", ["cost-bands", "bands", "blocks"])
def test_bench_tile_layouts_cover_the_frame(gv, layout):
    """bench.py --tile-layout: every layout gives every 4K tile to exactly one of 8 ranks; cost bands from a
    cost-class map balance the summed cost (the split bench.py's tile branch and --rank-balance use)."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)  # no GPU work at import
    dist = importlib.import_module("3dgvrt_lightfield_amd.dist")
    W, H, world = 3840, 2160, 8
    cls = np.random.default_rng(5).integers(0, 40, size=(1, 270, 480), dtype=np.uint8)
    parts = bench.split_tiles(dist, layout, W, H, world, cls)
    lin = np.concatenate([p[:, 1].astype(np.int64) * 480 + p[:, 0] for p in parts])
    assert np.array_equal(np.sort(lin), np.arange(480 * 270))
    if layout == "cost-bands":
        w = dist.cost_weights(cls).reshape(-1)
        sums = [w[p[:, 1].astype(np.int64) * 480 + p[:, 0]].sum() for p in parts]
        assert max(sums) <= 1.001 * np.mean(sums) + w.max()
