"""Multi-GPU frame split + exchange: one process per GPU, scene and BVH replicated per
rank, one exchange per frame.

  * tile split  (strong scaling, config 4): by default contiguous bands of the frame's 64x64-pixel blocks
    (8x8 of the kernel's 8x8 tiles), cut where the summed per-tile cost of a calibration frame reaches
    k/N of the total (band_tiles over cost_weights; bench.py --tile-layout cost-bands), or 64x64-pixel
    blocks round-robin over ranks (rank_tiles, --tile-layout blocks); each rank renders its tiles
    tile-packed, the parts go to rank 0 with exact-size point-to-point sends (torch.distributed, backend
    'nccl' = RCCL over xGMI on MI355X, 'gloo' on CPU for tests) and are scattered into the frame
    (gvrt_unpack_tiles_rgba8 on the GPU, unpack_tiles_host on the CPU).
  * view split  (light-field config 5, and one view per rank for the weak-scaling line): whole views,
    cost-balanced (balanced_views) when there are more views than ranks, else round-robin (rank_views).

`FrameExchange` is the double-buffered exchange bench.py runs; the renderer and the rank-0 assembly are
injected, so the same object is driven by the gloo tests on CPU (tests/test_dist.py).  `launch_ranks`
turns `bench.py --gpus N` started as one plain process into N ranks.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys

import numpy as np

from .renderer import tiles_for_rank


def rank_tiles(width, height, ncams, world, block=8):
    """Tile lists of every rank (uint16 [n, 4] rows of (tx, ty, cam, 0))."""
    return [tiles_for_rank(width, height, ncams, r, world, block) for r in range(world)]


# 2^(k/4), k = 0..3, as exact decimal literals: cost_weights is 2^(c div 4) x QUARTER_OCTAVES[c mod 4], bit for
# bit the same doubles as the C++ host's (gvrt_rccl.cpp), so both compute the same band cuts
QUARTER_OCTAVES = (1.0, 1.189207115002721, 1.4142135623730951, 1.681792830507429)


def cost_weights(classes):
    """Relative cost of a tile from its class (gvrt_read_tile_costs: 4 classes per octave of wave cycles)."""
    c = np.asarray(classes, np.int64)
    return np.ldexp(np.asarray(QUARTER_OCTAVES, np.float64)[c & 3], c >> 2)


def band_tiles(width, height, world, costs=None, ncams=1, block=8):
    """Contiguous parts of the frame, one per rank: the tiles in the order of rank_tiles' blocks (block x block
    tiles, blocks row-major, tiles row-major inside a block) cut into `world` runs of equal tile count, or of
    equal summed cost when `costs` (per-tile weights [ncams, ty, tx], e.g. cost_weights of a previous frame's
    classes) is given.  A part is then a band of block rows (its tiles share BVH nodes and records in that
    GPU's caches, and the block order keeps the XCD dealing of each cost class compact), where the block
    round-robin of rank_tiles scatters each part over the whole frame.  world = 1 gives rank_tiles' list.
    Every rank computes the same cuts from the same costs.  Returns uint16 [n, 4] rows of (tx, ty, cam, 0)."""
    rows = tiles_for_rank(width, height, ncams, 0, 1, block).astype(np.int64)
    tx_n, ty_n = (width + 7) // 8, (height + 7) // 8
    n = rows.shape[0]
    if costs is None:
        w = np.ones(n)
    else:
        c = np.asarray(costs, np.float64)
        if c.size != ncams * ty_n * tx_n:
            raise ValueError("costs must hold one weight per tile")
        w = c.reshape(ncams, ty_n, tx_n)[rows[:, 2], rows[:, 1], rows[:, 0]]
    cum = np.concatenate([[0.0], np.cumsum(w)])
    # cut k: the first list position whose prefix weight reaches k/world of the total
    cuts = [0] + [int(np.searchsorted(cum, cum[-1] * k / world, side="left")) for k in range(1, world)] + [n]
    cuts = np.maximum.accumulate(np.minimum(cuts, n))
    rows = rows.astype(np.uint16)
    return [rows[cuts[r]:cuts[r + 1]] for r in range(world)]


def rank_views(views, world):
    """Views of every rank, round-robin (config 5 shards whole views over GPUs)."""
    return [list(range(r, views, world)) for r in range(world)]


def balanced_views(costs, world):
    """Cost-weighted view assignment (config 5 on N ranks): every rank gets floor or ceil(views / world) views, and
    the views are placed costliest first, each on the rank with the least cost so far among those with room
    (longest-processing-time list scheduling with a count bound; ties by rank, then view index, so every rank
    computes the same assignment from the same costs).  Views of a rank are returned in increasing index."""
    costs = [float(c) for c in costs]
    n = len(costs)
    cap = [n // world + (1 if r < n % world else 0) for r in range(world)]
    load = [0.0] * world
    out = [[] for _ in range(world)]
    for v in sorted(range(n), key=lambda i: (-costs[i], i)):
        r = min((rr for rr in range(world) if len(out[rr]) < cap[rr]), key=lambda rr: (load[rr], rr))
        out[r].append(v)
        load[r] += costs[v]
    return [sorted(g) for g in out]


def unpack_tiles_host(packed, tiles, width, height, ncams=1, frame=None):
    """Host mirror of k_unpack (gvrt_render.hip): packed[i*64 + lane] -> frame[cam][ty*8 + lane//8][tx*8 + lane%8]."""
    packed = np.asarray(packed).reshape(-1, 64, packed.shape[-1] if packed.ndim > 1 else 1)
    if frame is None:
        frame = np.zeros((ncams, height, width, packed.shape[-1]), packed.dtype)
    lane = np.arange(64)
    for i, (tx, ty, cam, _) in enumerate(np.asarray(tiles, np.int64)):
        px = tx * 8 + (lane & 7)
        py = ty * 8 + (lane >> 3)
        ok = (px < width) & (py < height)
        frame[cam, py[ok], px[ok]] = packed[i, ok]
    return frame


class FrameExchange:
    """Double-buffered frame exchange, the one exchange step per frame of SURVEY §8e.

    Every rank owns `nbuf` send buffers of exactly its own part size; rank 0 owns `nbuf` receive buffers per other
    rank, each exactly that rank's part size.  The exchange is point to point (batch_isend_irecv: every rank r > 0
    sends its part to rank 0, rank 0 receives each; rank 0's own part never leaves its send buffer), so unequal
    parts move no padding (round 3 gathered every part padded to the largest one: up to 28 % extra bytes with cost
    bands).  step(render) waits until the exchange that last used buffer b has completed (and lets rank 0 assemble
    that frame), renders the next frame into buffer b, and posts its sends / receives asynchronously, so the
    exchange of frame i (RCCL on its own stream) overlaps the render of frame i + 1 (the library's HIP stream).
    drain() completes every outstanding frame.

      render(buf)             writes this rank's part of the next frame into `buf` (its send buffer)
      assemble(parts, frame)  rank 0 only: builds the frame from the parts (list of world tensors, rank r's of its
                              part size); frame counts from 0
      sync()                  called after an exchange completed and before its buffers are reused or read by
                              another stream (torch.cuda.current_stream().synchronize on the GPU)
      mark(name)              optional, probe() only: called at "rendered" (render posted), "exchanged" (the
                              exchange waited for) and "assembled"; the bench records HIP events there
    """

    def __init__(self, dist, rank, world, part_sizes, item_shape, dtype, device="cpu", nbuf=2, assemble=None,
                 sync=None):
        import torch

        self.dist, self.rank, self.world = dist, rank, world
        self.part_sizes = [int(s) for s in part_sizes]
        self.item_shape = tuple(item_shape)
        self.send = [torch.zeros((self.part_sizes[rank],) + self.item_shape, dtype=dtype, device=device)
                     for _ in range(nbuf)]
        self.recv = [[None if r == 0 else torch.empty((self.part_sizes[r],) + self.item_shape, dtype=dtype,
                                                      device=device) for r in range(world)] if rank == 0 else None
                     for _ in range(nbuf)]
        self.pending = [None] * nbuf
        self.frame_of = [None] * nbuf
        self.nbuf = nbuf
        self.assemble = assemble
        self.sync = sync
        self.frames = 0
        item_bytes = int(np.prod(self.item_shape, dtype=np.int64)) * torch.empty((), dtype=dtype).element_size()
        # what crosses the links per frame (rank r > 0's part to rank 0), and what a padded gather moved instead
        self.exchange_bytes = sum(self.part_sizes[1:]) * item_bytes
        self.padded_gather_bytes = (world - 1) * max(self.part_sizes) * item_bytes

    def parts(self, b):
        """Rank 0: every rank's part of the frame in buffer b (rank 0's own part is its send buffer)."""
        return [self.send[b]] + list(self.recv[b][1:])

    def _post(self, b):
        d = self.dist
        if self.rank == 0:
            ops = [d.P2POp(d.irecv, self.recv[b][r], r) for r in range(1, self.world) if self.part_sizes[r]]
        else:
            ops = [d.P2POp(d.isend, self.send[b], 0)] if self.part_sizes[self.rank] else []
        return d.batch_isend_irecv(ops) if ops else []

    def _finish(self, b):
        if self.pending[b] is None:
            return
        for w in self.pending[b]:
            w.wait()
        if self.sync:
            self.sync()
        if self.rank == 0 and self.assemble:
            self.assemble(self.parts(b), self.frame_of[b])
        self.pending[b] = None

    def step(self, render):
        b = self.frames % self.nbuf
        self._finish(b)
        render(self.send[b])
        self.pending[b] = self._post(b)
        self.frame_of[b] = self.frames
        self.frames += 1

    def drain(self):
        for k in range(self.nbuf):
            self._finish((self.frames + k) % self.nbuf)

    def probe(self, render, mark, barrier=None):
        """One frame with nothing else in flight, for the per-phase times of the strong-scaling record: render,
        (barrier: every rank has rendered), exchange, wait, assemble, with mark() at each boundary ("rendered",
        "posted", "exchanged", "assembled").  Call after drain()."""
        self.drain()
        b = self.frames % self.nbuf
        render(self.send[b])
        mark("rendered")
        if barrier:
            barrier()
        mark("posted")
        w = self._post(b)
        for x in w:
            x.wait()
        mark("exchanged")
        if self.sync:
            self.sync()
        if self.rank == 0 and self.assemble:
            self.assemble(self.parts(b), self.frames)
        mark("assembled")
        self.frames += 1


def gather_tiles(dist, part, rank, world, sizes, device=None):
    """Gather tile-packed parts (uint8 [n_r*64, 4] tensors) to rank 0 (one synchronous exchange)."""
    ex = FrameExchange(dist, rank, world, sizes, part.shape[1:], part.dtype, part.device, nbuf=1)
    out = []
    ex.assemble = lambda parts, _f: out.extend(p.clone() for p in parts)
    ex.step(lambda buf: buf.copy_(part))
    ex.drain()
    return out if rank == 0 else None


def render_split_frame(dist, render_fn, width, height, rank, world, block=8, device="cpu", unpack_fn=None):
    """Render one frame split over `world` ranks and assemble it on rank 0.

    render_fn(tiles) -> uint8 tensor [len(tiles)*64, 4] (tile-packed rgba8 of this rank's tiles).
    unpack_fn(packed_tensor, tiles, frame_tensor) assembles on rank 0 (defaults to the host mirror).
    Returns the [H, W, 4] frame on rank 0, None elsewhere."""
    import torch

    all_tiles = rank_tiles(width, height, 1, world, block)
    part = render_fn(all_tiles[rank])
    sizes = [t.shape[0] * 64 for t in all_tiles]
    parts = gather_tiles(dist, part, rank, world, sizes)
    if rank != 0:
        return None
    if unpack_fn is None:
        frame = np.zeros((1, height, width, 4), np.uint8)
        for p, t in zip(parts, all_tiles):
            unpack_tiles_host(p.cpu().numpy(), t, width, height, 1, frame)
        return torch.from_numpy(frame[0])
    frame = torch.zeros((height, width, 4), dtype=torch.uint8, device=device)
    for p, t in zip(parts, all_tiles):
        unpack_fn(p, t, frame)
    return frame


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(nproc, script, argv, env=None):
    """One process per GPU: when `script --gpus N` runs as a plain process (no WORLD_SIZE, or WORLD_SIZE 1)
    with N > 1, start its N ranks as children (`torch.distributed.run`, one node, rendezvous on 127.0.0.1)
    and return their exit code.  Returns None when this process already is one rank of an N-rank job (or
    N == 1): the caller then goes on as that rank.  A job whose WORLD_SIZE is neither 1 nor N is refused.
    Call before anything touches the GPU (the children do the GPU work; nothing here is exec'd)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == nproc:
        return None
    if world > 1:
        raise SystemExit(f"launched with WORLD_SIZE={world} but --gpus {nproc}")
    if nproc <= 1:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", script, *argv]
    e = dict(os.environ if env is None else env)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only (RCCL / tensor sharing across ranks)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    return subprocess.run(cmd, env=e).returncode
