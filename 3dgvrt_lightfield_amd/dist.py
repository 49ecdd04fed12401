"""Multi-GPU frame split + gather: one process per GPU, scene and LBVH replicated per
rank, one exchange per frame.

  * tile split  (strong scaling): 64x64-pixel blocks (8x8 of the kernel's 8x8 tiles) round-robin
    over ranks; each rank renders its tiles tile-packed, the parts are gathered to rank 0 with
    torch.distributed (backend 'nccl' = RCCL over xGMI on MI355X, 'gloo' on CPU for tests) and
    scattered into the frame (gvrt_unpack_tiles_rgba8 on the GPU, unpack_tiles_host on the CPU).
  * view split  (weak scaling, light-field config 5): whole views round-robin over ranks.

The renderer is injected (`render_fn`) so the collective plumbing is testable without a GPU.
"""
from __future__ import annotations

import numpy as np

from .renderer import tiles_for_rank


def rank_tiles(width, height, ncams, world, block=8):
    """Tile lists of every rank (uint16 [n, 4] rows of (tx, ty, cam, 0))."""
    return [tiles_for_rank(width, height, ncams, r, world, block) for r in range(world)]


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


def gather_tiles(dist, part, rank, world, sizes, device=None):
    """Gather tile-packed parts (uint8 [n_r*64, 4] tensors) to rank 0.  NCCL/gloo gather needs equal
    shapes, so every part is padded to the largest; rank 0 gets the unpadded list."""
    import torch

    maxn = max(sizes)
    send = torch.zeros((maxn, part.shape[1]), dtype=part.dtype, device=part.device)
    send[: part.shape[0]].copy_(part)
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
    dist.gather(send, bufs, dst=0)
    if rank != 0:
        return None
    return [b[:s] for b, s in zip(bufs, sizes)]


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
