#!/usr/bin/env python3
"""Benchmark of the Particle Rendering hot path (BASELINE.json metric: Mrays/s + fps @1920x1080, 1M
Gaussians; PSNR vs the reference restated by the CPU oracle).

Workload at N=1: config 2 ("bicycle" stand-in, 1M synthetic Gaussians, seed 1, 1920x1080, orbit
camera r=4 / elev 20 / fovy 50, ray-query variant).  A step = one Particle Rendering pass over one
1920x1080 view with the scene, proxies and BVH resident in HBM (enclosing + BVH build are
one-shot and reported separately; by default the static-scene quality build, `--build fast` for the
1.4 ms device LBVH).  With --gpus N each rank renders its own view of an N-camera
light-field rig (config 5 shards views over GPUs) and the frames are gathered to rank 0 with RCCL
(torch.distributed 'nccl'): per-GPU work is fixed, so scaling is weak.  `--split tiles` instead
splits ONE frame into 64x64 blocks round-robin over ranks (strong scaling) and gathers the
tile-packed parts.

    python bench.py --gpus 1 --steps 20 --warmup 3
"""
import argparse
import importlib
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md chip table


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="bicycle", choices=["bicycle", "garden", "truck", "lightfield", "config1"])
    ap.add_argument("--split", default="views", choices=["views", "tiles"])
    ap.add_argument("--mode", default="fast", choices=["fast", "literal"])
    ap.add_argument("--ply", default=None, help="render this 3DGS .ply (e.g. Mip-NeRF360 bicycle) instead of the "
                                                  "synthetic stand-in of --config (same camera and resolution)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stats", action="store_true", help="skip the LITERAL stats pass (roofline bytes)")
    ap.add_argument("--build", default="quality", choices=["quality", "fast"],
                    help="quality: host binned-SAH tree + SAH-optimal 4-wide collapse (the static-scene build, as "
                         "the reference's PREFER_FAST_TRACE BLAS); fast: device LBVH + greedy collapse (~1.4 ms)")
    return ap.parse_args()


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        world = max(world, 1)
    import torch
    import torch.distributed as dist

    gv = importlib.import_module("3dgvrt_lightfield_amd")
    distributed = world > 1
    if distributed:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)

    gen, W, H, ncams_cfg = gv.scene.CONFIGS[args.config]
    if args.ply:  # "if bicycle.ply is supplied, use it instead and say so"
        splats = gv.SplatSet()
        if not gv.PLYLoader().loadPLYModel(args.ply, splats):
            raise SystemExit(f"cannot load {args.ply}")
    else:
        splats = gv.scene.make(**gen)
    n_input = splats["positions"].size // 3

    r = gv.Renderer(local_rank)
    bkw = dict(builder=2, collapse=1) if args.build == "quality" else {}
    m = r.prepare(splats, **bkw)
    first_build = r.stats()  # includes the one-time lazy loading of the build kernels' code objects
    m = r.prepare(splats, **bkw)    # steady-state scene build (what a scene change costs)
    st0 = r.stats()

    # cameras: an N-view planar rig around the config-2 orbit camera (view 0 = the config camera)
    if args.config == "config1":
        eye, fovy = (0.0, 0.0, 3.0), gv.camera.FOV_Y
    else:
        eye, fovy = gv.camera.orbit_eye(4.0, 20.0, 30.0), 50.0  # = scene.mipnerf_camera (view 0)
    target = (0.0, 0.0, 0.0)
    views = world if args.split == "views" else 1
    views = max(views, ncams_cfg if args.config == "lightfield" else 1)
    vis, pi = gv.camera.lightfield_grid_rig(eye, target, (0.0, 1.0, 0.0), nx=views, ny=1, spacing=0.1,
                                            fovy_deg=fovy, aspect=gv.camera.aspect_ratio(W, H))
    vis = vis.reshape(views, 16)
    if args.split == "views":
        my_views = [v for v in range(views) if v % world == rank]
        vi = np.ascontiguousarray(vis[my_views].reshape(-1))
        ncams = len(my_views)
        tiles = None
        rays_per_rank = W * H * ncams
        frame = torch.zeros((ncams, H, W, 4), dtype=torch.uint8, device=dev)
    else:
        vi = np.ascontiguousarray(vis[0])
        ncams = 1
        tiles = gv.tiles_for_rank(W, H, 1, rank, world, block=8)
        rays_per_rank = int(tiles.shape[0]) * 64
        frame = torch.zeros((tiles.shape[0] * 64, 4), dtype=torch.uint8, device=dev)
    mode = gv.MODE_FAST if args.mode == "fast" else gv.MODE_LITERAL
    params = r.render_params(mode=mode)

    # Double-buffered frame exchange: the RCCL gather of frame i (torch's stream, async) runs while
    # frame i+1 renders on the library's own HIP stream; a buffer is reused only after its gather
    # completed.  Tile split: rank 0 scatters the gathered parts into the full frame
    # (gvrt_unpack_tiles_rgba8), as SURVEY §8e's one exchange step per frame.
    nbuf = 2 if distributed else 1
    frames = [frame] + [torch.zeros_like(frame) for _ in range(nbuf - 1)]
    rank_tiles = [gv.tiles_for_rank(W, H, 1, q, world, block=8) for q in range(world)] if args.split == "tiles" else None
    if distributed and args.split == "tiles":
        # NCCL gather needs equal sizes: pad every rank's part to the largest
        maxs = max(t.shape[0] for t in rank_tiles) * 64
        sendbufs = [torch.zeros((maxs, 4), dtype=torch.uint8, device=dev) for _ in range(nbuf)]
        gathered = [[torch.empty((maxs, 4), dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
                    for _ in range(nbuf)]
        full = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev) if rank == 0 else None
    elif distributed:
        gathered = [[torch.empty_like(frame) for _ in range(world)] if rank == 0 else None for _ in range(nbuf)]
    pending = [None] * nbuf

    kernel_ms = []

    def finish(b):
        if pending[b] is None:
            return
        pending[b].wait()
        torch.cuda.current_stream().synchronize()  # the library's stream reads / overwrites this buffer next
        if args.split == "tiles" and rank == 0:
            for q in range(world):
                r.unpack_tiles_rgba8(gathered[b][q].data_ptr(), rank_tiles[q], W, H, full.data_ptr())
        pending[b] = None

    it = [0]

    # One GPU: frames are queued back to back (gvrt_render_async; one host round trip per K frames instead of
    # one per frame); the kernel time is the mean over the queued launches (HIP event pairs), read at sync.
    # Several ranks: synchronous renders, each frame handed to the RCCL gather as soon as it is done.
    use_async = not distributed

    def step():
        b = it[0] % nbuf
        it[0] += 1
        finish(b)
        r.render_device(vi, pi, W, H, ncams, params=params, tiles=tiles, rgba8_ptr=frames[b].data_ptr(),
                        packed=args.split == "tiles", async_=use_async)
        if not use_async:
            kernel_ms.append(r.render_ms())
        if distributed:
            if args.split == "views":
                pending[b] = dist.gather(frames[b], gathered[b] if rank == 0 else None, dst=0, async_op=True)
            else:
                sendbufs[b][: frames[b].shape[0]].copy_(frames[b])
                pending[b] = dist.gather(sendbufs[b], gathered[b] if rank == 0 else None, dst=0, async_op=True)

    def drain():
        for b in range(nbuf):
            finish(b)

    for _ in range(args.warmup):
        step()
    drain()
    if use_async:
        r.sync()
    kernel_ms.clear()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()  # every frame of the timed steps is rendered and gathered (and scattered) inside the clock
    if use_async:
        r.sync()  # every queued frame finished inside the clock
        kernel_ms.append(r.render_ms())  # mean over the K launches
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        rays_t = torch.tensor([rays_per_rank], dtype=torch.float64, device=dev)
        dist.all_reduce(rays_t)
        total_rays_per_step = float(rays_t.item())
    else:
        total_rays_per_step = float(rays_per_rank)

    ms_per_step = elapsed / args.steps * 1e3
    mrays = total_rays_per_step * args.steps / elapsed / 1e6
    kern_avg = float(np.mean(kernel_ms)) if kernel_ms else float("nan")

    result = None
    if rank == 0:
        # ---- roofline: algorithmic bytes of the reference algorithm on this input (LITERAL counters)
        roof = None
        lit_stats = None
        if not args.no_stats:
            r.set_stats(True)
            r.render(vi[:16], pi, W, H, 1, params=r.render_params(mode=gv.MODE_LITERAL), rgba8=False, rgba32f=False)
            lit_stats = r.stats()
            r.set_stats(False)
            rays1 = W * H
            bytes_per_launch = (48.0 * lit_stats["crossings"] + 192.0 * lit_stats["accepted"] + 4.0 * rays1) * (
                rays_per_rank / rays1)
            achieved = bytes_per_launch / (kern_avg * 1e-3) / 1e9
            traffic = None
            pmc = os.path.join(ROOT, "profiles", f"pmc_{args.config}.json")
            if os.path.exists(pmc):
                try:
                    traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
                except Exception:
                    traffic = None
            roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                    "algorithmic_bytes_per_launch": bytes_per_launch,
                    "kernel_ms_avg": round(kern_avg, 4), "kernel": "k_render<FAST,K=24,packed>"}

        # ---- CPU baseline (oracle restatement, all host threads we use), PSNR vs oracle on the sample
        cpu = None
        psnr = None
        if not args.no_cpu_baseline and world == 1:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O

            threads = min(16, os.cpu_count() or 1)
            e = O.enclose(splats)
            sc = O.Scene(e, proxy_mode=1)
            probe = np.arange(0, W * H, 2003, dtype=np.uint64)
            t = time.perf_counter()
            sc.render(vi[:16], pi, W, H, subset=probe, threads=threads)
            rate = len(probe) / max(time.perf_counter() - t, 1e-6)
            nsub = int(min(W * H, max(len(probe), rate * args.cpu_seconds)))
            stride = max(1, (W * H) // nsub)
            sub = np.arange(0, W * H, stride, dtype=np.uint64)
            t = time.perf_counter()
            ref = sc.render(vi[:16], pi, W, H, subset=sub, threads=threads)
            dt = time.perf_counter() - t
            # and on one core, a strided sample sized for ~3 s
            n1 = int(min(W * H, max(256, rate / threads * 3.0)))
            sub1 = np.arange(0, W * H, max(1, (W * H) // n1), dtype=np.uint64)
            t = time.perf_counter()
            sc.render(vi[:16], pi, W, H, subset=sub1, threads=1)
            dt1 = time.perf_counter() - t
            cpu = {"value": round(len(sub) / dt / 1e6, 6), "unit": "Mrays/s", "cores": threads, "kind": "port",
                   "sample": f"{len(sub)} rays (every {stride}th pixel of view 0), oracle analytic-proxy literal "
                             f"ray-march, {dt:.1f} s on {threads} threads",
                   "value_1core": round(len(sub1) / dt1 / 1e6, 6),
                   "sample_1core": f"{len(sub1)} rays (strided over view 0), {dt1:.1f} s on 1 thread"}
            img = r.render(vi[:16], pi, W, H, 1, params=params, rgba32f=True, rgba8=True)
            got = img["rgba8"].reshape(-1, 4)[sub.astype(np.int64)]
            psnr = gv.psnr_rgb(got, gv.quantize_rgba8(ref["rgba32f"]))

        result = {
            "metric": "Mrays/s + fps @1920x1080, 1M Gaussians; PSNR vs Vulkan reference",
            "value": round(mrays, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak" if args.split == "views" else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": (f"real scene {os.path.basename(args.ply)}" if args.ply
                     else "synthetic (seeded stand-in scene, SURVEY §8d)"),
            "config": {"workload": f"{args.config}: {n_input} {'PLY' if args.ply else 'synthetic'} Gaussians, {W}x{H}, "
                                   f"{'one view per rank' if args.split == 'views' else 'one frame tile-split'}, "
                                   f"ray-query variant, {args.mode} k-buffer",
                       "gaussians": n_input, "survivors": m, "width": W, "height": H,
                       "views": views, "split": args.split, "parallelism": f"{args.split}{world}",
                       "build": ("quality: host binned-SAH tree + SAH-optimal 4-wide collapse" if args.build == "quality"
                                 else "fast: device LBVH + greedy 4-wide collapse")},
            "fps": round(1e3 / ms_per_step, 2),
            "kernel_ms": round(kern_avg, 4),
            "kernel_mrays": round(rays_per_rank / (kern_avg * 1e-3) / 1e6, 3) if kern_avg == kern_avg else None,
            "psnr_vs_oracle_db": None if psnr is None else (round(psnr, 2) if math.isfinite(psnr) else "inf"),
            "enclose_ms": round(st0["enclose_ms"], 3),
            "accel_ms": round(st0["accel_ms"], 3),
            "first_build_ms": round(first_build["enclose_ms"] + first_build["accel_ms"], 3),
            "bvh_depth": st0["bvh_depth"],
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if lit_stats:
            result["reference_counters"] = {"crossings_per_ray": lit_stats["crossings"] / (W * H),
                                            "accepted_per_ray": lit_stats["accepted"] / (W * H),
                                            "rounds_per_ray": lit_stats["rounds"] / (W * H)}
        print(json.dumps(result), flush=True)
    r.close()
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
