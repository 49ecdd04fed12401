#!/usr/bin/env python3
"""Benchmark of the Particle Rendering hot path (BASELINE.json metric: Mrays/s + fps @1920x1080, 1M
Gaussians; PSNR vs the reference restated by the CPU oracle).

Workload at N=1: config 2 ("bicycle" stand-in, 1M synthetic Gaussians, seed 1, 1920x1080, orbit
camera r=4 / elev 20 / fovy 50, ray-query variant).  A step = one Particle Rendering pass over one
1920x1080 view with the scene, proxies and BVH resident in HBM (enclosing + BVH build are
one-shot and reported separately; by default the static-scene quality build on the device (binned SAH +
SAH-optimal collapse, ~9 ms at 1M, with the reference's SplitBLAS grid applied to proxies spanning 3+ of its 10
cells: renderer.QUALITY_BUILD), `--build fast` for the ~1.5 ms device LBVH).

Several GPUs: `python bench.py --gpus N` started as one process launches its N ranks
itself (torch.distributed.run, one process per GPU; dist.launch_ranks); launched by torch.distributed.run
with WORLD_SIZE = N it is one of them.  `--split views` (default; config 5) gives each rank its own
view(s) of a light-field camera rig: weak scaling.  `--split tiles` (default for `--config truck`,
config 4) splits ONE frame into 64x64 blocks round-robin over ranks: strong scaling.  Either way the
ranks' parts go to rank 0 through dist.FrameExchange (double-buffered RCCL gather, tile parts scattered
into the frame by gvrt_unpack_tiles_rgba8).

At N=1 the line also carries the HBM traffic of the render kernel measured by rocprofv3 PMC passes of
this same command (FETCH_SIZE, WRITE_SIZE, VALU issue; child processes started before this process
touches the GPU), and the CPU baseline (the oracle restatement on the host's CPU share).

    python bench.py --gpus 1 --steps 20 --warmup 3
"""
import argparse
import csv
import glob
import hashlib
import importlib
import json
import math
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md chip table
L2_PEAK_GBS = 34500.0  # aggregate L2 of the 8 XCDs (MI355X_MICROARCH.md, L2 per XCD: ~34.5 TB/s)
L2_LAT_CYC = 200.0     # global_load L2-hit latency, ~180-225 cycles (MI355X_MICROARCH.md, per-instruction constants)
# VALU issue: 256 CUs x 4 SIMD-32s, a wave64 VALU instruction occupies its SIMD for 2 cycles (MI355X_MICROARCH.md);
# the clock is the one measured over the dispatch (GRBM_GUI_ACTIVE counts cycles on each of the 8 XCDs)
N_SIMD = 256 * 4
N_XCD = 8


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="bicycle",
                    choices=["bicycle", "garden", "truck", "lightfield", "config1", "dense", "trained"])
    ap.add_argument("--split", default="auto", choices=["auto", "views", "tiles"],
                    help="auto: tiles for --config truck (config 4, strong scaling), else views")
    ap.add_argument("--mode", default="fast", choices=["fast", "literal"])
    ap.add_argument("--ply", default=None, help="render this 3DGS .ply (e.g. Mip-NeRF360 bicycle) instead of the "
                                                  "synthetic stand-in of --config (same camera and resolution)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stats", action="store_true", help="skip the LITERAL stats pass (roofline bytes)")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC passes (roofline.traffic, VALU)")
    ap.add_argument("--exchange", action="store_true",
                    help="run the multi-GPU frame-exchange path even with one rank (torch.distributed.run "
                         "--nproc-per-node 1: rehearses the N-rank step on one GPU)")
    ap.add_argument("--tile-layout", default="cost-bands", choices=["cost-bands", "bands", "blocks"],
                    help="tile split: contiguous row-major bands of equal cost (rank 0 measures the per-tile costs of "
                         "the full frame once at set-up and broadcasts them), bands of equal tile count, or 64x64-pixel "
                         "blocks round-robin")
    ap.add_argument("--camera-path", default="static", choices=["static", "orbit"],
                    help="static: every frame renders the config camera (the headline); orbit: the camera's azimuth "
                         "advances by --orbit-step degrees per frame (a moving camera: the reference's frame loop "
                         "updates the camera every frame, base/VulkanRTBase.cpp:395-440, base/camera.hpp:229-281)")
    ap.add_argument("--orbit-step", type=float, default=0.5, help="degrees of azimuth per frame (--camera-path orbit)")
    ap.add_argument("--rank-balance", type=int, default=0,
                    help="one GPU only: also time each of N ranks' parts of the split (tile lists of --split tiles, "
                         "view groups of --split views) as that rank would render it, and report the imbalance")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=0|1",
                    help="per-handle tuning switch (gvrt_set_option; names in _lib.OPTIONS), for same-box A/B runs; "
                         "none of them changes an image")
    ap.add_argument("--strong", default="bicycle,truck",
                    help="N-rank runs (--gpus N > 1, or --exchange): strong-scaling sub-records of these frames "
                         "(bicycle: the config-2 1080p frame, truck: the config-4 4K frame), each tile-split over the "
                         "ranks in cost bands and exchanged to rank 0; 'none' to skip")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the `configs` sub-record of the default one-GPU line (garden, truck 4K, light field, dense, "
                         "trained stand-in, orbit 0.5 and 2 deg: kernel ms, Mrays/s, VALU issue, visits per wave, "
                         "first frame)")
    ap.add_argument("--configs-child", action="store_true", help=argparse.SUPPRESS)  # PMC child of the configs record
    ap.add_argument("--pmc-keep", default=None, metavar="DIR",
                    help="keep the per-dispatch PMC rows of the line's own passes as DIR/bench_pmc.json (profiles/)")
    ap.add_argument("--strong-budget-s", type=float, default=300.0,
                    help="N-rank runs: a strong-scaling sub-record starts only while the run's wall time is below this "
                         "(rank 0 decides, every rank follows); later ones are listed as skipped, so the line still prints")
    ap.add_argument("--build", default="quality", choices=["quality", "fast"],
                    help="quality: device binned-SAH tree + SAH-optimal 4-wide collapse + large-proxy SplitBLAS pieces (the static-scene build, "
                         "as the reference's PREFER_FAST_TRACE BLAS); fast: device LBVH + greedy collapse")
    args = ap.parse_args()
    if args.split == "auto":
        args.split = "tiles" if args.config == "truck" else "views"
    return args


# ------------------------------------------------------------------------------------------------ host
def cpu_share():
    """CPUs this job may use on the host (affinity, cgroup quota, OMP_NUM_THREADS) and the node's CPU model."""
    n_aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = n_aff
    if quota:
        threads = min(threads, max(1, int(math.floor(quota))))
    if omp and omp.isdigit():
        threads = min(threads, int(omp))
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"threads": max(1, threads), "nproc": os.cpu_count(), "affinity": n_aff, "cgroup_quota_cpus": quota,
            "omp_num_threads": omp, "model": model}


# ------------------------------------------------------------------------------------------------ PMC
def pmc_passes(args):
    """roofline.traffic and the VALU-issue roofline from rocprofv3 PMC passes of THIS command (a short run:
    5 timed + 1 warmup FAST launches after the unordered first frame, which is not averaged; no CPU baseline /
    stats), one counter set per pass as MI355X_MICROARCH.md
    prescribes (FETCH_SIZE and WRITE_SIZE cannot share a pass).  Runs as child processes before this process
    touches the GPU.  Returns per-dispatch averages of the k_render kernel, or {"error": ...}."""
    exe = shutil.which("rocprofv3")
    if not exe:
        return {"error": "rocprofv3 not found"}
    child = [sys.executable, os.path.abspath(__file__), "--gpus", "1", "--steps", "5", "--warmup", "1",
             "--config", args.config, "--split", args.split, "--mode", args.mode, "--build", args.build,
             "--no-cpu-baseline", "--no-stats", "--no-pmc", "--no-configs"]
    if args.ply:
        child += ["--ply", args.ply]
    for kv in args.option:
        child += ["--option", kv]
    if args.camera_path != "static":
        child += ["--camera-path", args.camera_path, "--orbit-step", str(args.orbit_step)]
    out = {}
    kept = []
    # (8 SQ counters and 1 GRBM counter fit one pass; FETCH_SIZE / WRITE_SIZE need TCC passes of their own)
    passes = [["FETCH_SIZE"], ["WRITE_SIZE"],
              ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY",
               "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "GRBM_GUI_ACTIVE"],
              # what the kernel asks of the cache hierarchy: L2 requests and hits, the scalar cache,
              # the vector L1 (3 TCC, 2 TCP, 2 SQ, 1 GRBM counters: within one pass's limits)
              ["TCC_REQ_sum", "TCC_HIT_sum", "TCC_MISS_sum", "TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum",
               "SQC_DCACHE_REQ", "SQC_DCACHE_MISSES", "GRBM_GUI_ACTIVE"]]
    tmp = tempfile.mkdtemp(prefix="gvrt_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        for i, counters in enumerate(passes):
            d = os.path.join(tmp, f"p{i}")
            cmd = ["timeout", "-s", "KILL", "150", exe, "--pmc", *counters, "--kernel-include-regex", "k_render",
                   "-d", d, "-o", "run", "--output-format", "csv", "--", *child]
            r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, timeout=200,
                               env=dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp")))
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if r.returncode != 0 or not files:
                out.setdefault("error", f"pass {counters}: rc {r.returncode} {r.stderr[-300:]}")
                break
            # the timed launches only: FAST k_render dispatches of the frame's grid (config 5's per-view
            # calibration renders and any LITERAL counter launch have other grids / kernels)
            rows = [row for f in files for row in csv.DictReader(open(f))
                    if "k_render<false" in row.get("Kernel_Name", "")]
            grid = max((int(row.get("Grid_Size", 0) or 0) for row in rows), default=0)
            rows = [row for row in rows if int(row.get("Grid_Size", 0) or 0) == grid]
            # not the first launch: it has no previous per-tile costs (supertile order), the timed ones are ordered
            first = min((int(row["Dispatch_Id"]) for row in rows), default=-1)
            rows = [row for row in rows if int(row["Dispatch_Id"]) != first]
            agg, cnt = {}, {}
            for row in rows:
                k = row["Counter_Name"]
                agg[k] = agg.get(k, 0.0) + float(row["Counter_Value"])
                cnt[k] = cnt.get(k, 0) + 1
            out.update({k: agg[k] / cnt[k] for k in agg})
            out["dispatches"] = max(cnt.values()) if cnt else 0
            if args.pmc_keep:  # the rows behind these averages, for profiles/ (scripts/reproduce_line.py)
                kept.extend({"pass": i, "dispatch": int(row["Dispatch_Id"]), "grid": int(row.get("Grid_Size", 0) or 0),
                             "counter": row["Counter_Name"], "value": float(row["Counter_Value"])} for row in rows)
    except subprocess.TimeoutExpired:
        out.setdefault("error", "PMC pass timed out")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    if args.pmc_keep:
        os.makedirs(args.pmc_keep, exist_ok=True)
        with open(os.path.join(args.pmc_keep, "bench_pmc.json"), "w") as f:
            json.dump({"command": child, "passes": passes, "averages": out, "rows": kept}, f, indent=0)
    return out


# ------------------------------------------------------------------------------------------------ configs record
# the other BASELINE configurations in the line the driver runs, one compact record each, measured with
# the headline's protocol (first frame alone, then W warm-up and K timed frames queued back to back, barrier-free one
# GPU).  (label, scene config, camera path)
CONFIG_SET = (("garden", "garden", "static"), ("truck_4k", "truck", "static"), ("lightfield_16", "lightfield", "static"),
              ("dense", "dense", "static"), ("trained", "trained", "static"), ("orbit_0.5deg", "bicycle", "orbit"),
              ("orbit_2deg", "bicycle", "orbit"))
ORBIT_STEPS = {"orbit_0.5deg": 0.5, "orbit_2deg": 2.0}  # degrees of azimuth per frame of the orbit entries


def scene_cached(gv, gen):
    """The seeded stand-in scene; with GVRT_SCENE_CACHE set, generated once and shared (np.save files) between the
    configs record's PMC child and the line's own process, which would otherwise both spend ~20 s generating."""
    d = os.environ.get("GVRT_SCENE_CACHE")
    if not d:
        return gv.scene.make(**gen)
    path = os.path.join(d, f"{gen['kind']}_{gen['n']}_{gen['seed']}.npz")
    if os.path.exists(path):
        with np.load(path) as z:
            return {k: z[k] for k in z.files}
    sp = gv.scene.make(**gen)
    tmp = path + f".{os.getpid()}.npz"
    np.savez(tmp, **sp)
    os.replace(tmp, path)
    return sp


def config_frames(gv, name, path, nframes, step=0.5):
    """Per-frame cameras of one configs-record entry: the config camera (config 5: the centred 16-view rig, as
    `--config lightfield`), or for the orbit path azimuth 30 + k * step in frame k."""
    _, W, H, ncams = gv.scene.CONFIGS[name]
    views = ncams if name == "lightfield" else 1

    def rig(k):
        az = 30.0 + (k * step if path == "orbit" else 0.0)
        v, p = gv.camera.lightfield_grid_rig(gv.camera.orbit_eye(4.0, 20.0, az), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0),
                                             nx=views, ny=1, spacing=0.1, fovy_deg=50.0,
                                             aspect=gv.camera.aspect_ratio(W, H), centred=name == "lightfield")
        return np.ascontiguousarray(np.asarray(v, np.float32).reshape(-1)), p

    frames = [rig(k) for k in range(nframes)] if path == "orbit" else [rig(0)] * nframes
    return frames, W, H, views


def run_config_set(gv, torch, steps, warmup, bicycle_r=None, literal=True, bkw=None):
    """Each CONFIG_SET entry with the headline's timing protocol; returns {label: record} and the number of FAST
    k_render launches of each entry in launch order (the PMC child's manifest)."""
    dev = torch.device("cuda", torch.cuda.current_device())
    recs, manifest = {}, []
    scenes = {}
    for label, name, path in CONFIG_SET:
        gen, _, _, _ = gv.scene.CONFIGS[name]
        key = (gen["kind"], gen["n"], gen["seed"])
        own = False
        if key == ("mipnerf", 1_000_000, 1) and bicycle_r is not None:
            r = bicycle_r
            m = bicycle_r.m
        else:
            if key not in scenes:
                scenes.clear()
                scenes[key] = scene_cached(gv, gen)
            r, own = gv.Renderer(dev.index), True
            m = r.prepare(scenes[key], **(bkw or {}))
        nframes = 1 + warmup + steps
        step = ORBIT_STEPS.get(label, 0.5)
        frames, W, H, views = config_frames(gv, name, path, nframes, step)
        params = r.render_params(mode=gv.MODE_FAST)
        buf = torch.zeros((views * H * W * 4,), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        t = time.perf_counter()
        r.render_device(frames[0][0], frames[0][1], W, H, views, params=params, rgba8_ptr=buf.data_ptr())
        torch.cuda.synchronize()
        first_wall = (time.perf_counter() - t) * 1e3
        first_ms = r.render_ms()
        for k in range(1, 1 + warmup):
            r.render_device(frames[k][0], frames[k][1], W, H, views, params=params, rgba8_ptr=buf.data_ptr(),
                            async_=True)
        r.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(1 + warmup, nframes):
            r.render_device(frames[k][0], frames[k][1], W, H, views, params=params, rgba8_ptr=buf.data_ptr(),
                            async_=True)
        r.sync()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kms = float(r.render_ms())
        rays = W * H * views
        rec = {"config": f"{name}: {gen['n']} Gaussians ({m} survivors), {W}x{H}" + (f" x {views} views" if views > 1 else "")
                         + (f", camera orbiting {step} deg per frame" if path == "orbit" else ""),
               "rays_per_step": rays, "kernel_ms": round(kms, 4), "ms_per_step": round(el / steps * 1e3, 4),
               "mrays": round(rays * steps / el / 1e6, 1), "kernel_mrays": round(rays / (kms * 1e-3) / 1e6, 1),
               "first_frame_kernel_ms": round(first_ms, 4), "first_frame_wall_ms": round(first_wall, 4)}
        if path == "static":
            rec["frame_sha1"] = hashlib.sha1(buf.cpu().numpy().tobytes()).hexdigest()
        if literal:
            # SURVEY §8d's algorithmic bytes from the reference algorithm's counters (LITERAL, frame-0 camera)
            r.set_stats(True)
            r.render(frames[0][0], frames[0][1], W, H, views, params=r.render_params(mode=gv.MODE_LITERAL),
                     rgba8=False, rgba32f=False)
            st = r.stats()
            r.set_stats(False)
            b = 48.0 * st["crossings"] + 192.0 * st["accepted"] + 4.0 * rays
            # the reference algorithm's gather bytes (no fraction: packet traversal shares them, see the roofline)
            rec["reference_gather_bytes"] = b
            rec["reference_gather_equiv_gbs"] = round(b / (kms * 1e-3) / 1e9, 1)
            # traversal diagnostics of the product traversal (the FAST counter kernel): visits per wave
            r.set_stats(True)
            r.render(frames[0][0], frames[0][1], W, H, views, params=r.render_params(mode=gv.MODE_FAST),
                     rgba8=False, rgba32f=False)
            sf = r.stats()
            r.set_stats(False)
            waves = views * ((W + 7) // 8) * ((H + 7) // 8)
            rec["node_visits_per_wave"] = round(sf["wave_node_visits"] / waves, 2)
            rec["leaf_visits_per_wave"] = round(sf["wave_leaf_visits"] / waves, 2)
            rec["rounds_per_wave"] = round(sf["wave_rounds"] / waves, 3)
        manifest.append([label, nframes])
        recs[label] = rec
        del buf
        if own:
            r.close()
    return recs, manifest


def configs_pmc(args):
    """One rocprofv3 SQ pass over a child that renders CONFIG_SET (5 timed + 1 warm-up frames each): the VALU-issue
    fraction of each entry's ordered launches, attributed by dispatch order (the child's manifest).  Before this
    process touches the GPU.  Returns {label: {...}} or {"error": ...}."""
    exe = shutil.which("rocprofv3")
    if not exe:
        return {"error": "rocprofv3 not found"}
    steps, warmup = 5, 1
    child = [sys.executable, os.path.abspath(__file__), "--configs-child", "--steps", str(steps), "--warmup",
             str(warmup), "--build", args.build]
    counters = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "GRBM_GUI_ACTIVE"]
    tmp = tempfile.mkdtemp(prefix="gvrt_cfgpmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        d = os.path.join(tmp, "p")
        cmd = ["timeout", "-s", "KILL", "240", exe, "--pmc", *counters, "--kernel-include-regex", "k_render",
               "-d", d, "-o", "run", "--output-format", "csv", "--", *child]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300,
                           env=dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp")))
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode != 0 or not files or not lines:
            return {"error": f"configs pass: rc {r.returncode} {r.stderr[-300:]}"}
        manifest = json.loads(lines[-1])["manifest"]
        per = {}
        for f in files:
            for row in csv.DictReader(open(f)):
                if "k_render<false" in row.get("Kernel_Name", ""):
                    per.setdefault(int(row["Dispatch_Id"]), {})[row["Counter_Name"]] = float(row["Counter_Value"])
        ids = sorted(per)
        need = sum(n for _, n in manifest)
        if len(ids) != need:
            return {"error": f"configs pass: {len(ids)} k_render dispatches, manifest {need}"}
        out, i = {}, 0
        for label, n in manifest:
            seg = [per[k] for k in ids[i + n - steps:i + n]]  # the timed (cost-ordered) launches
            i += n
            fr = [2.0 * x["SQ_INSTS_VALU"] / (N_SIMD * x["GRBM_GUI_ACTIVE"] / N_XCD) for x in seg]
            wc = sum(x["SQ_WAVE_CYCLES"] for x in seg)
            out[label] = {"valu_issue_frac": round(float(np.mean(fr)), 4),
                          "valu_per_wave": round(sum(x["SQ_INSTS_VALU"] for x in seg) / max(sum(x["SQ_WAVES"] for x in seg), 1), 1),
                          "wave_cycles": {"issuing": round(sum(x["SQ_ACTIVE_INST_ANY"] for x in seg) / wc, 4),
                                          "waiting_on_memory": round(sum(x["SQ_WAIT_ANY"] for x in seg) / wc, 4)}}
        return out
    except subprocess.TimeoutExpired:
        return {"error": "configs PMC pass timed out"}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def tile_cost_calibration(r, vi, pi, W, H, params):
    """Per-tile cost classes of the full frame (gvrt_read_tile_costs after two launches, the second cost-ordered),
    for the cost-weighted band split; before the timed region."""
    import torch
    buf = torch.zeros((H, W, 4), dtype=torch.uint8, device=torch.device("cuda", torch.cuda.current_device()))
    for _ in range(2):
        r.render_device(vi, pi, W, H, 1, params=params, rgba8_ptr=buf.data_ptr())
    return r.tile_costs(W, H)


def split_tiles(dist_mod, layout, W, H, world, classes=None):
    """Every rank's tile list for the tile split (--tile-layout)."""
    if layout == "blocks":
        return dist_mod.rank_tiles(W, H, 1, world, block=8)
    return dist_mod.band_tiles(W, H, world, costs=dist_mod.cost_weights(classes) if layout == "cost-bands" else None)


def view_cost_calibration(r, vis, pi, W, H, params, reps=2):
    """Kernel ms of each view of the rig rendered alone (the last of `reps` launches: cost-ordered)."""
    import torch
    buf = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    out = []
    for v in np.asarray(vis, np.float32).reshape(-1, 16):
        for _ in range(reps):
            r.render_device(np.ascontiguousarray(v), pi, W, H, 1, params=params, rgba8_ptr=buf.data_ptr())
        out.append(float(r.render_ms()))
    return out


def strong_scaling_record(gv, dist_mod, dist, r, vi, pi, W, H, params, rank, world, dev, label, steps=10, warmup=3,
                          probes=3):
    """One frame tile-split over every rank in cost bands, all ranks together:
    rank 0 measures the full frame's per-tile costs (two launches; the second one's kernel time is the one-GPU
    figure), one broadcast gives every rank the classes and the same band cuts, and the split frame runs through
    dist.FrameExchange (exact-size point-to-point sends to rank 0, rank-0 scatter by gvrt_unpack_tiles_rgba8) --
    pipelined for `steps` frames (barrier + sync on both sides, the max over ranks), then `probes` frames one at a
    time with HIP events around each phase: this rank's render (kernel ms from the handle), the exchange (after a
    barrier, so it is the transfer and not a wait for a slower rank's render) and rank 0's assembly.  Returns the
    record on rank 0 (None elsewhere); the assembled frame is checked against rank 0's one-GPU frame."""
    import torch
    H8, W8 = (H + 7) // 8, (W + 7) // 8
    classes = (tile_cost_calibration(r, vi, pi, W, H, params) if rank == 0 else np.zeros((1, H8, W8), np.uint8))
    one_ms = r.render_ms() if rank == 0 else 0.0
    t = torch.from_numpy(np.ascontiguousarray(classes)).to(dev)
    dist.broadcast(t, src=0)
    classes = t.cpu().numpy()
    all_tiles = split_tiles(dist_mod, "cost-bands", W, H, world, classes)
    tiles = all_tiles[rank]
    sizes = [int(x.shape[0]) * 64 for x in all_tiles]
    full = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev) if rank == 0 else None

    def assemble(parts, _k):
        for p, tl in zip(parts, all_tiles):
            if tl.shape[0]:
                r.unpack_tiles_rgba8(p.data_ptr(), tl, W, H, full.data_ptr())

    ex = dist_mod.FrameExchange(dist, rank, world, sizes, (4,), torch.uint8, dev, nbuf=2, assemble=assemble)

    def render_into(buf):
        if tiles.shape[0]:
            r.render_device(vi, pi, W, H, 1, params=params, tiles=tiles, rgba8_ptr=buf.data_ptr(), packed=True,
                            async_=True)

    for _ in range(warmup):
        ex.step(render_into)
    ex.drain()
    r.sync()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ex.step(render_into)
    ex.drain()
    r.sync()
    torch.cuda.synchronize()
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    ms_frame = float(el.item()) / steps * 1e3
    pipe_kms = r.render_ms() if tiles.shape[0] else 0.0  # mean over the pipelined launches
    # per-phase probes, one frame at a time
    pk, px, pa = [], [], []
    for _ in range(probes):
        evs = {}

        def mark(name):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            evs[name] = e

        def barrier():
            torch.cuda.current_stream().synchronize()
            dist.barrier()

        ex.probe(render_into, mark, barrier=barrier)
        r.sync()
        torch.cuda.synchronize()
        pk.append(r.render_ms() if tiles.shape[0] else 0.0)
        px.append(evs["posted"].elapsed_time(evs["exchanged"]))
        pa.append(evs["exchanged"].elapsed_time(evs["assembled"]))
    mine = torch.tensor([pipe_kms, float(np.median(pk)), float(np.median(px)), float(np.median(pa)), sizes[rank] * 4.0],
                        dtype=torch.float64, device=dev)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    if rank != 0:
        return None
    per = torch.stack(allr).cpu().numpy()
    got = hashlib.sha1(full.cpu().numpy().tobytes()).hexdigest()
    ref = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)
    r.render_device(vi, pi, W, H, 1, params=params, rgba8_ptr=ref.data_ptr())
    torch.cuda.synchronize()
    one_sha = hashlib.sha1(ref.cpu().numpy().tobytes()).hexdigest()
    return {"frame": label, "layout": "cost-bands", "ranks": world, "steps": steps,
            "ms_per_frame": round(ms_frame, 4), "mrays": round(W * H / (ms_frame * 1e-3) / 1e6, 1),
            "one_gpu_kernel_ms": round(one_ms, 4),
            "tiles_per_rank": [int(x.shape[0]) for x in all_tiles],
            "kernel_ms_per_rank": [round(float(x), 4) for x in per[:, 0]],
            "probe_kernel_ms_per_rank": [round(float(x), 4) for x in per[:, 1]],
            "exchange_ms_per_rank": [round(float(x), 4) for x in per[:, 2]],
            "assemble_ms": round(float(per[0, 3]), 4),
            "exchange_bytes": int(ex.exchange_bytes), "padded_gather_bytes_round3": int(ex.padded_gather_bytes),
            "bytes_sent_per_rank": [int(x) for x in per[:, 4]],
            "identical_to_one_gpu": got == one_sha, "frame_sha1": got,
            "note": "pipelined: FrameExchange double-buffered, the exchange of frame i under the render of i+1; "
                    "probe_*: one frame at a time, the exchange timed after a barrier (transfer only), assembly on "
                    "rank 0 (gvrt_unpack_tiles_rgba8); rank r > 0 sends its exact part, rank 0's part stays put"}


def rank_balance(args, r, gv, dist_mod, vi_all, pi, W, H, views, params, full_ms, reps=4, view_costs=None):
    """Strong-scaling imbalance measured on one GPU: each of N ranks' parts of the split rendered alone, as that
    rank renders it (its own cost-ordered dispatch: the part is rendered `reps` times, the first launch of a
    list being unordered, and the later ones' median kept).  Tile split: the 64x64-block round-robin tile
    lists of dist.rank_tiles; view split: dist.rank_views of the rig.  implied_efficiency = full-workload
    kernel time / (N x slowest part): the N-GPU efficiency this imbalance allows (gather not included)."""
    import torch
    n = args.rank_balance
    dev = torch.device("cuda", 0)
    ms = []
    layouts = {}
    if args.split == "tiles":
        def time_parts(parts):
            buf = torch.zeros((max(t.shape[0] for t in parts) * 64, 4), dtype=torch.uint8, device=dev)
            out = []
            for t in parts:
                got = []
                for _ in range(reps):
                    r.render_device(vi_all[:16], pi, W, H, 1, params=params, tiles=t, rgba8_ptr=buf.data_ptr(),
                                    packed=True)
                    got.append(r.render_ms())
                out.append(float(np.median(got[1:])))
            return out

        # the full frame's per-tile costs (two launches: the second is cost-ordered and records them again)
        fbuf = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)
        for _ in range(2):
            r.render_device(vi_all[:16], pi, W, H, 1, params=params, rgba8_ptr=fbuf.data_ptr())
        classes = r.tile_costs(W, H)
        costs = dist_mod.cost_weights(classes)
        alts = {k: split_tiles(dist_mod, k, W, H, n, classes) for k in ("cost-bands", "bands", "blocks")
                if k != args.tile_layout}
        parts = split_tiles(dist_mod, args.tile_layout, W, H, n, classes)
        # every layout timed twice, in turn, and the second pass kept (the first parts timed in a process ran
        # up to 10 % slower, whichever layout they belonged to)
        for lay in [parts, *alts.values()]:
            time_parts(lay)
        ms = time_parts(parts)
        for name, p in alts.items():
            pm = time_parts(p)
            est = [float(costs.reshape(-1)[(t[:, 1].astype(np.int64) * ((W + 7) // 8) + t[:, 0])].sum()) for t in p]
            layouts[name] = {"tiles": [int(t.shape[0]) for t in p], "kernel_ms": [round(x, 4) for x in pm],
                             "max_over_mean": round(max(pm) / float(np.mean(pm)), 4),
                             "implied_efficiency": round(full_ms / (n * max(pm)), 4),
                             "cost_max_over_mean_est": round(max(est) / float(np.mean(est)), 4)}
        what = (f"{n} tile lists, layout {args.tile_layout}, "
                f"{min(t.shape[0] for t in parts)}..{max(t.shape[0] for t in parts)} tiles each")
    else:
        vis = np.asarray(vi_all, np.float32).reshape(-1, 16)
        rr = dist_mod.rank_views(views, n)
        groups = dist_mod.balanced_views(view_costs, n) if view_costs else rr
        buf = torch.zeros((max(len(g) for g in groups), H, W, 4), dtype=torch.uint8, device=dev)
        for g in groups:
            if not g:
                continue
            got = []
            for _ in range(reps):
                r.render_device(np.ascontiguousarray(vis[g].reshape(-1)), pi, W, H, len(g), params=params,
                                rgba8_ptr=buf.data_ptr())
                got.append(r.render_ms())
            ms.append(float(np.median(got[1:])))
        what = (f"{n} view groups of the {views}-view rig ({len(groups[0])} views each), "
                + ("cost-balanced (dist.balanced_views: " + str(groups) + ")" if view_costs else "round-robin"))
    mean, mx = float(np.mean(ms)), float(np.max(ms))
    extra = {}
    if args.split != "tiles" and view_costs:
        # the round-robin assignment the balancing replaces, from the same per-view costs
        rrc = [sum(view_costs[v] for v in g) for g in dist_mod.rank_views(views, n)]
        bc = [sum(view_costs[v] for v in g) for g in groups]
        extra = {"view_ms": [round(x, 4) for x in view_costs],
                 "round_robin_max_over_mean_est": round(max(rrc) / float(np.mean(rrc)), 4),
                 "balanced_max_over_mean_est": round(max(bc) / float(np.mean(bc)), 4)}
    if layouts:
        extra["other_layouts"] = layouts
    return {**extra, "ranks": n, "parts": what, "kernel_ms": [round(x, 4) for x in ms], "max_over_mean": round(mx / mean, 4),
            "full_kernel_ms": round(full_ms, 4), "implied_efficiency": round(full_ms / (n * mx), 4),
            "note": "each part alone on one GPU with its own cost-ordered dispatch; median of the ordered launches"}


T_START = time.perf_counter()


def main():
    args = parse()
    dist_mod = importlib.import_module("3dgvrt_lightfield_amd.dist")  # no GPU work at import
    rc = dist_mod.launch_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:])
    if rc is not None:  # this process started the N ranks; rank 0 printed the line
        sys.exit(rc)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1 or (args.exchange and "RANK" in os.environ)
    if args.configs_child:  # the configs record's PMC child: render CONFIG_SET, print the launch manifest
        import torch
        gv = importlib.import_module("3dgvrt_lightfield_amd")
        bkw = dict(gv.QUALITY_BUILD) if args.build == "quality" else {}
        _, manifest = run_config_set(gv, torch, args.steps, args.warmup, literal=False, bkw=bkw)
        print(json.dumps({"manifest": manifest}), flush=True)
        return
    with_configs = (not distributed and world == 1 and not args.no_configs and args.config == "bicycle" and not args.ply
                    and args.camera_path == "static" and args.mode == "fast" and args.split == "views")
    cache_dir = None
    if with_configs and not os.environ.get("GVRT_SCENE_CACHE"):
        cache_dir = tempfile.mkdtemp(prefix="gvrt_scenes_", dir=os.environ.get("TMPDIR", "/tmp"))
        os.environ["GVRT_SCENE_CACHE"] = cache_dir
    pmc = None
    cfg_pmc = None
    if not distributed and not args.no_pmc:
        pmc = pmc_passes(args)  # before this process touches the GPU
        if with_configs:
            cfg_pmc = configs_pmc(args)

    import torch
    import torch.distributed as dist

    gv = importlib.import_module("3dgvrt_lightfield_amd")
    if distributed:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        world = dist.get_world_size()
        rank = dist.get_rank()
    if world != args.gpus:
        print(f"bench: {world} ranks but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
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
    for kv in args.option:
        name, _, val = kv.partition("=")
        r.set_option(name, int(val))
    bkw = dict(gv.QUALITY_BUILD) if args.build == "quality" else {}
    m = r.prepare(splats, **bkw)
    first_build = r.stats()  # includes the one-time lazy loading of the build kernels' code objects
    m = r.prepare(splats, **bkw)    # steady-state scene build (what a scene change costs)
    st0 = r.stats()

    # cameras: an N-view planar rig starting at the config camera (view 0 = the config camera for any N);
    # config 5 (lightfield) is its centred 16-view array
    # --camera-path orbit: frame k's rig sits at azimuth 30 + k * orbit_step (the static headline: k = 0 always)
    views = world if args.split == "views" else 1
    views = max(views, ncams_cfg if args.config == "lightfield" else 1)

    def rig(k):
        if args.config == "config1":
            eye, fovy = (0.0, 0.0, 3.0), gv.camera.FOV_Y
        else:
            az = 30.0 + (k * args.orbit_step if args.camera_path == "orbit" else 0.0)
            eye, fovy = gv.camera.orbit_eye(4.0, 20.0, az), 50.0  # k = 0: scene.mipnerf_camera (view 0)
        v, p = gv.camera.lightfield_grid_rig(eye, (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), nx=views, ny=1, spacing=0.1,
                                             fovy_deg=fovy, aspect=gv.camera.aspect_ratio(W, H),
                                             centred=args.config == "lightfield")
        return v.reshape(views, 16), p

    nframes = 1 + args.warmup + args.steps
    rigs = [rig(k) for k in range(nframes)] if args.camera_path == "orbit" else [rig(0)] * nframes
    vis, pi = rigs[0]
    mode = gv.MODE_FAST if args.mode == "fast" else gv.MODE_LITERAL
    params = r.render_params(mode=mode)
    view_costs = None
    if args.split == "views":
        all_views = dist_mod.rank_views(views, world)
        if views > world:
            # more views than ranks (config 5): views differ in cost (measured up to 1.4x), so they are assigned by
            # cost: rank 0 times each view alone once (its second launch, cost-ordered), every rank gets the costs
            # (one broadcast at set-up, not per frame) and computes the same assignment (dist.balanced_views)
            view_costs = view_cost_calibration(r, rigs[0][0], rigs[0][1], W, H, params) if rank == 0 else [0.0] * views
            if distributed:
                t = torch.tensor(view_costs, dtype=torch.float64, device=dev)
                dist.broadcast(t, src=0)
                view_costs = t.cpu().tolist()
            all_views = dist_mod.balanced_views(view_costs, world)
        my_views = all_views[rank]
        frame_vi = [np.ascontiguousarray(v[my_views].reshape(-1)) for v, _ in rigs]
        ncams = len(my_views)
        tiles = None
        rays_per_rank = W * H * ncams
        part_sizes, item_shape = [len(v) for v in all_views], (H, W, 4)
    else:
        frame_vi = [np.ascontiguousarray(v[0]) for v, _ in rigs]
        ncams = 1
        classes = None
        if args.tile_layout == "cost-bands":
            # the frame's tiles differ in cost (4x on bicycle): rank 0 measures them once, every rank gets the
            # classes (one broadcast at set-up, not per frame) and computes the same band cuts
            classes = (tile_cost_calibration(r, frame_vi[0], pi, W, H, params) if rank == 0
                       else np.zeros((1, (H + 7) // 8, (W + 7) // 8), np.uint8))
            if distributed:
                t = torch.from_numpy(classes).to(dev)
                dist.broadcast(t, src=0)
                classes = t.cpu().numpy()
        all_tiles = split_tiles(dist_mod, args.tile_layout, W, H, world, classes)
        tiles = all_tiles[rank]
        rays_per_rank = int(tiles.shape[0]) * 64
        part_sizes, item_shape = [t.shape[0] * 64 for t in all_tiles], (4,)
    packed = args.split == "tiles"
    kernel_ms = []
    full = None
    frame_k = [0]  # frames rendered so far (frame_vi index)

    def next_vi():
        v = frame_vi[min(frame_k[0], nframes - 1)]
        frame_k[0] += 1
        return v

    if distributed:
        # one exchange step per frame: dist.FrameExchange, double-buffered RCCL gather to rank 0
        if packed and rank == 0:
            full = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)

        def assemble(parts, _frame):  # rank 0: tile parts -> the frame (gvrt_unpack_tiles_rgba8)
            if packed:
                for p, t in zip(parts, all_tiles):
                    r.unpack_tiles_rgba8(p.data_ptr(), t, W, H, full.data_ptr())

        # Frames are queued as on one GPU (gvrt_render_async), on torch's stream (gvrt_set_stream): the
        # gather of a frame is posted behind its render, the wait for the gather that last used a buffer
        # (work.wait) precedes the next render into it, all ordered on the device with no host round trip.
        xs = torch.cuda.Stream(dev)  # not the null stream: the handle's own stream does not order with it
        torch.cuda.synchronize()
        torch.cuda.set_stream(xs)
        r.set_stream(xs.cuda_stream)
        ex = dist_mod.FrameExchange(dist, rank, world, part_sizes, item_shape, torch.uint8, dev, nbuf=2,
                                    assemble=assemble, sync=None)

        def render_into(buf):
            r.render_device(next_vi(), pi, W, H, ncams, params=params, tiles=tiles, rgba8_ptr=buf.data_ptr(),
                            packed=packed, async_=True)

        def step():
            ex.step(render_into)

        def drain():
            ex.drain()
            r.sync()
            kernel_ms.append(r.render_ms())  # mean over the queued launches
    else:
        # One GPU: frames are queued back to back (gvrt_render_async; one host round trip per K frames instead
        # of one per frame); the kernel time is the mean over the queued launches (HIP event pairs), at sync.
        frame = torch.zeros((part_sizes[0],) + item_shape, dtype=torch.uint8, device=dev)

        def step():
            r.render_device(next_vi(), pi, W, H, ncams, params=params, tiles=tiles, rgba8_ptr=frame.data_ptr(),
                            packed=packed, async_=True)

        def drain():
            r.sync()
            kernel_ms.append(r.render_ms())  # mean over the queued launches

    # the first frame of a frame size has no previous per-tile costs: it is dispatched in supertile order
    # (frame 0, rendered synchronously and timed on its own; the handle orders every later frame)
    first_buf = torch.zeros((part_sizes[0],) + item_shape, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t_ff = time.perf_counter()
    r.render_device(next_vi(), pi, W, H, ncams, params=params, tiles=tiles, rgba8_ptr=first_buf.data_ptr(),
                    packed=packed)
    torch.cuda.synchronize()
    first_frame_wall_ms = (time.perf_counter() - t_ff) * 1e3  # host call + the unordered launch, synchronous
    first_frame_ms = r.render_ms()
    del first_buf
    for _ in range(args.warmup):
        step()
    drain()
    kernel_ms.clear()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()  # every frame of the timed steps is rendered (and gathered and assembled) inside the clock
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

    # digest of view 0 as rank 0 holds it after the exchange (tile split: the assembled frame, equal for any N)
    digest = None
    if rank == 0:
        if distributed:
            if packed:
                img = full
            else:  # view 0 in the part of the rank that rendered it
                r0 = next(k for k, g in enumerate(all_views) if 0 in g)
                img = ex.parts((ex.frames - 1) % ex.nbuf)[r0][all_views[r0].index(0)]
        else:
            img = frame if not packed else None
            if packed:  # one rank: unpack the whole frame's tiles
                img = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)
                r.unpack_tiles_rgba8(frame.data_ptr(), tiles, W, H, img.data_ptr())
            else:
                img = frame[my_views.index(0)]
        torch.cuda.synchronize()
        digest = hashlib.sha1(img.cpu().numpy().tobytes()).hexdigest()

    # ---- strong-scaling sub-records (N-rank runs): one frame tile-split over all ranks, every rank taking part
    strong = []
    if distributed and args.strong != "none":
        for name in [x for x in args.strong.split(",") if x]:
            # the wall-time budget: rank 0's clock decides for every rank (one broadcast), so no rank waits in a
            # sub-record its peers skipped
            go = torch.tensor([1.0 if time.perf_counter() - T_START < args.strong_budget_s else 0.0], device=dev)
            dist.broadcast(go, src=0)
            if go.item() == 0.0:
                if rank == 0:
                    strong.append({"frame": name, "skipped": f"wall-time budget {args.strong_budget_s:.0f} s reached "
                                                              f"({time.perf_counter() - T_START:.0f} s into the run)"})
                continue
            t_rec = time.perf_counter()
            if name == "bicycle" and args.config == "bicycle" and not args.ply:
                rs, own = r, False
            else:
                gen_s, _, _, _ = gv.scene.CONFIGS[name]
                rs, own = gv.Renderer(local_rank), True
                rs.prepare(gv.scene.make(**gen_s), **bkw)
                rs.set_stream(torch.cuda.current_stream().cuda_stream)
            _, Ws, Hs, _ = gv.scene.CONFIGS[name]
            vs, ps = gv.scene.mipnerf_camera(Ws, Hs)
            rec = strong_scaling_record(gv, dist_mod, dist, rs, np.ascontiguousarray(vs, np.float32), ps, Ws, Hs,
                                        rs.render_params(mode=mode), rank, world, dev,
                                        f"{name} {Ws}x{Hs} ({'config 2' if name == 'bicycle' else 'config 4'})")
            if own:
                rs.close()
            if rec:
                rec["wall_s"] = round(time.perf_counter() - t_rec, 2)  # scene build, calibration and the timed frames
                strong.append(rec)

    if rank == 0:
        # ---- roofline.  The binding resource, from the PMC passes of this command: instruction issue.  The kernel
        # moves ~0.2 GB per launch through HBM (2-3 % of 8 TB/s) and its waves spend their lifetime issuing (~42 %),
        # waiting on dependent scalar loads (~38 %) or ready behind other waves' issue (~20 %); the busiest unit is
        # the SIMDs' VALU pipe: frac = 2 x VALU wave-instructions / (1024 SIMDs x the dispatch's cycles), <= 1 by
        # construction.  Beside it what the kernel asks of the cache hierarchy (L2 requests against
        # the L2 peak, the scalar cache, the vector L1) and a latency account (dependent scalar loads per wave x the
        # L2 hit latency / the wave lifetime); `binding` names the largest of the three fractions.
        # roofline.reference_gather keeps SURVEY §8d's algorithmic bytes (the reference algorithm's one-ray-at-a-time
        # gathers, from the LITERAL counters) as a plain figure: packet traversal shares those gathers across a wave's
        # 64 rays, so it is neither a bound nor a physical rate.
        roof = None
        lit_stats = None
        fast_stats = None
        logical = None
        vi = frame_vi[0]  # the frame-0 camera (the static headline's) for the counters and the CPU baseline
        if not args.no_stats:
            r.set_stats(True)
            r.render(vi[:16], pi, W, H, 1, params=r.render_params(mode=gv.MODE_LITERAL), rgba8=False, rgba32f=False)
            lit_stats = r.stats()
            r.set_stats(False)
            rays1 = W * H
            bytes_per_launch = (48.0 * lit_stats["crossings"] + 192.0 * lit_stats["accepted"] + 4.0 * rays1) * (
                rays_per_rank / rays1)
            achieved = bytes_per_launch / (kern_avg * 1e-3) / 1e9
            logical = {"bytes_per_launch": bytes_per_launch, "equivalent_gbs": round(achieved, 1),
                       "note": "SURVEY §8d: sum over rays of 48 B per crossing + 192 B per accepted crossing + 4 B (the "
                               "reference algorithm's LITERAL counters) / kernel time.  Not a bound and not a physical "
                               "rate: the packet traversal issues one scalar gather per wave where this counts 64"}
            # the product traversal's visits (FAST counter kernel, same traversal as the timed kernel)
            r.set_stats(True)
            r.render(vi[:16], pi, W, H, 1, params=r.render_params(mode=gv.MODE_FAST), rgba8=False, rgba32f=False)
            fast_stats = r.stats()
            r.set_stats(False)
        traffic = None
        if pmc and "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
            # FETCH_SIZE in KiB, half-counted on gfx950 (x2); WRITE_SIZE in KiB (MI355X_MICROARCH.md, HBM)
            traffic = pmc["FETCH_SIZE"] * 1024 * 2 + pmc["WRITE_SIZE"] * 1024
        kern = "k_render<FAST,K=32,packed>" if args.mode == "fast" else "k_render<LITERAL,K=16>"
        if pmc and "SQ_INSTS_VALU" in pmc and pmc.get("GRBM_GUI_ACTIVE"):
            cyc = pmc["GRBM_GUI_ACTIVE"] / N_XCD  # shader cycles of the dispatch
            clock = cyc / (kern_avg * 1e-3)
            rate = pmc["SQ_INSTS_VALU"] / (kern_avg * 1e-3)
            peak = N_SIMD * clock / 2.0
            waves = max(pmc.get("SQ_WAVES", 1), 1)
            roof = {"bound": "issue", "achieved": rate, "peak": peak, "unit": "VALU wave-instr/s",
                    "frac": round(2.0 * pmc["SQ_INSTS_VALU"] / (N_SIMD * cyc), 4), "traffic": traffic,
                    "binding_unit": "SIMD VALU issue: a wave64 VALU instruction holds a SIMD-32 for 2 cycles; peak = "
                                    "1024 SIMDs x the dispatch's clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time) / 2",
                    "clock_ghz": round(clock / 1e9, 4),
                    "valu_per_wave": pmc["SQ_INSTS_VALU"] / waves,
                    "salu_per_wave": pmc.get("SQ_INSTS_SALU", 0) / waves,
                    "smem_per_wave": pmc.get("SQ_INSTS_SMEM", 0) / waves}
            if pmc.get("SQ_WAVE_CYCLES"):
                wc = pmc["SQ_WAVE_CYCLES"]
                roof["wave_cycles"] = {"issuing": round(pmc.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4),
                                       "waiting_on_memory": round(pmc.get("SQ_WAIT_ANY", 0) / wc, 4),
                                       "ready_not_issued": round(pmc.get("SQ_WAIT_INST_ANY", 0) / wc, 4)}
        else:  # no PMC passes (--no-pmc or rocprofv3 missing): nothing measured binds
            roof = {"bound": "unmeasured", "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": traffic,
                    "note": "no PMC passes: " + str((pmc or {}).get("error", "--no-pmc"))}
        if roof is not None and traffic is not None and "wave_cycles" in roof:
            # the binding unit is the busier of the two measured resources: VALU issue or HBM bytes
            hbm_frac = traffic / (kern_avg * 1e-3) / 1e9 / HBM_PEAK_GBS
            if hbm_frac > roof["frac"]:
                roof.update({"bound": "hbm", "achieved": traffic / (kern_avg * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(hbm_frac, 4), "valu_issue_frac": roof["frac"]})
        if roof is not None:
            roof["kernel_ms_avg"] = round(kern_avg, 4)
            roof["kernel"] = kern
            if logical:
                roof["reference_gather"] = logical
            if pmc and pmc.get("TCC_REQ_sum") is not None and pmc.get("SQ_WAVES"):
                # L2 (TCC) requests: each moves at most one 128-B line, so req x 128 B bounds the bytes L2 served
                l2_bytes = pmc["TCC_REQ_sum"] * 128.0
                l2_gbs = l2_bytes / (kern_avg * 1e-3) / 1e9
                hits = pmc.get("TCC_HIT_sum", 0.0)
                miss = pmc.get("TCC_MISS_sum", 0.0)
                sq_req = pmc.get("SQC_DCACHE_REQ", 0.0)
                roof["cache"] = {
                    "l2_requests": pmc["TCC_REQ_sum"], "l2_hit_rate": round(hits / max(hits + miss, 1.0), 4),
                    "l2_request_bytes_max": l2_bytes, "l2_gbs_max": round(l2_gbs, 1), "l2_peak_gbs": L2_PEAK_GBS,
                    "l2_frac": round(l2_gbs / L2_PEAK_GBS, 4),
                    "scalar_loads": pmc.get("SQ_INSTS_SMEM"),
                    "scalar_request_bytes": pmc.get("SQ_INSTS_SMEM", 0.0) * 64.0,
                    "scalar_cache_requests": sq_req,
                    "scalar_cache_hit_rate": round(1.0 - pmc.get("SQC_DCACHE_MISSES", 0.0) / max(sq_req, 1.0), 4),
                    "vector_l1_accesses": pmc.get("TCP_TOTAL_CACHE_ACCESSES_sum"),
                    "vector_l1_to_l2_reads": pmc.get("TCP_TCC_READ_REQ_sum"),
                    "note": "per launch.  Scalar loads are the wave-uniform node (2 x 64 B) and leaf-record (64 B) "
                            "fetches; vector L1 accesses are the per-lane record and SH loads of the composite; L2 "
                            "serves both.  l2_frac = TCC_REQ_sum x 128 B / kernel time / the guide's 34.5 TB/s L2 peak "
                            "(an upper bound on the bytes: a request moves at most one line)"}
            if fast_stats and pmc and pmc.get("SQ_WAVE_CYCLES") and pmc.get("SQ_WAVES"):
                waves = pmc["SQ_WAVES"]
                life = 4.0 * pmc["SQ_WAVE_CYCLES"] / waves  # SQ_WAVE_CYCLES counts quad-cycles
                nv = fast_stats["wave_node_visits"] / waves
                lv = fast_stats["wave_leaf_visits"] / waves
                roof["latency"] = {
                    "node_visits_per_wave": round(nv, 2), "leaf_visits_per_wave": round(lv, 2),
                    "rounds_per_wave": round(fast_stats["wave_rounds"] / waves, 3),
                    "wave_lifetime_cycles": round(life, 1), "l2_hit_latency_cycles": L2_LAT_CYC,
                    "frac": round((nv + lv) * L2_LAT_CYC / life, 4),
                    "note": "each node and leaf visit waits for one dependent scalar load (a node's two loads issue "
                            "together); frac = (node + leaf visits per wave) x the guide's L2-hit latency / the wave's "
                            "lifetime (4 x SQ_WAVE_CYCLES / SQ_WAVES): the share of a wave's life spent waiting on the "
                            "chain if every load hit L2 (Infinity Cache hits take ~545 cycles)"}
            fr = {"valu_issue": roof.get("valu_issue_frac", roof["frac"]) if roof["bound"] == "hbm" else roof["frac"],
                  "l2_bandwidth": roof.get("cache", {}).get("l2_frac"),
                  "dependent_load_latency": roof.get("latency", {}).get("frac")}
            fr = {k: v for k, v in fr.items() if v is not None}
            if fr:
                roof["binding"] = {"fractions": fr, "largest": max(fr, key=fr.get)}
            if traffic is not None:
                hb = traffic / (kern_avg * 1e-3) / 1e9
                roof["hbm"] = {"achieved": round(hb, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(hb / HBM_PEAK_GBS, 5),
                               "traffic_read_bytes": pmc["FETCH_SIZE"] * 1024 * 2,
                               "traffic_write_bytes": pmc["WRITE_SIZE"] * 1024}
            if pmc:
                roof["pmc"] = {k: v for k, v in pmc.items()}

        # ---- CPU baseline (oracle restatement on the host's CPU share), PSNR vs oracle on the sample
        cpu = None
        psnr = None
        if not args.no_cpu_baseline and world == 1:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O

            host = cpu_share()
            threads = host["threads"]
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
            ref = sc.render(vi[:16], pi, W, H, subset=sub, threads=threads, margin=True)
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
                   "sample_1core": f"{len(sub1)} rays (strided over view 0), {dt1:.1f} s on 1 thread",
                   "node": {"nproc": host["nproc"], "cpu_model": host["model"], "affinity_cpus": host["affinity"],
                            "cgroup_quota_cpus": host["cgroup_quota_cpus"], "omp_num_threads": host["omp_num_threads"],
                            "threads_used": "the job's CPU share: min(affinity, cgroup quota, OMP_NUM_THREADS)"}}
            img = r.render(vi[:16], pi, W, H, 1, params=params, rgba32f=True, rgba8=True)
            got = img["rgba8"].reshape(-1, 4)[sub.astype(np.int64)]
            psnr = gv.psnr_rgb(got, gv.quantize_rgba8(ref["rgba32f"]))
            gotf = img["rgba32f"].reshape(-1, 4)[sub.astype(np.int64)]
            amb = O.ambiguous(ref["margin"])
            d = np.abs(gotf[:, :3] - ref["rgba32f"][:, :3]).max(axis=1)
            cpu["parity"] = {"rays": int(len(sub)), "on_threshold": int(amb.sum()),
                             "max_abs_diff_off_threshold": float(d[~amb].max()) if (~amb).any() else 0.0,
                             "frac_beyond_1e-4_off_threshold": float((d[~amb] > 1e-4).mean()) if (~amb).any() else 0.0,
                             "frac_beyond_1e-4_all": float((d > 1e-4).mean())}

        # the host-buffer boundary (gvrt_render with host pointers: the frame staged in the handle's scratch and
        # copied over PCIe, the call returns when the host holds it): rgba8 of the same frame, not the bench value
        host_out = None
        if world == 1 and args.split == "views" and ncams == 1:
            for _ in range(2):
                r.render(frame_vi[0], pi, W, H, 1, params=params, rgba32f=False)
            reps = 10
            t0 = time.perf_counter()
            for _ in range(reps):
                r.render(frame_vi[0], pi, W, H, 1, params=params, rgba32f=False)
            hms = (time.perf_counter() - t0) * 1e3 / reps
            host_out = {"ms_per_frame": round(hms, 4), "mrays_per_s": round(W * H / hms / 1e3, 1),
                        "note": "gvrt_render into host rgba8 (staged + D2H copy over PCIe, synchronous), 10 frames"}

        # moving camera: the same views rendered as static frames (each view twice in a row, the second launch
        # ordered by its own costs), so the moving-camera penalty is measured on equal work
        orbit_static = None
        if args.camera_path == "orbit" and world == 1:
            import torch
            buf = torch.zeros((part_sizes[0],) + item_shape, dtype=torch.uint8, device=dev)
            ks = list(range(1 + args.warmup, nframes, max(1, args.steps // 10)))
            got = []
            for k in ks:
                for _ in range(2):
                    r.render_device(frame_vi[k], pi, W, H, ncams, params=params, tiles=tiles, rgba8_ptr=buf.data_ptr(),
                                    packed=packed)
                got.append(r.render_ms())
            orbit_static = {"kernel_ms": round(float(np.mean(got)), 4), "views": len(ks),
                            "note": "every ~10th timed view rendered twice as a static frame (second launch ordered by "
                                    "its own costs): the static cost of the same views"}
        balance = None
        if args.rank_balance > 1 and world == 1:
            if args.split == "views" and views > args.rank_balance:
                vc = view_cost_calibration(r, rigs[0][0], rigs[0][1], W, H, params)
            else:
                vc = None
            balance = rank_balance(args, r, gv, dist_mod, frame_vi[0], pi, W, H, views, params, kern_avg, view_costs=vc)

        # ---- the other BASELINE configurations, after everything else the line measures
        configs = None
        if with_configs:
            t_cfg = time.perf_counter()
            configs, _ = run_config_set(gv, torch, args.steps, args.warmup, bicycle_r=r, bkw=bkw)
            for label, rec in configs.items():
                if cfg_pmc and label in cfg_pmc:
                    rec.update(cfg_pmc[label])
                elif cfg_pmc and "error" in cfg_pmc:
                    rec["valu_issue_frac"] = None
            configs["_note"] = (f"each config timed as the headline ({args.warmup} warm-up + {args.steps} timed frames "
                                "queued back to back after an unordered first frame); valu_issue_frac from one rocprofv3 SQ "
                                "pass of a child rendering the same set (5 timed frames each); reference_gather_* = SURVEY "
                                "§8d bytes of the reference's one-ray-at-a-time gathers (LITERAL counters), not a physical "
                                "rate; node / leaf visits and rounds per wave from the FAST counter kernel; whole record "
                                f"{time.perf_counter() - t_cfg:.1f} s")
            if cfg_pmc and "error" in cfg_pmc:
                configs["_pmc_error"] = cfg_pmc["error"]
        if cache_dir:
            shutil.rmtree(cache_dir, ignore_errors=True)

        result = {
            "metric": "Mrays/s + fps @1920x1080, 1M Gaussians; PSNR vs Vulkan reference",
            "value": round(mrays, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            # weak: each rank's work is fixed as N grows (one view per rank); strong: the total is fixed (one frame
            # tile-split, or the 16-view light field over N <= 16 ranks)
            "scaling": "weak" if args.split == "views" and views == world else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": (f"real scene {os.path.basename(args.ply)}" if args.ply
                     else "synthetic (seeded stand-in scene, SURVEY §8d)"),
            "config": {"workload": f"{args.config}: {n_input} {'PLY' if args.ply else 'synthetic'} Gaussians, {W}x{H}, "
                                   f"{'one view per rank' if args.split == 'views' else 'one frame tile-split'}, "
                                   f"ray-query variant, {args.mode} k-buffer",
                       "gaussians": n_input, "survivors": m, "width": W, "height": H,
                       "views": views, "split": args.split, "parallelism": f"{args.split}{world}",
                       **({"tile_layout": args.tile_layout} if args.split == "tiles" else {}),
                       "dispatch": "tiles costliest-first by the previous frame's per-tile cost, each cost class "
                                   "dealt to the 8 XCDs in contiguous chunks (handle options tile_order=0: supertile order; "
                                   "tile_xcd=0: no dealing)",
                       "build": ("quality: device binned-SAH tree + SAH-optimal 4-wide collapse, proxies spanning 3+ "
                                 "of 10 SplitBLAS cells split into cell pieces" if args.build == "quality"
                                 else "fast: device LBVH + greedy 4-wide collapse")},
            "fps": round(1e3 / ms_per_step, 2),
            "kernel_ms": round(kern_avg, 4),
            "kernel_mrays": round(rays_per_rank / (kern_avg * 1e-3) / 1e6, 3) if kern_avg == kern_avg else None,
            "psnr_vs_oracle_db": None if psnr is None else (round(psnr, 2) if math.isfinite(psnr) else "inf"),
            "frame_sha1": digest,
            "options": {kv.partition("=")[0]: int(kv.partition("=")[2]) for kv in args.option} or None,
            "camera_path": (f"orbit: azimuth 30 + {args.orbit_step} deg per frame (every frame a new camera; the "
                            f"cost order of each frame from its predecessor)" if args.camera_path == "orbit"
                            else "static: every frame the config camera"),
            "first_frame_kernel_ms": round(first_frame_ms, 4),
            "first_frame_wall_ms": round(first_frame_wall_ms, 4),
            "enclose_ms": round(st0["enclose_ms"], 3),
            "accel_ms": round(st0["accel_ms"], 3),
            "first_build_ms": round(first_build["enclose_ms"] + first_build["accel_ms"], 3),
            "bvh_depth": st0["bvh_depth"],
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if balance:
            result["rank_balance"] = balance
        if strong:
            result["strong_scaling"] = strong
        if orbit_static:
            result["orbit_same_views_static"] = orbit_static
        if configs:
            result["configs"] = configs
        if host_out:
            result["host_output_pcie"] = host_out
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
