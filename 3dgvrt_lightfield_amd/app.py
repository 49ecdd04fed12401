"""Headless host application around libgvrt.so: the `VulkanFullRT` analogue of SURVEY §8b ("gvrt_app").

Mirrors what the reference application does around the hot path, minus window / swapchain:

  prepare()          VulkanFullRT::prepare (VulkanFullRT.cpp:1990-2113): load PLY (or a synthetic
                     SURVEY §8d scene), Gaussian Enclosing pass, acceleration structure
  draw()             VulkanFullRT::draw (:2115): one Particle Rendering pass for one camera
  eval capture       VulkanFullRT.cpp:2127-2161 (EVAL_QUALITY): render every camera of a NeRF
                     `transforms_*.json` and write `r_<i>.png` (RGBA, stbi_write_png layout)
  light field        computeGaussianLightField (:1900-1976): ring rig (4 views) or the config-5 grid,
                     one batched launch, a PNG per view plus `rayDirs` ([cam][x][y] float4, .npy)
  hit counts         printRayHitCounts (:2182-2195): accepted hits per pixel, "%u " per pixel, one
                     line per row (`rayHitCountsOutput.txt`)
  benchmark          vks::Benchmark (base/benchmark.hpp:37-104): warm-up seconds, then timed frames for
                     `duration` seconds; `fps.txt` CSV "device,driverversion,duration (ms),frames,fps"
                     (fixed, 4 decimals) and optional "frame,ms" rows
  psnr / ssim        results/evaluations/eval_quality.py:9-62: per-image PSNR over the 3 colour channels
                     (peak 255) and SSIM as skimage.structural_similarity(channel_axis=-1, win_size=7)
                     with its defaults (uniform 7x7 window, sample covariance, K1 0.01, K2 0.03,
                     data range 255), averaged over the files present in both folders

CLI:  python -m 3dgvrt_lightfield_amd.app {render,eval,lightfield,hitcounts,bench,psnr} ...
"""
import argparse
import importlib
import os
import sys
import time

import numpy as np

gv = importlib.import_module(__package__ or "3dgvrt_lightfield_amd")
camera = gv.camera


# ---------------------------------------------------------------------------------------- images
def save_png(path, rgba8):
    from PIL import Image  # PNG writer only; the product path never needs it
    a = np.ascontiguousarray(rgba8, np.uint8)
    Image.fromarray(a, "RGBA" if a.shape[-1] == 4 else "RGB").save(path)


def load_png_rgb(path):
    """cv2.imread(path) (IMREAD_COLOR) drops alpha; PSNR/SSIM are channel-order independent."""
    from PIL import Image
    return np.asarray(Image.open(path).convert("RGB"), np.uint8)


def write_hit_counts_txt(path, counts):
    c = np.asarray(counts, np.uint32)
    with open(path, "w") as fh:
        for row in c.reshape(c.shape[-2], c.shape[-1]):
            fh.write("".join(f"{int(v)} " for v in row))
            fh.write("\n")


def psnr(img1, img2):
    """eval_quality.py:9-14."""
    mse = np.mean((img1.astype(np.float32) - img2.astype(np.float32)) ** 2)
    if mse == 0:
        return float("inf")
    return 10 * np.log10((255.0 ** 2) / mse)


def ssim(img1, img2, win_size=7):
    """skimage.metrics.structural_similarity(img1, img2, channel_axis=-1, win_size=7) for uint8 input,
    restated with its documented defaults (skimage is not installed here: parity unpinned)."""
    from scipy.ndimage import uniform_filter
    h, w = img1.shape[:2]
    if min(h, w) < win_size:  # eval_quality.py:21-24
        win_size = min(h, w) if min(h, w) % 2 == 1 else min(h, w) - 1
    x_all = img1.astype(np.float64)
    y_all = img2.astype(np.float64)
    R = 255.0
    c1, c2 = (0.01 * R) ** 2, (0.03 * R) ** 2
    npx = win_size ** 2
    cov_norm = npx / (npx - 1.0)
    pad = (win_size - 1) // 2
    vals = []
    for ch in range(x_all.shape[-1]):
        x, y = x_all[..., ch], y_all[..., ch]
        ux, uy = uniform_filter(x, win_size), uniform_filter(y, win_size)
        uxx, uyy, uxy = uniform_filter(x * x, win_size), uniform_filter(y * y, win_size), uniform_filter(x * y, win_size)
        vx, vy, vxy = cov_norm * (uxx - ux * ux), cov_norm * (uyy - uy * uy), cov_norm * (uxy - ux * uy)
        s = ((2 * ux * uy + c1) * (2 * vxy + c2)) / ((ux * ux + uy * uy + c1) * (vx + vy + c2))
        vals.append(s[pad:s.shape[0] - pad, pad:s.shape[1] - pad].mean())
    return float(np.mean(vals))


def compare_dirs(gt_dir, test_dir, with_ssim=True):
    """eval_quality.py main loop for one test folder: returns ({file: (psnr, ssim)}, avg_psnr, avg_ssim)."""
    res = {}
    for fname in sorted(os.listdir(gt_dir)):
        tp = os.path.join(test_dir, fname)
        if not os.path.exists(tp):
            continue
        a, b = load_png_rgb(os.path.join(gt_dir, fname)), load_png_rgb(tp)
        res[fname] = (psnr(a, b), ssim(a, b) if with_ssim else float("nan"))
    p = [v[0] for v in res.values()]
    s = [v[1] for v in res.values()]
    return res, (sum(p) / len(p) if p else float("nan")), (sum(s) / len(s) if s else float("nan"))


# ---------------------------------------------------------------------------------------- benchmark
class Benchmark:
    """vks::Benchmark (base/benchmark.hpp:22-104)."""

    def __init__(self, warmup=1.0, duration=10.0, filename="fps.txt", output_frame_times=False):
        self.warmup, self.duration, self.filename = warmup, duration, filename
        self.output_frame_times = output_frame_times
        self.frame_times = []
        self.runtime = 0.0
        self.device, self.driver = "unknown", "unknown"

    def run(self, render_fn, sync_fn):
        t_meas = 0.0
        while t_meas < self.warmup * 1000.0:  # benchmark.hpp:50-56
            t0 = time.perf_counter()
            render_fn()
            sync_fn()
            t_meas += (time.perf_counter() - t0) * 1000.0
        while self.runtime < self.duration * 1000.0:  # :60-66
            t0 = time.perf_counter()
            render_fn()
            sync_fn()
            dt = (time.perf_counter() - t0) * 1000.0
            self.runtime += dt
            self.frame_times.append(dt)
        return len(self.frame_times) / (self.runtime / 1000.0)

    def save_results(self):
        n = len(self.frame_times)
        with open(self.filename, "w") as fh:  # benchmark.hpp:77-104
            fh.write("device,driverversion,duration (ms),frames,fps\n")
            fh.write(f"{self.device},{self.driver},{self.runtime:.4f},{n},{n / (self.runtime / 1000.0):.4f}\n")
            if self.output_frame_times:
                fh.write("\nframe,ms\n")
                for i, t in enumerate(self.frame_times):
                    fh.write(f"{i},{t:.4f}\n")


# ---------------------------------------------------------------------------------------- app
class GvrtApp:
    """prepare() / draw() around one gvrt handle (one device, one stream)."""

    def __init__(self, device=0):
        self.r = gv.Renderer(device)
        self.splats = None
        self.m = 0

    def close(self):
        self.r.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def prepare(self, ply=None, config=None, **enclosing):
        if ply:
            s = gv.SplatSet()
            if not gv.PLYLoader().loadPLYModel(ply, s):
                raise gv.GvrtError(-6, f"cannot load {ply}")  # GVRT_ERR_IO
            self.splats = s
        else:
            gen = gv.scene.CONFIGS[config or "config1"][0]
            self.splats = gv.scene.make(**gen)
        self.m = self.r.prepare(self.splats, **enclosing)
        return self.m

    def draw(self, view_inv, proj_inv, width, height, **kw):
        return self.r.render(view_inv, proj_inv, width, height, **kw)

    # EVAL_QUALITY capture
    def eval_capture(self, transforms_json, out_dir, width=800, height=800, **kw):
        vis, pi = camera.nerf_eval_matrices(transforms_json, width, height)  # setDatasetCamera per frame
        os.makedirs(out_dir, exist_ok=True)
        for i, vi in enumerate(vis):
            img = self.draw(vi, pi, width, height, rgba32f=False, **kw)["rgba8"][0]
            save_png(os.path.join(out_dir, f"r_{i}.png"), img)
        return len(vis)

    def light_field(self, out_dir, rig="ring", width=180, height=180, **kw):
        if rig == "ring":  # computeGaussianLightField: RT-pipeline semantics (+0.5, alpha 1)
            vi, pi = camera.lightfield_ring_rig(self.splats["positions"], 4, width, height)
            kw = dict(dict(pixel_offset=0.5, alpha_init=1.0), **kw)
        else:  # config 5 grid
            vi, pi = camera.lightfield_grid_rig(camera.orbit_eye(4.0, 20.0, 90.0), (0.0, 0.0, 0.0), nx=4, ny=4,
                                                spacing=0.1, aspect=camera.aspect_ratio(width, height))
        ncams = len(vi) // 16
        out = self.draw(vi, pi, width, height, ncams=ncams, rgba32f=False, ray_dirs=True, ray_dirs_layout=1, **kw)
        os.makedirs(out_dir, exist_ok=True)
        for c in range(ncams):
            save_png(os.path.join(out_dir, f"view_{c}.png"), out["rgba8"][c])
        np.save(os.path.join(out_dir, "rayDirs.npy"), out["ray_dirs"].reshape(ncams, width, height, 4))
        return ncams

    def hit_counts(self, view_inv, proj_inv, width, height, path, **kw):
        out = self.draw(view_inv, proj_inv, width, height, rgba8=False, rgba32f=False, hit_counts=True, **kw)
        write_hit_counts_txt(path, out["hit_counts"][0])
        return out["hit_counts"][0]

    def benchmark(self, view_inv, proj_inv, width, height, warmup=1.0, duration=10.0, filename="fps.txt",
                  frame_times=False, **kw):
        torch = importlib.import_module("torch")  # device buffer + synchronize (plumbing)
        frame = torch.empty((height, width, 4), dtype=torch.uint8, device="cuda")
        b = Benchmark(warmup, duration, filename, frame_times)
        props = gv.device_properties(self.r.device)  # the deviceName / driverVersion fps.txt reports
        b.device, b.driver = props["device_name"].replace(",", " "), str(props["driver_version"])
        fps = b.run(lambda: self.r.render_device(view_inv, proj_inv, width, height, rgba8_ptr=frame.data_ptr(), **kw),
                    torch.cuda.synchronize)
        b.save_results()
        return fps, b


def _camera_for(args, splats):
    if args.config in (None, "config1") and not args.ply:
        return gv.scene.config1_camera(args.width, args.height)
    return gv.scene.mipnerf_camera(args.width, args.height)


def main(argv=None):
    ap = argparse.ArgumentParser(prog="gvrt_app", description=__doc__.split("\n")[0])
    ap.add_argument("cmd", choices=["render", "eval", "lightfield", "hitcounts", "bench", "psnr"])
    ap.add_argument("--ply")
    ap.add_argument("--config", default=None, help="synthetic scene (SURVEY §8d): " + ", ".join(gv.scene.CONFIGS))
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--out", default="gvrt_out")
    ap.add_argument("--transforms", help="NeRF transforms_*.json for eval")
    ap.add_argument("--rig", default="ring", choices=["ring", "grid"])
    ap.add_argument("--variant", default="rq", choices=["rq", "rt"], help="ray query (+0, alpha 0) or RT pipeline")
    ap.add_argument("--duration", type=float, default=10.0)
    ap.add_argument("--warmup", type=float, default=1.0)
    ap.add_argument("--frametimes", action="store_true")
    ap.add_argument("--build", default="fast", choices=["fast", "quality"],
                    help="fast: device LBVH (~1.5 ms at 1M); quality: device binned SAH + SAH-optimal collapse (~9 ms; static scenes)")
    ap.add_argument("--split-cells", type=int, default=0,
                    help="SplitBLAS analogue: grid cells on the longest axis (reference: 10; 0 = off)")
    ap.add_argument("--gt", help="psnr: ground-truth folder")
    ap.add_argument("--test", help="psnr: folder to score")
    args = ap.parse_args(argv)

    if args.cmd == "psnr":
        res, p, s = compare_dirs(args.gt, args.test)
        for f, (pp, ss) in res.items():
            print(f"{f}: PSNR={pp:.2f}, SSIM={ss:.4f}")
        print(f"{os.path.basename(os.path.normpath(args.test))} Average → PSNR: {p:.2f}, SSIM: {s:.4f}")
        return 0

    kw = dict(pixel_offset=0.5, alpha_init=1.0) if args.variant == "rt" else {}
    with GvrtApp(0) as app:
        bkw = dict(builder=2, collapse=1) if args.build == "quality" else {}
        m = app.prepare(ply=args.ply, config=args.config, split_cells=args.split_cells, **bkw)
        print(f"prepared: {m} Gaussians after the enclosing pass; stats {app.r.stats()}")
        if args.cmd == "eval":
            n = app.eval_capture(args.transforms, args.out, args.width, args.height, **kw)
            print(f"wrote {n} views to {args.out}")
        elif args.cmd == "lightfield":
            n = app.light_field(args.out, args.rig, args.width, args.height, **kw)
            print(f"wrote {n} views + rayDirs.npy to {args.out}")
        else:
            vi, pi = _camera_for(args, app.splats)
            if args.cmd == "render":
                os.makedirs(args.out, exist_ok=True)
                img = app.draw(vi, pi, args.width, args.height, rgba32f=False, **kw)["rgba8"][0]
                save_png(os.path.join(args.out, "frame.png"), img)
            elif args.cmd == "hitcounts":
                os.makedirs(args.out, exist_ok=True)
                app.hit_counts(vi, pi, args.width, args.height, os.path.join(args.out, "rayHitCountsOutput.txt"), **kw)
            elif args.cmd == "bench":
                fps, b = app.benchmark(vi, pi, args.width, args.height, args.warmup, args.duration,
                                       os.path.join(args.out, "fps.txt") if os.path.isdir(args.out) else "fps.txt",
                                       args.frametimes, **kw)
                print(f"frames : {len(b.frame_times)}\nfps    : {fps:.2f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
