"""Host application pieces (3dgvrt_lightfield_amd/app.py) that need no GPU: the eval_quality.py
metrics, the fps.txt benchmark CSV (base/benchmark.hpp) and the hit-count text dump
(VulkanFullRT.cpp:2182-2195).  The GPU end of the app is in test_gpu_app.py."""
import importlib
import os

import numpy as np
import pytest

app = importlib.import_module("3dgvrt_lightfield_amd.app")


def _ssim_direct(a, b, win=7):
    """Slow restatement of the same SSIM definition (uniform window, sample covariance), interior only."""
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    c1, c2 = (0.01 * 255) ** 2, (0.03 * 255) ** 2
    pad = win // 2
    out = []
    for ch in range(a.shape[-1]):
        vals = []
        for y in range(pad, a.shape[0] - pad):
            for x in range(pad, a.shape[1] - pad):
                pa = a[y - pad:y + pad + 1, x - pad:x + pad + 1, ch].ravel()
                pb = b[y - pad:y + pad + 1, x - pad:x + pad + 1, ch].ravel()
                ma, mb = pa.mean(), pb.mean()
                va, vb = pa.var(ddof=1), pb.var(ddof=1)
                cov = ((pa - ma) * (pb - mb)).sum() / (pa.size - 1)
                vals.append(((2 * ma * mb + c1) * (2 * cov + c2)) / ((ma * ma + mb * mb + c1) * (va + vb + c2)))
        out.append(np.mean(vals))
    return float(np.mean(out))


def test_psnr_formula():
    a = np.zeros((4, 4, 3), np.uint8)
    b = a.copy()
    assert app.psnr(a, b) == float("inf")
    b[0, 0, 0] = 255  # MSE = 255^2 / 48
    assert abs(app.psnr(a, b) - 10 * np.log10(48.0)) < 1e-5


def test_ssim_matches_direct_definition():
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (20, 23, 3), dtype=np.uint8)
    b = np.clip(a.astype(int) + rng.integers(-30, 31, a.shape), 0, 255).astype(np.uint8)
    assert abs(app.ssim(a, a) - 1.0) < 1e-12
    assert abs(app.ssim(a, b) - _ssim_direct(a, b)) < 1e-9


def test_compare_dirs_and_png_roundtrip(tmp_path):
    pytest.importorskip("PIL")
    rng = np.random.default_rng(1)
    gt, te = tmp_path / "gt", tmp_path / "te"
    gt.mkdir()
    te.mkdir()
    imgs = []
    for i in range(3):
        im = rng.integers(0, 256, (16, 16, 4), dtype=np.uint8)
        imgs.append(im)
        app.save_png(str(gt / f"r_{i}.png"), im)
        if i < 2:  # r_2 missing from the test folder: skipped, as eval_quality.py does
            app.save_png(str(te / f"r_{i}.png"), im if i == 0 else 255 - im)
    np.testing.assert_array_equal(app.load_png_rgb(str(gt / "r_1.png")), imgs[1][..., :3])
    res, p, s = app.compare_dirs(str(gt), str(te))
    assert sorted(res) == ["r_0.png", "r_1.png"]
    assert res["r_0.png"][0] == float("inf") and res["r_0.png"][1] == pytest.approx(1.0)
    assert res["r_1.png"][0] == pytest.approx(app.psnr(imgs[1][..., :3], 255 - imgs[1][..., :3]))


def test_hit_counts_text_layout(tmp_path):
    c = np.arange(6, dtype=np.uint32).reshape(2, 3)
    path = tmp_path / "rayHitCountsOutput.txt"
    app.write_hit_counts_txt(str(path), c)
    assert path.read_text() == "0 1 2 \n3 4 5 \n"


# SHA-1 of the reference's own printRayHitCounts output (results/texts/rayHitCountsOutput.txt, written by
# VulkanFullRT.cpp:2182-2195 at 1920x1080).  Every count in that file is 0, so it pins the layout only.
REF_HIT_COUNTS_SHA1 = "e4b66ece2d1699ddc198bd6c23a8b47a9246821b"


def test_hit_counts_text_matches_reference_file(tmp_path):
    import hashlib
    path = tmp_path / "rayHitCountsOutput.txt"
    app.write_hit_counts_txt(str(path), np.zeros((1080, 1920), np.uint32))
    assert hashlib.sha1(path.read_bytes()).hexdigest() == REF_HIT_COUNTS_SHA1


def test_benchmark_csv_layout(tmp_path):
    b = app.Benchmark(warmup=0.0, duration=0.02, filename=str(tmp_path / "fps.txt"), output_frame_times=True)
    b.device, b.driver = "dev", "7.2"
    fps = b.run(lambda: None, lambda: None)
    assert fps > 0 and len(b.frame_times) > 0
    b.save_results()
    lines = (tmp_path / "fps.txt").read_text().split("\n")
    assert lines[0] == "device,driverversion,duration (ms),frames,fps"
    f = lines[1].split(",")
    assert f[0] == "dev" and f[1] == "7.2" and int(f[3]) == len(b.frame_times)
    assert f[2].split(".")[1].__len__() == 4 and f[4].split(".")[1].__len__() == 4
    assert lines[2] == "" and lines[3] == "frame,ms" and lines[4].startswith("0,")
