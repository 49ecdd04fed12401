"""The C++ host layer (3dgvrt_lightfield_amd/host/, binary gvrt_app) without a GPU: the reference's
Camera / CameraLoader / glm matrix conventions agree with the Python mirror (camera.py, itself checked
in test_oracle_kat.py::test_camera_math), and the PNG writer produces a file a standard decoder reads
back bit for bit.  GPU flows of the same binary: tests/test_gpu_app.py."""
import json
import math
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APP = os.path.join(ROOT, "3dgvrt_lightfield_amd", "gvrt_app")


def run(*args):
    assert os.path.exists(APP), "gvrt_app not built (__graft_entry__.build())"
    r = subprocess.run([APP, *args], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return r.stdout


def mats(out):
    d = {}
    for line in out.splitlines():
        k, *v = line.split()
        d[k] = np.array([float(x) for x in v], np.float32)
    return d


def test_usage_and_png_roundtrip(tmp_path):
    r = subprocess.run([APP], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage: gvrt_app" in r.stderr
    Image = pytest.importorskip("PIL.Image")
    for w, h in ((37, 23), (300, 260)):  # the second spans several stored deflate blocks
        p = str(tmp_path / f"t{w}.png")
        run("png", p, "--width", str(w), "--height", str(h))
        a = np.asarray(Image.open(p))
        assert a.shape == (h, w, 4)
        y, x = np.mgrid[0:h, 0:w]
        exp = np.stack([x * 255 // max(w - 1, 1), y * 255 // max(h - 1, 1), (x ^ y) & 0xFF, 255 - ((x + y) & 0x7F)], -1)
        np.testing.assert_array_equal(a, exp.astype(np.uint8))


def test_camera_presets_match_python(gv):
    W, H = 64, 48
    m = mats(run("cameras", "--width", str(W), "--height", str(H)))
    vi, pi = gv.scene.config1_camera(W, H)
    np.testing.assert_allclose(m["config1_view_inv"], vi, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(m["config1_proj_inv"], pi, rtol=1e-6, atol=1e-6)
    vi, pi = gv.scene.mipnerf_camera(W, H)
    np.testing.assert_allclose(m["orbit_view_inv"], vi, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(m["orbit_proj_inv"], pi, rtol=1e-6, atol=1e-6)
    c = gv.camera.Camera()
    c.set_position((0.5, -1.0, 2.0))
    c.set_rotation((10.0, 20.0, 30.0))
    np.testing.assert_allclose(m["euler_view"], gv.camera.colmajor(c.view), rtol=1e-6, atol=1e-6)


def test_nerf_transforms_loader_matches_python(gv, tmp_path):
    frames = []
    rng = np.random.default_rng(5)
    for k in range(3):
        q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
        c2w = np.eye(4)
        c2w[:3, :3], c2w[:3, 3] = q, rng.normal(size=3) * 3
        frames.append({"file_path": f"./val/r_{k}", "rotation": 0.01, "transform_matrix": c2w.tolist()})
    tj = tmp_path / "transforms_val.json"
    tj.write_text(json.dumps({"camera_angle_x": 0.6911112070083618, "frames": frames}, indent=4))
    m = mats(run("cameras", "--transforms", str(tj)))
    angle, views = gv.camera.load_nerf_cameras(str(tj))
    assert math.isclose(angle, 0.6911112070083618)
    for k, w2c in enumerate(views):
        np.testing.assert_allclose(m[f"nerf_w2c_{k}"], gv.camera.colmajor(w2c), rtol=1e-6, atol=1e-6)
