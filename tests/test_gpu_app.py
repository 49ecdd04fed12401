"""The headless app (3dgvrt_lightfield_amd/app.py) end to end on the GPU: PLY -> prepare -> eval capture
(r_<i>.png per NeRF camera), light-field batch (PNG per view + rayDirs), hit-count dump, fps.txt."""
import importlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
app = importlib.import_module("3dgvrt_lightfield_amd.app")


def test_app_eval_lightfield_hitcounts_bench(gv, tmp_path):
    pytest.importorskip("PIL")
    splats = gv.scene.config1(n=2000)
    ply = str(tmp_path / "scene.ply")
    gv.save_ply(ply, splats)
    # a NeRF transforms file with two cameras on a circle, looking at the origin
    frames = []
    for a in (0.0, 0.7):
        eye = np.array([3 * np.sin(a), 0.0, 3 * np.cos(a)])
        f = -eye / np.linalg.norm(eye)
        r = np.cross(f, [0.0, 1.0, 0.0]); r /= np.linalg.norm(r)
        u = np.cross(r, f)
        c2w = np.eye(4); c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = r, u, -f, eye
        frames.append({"file_path": "./val/r_x", "transform_matrix": c2w.tolist()})
    tj = tmp_path / "transforms_val.json"
    tj.write_text(json.dumps({"camera_angle_x": 0.69, "frames": frames}))

    with app.GvrtApp(0) as a:
        m = a.prepare(ply=ply)
        assert m > 0
        out = tmp_path / "eval"
        assert a.eval_capture(str(tj), str(out), 64, 64) == 2
        r0 = app.load_png_rgb(str(out / "r_0.png"))
        # the PNG is exactly the frame draw() returns for that camera
        vis, pi = gv.camera.nerf_eval_matrices(str(tj), 64, 64)
        img = a.draw(vis[0], pi, 64, 64, rgba32f=False)["rgba8"][0]
        np.testing.assert_array_equal(r0, img[..., :3])
        assert img[..., 3].max() > 0  # the camera sees the scene

        lf = tmp_path / "lf"
        assert a.light_field(str(lf), "ring", 48, 48) == 4
        assert sorted(os.listdir(lf)) == ["rayDirs.npy", "view_0.png", "view_1.png", "view_2.png", "view_3.png"]
        d = np.load(str(lf / "rayDirs.npy"))
        assert d.shape == (4, 48, 48, 4)

        vi, pi = gv.scene.config1_camera(32, 32)
        hc = a.hit_counts(vi, pi, 32, 32, str(tmp_path / "rayHitCountsOutput.txt"))
        rows = (tmp_path / "rayHitCountsOutput.txt").read_text().splitlines()
        assert len(rows) == 32 and [int(v) for v in rows[5].split()] == hc[5].tolist()

        fps, b = a.benchmark(vi, pi, 32, 32, warmup=0.05, duration=0.2, filename=str(tmp_path / "fps.txt"))
        assert fps > 0
        assert (tmp_path / "fps.txt").read_text().startswith("device,driverversion,duration (ms),frames,fps\n")


def test_bench_on_a_ply(gv, tmp_path):
    """bench.py --ply renders a supplied scene instead of the synthetic stand-in and says so."""
    import subprocess
    import sys
    ply = str(tmp_path / "scene.ply")
    gv.save_ply(ply, gv.scene.config1(n=5000))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--ply", ply, "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["data"] == "real scene scene.ply" and line["config"]["gaussians"] == 5000
    assert line["value"] > 0 and line["roofline"]["frac"] > 0
    # the roofline names its binding unit (instruction issue, from the PMC passes) and is a bound
    roof = line["roofline"]
    assert roof["bound"] in ("issue", "hbm") and roof["frac"] <= 1.0, roof
    # the bound names the busier resource: VALU issue unless the HBM fraction is larger
    assert (roof["bound"] == "hbm") == (roof["hbm"]["frac"] > roof.get("valu_issue_frac", roof["frac"])), roof
    assert 0.0 < roof["hbm"]["frac"] < 1.0
    # round 6: the reference-gather figure carries no bound and no fraction; every fraction the line
    # states is <= 1 and the largest names the binding unit
    assert "bound" not in roof["reference_gather"] and "frac" not in roof["reference_gather"]
    fr = roof["binding"]["fractions"]
    assert all(0.0 <= v <= 1.0 for v in fr.values()) and roof["binding"]["largest"] == max(fr, key=fr.get), roof
    assert 0.0 < roof["cache"]["l2_hit_rate"] <= 1.0 and roof["latency"]["node_visits_per_wave"] > 0


def test_cpp_app_flows_match_python(gv, tmp_path):
    """The C++ gvrt_app (host/gvrt_host.cpp: PLYLoader, Camera, CameraLoader, vks::Benchmark, VulkanFullRT
    flows) on the GPU: its frames equal the Python mirror's for the same cameras."""
    Image = pytest.importorskip("PIL.Image")
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "3dgvrt_lightfield_amd", "gvrt_app")
    splats = gv.scene.config1(n=3000)
    ply = str(tmp_path / "scene.ply")
    gv.save_ply(ply, splats)

    def app_run(*args):
        r = subprocess.run([exe, *args, "--ply", ply], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        return r.stdout

    W = H = 64
    out = tmp_path / "cpp"
    app_run("render", "--camera", "config1", "--width", str(W), "--height", str(H), "--out", str(out))
    got = np.asarray(Image.open(out / "frame.png"))
    with app.GvrtApp(0) as a:
        a.prepare(ply=ply)
        vi, pi = gv.scene.config1_camera(W, H)
        ref = a.draw(vi, pi, W, H, rgba32f=False)["rgba8"][0]
        np.testing.assert_array_equal(got, ref)  # bit-identical camera matrices -> the same frame
        hc = a.hit_counts(vi, pi, W, H, str(tmp_path / "py_hits.txt"))
        lf_ref = a.draw(*gv.camera.lightfield_ring_rig(a.splats["positions"], 4, 48, 48), 48, 48, ncams=4,
                        rgba32f=False, pixel_offset=0.5, alpha_init=1.0)["rgba8"]
    assert got[..., 3].max() > 0
    app_run("hitcounts", "--camera", "config1", "--width", str(W), "--height", str(H), "--out", str(out))
    rows = (out / "rayHitCountsOutput.txt").read_text().splitlines()
    cpp_hc = np.array([[int(v) for v in r.split()] for r in rows])
    np.testing.assert_array_equal(cpp_hc, hc)
    app_run("lightfield", "--width", "48", "--height", "48", "--out", str(out / "lf"))
    for c in range(4):
        v = np.asarray(Image.open(out / "lf" / f"view_{c}.png"))
        np.testing.assert_array_equal(v, lf_ref[c])
    d = np.fromfile(out / "lf" / "rayDirs.bin", np.float32).reshape(4, 48, 48, 4)
    np.testing.assert_allclose(np.linalg.norm(d[..., :3], axis=-1), 1.0, atol=1e-5)
    s = app_run("bench", "--camera", "config1", "--width", "32", "--height", "32", "--duration", "1", "--warmup", "0",
                "--out", str(out))
    assert "Benchmark finished" in s and "fps    : " in s
    assert (out / "fps.txt").read_text().startswith("device,driverversion,duration (ms),frames,fps\n")


@pytest.mark.parametrize("layout", ["cost-bands", "blocks"])
def test_cpp_rccl_split_frame_one_rank(gv, tmp_path, layout):
    """The native multi-GPU path of the C++ host (host/gvrt_rccl.h SplitFrame: ncclCommInitRank, this rank's
    tiles rendered tile-packed, grouped ncclSend / ncclRecv to rank 0, gvrt_unpack_tiles_rgba8) with a one-rank
    communicator: rank 0 sends its part to itself through RCCL, and the gathered frame equals the one-GPU frame
    byte for byte (the app checks and prints it).  cost-bands: rank 0's calibration renders, gvrt_read_tile_costs
    and the ncclBroadcast of the classes run first."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "3dgvrt_lightfield_amd", "gvrt_app")
    ply = str(tmp_path / "scene.ply")
    gv.save_ply(ply, gv.scene.config1(n=3000))
    import subprocess
    for W, H in ((256, 256), (200, 120)):
        r = subprocess.run([exe, "split", "--ply", ply, "--rank", "0", "--world", "1", "--id-file",
                            str(tmp_path / f"rccl_{W}.id"), "--frames", "4", "--camera", "config1", "--width", str(W),
                            "--height", str(H), "--layout", layout, "--out", str(tmp_path / f"split_{W}")],
                           capture_output=True, text=True, timeout=180,
                           env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
        assert r.returncode == 0, r.stderr[-2000:]
        line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
        import json
        d = json.loads(line)
        assert d["identical_to_one_gpu"] is True and d["world"] == 1 and d["ms_per_frame"] > 0


def _split(exe, ply, tmp_path, tag, *extra, timeout=180):
    import subprocess
    return subprocess.run([exe, "split", "--ply", ply, "--rank", "0", "--world", "1", "--id-file",
                           str(tmp_path / f"rccl_{tag}.id"), "--out", str(tmp_path / f"split_{tag}"), *extra],
                          capture_output=True, text=True, timeout=timeout,
                          env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def test_cpp_rccl_split_views_one_rank(gv, tmp_path):
    """Config 5 through the native C++ path: SplitFrame::VIEWS over a 16-view light-field rig --
    rank 0 times each view alone, one ncclBroadcast of the costs (with its status word), balanced_views, this rank's
    views in one batched launch, each view sent whole into its slot of the rig frame -- with a one-rank
    communicator: the gathered 16 views equal one batched render of the rig on this GPU byte for byte."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "3dgvrt_lightfield_amd", "gvrt_app")
    ply = str(tmp_path / "scene.ply")
    gv.save_ply(ply, gv.scene.config1(n=3000))
    import json
    r = _split(exe, ply, tmp_path, "views", "--frames", "3", "--width", "96", "--height", "64", "--layout", "views",
               "--views", "16")
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["identical_to_one_gpu"] is True and d["views"] == 16 and d["assignment"] == [list(range(16))]


def test_cpp_rccl_split_calibration_failure_is_a_status(gv, tmp_path):
    """a failed tile-cost calibration on rank 0 (here injected: the handle's tile_order is off, so
    gvrt_read_tile_costs has no costs to read) travels with the status word of the one broadcast every rank enters:
    SplitFrame reports it as a status and the app exits with it, promptly, instead of leaving peers in a
    collective."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "3dgvrt_lightfield_amd", "gvrt_app")
    ply = str(tmp_path / "scene.ply")
    gv.save_ply(ply, gv.scene.config1(n=2000))
    r = _split(exe, ply, tmp_path, "fail", "--frames", "2", "--width", "64", "--height", "64", "--layout",
               "cost-bands", "--tile-order-off", timeout=120)
    assert r.returncode == 1, (r.returncode, r.stdout[-500:], r.stderr[-1000:])
    assert "tile-cost calibration failed on rank 0" in r.stderr and "gvrt_read_tile_costs" in r.stderr
