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
    """name -> 16 uint32 bit patterns (glm memory order) as gvrt_app cameras prints them."""
    d = {}
    for line in out.splitlines():
        k, *v = line.split()
        d[k] = np.array([int(x, 16) for x in v], np.uint32)
    return d


def bits(m):
    return np.asarray(m, np.float32).reshape(16).view(np.uint32)


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
    """C++ (gvrt_math.h, float32 glm order) == Python (camera.py), bit for bit."""
    cam = gv.camera
    for W, H in ((64, 48), (1920, 1080)):
        m = mats(run("cameras", "--width", str(W), "--height", str(H), "--position", "0.5,-1,2", "--rotation", "10,20,30"))
        vi, pi = gv.scene.config1_camera(W, H)
        assert np.array_equal(m["config1_view_inv"], bits(vi)) and np.array_equal(m["config1_proj_inv"], bits(pi))
        vi, pi = gv.scene.mipnerf_camera(W, H)
        assert np.array_equal(m["orbit_view_inv"], bits(vi)) and np.array_equal(m["orbit_proj_inv"], bits(pi))
        c = cam.Camera()
        c.setPerspective(cam.FOV_Y, cam.aspect_ratio(W, H), cam.NEAR_PLANE, cam.FAR_PLANE)
        c.setPosition((0.5, -1.0, 2.0))
        c.setRotation((10.0, 20.0, 30.0))
        vi, pi = c.matrices_inverse()
        assert np.array_equal(m["euler_view"], bits(c.matrices.view))
        assert np.array_equal(m["euler_view_inv"], bits(vi)) and np.array_equal(m["euler_proj_inv"], bits(pi))


def test_nerf_transforms_and_ring_rig_match_python(gv, tmp_path):
    frames = []
    rng = np.random.default_rng(5)
    for k in range(3):
        q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
        c2w = np.eye(4)
        c2w[:3, :3], c2w[:3, 3] = q, rng.normal(size=3) * 3
        frames.append({"file_path": f"./val/r_{k}", "rotation": 0.01, "transform_matrix": c2w.tolist()})
    tj = tmp_path / "transforms_val.json"
    tj.write_text(json.dumps({"camera_angle_x": 0.6911112070083618, "frames": frames}, indent=4))
    splats = gv.scene.config1(n=500)
    ply = str(tmp_path / "s.ply")
    gv.save_ply(ply, splats)
    W, H = 800, 600
    m = mats(run("cameras", "--width", str(W), "--height", str(H), "--transforms", str(tj), "--ply", ply))
    vis, pi = gv.camera.nerf_eval_matrices(str(tj), W, H)
    _, w2cs = gv.camera.load_nerf_cameras(str(tj), W, H)
    for k in range(3):
        assert np.array_equal(m[f"nerf_w2c_{k}"], bits(w2cs[k]))
        assert np.array_equal(m[f"nerf_view_inv_{k}"], bits(vis[k]))
        assert np.array_equal(m[f"nerf_proj_inv_{k}"], bits(pi))
    vi, pi = gv.camera.lightfield_ring_rig(splats["positions"], 4, W, H)
    for c in range(4):
        assert np.array_equal(m[f"ring_view_inv_{c}"], bits(vi[16 * c:16 * c + 16]))
    assert np.array_equal(m["ring_proj_inv"], bits(pi))


REF_CAM = os.path.join(ROOT, "oracle", "_ref", "ref_camera_dump")


@pytest.mark.skipif(not os.path.exists(REF_CAM), reason="oracle/_ref not built (needs /root/reference)")
def test_cpp_cameras_bit_identical_to_reference(gv, tmp_path):
    """gvrt_app's Camera / CameraLoader / light-field rig against the reference's own camera.hpp /
    LoadCamera.hpp / glm built from its sources (oracle/_ref/ref_camera_dump)."""
    def hx(*v):
        return " ".join(float(np.float32(x)).hex() for x in v)

    tj = tmp_path / "transforms_val.json"
    tj.write_text(json.dumps({"camera_angle_x": 0.5, "frames": [
        {"file_path": "a", "transform_matrix": [[0.6, -0.8, 0.0, 1.5], [0.8, 0.6, 0.0, -2.25], [0.0, 0.0, 1.0, 3.0],
                                                [0.0, 0.0, 0.0, 1.0]]}]}))
    splats = gv.scene.config1(n=400)
    ply = str(tmp_path / "s.ply")
    gv.save_ply(ply, splats)
    pf = tmp_path / "pos.f32"
    pf.write_bytes(np.ascontiguousarray(splats["positions"], np.float32).tobytes())
    W, H = 640, 360
    m = mats(run("cameras", "--width", str(W), "--height", str(H), "--transforms", str(tj), "--ply", ply,
                 "--position", "1.25,-0.5,3", "--rotation", "-20,35,10"))
    cam = gv.camera
    asp = cam.aspect_ratio(W, H)
    lines = [f"euler {hx(1.25, -0.5, 3, -20, 35, 10, cam.FOV_Y, asp, cam.NEAR_PLANE, cam.FAR_PLANE)}",
             f"nerf {tj} {W} {H} {hx(cam.NEAR_PLANE)} {hx(cam.FAR_PLANE)}",
             f"lfring {pf} 400 {W} {H} 4",
             f"lookat {hx(0, 0, 3, 0, 0, 0, 0, 1, 0)}", f"persp {hx(cam.FOV_Y, asp, cam.NEAR_PLANE, cam.FAR_PLANE)}"]
    r = subprocess.run([REF_CAM], input="\n".join(lines) + "\n", capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    ref = [np.array([int(x, 16) for x in ln.split()], np.uint32) for ln in r.stdout.splitlines() if len(ln.split()) == 16]
    assert np.array_equal(m["euler_view"], ref[0]) and np.array_equal(m["euler_view_inv"], ref[1])
    assert np.array_equal(m["euler_proj_inv"], ref[3])
    assert np.array_equal(m["nerf_w2c_0"], ref[4]) and np.array_equal(m["nerf_view_inv_0"], ref[5])
    assert np.array_equal(m["nerf_proj_inv_0"], ref[7])
    for c in range(4):
        assert np.array_equal(m[f"ring_view_inv_{c}"], ref[8 + c])
    assert np.array_equal(m["ring_proj_inv"], ref[12])
    assert np.array_equal(m["config1_view_inv"], ref[14]) and np.array_equal(m["config1_proj_inv"], ref[16])


def test_reference_host_interfaces_compile_and_run(gv, tmp_path):
    """The reference's host interfaces kept intact (north_star): tests/cpp/host_interfaces.cpp asserts each
    member-function type and calls it with the reference's argument types; it links libgvrt.so and runs the
    host-side parts (PLY loader, NeRF camera loader, Camera, vks::Benchmark) without a GPU."""
    pkg = os.path.join(ROOT, "3dgvrt_lightfield_amd")
    exe = str(tmp_path / "host_interfaces")
    r = subprocess.run(["g++", "-O1", "-std=c++17", "-ffp-contract=off", "-Wall", "-Werror", "-I", os.path.join(pkg, "host"),
                        os.path.join(ROOT, "tests", "cpp", "host_interfaces.cpp"), os.path.join(pkg, "host", "gvrt_host.cpp"),
                        "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-L", pkg, "-lgvrt", "-L/opt/rocm/lib",
                        "-lamdhip64", f"-Wl,-rpath,{pkg}", "-Wl,-rpath,/opt/rocm/lib", "-o", exe],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    ply = str(tmp_path / "s.ply")
    gv.save_ply(ply, gv.scene.config1(n=300))
    tj = tmp_path / "transforms_val.json"
    tj.write_text(json.dumps({"camera_angle_x": 0.69, "frames": [
        {"file_path": "a", "transform_matrix": [[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 4], [0, 0, 0, 1]]}]}))
    r = subprocess.run([exe, ply, str(tj)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "splats 300 frames 1 cams 1" in r.stdout and "bench 5 5" in r.stdout
    assert "Benchmark finished" in r.stdout and "device : host-check" in r.stdout


REF_BENCH = os.path.join(ROOT, "oracle", "_ref", "ref_bench_dump")


@pytest.mark.skipif(not os.path.exists(REF_BENCH), reason="oracle/_ref not built (needs /root/reference)")
def test_benchmark_fps_txt_matches_reference(tmp_path):
    """vks::Benchmark::saveResults of the C++ host layer writes the reference's fps.txt byte for byte, and
    run() / saveResults print the same console lines (base/benchmark.hpp:37-104, built from the reference's
    sources by oracle/ref.mk): same device line, duration, frame count, fps, per-frame table and
    best / worst / avg.  Both sides enter the frame times as run()'s loop does."""
    pkg = os.path.join(ROOT, "3dgvrt_lightfield_amd")
    exe = str(tmp_path / "bench_results")
    r = subprocess.run(["g++", "-O1", "-std=c++17", "-ffp-contract=off", "-Wall", "-Werror", "-I", os.path.join(pkg, "host"),
                        os.path.join(ROOT, "tests", "cpp", "bench_results.cpp"), os.path.join(pkg, "host", "gvrt_host.cpp"),
                        "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-L", pkg, "-lgvrt", "-L/opt/rocm/lib",
                        "-lamdhip64", f"-Wl,-rpath,{pkg}", "-Wl,-rpath,/opt/rocm/lib", "-o", exe],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rng = np.random.default_rng(11)
    cases = [
        ("AMD Instinct MI355X", "70200", "1", ["1.25", "0.875", "3.0000001"]),
        ("AMD Instinct MI355X", "70200", "0", ["1.3046", "1.2947"]),
        ("gfx950 node 7", "4294967295", "1", [repr(float(x)) for x in rng.uniform(0.2, 40.0, 257)]),
        ("x", "0", "1", ["1e-9", "12345.678901234"]),
    ]
    for k, (dev, drv, ft, times) in enumerate(cases):
        outs = []
        for prog in (REF_BENCH, exe):
            f = tmp_path / f"fps_{k}_{os.path.basename(prog)}.txt"
            p = subprocess.run([prog, str(f), dev, drv, ft, *times], capture_output=True, text=True, timeout=60)
            assert p.returncode == 0, p.stderr
            outs.append((f.read_bytes(), p.stdout))
        assert outs[0][0] == outs[1][0], (outs[0][0][:300], outs[1][0][:300])
        assert outs[0][1] == outs[1][1], (outs[0][1], outs[1][1])
        assert outs[0][0].startswith(b"device,driverversion,duration (ms),frames,fps\n" + dev.encode() + b"," + drv.encode())


@pytest.mark.parametrize("W,H,world", [(3840, 2160, 8), (1920, 1080, 3), (100, 60, 2), (8, 8, 4)])
def test_cpp_split_tiles_match_python(gv, W, H, world):
    """The C++ host's tile split (gvrt_rccl.h rank_tiles, the native RCCL path) deals the same 64x64-pixel blocks
    to the same ranks as the Python layer (renderer.tiles_for_rank / dist.rank_tiles), and covers every tile
    once."""
    seen = []
    for rank in range(world):
        out = run("tiles", "--rank", str(rank), "--world", str(world), "--width", str(W), "--height", str(H))
        got = np.array([[int(v) for v in l.split()] for l in out.splitlines()], np.int64).reshape(-1, 3)
        ref = gv.tiles_for_rank(W, H, 1, rank, world, block=8).astype(np.int64)[:, :3]
        np.testing.assert_array_equal(got, ref)
        seen.extend(map(tuple, got))
    assert len(seen) == len(set(seen)) == ((W + 7) // 8) * ((H + 7) // 8)


@pytest.mark.parametrize("W,H,world", [(3840, 2160, 8), (1920, 1080, 3), (100, 60, 2)])
def test_cpp_cost_bands_match_python(gv, tmp_path, W, H, world):
    """The C++ host's cost-weighted band split (gvrt_rccl.h band_tiles, SplitFrame::COST_BANDS) cuts the same
    bands as the Python layer (dist.band_tiles over dist.cost_weights) from the same cost classes: the weights
    are the same doubles on both sides (2^(c div 4) x an exact quarter-octave literal)."""
    import importlib
    dist = importlib.import_module("3dgvrt_lightfield_amd.dist")
    tx_n, ty_n = (W + 7) // 8, (H + 7) // 8
    cls = np.random.default_rng(W + world).integers(0, 64, size=(ty_n, tx_n), dtype=np.uint8)
    f = tmp_path / "classes.bin"
    f.write_bytes(cls.tobytes())
    ref = dist.band_tiles(W, H, world, costs=dist.cost_weights(cls[None]))
    for rank in range(world):
        out = run("tiles", "--rank", str(rank), "--world", str(world), "--width", str(W), "--height", str(H),
                  "--layout", "bands", "--costs", str(f))
        got = np.array([[int(v) for v in l.split()] for l in out.splitlines()], np.int64).reshape(-1, 3)
        np.testing.assert_array_equal(got, ref[rank].astype(np.int64)[:, :3])


@pytest.mark.parametrize("views,world,seed", [(16, 8, 0), (16, 3, 1), (16, 16, 2), (7, 2, 3), (5, 8, 4), (16, 5, 5)])
def test_cpp_balanced_views_match_python(views, world, seed):
    """The C++ host's view split (gvrt_rccl.h balanced_views, SplitFrame::VIEWS: config 5 on N GPUs) assigns the same
    views to the same ranks as the Python layer (dist.balanced_views) from the same per-view costs, ties included
    (costs drawn from a few values, so equal costs occur), and every view once."""
    import importlib
    dist = importlib.import_module("3dgvrt_lightfield_amd.dist")
    rng = np.random.default_rng(seed)
    costs = rng.choice([0.72, 0.9, 1.1, 1.25, 1.4], size=views) * rng.choice([1.0, 1.0, 1.003], size=views)
    out = run("views", "--costs", ",".join(repr(float(c)) for c in costs), "--world", str(world))
    lines = out.splitlines()
    got = [[int(v) for v in l.split()] for l in lines] + [[] for _ in range(world - len(lines))]
    assert got == dist.balanced_views(costs.tolist(), world)
    assert sorted(v for g in got for v in g) == list(range(views))


@pytest.fixture(scope="module")
def split_fake(tmp_path_factory):
    """tests/cpp/split_fake.cpp: host/gvrt_split.cpp (the SplitFrame the RCCL build ships, unchanged) over an
    in-process backend whose ranks are threads (no GPU, no RCCL)."""
    pkg = os.path.join(ROOT, "3dgvrt_lightfield_amd")
    exe = str(tmp_path_factory.mktemp("split") / "split_fake")
    r = subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Werror", "-pthread", "-I", os.path.join(pkg, "host"),
                        os.path.join(ROOT, "tests", "cpp", "split_fake.cpp"), os.path.join(pkg, "host", "gvrt_split.cpp"),
                        "-o", exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


GVRT_ERR_OOM, GVRT_ERR_HIP, GVRT_ERR_RCCL = -2, -3, -8


@pytest.mark.parametrize("world", [2, 8])
@pytest.mark.parametrize("scenario", ["healthy", "healthy_views", "setup_fail", "stop", "group_fail", "render_fail"])
def test_split_frame_failure_paths_with_peers(split_fake, scenario, world):
    """SplitFrame's agree / bounded-wait / abort paths with real peers (SURVEY §5 "Failure detection":
    statuses, never an abort, replacing VK_CHECK_RESULT, base/VulkanTools.h:42-61), one thread per rank, the wait bound
    set to 1 s, the whole run under a hard 60 s limit:
      * healthy (cost bands; views): every frame assembled on rank 0 pixel for pixel, every rank GVRT_OK;
      * setup_fail: one rank's part-buffer allocation fails -> agree() gives every rank that status (GVRT_ERR_OOM);
      * stop: one rank stops taking part after its first frame -> every peer returns GVRT_ERR_RCCL within the bound;
      * group_fail: one rank's send fails inside the frame's group -> group_failed() ends the group and aborts it
        (GVRT_ERR_RCCL); every peer returns GVRT_ERR_RCCL within the bound;
      * render_fail: one rank's render fails -> it still enters the exchange, drains it, aborts (GVRT_ERR_HIP); every
        peer returns GVRT_ERR_RCCL within the bound."""
    r = subprocess.run([split_fake, scenario, str(world)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    ranks, victim, bound = d["ranks"], d["victim"], d["timeout_s"]
    peers = [x for x in ranks if x["rank"] != victim]
    v = ranks[victim]
    for x in ranks:  # no wait outlives its bound by much: at most two bounded waits per rank here
        assert x["seconds"] < 2 * bound + 1.0, x
    if scenario.startswith("healthy"):
        assert all(x["status"] == 0 and x["frames_ok"] == 4 for x in ranks), ranks
        assert ranks[0]["frame_ok"]
    elif scenario == "setup_fail":
        assert all(x["status"] == GVRT_ERR_OOM and x["frames_ok"] == 0 for x in ranks), ranks
        assert v["error"] == "part buffer" and all(x["error"] == "set-up failed on another rank" for x in peers)
    else:
        want_victim = {"stop": 0, "group_fail": GVRT_ERR_RCCL, "render_fail": GVRT_ERR_HIP}[scenario]
        assert v["status"] == want_victim and v["frames_ok"] == 1, v
        assert all(x["status"] == GVRT_ERR_RCCL for x in peers), peers
        assert all("no progress within" in x["error"] for x in peers), peers
        assert ranks[0]["frame_ok"]  # the frames completed before the failure were assembled correctly
