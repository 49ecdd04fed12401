"""Camera / ray-generation inputs pinned on the reference itself: the float32 host camera math
(camera.py) against the reference's own base/camera.hpp, base/LoadCamera.hpp and vendored glm
(lookAt, inverse, perspective_Vulkan_no_depth_reverse), compiled from their sources by oracle/ref.mk
into oracle/_ref/ref_camera_dump (test infrastructure only).  Every matrix must be BIT-identical:
these are the 32 floats per view that feed ray generation (raygen.rgen:116-121)."""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DUMP = os.path.join(ROOT, "oracle", "_ref", "ref_camera_dump")

pytestmark = pytest.mark.skipif(not os.path.exists(DUMP), reason="oracle/_ref not built (needs /root/reference)")


def hx(*vals):
    return " ".join(float(np.float32(v)).hex() for v in vals)


def ref(lines):
    """Run the reference driver; returns the printed matrices as uint32 words (16 per matrix)."""
    r = subprocess.run([DUMP], input="\n".join(lines) + "\n", capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = []
    for ln in r.stdout.splitlines():
        w = ln.split()
        if len(w) == 16:
            out.append(np.array([int(x, 16) for x in w], np.uint32))
        else:
            out.append(int(w[0]))
    return out


def bits(m):
    return np.asarray(m, np.float32).reshape(16).view(np.uint32)


def same(a, b, what):
    a, b = bits(a), np.asarray(b, np.uint32)
    assert np.array_equal(a, b), f"{what}: {a.view(np.float32)} vs {b.view(np.float32)}"


def test_config1_camera_bit_identical(gv):
    cam = gv.camera
    for W, H in ((256, 256), (64, 64), (160, 120)):
        vi, pi = gv.scene.config1_camera(W, H)
        v, vinv, p, pinv = ref([f"lookat {hx(0, 0, 3, 0, 0, 0, 0, 1, 0)}",
                                f"persp {hx(cam.FOV_Y, cam.aspect_ratio(W, H), cam.NEAR_PLANE, cam.FAR_PLANE)}"])
        same(vi, vinv, "config1 viewInverse")
        same(pi, pinv, "config1 projInverse")
        same(cam.look_at((0, 0, 3), (0, 0, 0), (0, 1, 0)), v, "config1 view")


def test_orbit_camera_bit_identical(gv):
    cam = gv.camera
    for az in (30.0, 0.0, 123.0, -75.5):
        W, H = 1920, 1080
        vi, pi = gv.scene.mipnerf_camera(W, H, azimuth_deg=az)
        eye = cam.orbit_eye(4.0, 20.0, az)
        _, vinv, _, pinv = ref([f"lookat {hx(*eye, 0, 0, 0, 0, 1, 0)}",
                                f"persp {hx(50.0, cam.aspect_ratio(W, H), cam.NEAR_PLANE, cam.FAR_PLANE)}"])
        same(vi, vinv, f"orbit {az} viewInverse")
        same(pi, pinv, f"orbit {az} projInverse")


def test_projection_matches_glm_float32(gv):
    """The verdict's example: glm float32 gives inverse(P) entries -199.950027 and -0.99999994."""
    cam = gv.camera
    P = cam.perspective_vulkan_no_depth_reverse(cam.radians(cam.FOV_Y), 1.0, cam.NEAR_PLANE, cam.FAR_PLANE)
    Pi = cam.inverse(P)
    assert Pi[2][3] == np.float32(-199.950027) and Pi[3][2] == np.float32(-0.99999994)


def test_random_lookat_and_perspective_bit_identical(gv):
    cam = gv.camera
    rng = np.random.default_rng(11)
    lines, cases = [], []
    for _ in range(300):
        eye = rng.normal(size=3).astype(np.float32) * 5
        tgt = rng.normal(size=3).astype(np.float32)
        up = rng.normal(size=3).astype(np.float32)
        fov = np.float32(rng.uniform(5, 150))
        asp = np.float32(rng.uniform(0.2, 5))
        zn = np.float32(rng.uniform(1e-3, 0.5))
        zf = np.float32(rng.uniform(1, 1000))
        lines += [f"lookat {hx(*eye, *tgt, *up)}", f"persp {hx(fov, asp, zn, zf)}"]
        cases.append((eye, tgt, up, fov, asp, zn, zf))
    out = ref(lines)
    for k, (eye, tgt, up, fov, asp, zn, zf) in enumerate(cases):
        v = cam.look_at(eye, tgt, up)
        p = cam.perspective_vulkan_no_depth_reverse(cam.radians(fov), asp, zn, zf)
        same(v, out[4 * k], f"view {k}")
        same(cam.inverse(v), out[4 * k + 1], f"viewInverse {k}")
        same(p, out[4 * k + 2], f"persp {k}")
        same(cam.inverse(p), out[4 * k + 3], f"projInverse {k}")


def test_euler_camera_bit_identical(gv):
    """camera.hpp Camera (N_IS_UP): setPerspective, setPosition, setRotation, updateUniformBuffer."""
    cam = gv.camera
    rng = np.random.default_rng(12)
    cases = [((0.5, -1.0, 2.0), (10.0, 20.0, 30.0)), ((0, 0, 0), (0, 0, 0)), ((1, 2, 3), (0, 45, 0)),
             ((0, -3, 0.5), (-30, 0, 0)), ((0, 0, 0), (0, 0, 90))]
    cases += [(tuple(rng.normal(size=3) * 3), tuple(rng.uniform(-180, 180, size=3))) for _ in range(100)]
    lines = [f"euler {hx(*p, *r, cam.FOV_Y, cam.aspect_ratio(1920, 1080), cam.NEAR_PLANE, cam.FAR_PLANE)}" for p, r in cases]
    out = ref(lines)
    for k, (p, r) in enumerate(cases):
        c = cam.Camera()
        c.setPerspective(cam.FOV_Y, cam.aspect_ratio(1920, 1080), cam.NEAR_PLANE, cam.FAR_PLANE)
        c.setPosition(p)
        c.setRotation(r)
        vi, pi = c.matrices_inverse()
        same(c.matrices.view, out[4 * k], f"euler view {k}")
        same(vi, out[4 * k + 1], f"euler viewInverse {k}")
        same(c.matrices.perspective, out[4 * k + 2], f"euler perspective {k}")
        same(pi, out[4 * k + 3], f"euler projInverse {k}")


def write_transforms(path, n=6, seed=5):
    frames = []
    rng = np.random.default_rng(seed)
    for k in range(n):
        q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
        c2w = np.eye(4)
        c2w[:3, :3], c2w[:3, 3] = q, rng.normal(size=3) * 3
        frames.append({"file_path": f"./val/r_{k}", "rotation": 0.012566370614359171,
                       "transform_matrix": c2w.tolist()})
    frames.append({"file_path": "./val/r_int", "transform_matrix": [[1, 0, 0, 0], [0, 0, -1, -4], [0, 1, 0, 1],
                                                                    [0, 0, 0, 1]]})
    path.write_text(json.dumps({"camera_angle_x": 0.6911112070083618, "frames": frames}, indent=4))
    return len(frames)


def test_nerf_transforms_cameras_bit_identical(gv, tmp_path):
    """CameraLoader::loadNerfCameraData + setDatasetCamera (EVAL_QUALITY sequence, VulkanFullRT.cpp:2150-2156)."""
    cam = gv.camera
    tj = tmp_path / "transforms_val.json"
    n = write_transforms(tj)
    for W, H in ((800, 800), (1920, 1080)):
        out = ref([f"nerf {tj} {W} {H} {hx(cam.NEAR_PLANE)} {hx(cam.FAR_PLANE)}"])
        assert out[0] == n
        vis, pi = cam.nerf_eval_matrices(str(tj), W, H)
        c = cam.Camera()
        c.setNearFar(cam.NEAR_PLANE, cam.FAR_PLANE)
        c.loadDatasetCamera("nerf", str(tj), W, H)
        for k in range(n):
            c.setDatasetCamera("nerf", k, cam.aspect_ratio(W, H))
            same(c.matrices.view, out[1 + 4 * k], f"nerf w2c {k}")
            same(vis[k], out[2 + 4 * k], f"nerf viewInverse {k}")
            same(c.matrices.perspective, out[3 + 4 * k], f"nerf perspective {k}")
            same(pi, out[4 + 4 * k], f"nerf projInverse {k}")


def test_lightfield_ring_rig_bit_identical(gv, config1, tmp_path):
    """calculateGaussianLightFieldSamples (VulkanFullRT.cpp:1518-1604) on the config-1 splats."""
    cam = gv.camera
    pos = np.ascontiguousarray(config1["positions"], np.float32)
    pf = tmp_path / "pos.f32"
    pf.write_bytes(pos.tobytes())
    for W, H in ((180, 180), (24, 24), (100, 40)):
        out = ref([f"lfring {pf} {pos.size // 3} {W} {H} 4"])
        vi, pi = cam.lightfield_ring_rig(pos, 4, W, H)
        for c in range(4):
            same(vi[16 * c:16 * c + 16], out[c], f"ring viewInverse {c}")
        same(pi, out[4], "ring projInverse")


def test_lightfield_grid_rig_glm_part_bit_identical(gv):
    """Config 5's planar rig (our definition): every camera's lookAt/inverse is glm's."""
    cam = gv.camera
    eye = cam.orbit_eye(4.0, 20.0, 30.0)
    vi, pi = cam.lightfield_grid_rig(eye, (0, 0, 0), nx=4, ny=4, spacing=0.1, aspect=cam.aspect_ratio(1920, 1080))
    f = cam.normalize(cam.sub(cam.vec3((0, 0, 0)), cam.vec3(eye)))
    s = cam.normalize(cam.cross(f, cam.vec3((0, 1, 0))))
    u = cam.cross(s, f)
    lines = []
    for j in range(4):
        for i in range(4):
            ox = (np.float32(i) - np.float32(1.5)) * np.float32(0.1)
            oy = (np.float32(j) - np.float32(1.5)) * np.float32(0.1)
            p = cam.add(cam.vec3(eye), cam.add(cam.scale(s, ox), cam.scale(u, oy)))
            lines.append(f"lookat {hx(*p, *cam.add(p, f), 0, 1, 0)}")
    out = ref(lines + [f"persp {hx(50.0, cam.aspect_ratio(1920, 1080), cam.NEAR_PLANE, cam.FAR_PLANE)}"])
    for k in range(16):
        same(vi[16 * k:16 * k + 16], out[2 * k + 1], f"grid viewInverse {k}")
    same(pi, out[33], "grid projInverse")
