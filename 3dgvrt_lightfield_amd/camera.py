"""Host camera math (the reference's glm-based camera path), as column-major float32 4x4s.

Reference: base/camera.hpp:31-58 (Camera::updateViewMatrix), :157-182 (setPerspective),
base/LoadCamera.hpp:45-147 (CameraLoader: NeRF transforms_*.json), the modified glm
`perspective_Vulkan_no_depth_reverse` (external/glm/glm/gtc/matrix_transform.inl:274-290),
VulkanFullRT::updateUniformBuffer (VulkanFullRT.cpp:1331-1349: viewInverse = inverse(view),
projInverse = inverse(perspective)) and the light-field rig
VulkanFullRT::calculateGaussianLightFieldSamples (VulkanFullRT.cpp:1518-1628).

Matrices are numpy (row, col) in math convention; `colmajor()` gives the 16 floats the
C-ABI (and GLSL) expects.
"""
from __future__ import annotations

import json
import math

import numpy as np

FOV_Y = 39.6          # base/Define.h:33
NEAR_PLANE = 0.005    # base/Define.h:34
FAR_PLANE = 20.0      # base/Define.h:35
FLT_MIN = np.float32(1.1754943508222875e-38)


def colmajor(m):
    return np.ascontiguousarray(np.asarray(m, dtype=np.float32).T.reshape(16))


def normalize(v):
    v = np.asarray(v, dtype=np.float64)
    return v / np.linalg.norm(v)


def look_at(eye, center, up):
    """glm::lookAt (right-handed, glm/ext/matrix_transform.inl lookAtRH)."""
    eye = np.asarray(eye, np.float64)
    f = normalize(np.asarray(center, np.float64) - eye)
    s = normalize(np.cross(f, up))
    u = np.cross(s, f)
    m = np.eye(4)
    m[0, :3] = s
    m[1, :3] = u
    m[2, :3] = -f
    m[0, 3] = -np.dot(s, eye)
    m[1, 3] = -np.dot(u, eye)
    m[2, 3] = np.dot(f, eye)
    return m


def perspective_vulkan_no_depth_reverse(fovy_rad, aspect, znear, zfar):
    """matrix_transform.inl:276-290 (Result[1][1] = -1/tan: row 0 of the image is the top)."""
    t = math.tan(fovy_rad / 2.0)
    m = np.zeros((4, 4))
    m[0, 0] = 1.0 / (aspect * t)
    m[1, 1] = -1.0 / t
    m[3, 2] = -1.0
    m[2, 2] = -zfar / (zfar - znear)
    m[2, 3] = -(zfar * znear) / (zfar - znear)
    return m


def inverse(m):
    return np.linalg.inv(np.asarray(m, np.float64))


def camera_matrices(view, proj):
    """(viewInverse, projInverse) column-major float32, as updateUniformBuffer uploads them."""
    return colmajor(inverse(view)), colmajor(inverse(proj))


def pinhole(eye, target, up=(0.0, 1.0, 0.0), fovy_deg=FOV_Y, aspect=1.0, znear=NEAR_PLANE, zfar=FAR_PLANE):
    view = look_at(eye, target, up)
    proj = perspective_vulkan_no_depth_reverse(math.radians(fovy_deg), aspect, znear, zfar)
    return camera_matrices(view, proj)


def orbit_camera(radius, elevation_deg, azimuth_deg, target=(0.0, 0.0, 0.0), fovy_deg=50.0, aspect=16 / 9):
    el, az = math.radians(elevation_deg), math.radians(azimuth_deg)
    eye = np.array([radius * math.cos(el) * math.sin(az), radius * math.sin(el), radius * math.cos(el) * math.cos(az)])
    return pinhole(eye + np.asarray(target), target, (0.0, 1.0, 0.0), fovy_deg, aspect)


class Camera:
    """base/camera.hpp Camera (Euler-angle camera, N_IS_UP axes of base/Define.h:63)."""

    def __init__(self):
        self.rotation = np.zeros(3)
        self.position = np.zeros(3)
        self.view = np.eye(4)
        self.perspective = np.eye(4)
        self.fov = FOV_Y
        self.znear = NEAR_PLANE
        self.zfar = FAR_PLANE

    @staticmethod
    def _rotate_axis(rad, u, v, n):  # camera.hpp rotateAxis: rotate u, v -> n
        s, c = math.sin(rad), math.cos(rad)
        v = normalize(v * c + np.cross(u, v) * s)
        n = normalize(np.cross(u, v))
        return u, v, n

    def update_view_matrix(self):  # camera.hpp:31-58 (N_IS_UP)
        u = np.array([1.0, 0.0, 0.0])
        v = np.array([0.0, 0.0, 1.0])
        n = np.array([0.0, -1.0, 0.0])
        if math.radians(self.rotation[1]) != 0:
            v, n, u = self._rotate_axis(math.radians(self.rotation[1]), v, n, u)
        if math.radians(self.rotation[0]) != 0:
            u, v, n = self._rotate_axis(math.radians(self.rotation[0]), u, v, n)
        if math.radians(self.rotation[2]) != 0:
            n, u, v = self._rotate_axis(math.radians(self.rotation[2]), n, u, v)
        rot = np.eye(4)
        rot[:3, 0], rot[:3, 1], rot[:3, 2] = u, v, n  # glm::mat4(vec4(u),vec4(v),vec4(n),...) columns
        tr = np.eye(4)
        tr[:3, 3] = -self.position
        self.view = rot.T @ tr  # glm::translate(transpose(rot), -position)

    def set_position(self, p):
        self.position = np.asarray(p, np.float64)
        self.update_view_matrix()

    def set_rotation(self, r):
        self.rotation = np.asarray(r, np.float64)
        self.update_view_matrix()

    def set_perspective(self, fov, aspect, znear, zfar):  # camera.hpp:157-182
        self.fov, self.znear, self.zfar = fov, znear, zfar
        self.perspective = perspective_vulkan_no_depth_reverse(math.radians(fov), aspect, znear, zfar)

    def matrices(self):
        return camera_matrices(self.view, self.perspective)


def load_nerf_cameras(path):
    """CameraLoader::loadNerfCameraData + c2wTow2cRT (LoadCamera.hpp:57-85, :124-147).

    Returns (camera_angle_x, [view matrices (w2c)]).  camera.setNerfCamera uses the w2c as the
    view matrix; the fovy actually used is FOV_Y (camera.hpp setDatasetCamera overrides it)."""
    with open(path) as fh:
        j = json.load(fh)
    views = []
    for fr in j["frames"]:
        c2w = np.asarray(fr["transform_matrix"], np.float64)
        r, t = c2w[:3, :3], c2w[:3, 3]
        w2c = np.eye(4)
        w2c[:3, :3] = r.T
        w2c[:3, 3] = -r.T @ t
        views.append(w2c)
    return float(j["camera_angle_x"]), views


def lightfield_ring_rig(positions, ncams=4, width=180, height=180):
    """VulkanFullRT::calculateGaussianLightFieldSamples (VulkanFullRT.cpp:1518-1628).

    bbox of the raw positions with max initialised to FLT_MIN (Q15), cameras at
    center +- maxR on x and y, lookAt(up = +z), 135 deg fov with aspect = (float)(width/height)
    (integer division, Q15).  Returns (viewInverse [ncams*16], projInverse [16])."""
    p = np.asarray(positions, np.float32).reshape(-1, 3)
    mn = np.minimum(p.min(axis=0), np.float32(np.finfo(np.float32).max))
    mx = np.maximum(p.max(axis=0), FLT_MIN)
    center = ((mn + mx) / 2).astype(np.float64)
    maxr = float(np.max(mx - mn)) / 2
    cams = [center + [maxr, 0, 0], center + [0, maxr, 0], center - [maxr, 0, 0], center - [0, maxr, 0]]
    vis = [colmajor(inverse(look_at(cams[i % 4], center, (0.0, 0.0, 1.0)))) for i in range(ncams)]
    proj = perspective_vulkan_no_depth_reverse(math.radians(135.0), float(width // height), NEAR_PLANE, FAR_PLANE)
    return np.concatenate(vis), colmajor(inverse(proj))


def lightfield_grid_rig(eye, target, up=(0.0, 1.0, 0.0), nx=4, ny=4, spacing=0.1, fovy_deg=50.0, aspect=16 / 9):
    """Config 5 camera array: nx*ny pinholes on a plane, parallel look direction."""
    eye = np.asarray(eye, np.float64)
    f = normalize(np.asarray(target, np.float64) - eye)
    s = normalize(np.cross(f, up))
    u = np.cross(s, f)
    proj = perspective_vulkan_no_depth_reverse(math.radians(fovy_deg), aspect, NEAR_PLANE, FAR_PLANE)
    vis = []
    for j in range(ny):
        for i in range(nx):
            off = (i - (nx - 1) / 2) * spacing * s + (j - (ny - 1) / 2) * spacing * u
            vis.append(colmajor(inverse(look_at(eye + off, eye + off + f, up))))
    return np.concatenate(vis), colmajor(inverse(proj))
