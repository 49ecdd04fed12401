"""Host camera math of the reference application, in float32 with glm's operation order, so the
matrices handed to the renderer are bit-identical to the ones the reference uploads.

Reference (paths relative to the reference root):
  * Camera — base/camera.hpp:31-58 (updateViewMatrix, N_IS_UP axes of base/Define.h:63),
    :124-141 (rotateAxis), :157-182 (setPerspective), :95-121 (setNerfCamera / setDatasetCamera /
    loadDatasetCamera);
  * CameraLoader — base/LoadCamera.hpp:45-56 (calcIntrinsics), :57-85 (c2wTow2cRT), :124-147
    (loadNerfCameraData);
  * glm 0.9.8 as vendored (external/glm): lookAtRH (gtc/matrix_transform.inl), the modified
    perspective_Vulkan_no_depth_reverse (:276-290), compute_inverse<mat4> (detail/func_matrix.inl:
    299-354), normalize = v * (1 / sqrt(dot(v, v))), dot3 = (x + y) + z, radians = deg * 0.0174...f;
  * VulkanFullRT::updateUniformBuffer (VulkanFullRT.cpp:1331-1349: viewInverse = inverse(view),
    projInverse = inverse(perspective)) and calculateGaussianLightFieldSamples (:1518-1604).

Every arithmetic step is one IEEE float32 operation in glm's order (numpy float32 scalars; no FMA,
as the reference's SSE build); sin/cos/tan/atan are the C library's sinf/cosf/tanf/atanf, which is
what `std::sin(float)` in camera.hpp / LoadCamera.hpp calls.  tests/test_camera_reference.py checks
every matrix bit for bit against the reference's own camera.hpp / LoadCamera.hpp / glm compiled from
its sources (oracle/ref.mk -> oracle/_ref/ref_camera_dump).

Matrices are float32 (4, 4) arrays in glm memory order: M[c][r] is column c, row r, so
`colmajor(M)` (the 16 floats of the C-ABI and of GLSL's mat4) is a plain reshape.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import json

import numpy as np

f32 = np.float32
FOV_Y = f32(39.6)          # base/Define.h:33 (39.6f)
NEAR_PLANE = f32(0.005)    # base/Define.h:34
FAR_PLANE = f32(20.0)      # base/Define.h:35
FLT_MIN = f32(1.1754943508222875e-38)
FLT_MAX = f32(3.4028234663852886e38)
RAD2DEGREE = 57.2957795131  # base/LoadCamera.hpp:20 (a double literal)

_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
for _fn in ("sinf", "cosf", "tanf", "atanf"):
    getattr(_libm, _fn).argtypes = [ctypes.c_float]
    getattr(_libm, _fn).restype = ctypes.c_float


def sinf(x):
    return f32(_libm.sinf(float(f32(x))))


def cosf(x):
    return f32(_libm.cosf(float(f32(x))))


def tanf(x):
    return f32(_libm.tanf(float(f32(x))))


def atanf(x):
    return f32(_libm.atanf(float(f32(x))))


def radians(deg):
    """glm::radians: degrees * static_cast<float>(0.01745329251994329576923690768489)."""
    return f32(deg) * f32(0.01745329251994329576923690768489)


def aspect_ratio(width, height):
    """(float)width / height, as VulkanFullRT computes the aspect (VulkanFullRT.cpp:2154)."""
    return f32(width) / f32(height)


# ------------------------------------------------------------------------------------ vec3 (glm order)
def vec3(v):
    return tuple(f32(x) for x in v)


def add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def scale(a, s):
    s = f32(s)
    return (a[0] * s, a[1] * s, a[2] * s)


def neg(a):
    return (-a[0], -a[1], -a[2])


def dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def cross(x, y):
    return (x[1] * y[2] - y[1] * x[2], x[2] * y[0] - y[2] * x[0], x[0] * y[1] - y[0] * x[1])


def normalize(v):
    v = vec3(v)
    return scale(v, f32(1) / np.sqrt(dot(v, v)))


# ------------------------------------------------------------------------------------ mat4 (glm layout)
def identity():
    return np.eye(4, dtype=np.float32)


def colmajor(m):
    """The 16 floats of a glm mat4 in memory order (what updateUniformBuffer uploads)."""
    return np.ascontiguousarray(np.asarray(m, np.float32).reshape(16))


def rowcol(m):
    """Math-convention view (row, col) of a glm-layout matrix (for tests doing linear algebra)."""
    return np.asarray(m, np.float32).T


def look_at(eye, center, up):
    """glm::lookAtRH (gtc/matrix_transform.inl)."""
    eye, center, up = vec3(eye), vec3(center), vec3(up)
    f = normalize(sub(center, eye))
    s = normalize(cross(f, up))
    u = cross(s, f)
    m = identity()
    for i in range(3):
        m[i][0] = s[i]
        m[i][1] = u[i]
        m[i][2] = -f[i]
    m[3][0] = -dot(s, eye)
    m[3][1] = -dot(u, eye)
    m[3][2] = dot(f, eye)
    return m


def perspective_vulkan_no_depth_reverse(fovy, aspect, znear, zfar):
    """glm::perspective_Vulkan_no_depth_reverse (matrix_transform.inl:276-290); fovy in radians
    (float32, e.g. `radians(deg)`).  Result[1][1] = -1/tan: image row 0 is the top."""
    fovy, aspect, znear, zfar = f32(fovy), f32(aspect), f32(znear), f32(zfar)
    t = tanf(fovy / f32(2))
    m = np.zeros((4, 4), np.float32)
    m[0][0] = f32(1) / (aspect * t)
    m[1][1] = -f32(1) / t
    m[2][3] = f32(-1)
    m[2][2] = -zfar / (zfar - znear)
    m[3][2] = -(zfar * znear) / (zfar - znear)
    return m


def inverse(m):
    """glm compute_inverse<mat4> (detail/func_matrix.inl:299-354): cofactors, SignA/SignB, one
    reciprocal of the determinant, every operation float32 in glm's order."""
    m = np.asarray(m, np.float32)

    def c2(a, b, c, d, e, f, g, h):  # m[a][b]*m[c][d] - m[e][f]*m[g][h]
        return m[a][b] * m[c][d] - m[e][f] * m[g][h]

    c00, c02, c03 = c2(2, 2, 3, 3, 3, 2, 2, 3), c2(1, 2, 3, 3, 3, 2, 1, 3), c2(1, 2, 2, 3, 2, 2, 1, 3)
    c04, c06, c07 = c2(2, 1, 3, 3, 3, 1, 2, 3), c2(1, 1, 3, 3, 3, 1, 1, 3), c2(1, 1, 2, 3, 2, 1, 1, 3)
    c08, c10, c11 = c2(2, 1, 3, 2, 3, 1, 2, 2), c2(1, 1, 3, 2, 3, 1, 1, 2), c2(1, 1, 2, 2, 2, 1, 1, 2)
    c12, c14, c15 = c2(2, 0, 3, 3, 3, 0, 2, 3), c2(1, 0, 3, 3, 3, 0, 1, 3), c2(1, 0, 2, 3, 2, 0, 1, 3)
    c16, c18, c19 = c2(2, 0, 3, 2, 3, 0, 2, 2), c2(1, 0, 3, 2, 3, 0, 1, 2), c2(1, 0, 2, 2, 2, 0, 1, 2)
    c20, c22, c23 = c2(2, 0, 3, 1, 3, 0, 2, 1), c2(1, 0, 3, 1, 3, 0, 1, 1), c2(1, 0, 2, 1, 2, 0, 1, 1)
    A = np.array
    fac0, fac1, fac2 = A([c00, c00, c02, c03]), A([c04, c04, c06, c07]), A([c08, c08, c10, c11])
    fac3, fac4, fac5 = A([c12, c12, c14, c15]), A([c16, c16, c18, c19]), A([c20, c20, c22, c23])
    v0 = A([m[1][0], m[0][0], m[0][0], m[0][0]])
    v1 = A([m[1][1], m[0][1], m[0][1], m[0][1]])
    v2 = A([m[1][2], m[0][2], m[0][2], m[0][2]])
    v3 = A([m[1][3], m[0][3], m[0][3], m[0][3]])
    inv0 = (v1 * fac0 - v2 * fac1) + v3 * fac2
    inv1 = (v0 * fac0 - v2 * fac3) + v3 * fac4
    inv2 = (v0 * fac1 - v1 * fac3) + v3 * fac5
    inv3 = (v0 * fac2 - v1 * fac4) + v2 * fac5
    sa = A([1, -1, 1, -1], np.float32)
    sb = A([-1, 1, -1, 1], np.float32)
    inv = np.stack([inv0 * sa, inv1 * sb, inv2 * sa, inv3 * sb]).astype(np.float32)
    row0 = A([inv[0][0], inv[1][0], inv[2][0], inv[3][0]])
    d = m[0] * row0
    det = (d[0] + d[1]) + (d[2] + d[3])
    return (inv * (f32(1) / det)).astype(np.float32)


def translate(m, v):
    """glm::translate(m, v): Result[3] = m[0]*v[0] + m[1]*v[1] + m[2]*v[2] + m[3]."""
    r = np.array(m, np.float32)
    r[3] = ((m[0] * f32(v[0]) + m[1] * f32(v[1])) + m[2] * f32(v[2])) + m[3]
    return r


def camera_matrices(view, proj):
    """(viewInverse, projInverse) as updateUniformBuffer uploads them (16 floats each)."""
    return colmajor(inverse(view)), colmajor(inverse(proj))


def pinhole(eye, target, up=(0.0, 1.0, 0.0), fovy_deg=FOV_Y, aspect=1.0, znear=NEAR_PLANE, zfar=FAR_PLANE):
    """glm::lookAt camera with perspective_Vulkan_no_depth_reverse(radians(fovy_deg)) (float32 inputs)."""
    view = look_at(eye, target, up)
    proj = perspective_vulkan_no_depth_reverse(radians(fovy_deg), aspect, znear, zfar)
    return camera_matrices(view, proj)


def orbit_eye(radius, elevation_deg, azimuth_deg, target=(0.0, 0.0, 0.0)):
    """Orbit position in float32: (r cos(el) sin(az), r sin(el), r cos(el) cos(az)) + target."""
    r = f32(radius)
    el, az = radians(elevation_deg), radians(azimuth_deg)
    ce = cosf(el)
    return add((r * ce * sinf(az), r * sinf(el), r * ce * cosf(az)), vec3(target))


def orbit_camera(radius, elevation_deg, azimuth_deg, target=(0.0, 0.0, 0.0), fovy_deg=50.0, aspect=f32(16) / f32(9)):
    return pinhole(orbit_eye(radius, elevation_deg, azimuth_deg, target), target, (0.0, 1.0, 0.0), fovy_deg, aspect)


class Camera:
    """base/camera.hpp Camera (Euler-angle camera, N_IS_UP axes of base/Define.h:63), float32.

    Mirrors the reference members and methods used on the render path: rotation / position
    (degrees / scene units), matrices.view / matrices.perspective (glm layout), setPerspective,
    updateAspectRatio, setPosition, setRotation, rotate, translate, setNearFar, loadDatasetCamera,
    setDatasetCamera, setNerfCamera, getCamNames."""

    class _Matrices:
        def __init__(self):
            self.perspective = identity()
            self.view = identity()

    def __init__(self):
        self.rotation = vec3((0, 0, 0))
        self.position = vec3((0, 0, 0))
        self.matrices = Camera._Matrices()
        self.fov = FOV_Y
        self.znear = NEAR_PLANE
        self.zfar = FAR_PLANE
        self.updated = True
        self.cameraLoader = CameraLoader()
        self.dataType = None

    # -- math-convention aliases kept for the Python callers
    @property
    def view(self):
        return self.matrices.view

    @property
    def perspective(self):
        return self.matrices.perspective

    @staticmethod
    def rotateAxis(rad, u, v, n):
        """camera.hpp:124-141: v = normalize(v cos + cross(u, v) sin); n = normalize(cross(u, v))."""
        s, c = sinf(rad), cosf(rad)
        v = normalize(add(scale(v, c), scale(cross(u, v), s)))
        n = normalize(cross(u, v))
        return u, v, n

    def updateViewMatrix(self):  # camera.hpp:31-58 (N_IS_UP)
        u, v, n = vec3((1, 0, 0)), vec3((0, 0, 1)), vec3((0, -1, 0))
        if radians(self.rotation[1]) != 0:
            v, n, u = self.rotateAxis(radians(self.rotation[1]), v, n, u)
        if radians(self.rotation[0]) != 0:
            u, v, n = self.rotateAxis(radians(self.rotation[0]), u, v, n)
        if radians(self.rotation[2]) != 0:
            n, u, v = self.rotateAxis(radians(self.rotation[2]), n, u, v)
        rot = identity()  # glm::mat4(vec4(u,0), vec4(v,0), vec4(n,0), vec4(0,0,0,1)): columns
        rot[0][:3], rot[1][:3], rot[2][:3] = u, v, n
        old = self.matrices.view
        self.matrices.view = translate(rot.T.copy(), neg(self.position))
        self.updated = self.updated or not np.array_equal(old, self.matrices.view)

    def setPosition(self, p):
        self.position = vec3(p)
        self.updateViewMatrix()

    def setRotation(self, r):
        self.rotation = vec3(r)
        self.updateViewMatrix()

    def rotate(self, delta):
        self.rotation = add(self.rotation, vec3(delta))
        self.updateViewMatrix()

    def setTranslation(self, t):
        self.setPosition(t)

    def translate(self, delta):
        self.position = add(self.position, vec3(delta))
        self.updateViewMatrix()

    def setPerspective(self, fov, aspect, znear, zfar):  # camera.hpp:157-182
        self.fov, self.znear, self.zfar = f32(fov), f32(znear), f32(zfar)
        self.matrices.perspective = perspective_vulkan_no_depth_reverse(radians(fov), aspect, znear, zfar)

    def updateAspectRatio(self, aspect):  # camera.hpp:184-198
        self.matrices.perspective = perspective_vulkan_no_depth_reverse(radians(self.fov), aspect, self.znear,
                                                                        self.zfar)

    def setNearFar(self, znear, zfar):
        self.znear, self.zfar = f32(znear), f32(zfar)

    def getNearClip(self):
        return self.znear

    def getFarClip(self):
        return self.zfar

    def getFov(self):
        return self.fov

    def getCamNames(self):
        return list(self.cameraLoader.camNames)

    def loadDatasetCamera(self, type_, path, width, height):  # camera.hpp:115-121
        if type_ == "nerf":
            self.cameraLoader.loadNerfCameraData(path, width, height, self.znear, self.zfar)
        self.dataType = type_

    def setNerfCamera(self, idx):  # camera.hpp:100-104
        self.matrices.view = self.cameraLoader.nerfCameras.frames[idx].transformMatrix.copy()

    def setDatasetCamera(self, type_, idx, aspect):  # camera.hpp:106-113
        if type_ == "nerf":
            self.setPerspective(self.cameraLoader.fovy, aspect, self.znear, self.zfar)
            self.setPerspective(FOV_Y, aspect, self.znear, self.zfar)
            self.setNerfCamera(idx)

    def matrices_inverse(self):
        """(viewInverse, projInverse) as updateUniformBuffer uploads them (VulkanFullRT.cpp:1342-1343)."""
        return camera_matrices(self.matrices.view, self.matrices.perspective)

    # snake_case aliases used by the Python app / tests
    set_position = setPosition
    set_rotation = setRotation
    set_perspective = setPerspective
    update_view_matrix = updateViewMatrix
    matrices_pair = matrices_inverse


class CameraFrame:
    def __init__(self):
        self.filePath = ""
        self.transformMatrix = identity()
        self.position = vec3((0, 0, 0))


class NerfCameraData:
    def __init__(self):
        self.cameraAngleX = f32(0)
        self.frames = []
        self.centers = []


class CameraLoader:
    """base/LoadCamera.hpp CameraLoader: loadNerfCameraData(path, width, height, znear, zfar)."""

    def __init__(self):
        self.nerfCameras = NerfCameraData()
        self.fovy = f32(0)
        self.camNames = []

    def calcIntrinsics(self, cameraAngleX, width, height, nearPlane, farPlane):  # LoadCamera.hpp:45-56
        fx = f32(0.5) * f32(width) / tanf(f32(0.5) * f32(cameraAngleX))
        fovy = f32(2) * atanf(f32(height) / (f32(2) * fx))
        self.fovy = f32(float(fovy) * RAD2DEGREE)  # float *= double

    def c2wTow2cRT(self, frame):  # LoadCamera.hpp:57-85: w2c = [R^T | -R^T T]
        m = frame.transformMatrix
        rinv = m[:3, :3].T.copy()  # glm::transpose(glm::mat3(m)) in glm layout
        t = m[3][:3]
        # mat3 * vec3 (glm): row r = m[0][r]*v.x + m[1][r]*v.y + m[2][r]*v.z, on -R_inv
        nr = -rinv
        tinv = tuple((nr[0][r] * t[0] + nr[1][r] * t[1]) + nr[2][r] * t[2] for r in range(3))
        w2c = identity()
        w2c[:3, :3] = rinv
        w2c[3][:3] = tinv
        frame.transformMatrix = w2c
        self.nerfCameras.centers.append(tinv)
        frame.position = neg(tinv)

    def loadNerfCameraData(self, jsonPath, width, height, znear, zfar):  # LoadCamera.hpp:124-147
        with open(jsonPath) as fh:
            j = json.load(fh)
        self.nerfCameras.cameraAngleX = f32(j["camera_angle_x"])
        self.calcIntrinsics(self.nerfCameras.cameraAngleX, width, height, znear, zfar)
        for i, fr in enumerate(j["frames"]):
            f = CameraFrame()
            f.filePath = fr.get("file_path", "")
            tm = fr["transform_matrix"]
            for row in range(4):
                for col in range(4):
                    f.transformMatrix[col][row] = f32(tm[row][col])
            self.c2wTow2cRT(f)
            self.nerfCameras.frames.append(f)
            self.camNames.append(str(i))


def load_nerf_cameras(path, width=800, height=800):
    """(camera_angle_x, [w2c view matrices in glm layout]) of a NeRF transforms_*.json."""
    cl = CameraLoader()
    cl.loadNerfCameraData(path, width, height, NEAR_PLANE, FAR_PLANE)
    return float(cl.nerfCameras.cameraAngleX), [f.transformMatrix for f in cl.nerfCameras.frames]


def nerf_eval_matrices(path, width, height):
    """The EVAL_QUALITY camera sequence (VulkanFullRT.cpp:2150-2156): for every frame,
    setDatasetCamera(nerf, i, (float)width / height) then updateUniformBuffer's inverses.
    Returns ([viewInverse 16 floats per frame], projInverse)."""
    cam = Camera()
    cam.setNearFar(NEAR_PLANE, FAR_PLANE)
    cam.loadDatasetCamera("nerf", path, width, height)
    vis, pi = [], None
    for i in range(len(cam.getCamNames())):
        cam.setDatasetCamera("nerf", i, aspect_ratio(width, height))
        vi, pi = cam.matrices_inverse()
        vis.append(vi)
    return vis, pi


def lightfield_ring_rig(positions, ncams=4, width=180, height=180):
    """VulkanFullRT::calculateGaussianLightFieldSamples (VulkanFullRT.cpp:1518-1604).

    bbox of the raw positions with max initialised to FLT_MIN (Q15), cameras at
    center +- maxR on x and y, lookAt(up = +z), 135 deg fov with aspect = (float)(width/height)
    (integer division, Q15).  Returns (viewInverse [ncams*16], projInverse [16])."""
    p = np.asarray(positions, np.float32).reshape(-1, 3)
    mn = np.minimum(p.min(axis=0), FLT_MAX) if len(p) else np.full(3, FLT_MAX, np.float32)
    mx = np.maximum(p.max(axis=0), FLT_MIN) if len(p) else np.full(3, FLT_MIN, np.float32)
    center = tuple((mn[k] + mx[k]) / f32(2) for k in range(3))
    cand = [mx[k] - mn[k] for k in range(3)]
    maxr = max(max(cand[0], cand[1]), cand[2]) / f32(2)
    cams = [(center[0] + maxr, center[1], center[2]), (center[0], center[1] + maxr, center[2]),
            (center[0] - maxr, center[1], center[2]), (center[0], center[1] - maxr, center[2])]
    vis = [colmajor(inverse(look_at(cams[i % 4], center, (0.0, 0.0, 1.0)))) for i in range(ncams)]
    proj = perspective_vulkan_no_depth_reverse(radians(135.0), f32(width // height), NEAR_PLANE, FAR_PLANE)
    return np.concatenate(vis), colmajor(inverse(proj))


def lightfield_grid_rig(eye, target, up=(0.0, 1.0, 0.0), nx=4, ny=4, spacing=0.1, fovy_deg=50.0,
                        aspect=f32(16) / f32(9), centred=True):
    """Config 5 camera array: nx*ny pinholes on a plane, parallel look direction, float32:
    f = normalize(target - eye), s = normalize(cross(f, up)), u = cross(s, f); camera (i, j) at
    eye + (ox * s + oy * u) with ox = (i - (nx-1)/2) * spacing, oy = (j - (ny-1)/2) * spacing (centred), or
    ox = i * spacing, oy = j * spacing (centred=False: camera (0, 0) is `eye` itself), looking at its
    position + f."""
    eye = vec3(eye)
    up = vec3(up)
    f = normalize(sub(vec3(target), eye))
    s = normalize(cross(f, up))
    u = cross(s, f)
    proj = perspective_vulkan_no_depth_reverse(radians(fovy_deg), aspect, NEAR_PLANE, FAR_PLANE)
    sp = f32(spacing)
    vis = []
    for j in range(ny):
        for i in range(nx):
            ox = ((f32(i) - f32(nx - 1) / f32(2)) if centred else f32(i)) * sp
            oy = ((f32(j) - f32(ny - 1) / f32(2)) if centred else f32(j)) * sp
            pos = add(eye, add(scale(s, ox), scale(u, oy)))
            vis.append(colmajor(inverse(look_at(pos, add(pos, f), up))))
    return np.concatenate(vis), colmajor(inverse(proj))
