"""Host-side mirror of the reference's model / renderer classes over the C-ABI.

  vk3DGRT::SplatSet, PLYLoader, Model   base/Vulkan3DGRTModel.h:15-52
  VulkanFullRT::prepare / draw          projects/VulkanFullRT/VulkanFullRT.cpp:1990-2178
  computeGaussianLightField             projects/VulkanFullRT/VulkanFullRT.cpp:1900-1976

Every GPU call goes to libgvrt.so; nothing here computes a pixel.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, lib

SPLAT_KEYS = (("positions", 3), ("f_dc", 3), ("f_rest", 45), ("opacity", 1), ("scale", 3), ("rotation", 4))

# The static-scene build the bench renders with (Renderer.prepare / build_accel keywords): the device binned-SAH
# tree with the SAH-optimal 4-wide collapse (the reference's PREFER_FAST_TRACE BLAS, VulkanFullRT.cpp:621) and
# the SplitBLAS grid of the reference (SPLIT_BLAS, NUMBER_OF_CELLS_PER_LONGEST_AXIS = 10, base/Define.h:45-47)
# applied to the large proxies only: those whose box overlaps at least 3 cells along an axis (a fifth of the
# scene) are split into cell pieces, the rest stay whole, and a scene without such proxies gets the unsplit tree.
QUALITY_BUILD = dict(builder=2, collapse=1, split_cells=10, split_min_span=3)


class SplatSet(dict):
    """vk3DGRT::SplatSet: SoA float32 arrays keyed like the C++ members."""

    def size(self):
        return self["positions"].size // 3 if "positions" in self else 0


class PLYLoader:
    """vk3DGRT::PLYLoader (Vulkan3DGRTModel.cpp:7-125) -> gvrt_ply_load."""

    def loadPLYModel(self, filename, output: SplatSet) -> bool:
        buf = _lib.SplatBuffers()
        st = lib().gvrt_ply_load(str(filename).encode(), C.byref(buf))
        if st != _lib.GVRT_OK:
            return False
        n = int(buf.n)
        try:
            for k, m in SPLAT_KEYS:
                p = getattr(buf, k)
                output[k] = np.ctypeslib.as_array(p, shape=(n * m,)).copy() if n else np.zeros(0, np.float32)
        finally:
            lib().gvrt_ply_free(C.byref(buf))
        return True


def save_ply(filename, splats):
    s, keep = _lib.make_splats_struct(splats)
    st = lib().gvrt_ply_save(str(filename).encode(), C.byref(s))
    check(st)


class Renderer:
    """One device, one handle: enclosing pass, LBVH, Particle Rendering pass."""

    def __init__(self, device=0):
        h = _lib.H()
        check(lib().gvrt_create(int(device), C.byref(h)))
        self.h = h
        self.device = device
        self.m = 0
        self._ms_stats = _lib.Stats()

    def close(self):
        if self.h:
            lib().gvrt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- Model::allocateAttributeBuffers
    def load_splats(self, splats):
        s, keep = _lib.make_splats_struct(splats)
        check(lib().gvrt_load_splats(self.h, C.byref(s)), self.h)

    @staticmethod
    def enclosing_params(**kw):
        p = _lib.EnclosingParams()
        lib().gvrt_default_enclosing_params(C.byref(p))
        for k, v in kw.items():
            setattr(p, k, v)
        return p

    @staticmethod
    def render_params(**kw):
        p = _lib.RenderParams()
        lib().gvrt_default_render_params(C.byref(p))
        for k, v in kw.items():
            if k == "aabb":
                p.aabb[:] = list(v)
            else:
                setattr(p, k, v)
        return p

    def build_enclosing(self, **kw):
        m = C.c_uint64(0)
        p = self.enclosing_params(**kw)
        check(lib().gvrt_build_enclosing(self.h, C.byref(p), C.byref(m)), self.h)
        self.m = int(m.value)
        self._emit = bool(p.emit_triangles)
        return self.m

    def read_enclosing(self, triangles=False):
        m = self.m
        dens = np.zeros(12 * m, np.float32)
        sh = np.zeros(48 * m, np.float32)
        src = np.zeros(m, np.uint32)
        verts = np.zeros(36 * m, np.float32) if triangles else None
        tris = np.zeros(60 * m, np.uint32) if triangles else None
        check(lib().gvrt_read_enclosing(self.h, _lib.vptr(dens), _lib.vptr(sh), _lib.vptr(verts), _lib.vptr(tris),
                                        _lib.vptr(src)), self.h)
        out = {"density": dens, "sh": sh, "src_index": src}
        if triangles:
            out["verts"], out["tris"] = verts, tris
        return out

    def build_accel(self, split_cells=0, builder=0, collapse=0, depth_budget=0, split_min_span=0):
        p = _lib.AccelParams()
        lib().gvrt_default_accel_params(C.byref(p))
        p.split_cells, p.builder, p.collapse = int(split_cells), int(builder), int(collapse)
        p.depth_budget, p.split_min_span = int(depth_budget), int(split_min_span)
        check(lib().gvrt_build_accel_ex(self.h, C.byref(p)), self.h)

    def prepare(self, splats, split_cells=0, builder=0, collapse=0, split_min_span=0, **enclosing):
        """VulkanFullRT::prepare: upload, enclose, build the acceleration structure."""
        self.load_splats(splats)
        m = self.build_enclosing(**enclosing)
        self.build_accel(split_cells=split_cells, builder=builder, collapse=collapse, split_min_span=split_min_span)
        return m

    def set_option(self, name, value):
        """gvrt_set_option: a per-handle tuning switch by name (_lib.OPTIONS), 0 or 1."""
        check(lib().gvrt_set_option(self.h, _lib.OPTIONS[name], int(value)), self.h)

    def get_option(self, name):
        v = C.c_int64(0)
        check(lib().gvrt_get_option(self.h, _lib.OPTIONS[name], C.byref(v)), self.h)
        return int(v.value)

    def tile_costs(self, width=None, height=None, ncams=1, ntiles=None):
        """gvrt_read_tile_costs: the last cost-ordered launch's per-tile cost classes (c: ~2^(c/4) k cycles).
        Full frame: uint8 [ncams, ceil(H/8), ceil(W/8)]; a caller tile list: ntiles=len(list), uint8 [ntiles]."""
        if ntiles is None:
            shape = (ncams, (height + 7) // 8, (width + 7) // 8)
        else:
            shape = (int(ntiles),)
        out = np.zeros(shape, np.uint8)
        check(lib().gvrt_read_tile_costs(self.h, out.ctypes.data, out.size), self.h)
        return out

    def set_stats(self, on=True):
        check(lib().gvrt_set_stats(self.h, 1 if on else 0), self.h)

    def stats(self):
        s = _lib.Stats()
        check(lib().gvrt_get_stats(self.h, C.byref(s)), self.h)
        out = {k: getattr(s, k) for k, _ in s._fields_ if not k.startswith("pad")}
        out["phase_cycles"] = list(out["phase_cycles"])
        return out

    def render_ms(self):
        """Device time of the last render kernel (gvrt_stats.render_ms) without building the stats dict."""
        s = self._ms_stats
        check(lib().gvrt_get_stats(self.h, C.byref(s)), self.h)
        return s.render_ms

    @staticmethod
    def tile_array(tiles):
        if tiles is None:
            return None, 0
        t = np.ascontiguousarray(np.asarray(tiles, np.uint16).reshape(-1, 4))
        return t, t.shape[0]

    def render(self, view_inv, proj_inv, width, height, ncams=1, params=None, tiles=None, rgba8=True,
               rgba32f=True, ray_dirs=False, hit_counts=False, packed=False, **kw):
        """Host-output render; returns dict of numpy arrays ([cam][H][W][...] or tile-packed)."""
        p = params if params is not None else self.render_params(**kw)
        vi = np.ascontiguousarray(view_inv, np.float32).reshape(-1)
        pi = np.ascontiguousarray(proj_inv, np.float32).reshape(16)
        if vi.size != 16 * ncams:
            raise ValueError("view_inv must hold 16*ncams floats")
        t, nt = self.tile_array(tiles)
        npix = nt * 64 if packed else width * height * ncams
        out = {}
        if rgba8:
            out["rgba8"] = np.zeros((npix, 4), np.uint8)
        if rgba32f:
            out["rgba32f"] = np.zeros((npix, 4), np.float32)
        if ray_dirs:
            out["ray_dirs"] = np.zeros((width * height * ncams, 4), np.float32)
        if hit_counts:
            out["hit_counts"] = np.zeros(npix, np.uint32)
        img = _lib.Image(_lib.vptr(out.get("rgba8")), _lib.vptr(out.get("rgba32f")), _lib.vptr(out.get("ray_dirs")),
                         _lib.vptr(out.get("hit_counts")), 0, 1 if packed else 0)
        check(lib().gvrt_render(self.h, C.byref(p), _lib.vptr(vi), _lib.vptr(pi), width, height, ncams,
                                _lib.vptr(t), nt, C.byref(img)), self.h)
        if not packed:
            for k in ("rgba8", "rgba32f"):
                if k in out:
                    out[k] = out[k].reshape(ncams, height, width, 4)
            if "hit_counts" in out:
                out["hit_counts"] = out["hit_counts"].reshape(ncams, height, width)
        return out

    def render_device(self, view_inv, proj_inv, width, height, ncams=1, params=None, tiles=None, rgba8_ptr=None,
                      rgba32f_ptr=None, ray_dirs_ptr=None, hit_counts_ptr=None, packed=False, async_=False, **kw):
        """Render into caller-owned device memory (e.g. torch tensor data_ptr()).  async_=True queues the
        frame (gvrt_render_async) and returns at once; sync() waits for the queued frames."""
        p = params if params is not None else self.render_params(**kw)
        vi = np.ascontiguousarray(view_inv, np.float32).reshape(-1)
        pi = np.ascontiguousarray(proj_inv, np.float32).reshape(16)
        if vi.size != 16 * ncams or pi.size != 16:
            raise ValueError("view_inv must hold 16*ncams floats and proj_inv 16")
        t, nt = self.tile_array(tiles)
        img = _lib.Image(rgba8_ptr, rgba32f_ptr, ray_dirs_ptr, hit_counts_ptr, 1, 1 if packed else 0)
        fn = lib().gvrt_render_async if async_ else lib().gvrt_render
        check(fn(self.h, C.byref(p), _lib.vptr(vi), _lib.vptr(pi), width, height, ncams, _lib.vptr(t), nt,
                 C.byref(img)), self.h)

    def sync(self):
        """gvrt_sync: wait for the frames queued by render_device(async_=True); render_ms() is then their mean."""
        check(lib().gvrt_sync(self.h), self.h)

    def set_stream(self, stream_ptr):
        """gvrt_set_stream: launch on this hipStream_t (an integer, e.g. torch.cuda.Stream().cuda_stream;
        0 / None: the handle's own stream — torch's default stream is the NULL stream, which the handle's
        non-blocking stream does not order with, so share a non-default torch stream)."""
        check(lib().gvrt_set_stream(self.h, C.c_void_p(stream_ptr or None)), self.h)

    def unpack_tiles_rgba8(self, packed_ptr, tiles, width, height, frame_ptr, ncams=1):
        """gvrt_unpack_tiles_rgba8: tile-packed rgba8 (device) -> frame [ncams][H][W][4] (device)."""
        t, nt = self.tile_array(tiles)
        check(lib().gvrt_unpack_tiles_rgba8(self.h, packed_ptr, _lib.vptr(t), nt, width, height, ncams, frame_ptr),
              self.h)

    def read_accel(self, which=1):
        """gvrt_read_accel: the binary tree (which=0, float32 [n, 16] rows: child boxes, then c0, c1, axis
        as int32 views), the 4-wide tree (which=1, [n, 32] rows), as raw 32-bit words (uint32), or (which=2,
        adaptive enclosing) each leaf's icosahedron half-width as float32 [n_leaves]."""
        n = C.c_uint64(0)
        check(lib().gvrt_read_accel(self.h, int(which), None, 0, C.byref(n)), self.h)
        if which == 2:
            hk = np.zeros(int(n.value), np.float32)
            if n.value:
                check(lib().gvrt_read_accel(self.h, 2, hk.ctypes.data, n.value, C.byref(n)), self.h)
            return hk
        words = 16 if which == 0 else 32
        out = np.zeros((int(n.value), words), np.uint32)
        if n.value:
            check(lib().gvrt_read_accel(self.h, int(which), out.ctypes.data, n.value, C.byref(n)), self.h)
        return out

    def device_buffers(self):
        """gvrt_get_device_buffers: device pointers of Model::Attributes and the enclosing outputs."""
        b = _lib.DeviceBuffers()
        check(lib().gvrt_get_device_buffers(self.h, C.byref(b)), self.h)
        return {k: getattr(b, k) for k, _ in b._fields_}


def device_properties(device=0):
    """gvrt_get_device_properties: name, driver version, CUs, memory, arch of a HIP device."""
    p = _lib.DeviceProperties()
    check(lib().gvrt_get_device_properties(int(device), C.byref(p)))
    return {"device_name": p.device_name.decode(), "driver_version": p.driver_version,
            "compute_units": p.compute_units, "total_memory": p.total_memory, "arch_name": p.arch_name.decode()}


def device_count():
    n = C.c_int(0)
    lib().gvrt_device_count(C.byref(n))
    return int(n.value)


def tiles_for_rank(width, height, ncams, rank, world, block=8):
    """Round-robin assignment of (block*8)^2-pixel blocks to ranks, as 8x8 tiles."""
    tx_n, ty_n = (width + 7) // 8, (height + 7) // 8
    bx_n, by_n = (tx_n + block - 1) // block, (ty_n + block - 1) // block
    out = []
    k = 0
    for c in range(ncams):
        for by in range(by_n):
            for bx in range(bx_n):
                if k % world == rank:
                    for ty in range(by * block, min((by + 1) * block, ty_n)):
                        for tx in range(bx * block, min((bx + 1) * block, tx_n)):
                            out.append((tx, ty, c, 0))
                k += 1
    return np.asarray(out, np.uint16).reshape(-1, 4)


def quantize_rgba8(rgba32f):
    """R8G8B8A8_UNORM store of imageStore: clamp to [0,1], round to nearest."""
    return (np.clip(np.asarray(rgba32f, np.float32), 0.0, 1.0) * np.float32(255.0) + np.float32(0.5)).astype(np.uint8)


def psnr_rgb(a8, b8):
    """results/evaluations/eval_quality.py:9-14 restated: MSE over RGB, peak 255."""
    a = np.asarray(a8, np.float64)[..., :3]
    b = np.asarray(b8, np.float64)[..., :3]
    mse = np.mean((a - b) ** 2)
    return float("inf") if mse == 0 else 20.0 * np.log10(255.0 / np.sqrt(mse))
