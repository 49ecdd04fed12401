"""ctypes binding of include/gvrt.h (libgvrt.so, built in-tree by `make -C 3dgvrt_lightfield_amd`).

The product path is the HIP library only: if libgvrt.so is missing or a GPU call fails, the
functions here raise -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))


def _lib_path():
    """libgvrt.so of this package; GVRT_LIB_PATH may select an A/B variant build, but only one built in-tree
    under this package (`make variant`, build/<name>/libgvrt.so): any other path is refused."""
    p = os.environ.get("GVRT_LIB_PATH")
    if not p:
        return os.path.join(_HERE, "libgvrt.so")
    rp = os.path.realpath(p)
    if not rp.startswith(os.path.realpath(_HERE) + os.sep) or os.path.basename(rp) != "libgvrt.so":
        raise RuntimeError(f"GVRT_LIB_PATH={p}: only a libgvrt.so built under {_HERE} may be loaded")
    return rp


LIB_PATH = _lib_path()

GVRT_OK = 0
STATUS_NAMES = {
    0: "GVRT_OK", -1: "GVRT_ERR_INVALID_ARG", -2: "GVRT_ERR_OOM", -3: "GVRT_ERR_HIP",
    -4: "GVRT_ERR_STATE", -5: "GVRT_ERR_NO_DEVICE", -6: "GVRT_ERR_IO", -7: "GVRT_ERR_UNSUPPORTED",
    -8: "GVRT_ERR_RCCL",
}
# per-handle tuning switches (gvrt_set_option; include/gvrt.h GVRT_OPT_*)
OPTIONS = {"tile_order": 0, "tile_xcd": 1, "octant_nodes": 2, "record_origins": 3, "box_slack": 4,
           "packed_kbuffer": 5, "order_spread": 6,
           "accept_boxes": 7, "optional_mem_mb": 8}
MODE_FAST = 0
MODE_LITERAL = 1


class GvrtError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class Splats(C.Structure):
    _fields_ = [("n", C.c_uint64)] + [(k, C.POINTER(C.c_float)) for k in
                                      ("positions", "f_dc", "f_rest", "opacity", "scale", "rotation")]


class SplatBuffers(C.Structure):
    _fields_ = Splats._fields_


class EnclosingParams(C.Structure):
    _fields_ = [("kernel_min_response", C.c_float), ("opts", C.c_uint32), ("degree", C.c_float),
                ("emit_triangles", C.c_uint32)]


class RenderParams(C.Structure):
    _fields_ = [("aabb", C.c_float * 6), ("min_transmittance", C.c_float),
                ("hit_min_gaussian_response", C.c_float), ("sph_eval_degree", C.c_uint32),
                ("alpha_min", C.c_float), ("pixel_offset", C.c_float), ("alpha_init", C.c_float),
                ("tmin_inclusive", C.c_uint32), ("mode", C.c_uint32), ("max_rounds", C.c_uint32),
                ("ray_dirs_layout", C.c_uint32), ("kbuffer_depth", C.c_uint32), ("reserved", C.c_uint32 * 4)]


class Tile(C.Structure):
    _fields_ = [("tx", C.c_uint16), ("ty", C.c_uint16), ("cam", C.c_uint16), ("pad", C.c_uint16)]


class Image(C.Structure):
    _fields_ = [("rgba8", C.c_void_p), ("rgba32f", C.c_void_p), ("ray_dirs", C.c_void_p),
                ("hit_counts", C.c_void_p), ("device_ptrs", C.c_uint32), ("packed", C.c_uint32)]


class AccelParams(C.Structure):
    _fields_ = [("split_cells", C.c_uint32), ("builder", C.c_uint32), ("collapse", C.c_uint32),
                ("depth_budget", C.c_uint32), ("split_min_span", C.c_uint32), ("reserved", C.c_uint32 * 3)]


class Stats(C.Structure):
    _fields_ = [("n_input", C.c_uint64), ("n_survivors", C.c_uint64), ("bvh_nodes", C.c_uint64),
                ("bvh_depth", C.c_uint32), ("bvh_depth4", C.c_uint32), ("rays", C.c_uint64),
                ("crossings", C.c_uint64), ("accepted", C.c_uint64), ("rounds", C.c_uint64),
                ("enclose_ms", C.c_float), ("accel_ms", C.c_float), ("render_ms", C.c_float),
                ("pad1", C.c_float), ("device_bytes", C.c_uint64), ("wave_node_visits", C.c_uint64),
                ("wave_leaf_visits", C.c_uint64), ("lane_leaf_tests", C.c_uint64),
                ("phase_cycles", C.c_uint64 * 4), ("wave_dead_visits", C.c_uint64),
                ("bvh_leaves", C.c_uint64), ("wave_rounds", C.c_uint64), ("wave_late_node_visits", C.c_uint64),
                ("bvh_builder", C.c_uint32), ("bvh_depth4_rebuilt", C.c_uint32)]


class DeviceProperties(C.Structure):
    _fields_ = [("device_name", C.c_char * 256), ("driver_version", C.c_uint32), ("compute_units", C.c_uint32),
                ("total_memory", C.c_uint64), ("arch_name", C.c_char * 64)]


class DeviceBuffers(C.Structure):
    _fields_ = [("n", C.c_uint64), ("positions", C.c_void_p), ("rotations", C.c_void_p), ("scales", C.c_void_p),
                ("densities", C.c_void_p), ("features_albedo", C.c_void_p), ("features_specular", C.c_void_p),
                ("m", C.c_uint64), ("vertices", C.c_void_p), ("indices", C.c_void_p),
                ("particle_density", C.c_void_p), ("particle_sph", C.c_void_p)]


H = C.c_void_p
_P = C.POINTER

# name -> (restype, argtypes); every symbol declared in include/gvrt.h
SIGNATURES = {
    "gvrt_abi_version": (C.c_int, []),
    "gvrt_build_info": (C.c_char_p, []),
    "gvrt_default_enclosing_params": (None, [_P(EnclosingParams)]),
    "gvrt_default_render_params": (None, [_P(RenderParams)]),
    "gvrt_create": (C.c_int32, [C.c_int, _P(H)]),
    "gvrt_destroy": (C.c_int32, [H]),
    "gvrt_last_error": (C.c_char_p, [H]),
    "gvrt_device_count": (C.c_int32, [_P(C.c_int)]),
    "gvrt_load_splats": (C.c_int32, [H, _P(Splats)]),
    "gvrt_build_enclosing": (C.c_int32, [H, _P(EnclosingParams), _P(C.c_uint64)]),
    "gvrt_read_enclosing": (C.c_int32, [H, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gvrt_build_accel": (C.c_int32, [H]),
    "gvrt_build_accel_ex": (C.c_int32, [H, _P(AccelParams)]),
    "gvrt_default_accel_params": (None, [_P(AccelParams)]),
    "gvrt_render": (C.c_int32, [H, _P(RenderParams), C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                C.c_uint32, C.c_void_p, C.c_uint64, _P(Image)]),
    "gvrt_render_async": (C.c_int32, [H, _P(RenderParams), C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                C.c_uint32, C.c_void_p, C.c_uint64, _P(Image)]),
    "gvrt_sync": (C.c_int32, [H]),
    "gvrt_set_stream": (C.c_int32, [H, C.c_void_p]),
    "gvrt_set_stats": (C.c_int32, [H, C.c_int]),
    "gvrt_set_option": (C.c_int32, [H, C.c_uint32, C.c_int64]),
    "gvrt_get_option": (C.c_int32, [H, C.c_uint32, _P(C.c_int64)]),
    "gvrt_get_device_properties": (C.c_int32, [C.c_int, _P(DeviceProperties)]),
    "gvrt_get_device_buffers": (C.c_int32, [H, _P(DeviceBuffers)]),
    "gvrt_read_accel": (C.c_int32, [H, C.c_int, C.c_void_p, C.c_uint64, _P(C.c_uint64)]),
    "gvrt_get_stats": (C.c_int32, [H, _P(Stats)]),
    "gvrt_unpack_tiles_rgba8": (C.c_int32, [H, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                            C.c_uint32, C.c_void_p]),
    "gvrt_read_tile_costs": (C.c_int32, [H, C.c_void_p, C.c_uint64]),
    "gvrt_ply_load": (C.c_int32, [C.c_char_p, _P(SplatBuffers)]),
    "gvrt_ply_free": (None, [_P(SplatBuffers)]),
    "gvrt_ply_save": (C.c_int32, [C.c_char_p, _P(Splats)]),
}

_lib = None


def lib():
    """Load libgvrt.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise GvrtError(-4, f"{LIB_PATH} is missing: run `make -C 3dgvrt_lightfield_amd` "
                                "(or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("GVRT_LIB_PATH") and not hasattr(L, name):
                continue  # an A/B variant built from an older revision may predate a symbol
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(status, handle=None):
    if status != GVRT_OK:
        msg = lib().gvrt_last_error(handle)
        raise GvrtError(status, msg.decode() if msg else "")


def fptr(a):
    return a.ctypes.data_as(_P(C.c_float))


def vptr(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def as_f32(a, n=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if n is not None and a.size != n:
        raise ValueError(f"expected {n} floats, got {a.size}")
    return a


def make_splats_struct(splats):
    """splats: dict/obj with positions,f_dc,f_rest,opacity,scale,rotation (SplatSet layout)."""
    get = (lambda k: splats[k]) if isinstance(splats, dict) else (lambda k: getattr(splats, k))
    n = get("positions").size // 3
    arrs = {k: as_f32(get(k), m * n) for k, m in
            (("positions", 3), ("f_dc", 3), ("f_rest", 45), ("opacity", 1), ("scale", 3), ("rotation", 4))}
    s = Splats(n, *[fptr(arrs[k]) for k in ("positions", "f_dc", "f_rest", "opacity", "scale", "rotation")])
    return s, arrs  # keep arrs alive while s is used
