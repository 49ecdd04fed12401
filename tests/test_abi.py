"""C-ABI checks without a GPU: libgvrt.so loads, exports every symbol include/gvrt.h declares, the
ctypes mirror has the C struct layouts, defaults match the reference constants, host-only entry
points (PLY loader) work, and GPU entry points fail with status codes instead of aborting."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "gvrt.h")


def header_functions():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gvrt_[a-z0-9_]+)\s*\(", txt)))


def test_every_declared_symbol_is_exported(gv):
    L = gv.lib()
    names = header_functions()
    assert len(names) >= 18
    for n in names:
        assert hasattr(L, n), f"libgvrt.so does not export {n}"
    from importlib import import_module
    sig = import_module("3dgvrt_lightfield_amd._lib").SIGNATURES
    assert set(names) == set(sig), set(names) ^ set(sig)


STRUCTS = {"gvrt_splats": "Splats", "gvrt_enclosing_params": "EnclosingParams", "gvrt_render_params": "RenderParams",
           "gvrt_tile": "Tile", "gvrt_image": "Image", "gvrt_stats": "Stats", "gvrt_splat_buffers": "SplatBuffers",
           "gvrt_accel_params": "AccelParams", "gvrt_device_properties": "DeviceProperties",
           "gvrt_device_buffers": "DeviceBuffers"}


def test_struct_layouts_match_header(gv):
    from importlib import import_module
    L = import_module("3dgvrt_lightfield_amd._lib")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "gvrt.h"', "int main(void){"]
    for cs, ps in STRUCTS.items():
        lines.append(f'printf("{cs} %zu\\n", sizeof({cs}));')
        for f, _ in getattr(L, ps)._fields_:
            lines.append(f'printf("{cs}.{f} %zu\\n", offsetof({cs}, {f}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(src, "w").write("\n".join(lines))
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), src, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split("\n")
    got = dict(line.rsplit(" ", 1) for line in out if line)
    for cs, ps in STRUCTS.items():
        st = getattr(L, ps)
        assert int(got[cs]) == C.sizeof(st), cs
        for f, _ in st._fields_:
            assert int(got[f"{cs}.{f}"]) == getattr(st, f).offset, f"{cs}.{f}"


def test_defaults_match_reference_constants(gv):
    p = gv.Renderer.render_params()
    assert list(p.aabb) == [-100, -100, -100, 100, 100, 100]            # VulkanUtils.h:53
    assert p.min_transmittance == pytest.approx(0.001)                  # VulkanUtils.h:54
    assert p.hit_min_gaussian_response == pytest.approx(0.0113)         # VulkanUtils.h:55
    assert p.sph_eval_degree == 3                                       # VulkanUtils.h:56
    assert p.alpha_min == pytest.approx(1 / 255)                        # 3dgs.glsl:16
    assert p.pixel_offset == 0.0 and p.alpha_init == 0.0 and p.tmin_inclusive == 0
    e = gv.Renderer.enclosing_params()
    assert e.kernel_min_response == pytest.approx(0.0113) and e.opts == 0 and e.degree == 4.0  # VulkanFullRT.cpp:1353-1356


def test_no_device_is_a_status_not_an_abort(gv):
    if gv.device_count() > 0:
        pytest.skip("a HIP device is present")
    h = C.c_void_p()
    st = gv.lib().gvrt_create(0, C.byref(h))
    assert st == -5 and not h.value                                     # GVRT_ERR_NO_DEVICE
    assert b"no HIP device" in gv.lib().gvrt_last_error(None)
    # NULL handles are rejected, never dereferenced
    assert gv.lib().gvrt_build_accel(None) == -1
    assert gv.lib().gvrt_render(None, None, None, None, 1, 1, 1, None, 0, None) == -1
    from importlib import import_module
    L = import_module("3dgvrt_lightfield_amd._lib")
    props = L.DeviceProperties()
    assert gv.lib().gvrt_get_device_properties(0, C.byref(props)) == -5
    assert gv.lib().gvrt_get_device_buffers(None, C.byref(L.DeviceBuffers())) == -1
    assert gv.lib().gvrt_set_option(None, 0, 1) == -1
    v = C.c_int64(7)
    assert gv.lib().gvrt_get_option(None, 0, C.byref(v)) == -1 and v.value == 7


def test_option_names_match_header(gv):
    """_lib.OPTIONS mirrors the GVRT_OPT_* values of include/gvrt.h."""
    from importlib import import_module
    L = import_module("3dgvrt_lightfield_amd._lib")
    txt = open(HDR).read()
    opts = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"#define GVRT_OPT_([A-Z_]+) (\d+)u", txt)}
    count = opts.pop("count")
    assert opts == L.OPTIONS and count == len(opts)


def test_lib_path_override_is_confined_to_the_package(tmp_path):
    """GVRT_LIB_PATH may only name a libgvrt.so built under the package (A/B variant builds)."""
    code = "import importlib; importlib.import_module('3dgvrt_lightfield_amd._lib')"
    for bad in (str(tmp_path / "libgvrt.so"), "/usr/lib/libm.so.6"):
        r = subprocess.run(["python3", "-c", code], cwd=ROOT, capture_output=True, text=True,
                           env=dict(os.environ, GVRT_LIB_PATH=bad))
        assert r.returncode != 0 and "only a libgvrt.so built under" in r.stderr


def test_ply_roundtrip_and_reorder(gv, tmp_path):
    s = gv.scene.config1(n=37, seed=5)
    path = tmp_path / "s.ply"
    gv.save_ply(path, s)
    got = gv.SplatSet()
    assert gv.PLYLoader().loadPLYModel(path, got)
    for k in s:
        np.testing.assert_array_equal(got[k], s[k], err_msg=k)
    assert got.size() == 37


def test_ply_ascii_channel_major_reorder(gv, tmp_path):
    """f_rest_{15c+i} in the file -> SplatSet.f_rest[3i+c] (Vulkan3DGRTModel.cpp:70-77); missing groups are zero."""
    names = ["x", "y", "z"] + [f"f_rest_{i}" for i in range(45)] + ["opacity", "f_dc_0", "f_dc_1", "f_dc_2"]
    hdr = "ply\nformat ascii 1.0\nelement camera 1\nproperty float a\nelement vertex 2\n" + \
          "".join(f"property float {n}\n" for n in names) + "element face 0\nproperty list uchar int vertex_indices\nend_header\n"
    rows = []
    for r in range(2):
        vals = [r, 2 * r, 3 * r] + [100 * r + i for i in range(45)] + [0.5 + r, 7, 8, 9]
        rows.append(" ".join(str(v) for v in vals))
    path = tmp_path / "a.ply"
    path.write_text(hdr + "1.5\n" + "\n".join(rows) + "\n")
    got = gv.SplatSet()
    assert gv.PLYLoader().loadPLYModel(path, got)
    fr = got["f_rest"].reshape(2, 15, 3)
    for r in range(2):
        for i in range(15):
            for c in range(3):
                assert fr[r, i, c] == 100 * r + 15 * c + i
    np.testing.assert_array_equal(got["scale"], 0)      # no scale_* properties -> zeros
    np.testing.assert_array_equal(got["rotation"], 0)
    np.testing.assert_array_equal(got["opacity"], [0.5, 1.5])
    np.testing.assert_array_equal(got["positions"], [0, 0, 0, 1, 2, 3])


def test_ply_missing_file_and_bad_header(gv, tmp_path):
    assert not gv.PLYLoader().loadPLYModel(tmp_path / "nope.ply", gv.SplatSet())
    bad = tmp_path / "bad.ply"
    bad.write_text("not a ply\n")
    assert not gv.PLYLoader().loadPLYModel(bad, gv.SplatSet())
