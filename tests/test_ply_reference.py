"""Row 1 parity, pinned on the reference itself: gvrt_ply_load vs the reference's own
vk3DGRT::PLYLoader::loadPLYModel (base/Vulkan3DGRTModel.cpp:7-125 + vendored miniply), built from
its sources by oracle/ref.mk into oracle/_ref/ref_ply_dump (test infrastructure only)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DUMP = os.path.join(ROOT, "oracle", "_ref", "ref_ply_dump")
KEYS = (("positions", 3), ("f_dc", 3), ("f_rest", 45), ("opacity", 1), ("scale", 3), ("rotation", 4))

pytestmark = pytest.mark.skipif(not os.path.exists(DUMP), reason="oracle/_ref not built (needs /root/reference)")


def ref_load(path, tmp_path):
    out = tmp_path / "dump.bin"
    r = subprocess.run([DUMP, str(path), str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = out.read_bytes()
    n = int(np.frombuffer(raw[:8], np.uint64)[0])
    arr = np.frombuffer(raw[8:], np.float32)
    res, off = {}, 0
    for k, m in KEYS:
        res[k] = arr[off: off + m * n]
        off += m * n
    return res


def ours(gv, path):
    s = gv.SplatSet()
    assert gv.PLYLoader().loadPLYModel(path, s)
    return s


def check_same(gv, path, tmp_path):
    a, b = ours(gv, path), ref_load(path, tmp_path)
    for k, _ in KEYS:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_binary_3dgs_ply(gv, tmp_path):
    s = gv.scene.config1(n=500, seed=9)
    p = tmp_path / "b.ply"
    gv.save_ply(p, s)
    check_same(gv, p, tmp_path)


def test_ascii_extra_elements_and_missing_groups(gv, tmp_path):
    names = ["x", "y", "z"] + [f"f_rest_{i}" for i in range(45)] + ["opacity", "f_dc_0", "f_dc_1", "f_dc_2"]
    hdr = "ply\nformat ascii 1.0\nelement camera 1\nproperty float a\nelement vertex 3\n" + \
          "".join(f"property float {n}\n" for n in names) + "end_header\n"
    rows = [" ".join(str(100 * r + i * 0.5) for i in range(len(names))) for r in range(3)]
    p = tmp_path / "a.ply"
    p.write_text(hdr + "1.5\n" + "\n".join(rows) + "\n")
    check_same(gv, p, tmp_path)


def test_double_and_reordered_properties(gv, tmp_path):
    rng = np.random.default_rng(3)
    names = ["rot_3", "rot_2", "rot_1", "rot_0", "opacity", "z", "y", "x", "scale_2", "scale_1", "scale_0",
             "f_dc_2", "f_dc_1", "f_dc_0"] + [f"f_rest_{i}" for i in reversed(range(45))]
    n = 7
    vals = rng.normal(size=(n, len(names)))
    hdr = "ply\nformat binary_little_endian 1.0\nelement vertex %d\n" % n + \
          "".join(f"property double {nm}\n" for nm in names) + "end_header\n"
    p = tmp_path / "d.ply"
    p.write_bytes(hdr.encode() + vals.astype("<f8").tobytes())
    check_same(gv, p, tmp_path)
