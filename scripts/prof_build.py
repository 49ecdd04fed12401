"""Driver for rocprofv3: builds the bench scene (enclose + accel) N times."""
import importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gv = importlib.import_module("3dgvrt_lightfield_amd")
cfg = os.environ.get("GVRT_CFG", "bicycle")
n = int(os.environ.get("GVRT_N", "5"))
bkw = dict(builder=int(os.environ.get("GVRT_B", "0")), collapse=int(os.environ.get("GVRT_C", "0")))
gen, W, H, _ = gv.scene.CONFIGS[cfg]
s = gv.scene.make(**gen)
with gv.Renderer(0) as r:
    for _ in range(n):
        r.prepare(s, **bkw)
        st = r.stats()
        print("enclose_ms", round(st["enclose_ms"], 3), "accel_ms", round(st["accel_ms"], 3), "nodes", st["bvh_nodes"])
