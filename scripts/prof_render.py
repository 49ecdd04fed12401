"""Minimal driver for rocprofv3: builds the bench scene and renders the bench view N times."""
import importlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gv = importlib.import_module("3dgvrt_lightfield_amd")
cfg = os.environ.get("GVRT_CFG", "bicycle")
n = int(os.environ.get("GVRT_N", "5"))
k = int(os.environ.get("GVRT_K", "0"))
gen, W, H, _ = gv.scene.CONFIGS[cfg]
s = gv.scene.make(**gen)
vi, pi = (gv.scene.mipnerf_camera(W, H) if cfg != "config1" else gv.scene.config1_camera(W, H))
opts = [kv.split("=") for kv in os.environ.get("GVRT_OPTS", "").split(",") if kv]
with gv.Renderer(0) as r:
    for name, val in opts:  # per-handle options (same-binary A/B), e.g. GVRT_OPTS=compact_nodes=1
        r.set_option(name, int(val))
    # the bench's default quality build (GVRT_BUILD=fast: device LBVH)
    r.prepare(s, **({} if os.environ.get("GVRT_BUILD") == "fast" else dict(gv.QUALITY_BUILD)))
    for _ in range(n):
        r.render(vi, pi, W, H, kbuffer_depth=k, rgba8=False, rgba32f=False)
    print("render_ms", r.stats()["render_ms"])
