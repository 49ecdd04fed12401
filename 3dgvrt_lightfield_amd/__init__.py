"""MI355X-native Gaussian ray tracer: the Particle Rendering hot path of wlckslxh/3DGVRT_lightfield.

Compute lives in libgvrt.so (hand-written HIP for gfx950 behind include/gvrt.h); this package
is the host-side mirror of the reference's loader / camera / renderer interfaces.  Import as
`importlib.import_module("3dgvrt_lightfield_amd")` (the directory name starts with a digit).
"""
try:  # torch first, so one HIP runtime serves both torch and libgvrt.so in one process
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C-ABI path
    torch = None

from . import camera, scene  # noqa: E402
from ._lib import GvrtError, LIB_PATH, MODE_FAST, MODE_LITERAL, lib  # noqa: E402
from .renderer import (QUALITY_BUILD, PLYLoader, Renderer, SplatSet, device_count, device_properties, psnr_rgb, quantize_rgba8,  # noqa: E402
                       save_ply, tiles_for_rank)

__all__ = ["camera", "scene", "GvrtError", "LIB_PATH", "MODE_FAST", "MODE_LITERAL", "lib", "QUALITY_BUILD", "PLYLoader",
           "Renderer", "SplatSet", "device_count", "device_properties", "psnr_rgb", "quantize_rgba8", "save_ply", "tiles_for_rank"]
