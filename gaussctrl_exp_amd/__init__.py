"""gaussctrl_exp_amd -- MI355X-native (gfx950) differentiable 3D Gaussian splatting
rasterizer behind the gsplat 0.1.2.1 Python API that Ubinya/gaussctrl_exp's
gaussctrl/gc_model.py calls.

Layout:
  csrc/                 hand-written HIP kernels + C ABI (include/gsplat_mi355x.h)
  _lib.py               ctypes binding (no CPU fallback)
  project_gaussians.py  sh.py  rasterize.py  utils.py   gsplat 0.1.2.1 surface
  camera.py             gc_model.py camera conventions (viewmat flip, projmat, tiles)
  scene.py              synthetic scenes + the gc_model render restatement
  formats.py            transforms.json / sparse_pc.ply / splatfacto ckpt loaders
  train.py              multi-view data-parallel train step (fused loss, fused Adam)
  exchange.py           data-parallel SH-gradient view exchange (RCCL all-gather)
  loss.py  optim.py     fused L1+SSIM loss, fused multi-tensor Adam
  quirks.py             the gsplat 0.1.2.1 [VERIFY] behaviour switch (GSPLAT_MI355X_QUIRKS)
  set_deterministic     bit-reproducible rasterize backward (GSPLAT_MI355X_DETERMINISTIC=1)

`import gsplat` (the top-level shim package) resolves to this implementation.
"""
from . import quirks
from ._lib import set_deterministic
from .project_gaussians import project_gaussians
from .rasterize import rasterize_gaussians, rasterize_gaussians_rgbd
from .sh import num_sh_bases, spherical_harmonics
from .utils import (bin_and_sort_gaussians, compute_cov2d_bounds,
                    compute_cumulative_intersects, get_tile_bin_edges,
                    map_gaussian_to_intersects)

__version__ = "0.1.2.1+mi355x"

__all__ = [
    "project_gaussians",
    "rasterize_gaussians",
    "rasterize_gaussians_rgbd",
    "spherical_harmonics",
    "num_sh_bases",
    "map_gaussian_to_intersects",
    "bin_and_sort_gaussians",
    "compute_cumulative_intersects",
    "compute_cov2d_bounds",
    "get_tile_bin_edges",
    "quirks",
    "set_deterministic",
]
