"""Drop-in `gsplat` package: the gsplat 0.1.2.1 Python API backed by the MI355X (gfx950)
kernels of gaussctrl_exp_amd.

/root/reference/gaussctrl/gc_model.py:32,35,36 imports
    from gsplat.sh import num_sh_bases, spherical_harmonics
    from gsplat.project_gaussians import project_gaussians
    from gsplat.rasterize import rasterize_gaussians
and nerfstudio 1.0.0 splatfacto imports the same names; with this directory on sys.path
those imports resolve here unchanged.
"""
import warnings

import torch

from gaussctrl_exp_amd import __version__
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import rasterize_gaussians
from gaussctrl_exp_amd.sh import spherical_harmonics
from gaussctrl_exp_amd.utils import (bin_and_sort_gaussians, compute_cov2d_bounds,
                                     compute_cumulative_intersects, get_tile_bin_edges,
                                     map_gaussian_to_intersects)

__all__ = [
    "__version__",
    "project_gaussians",
    "rasterize_gaussians",
    "spherical_harmonics",
    # utils
    "bin_and_sort_gaussians",
    "compute_cumulative_intersects",
    "compute_cov2d_bounds",
    "get_tile_bin_edges",
    "map_gaussian_to_intersects",
    # Function classes kept for backwards compatibility (gsplat 0.1.x __init__.py)
    "ProjectGaussians",
    "RasterizeGaussians",
    "BinAndSortGaussians",
    "ComputeCumulativeIntersects",
    "ComputeCov2dBounds",
    "GetTileBinEdges",
    "MapGaussiansToIntersects",
    "SphericalHarmonics",
    "NDRasterizeGaussians",
]


def _deprecated(name, fn):
    class _Deprecated(torch.autograd.Function):
        @staticmethod
        def forward(ctx, *args, **kwargs):
            warnings.warn(f"{name} is deprecated, use {fn.__name__} instead",
                          DeprecationWarning)
            return fn(*args, **kwargs)

        @classmethod
        def apply(cls, *args, **kwargs):
            warnings.warn(f"{name} is deprecated, use {fn.__name__} instead",
                          DeprecationWarning)
            return fn(*args, **kwargs)

    _Deprecated.__name__ = name
    return _Deprecated


MapGaussiansToIntersects = _deprecated("MapGaussiansToIntersects", map_gaussian_to_intersects)
ComputeCumulativeIntersects = _deprecated("ComputeCumulativeIntersects",
                                          compute_cumulative_intersects)
ComputeCov2dBounds = _deprecated("ComputeCov2dBounds", compute_cov2d_bounds)
GetTileBinEdges = _deprecated("GetTileBinEdges", get_tile_bin_edges)
BinAndSortGaussians = _deprecated("BinAndSortGaussians", bin_and_sort_gaussians)
ProjectGaussians = _deprecated("ProjectGaussians", project_gaussians)
RasterizeGaussians = _deprecated("RasterizeGaussians", rasterize_gaussians)
NDRasterizeGaussians = _deprecated("NDRasterizeGaussians", rasterize_gaussians)
SphericalHarmonics = _deprecated("SphericalHarmonics", spherical_harmonics)
