"""Binning utilities (gsplat 0.1.2.1 `gsplat/utils.py`), on the gfx950 kernels.

These expose the gsplat-layout intermediate tensors (64-bit isect_ids etc.) for callers
and tests; `rasterize_gaussians` itself uses the fused path in csrc/binning.hip.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib
from .ops import ops


def _bits_for(v: int) -> int:
    b = 0
    while (1 << b) <= v:
        b += 1
    return b


def map_gaussian_to_intersects(num_points: int, num_intersects: int, xys: Tensor,
                               depths: Tensor, radii: Tensor, cum_tiles_hit: Tensor,
                               tile_bounds: Tuple[int, int, int]) -> Tuple[Tensor, Tensor]:
    """(isect_ids [I] int64 = tile_id << 32 | depth bits, gaussian_ids [I] int32)."""
    xys, depths = xys.float().contiguous(), depths.float().contiguous()
    radii = radii.to(torch.int32).contiguous()
    cum_tiles_hit = cum_tiles_hit.to(torch.int32).contiguous()
    _lib.check_device("map_gaussian_to_intersects", xys, depths, radii, cum_tiles_hit)
    n = int(num_points)  # gsplat reads the first num_points entries
    if xys.shape[0] < n:
        raise ValueError("map_gaussian_to_intersects: num_points > xys.shape[0]")
    xys, depths, radii, cum_tiles_hit = xys[:n], depths[:n], radii[:n], cum_tiles_hit[:n]
    return ops().map_intersects(xys, depths, radii, cum_tiles_hit, int(tile_bounds[0]),
                                int(tile_bounds[1]), int(num_intersects))


def get_tile_bin_edges(num_intersects: int, isect_ids_sorted: Tensor,
                       tile_bounds: Optional[Tuple[int, int, int]] = None) -> Tensor:
    """tile_bins [rows, 2] int32 with [start, end) of each tile in the sorted list.

    gsplat 0.1.2.1 sizes the table by num_intersects (its signature has no tile count), and
    writes out of bounds when a tile id >= num_intersects.  Here rows = num_intersects by
    default with such writes dropped, or max(num_intersects, tiles) when tile_bounds is
    given."""
    rows = int(num_intersects)
    if tile_bounds is not None:
        rows = max(rows, int(tile_bounds[0]) * int(tile_bounds[1]))
    isect_ids_sorted = isect_ids_sorted.contiguous()
    _lib.check_device("get_tile_bin_edges", isect_ids_sorted)
    if isect_ids_sorted.numel() < int(num_intersects):
        raise ValueError("get_tile_bin_edges: num_intersects > isect_ids_sorted.numel()")
    return ops().tile_bins(isect_ids_sorted[:int(num_intersects)], rows)


def compute_cov2d_bounds(cov2d: Tensor) -> Tuple[Tensor, Tensor]:
    """(conics [N,3], radii [N,1] float) from upper-triangular 2D covariances [N,3]."""
    num_pts = cov2d.shape[0]
    assert num_pts > 0
    cov2d = cov2d.float().contiguous()
    dev = _lib.check_device("compute_cov2d_bounds", cov2d)
    conics = torch.empty((num_pts, 3), device=dev, dtype=torch.float32)
    radii = torch.empty((num_pts, 1), device=dev, dtype=torch.float32)
    _lib.call("gsplat_compute_cov2d_bounds", num_pts, _lib.ptr(cov2d), _lib.ptr(conics),
              _lib.ptr(radii), _lib.stream(dev))
    return conics, radii


def compute_cumulative_intersects(num_tiles_hit: Tensor) -> Tuple[int, Tensor]:
    """(num_intersects, inclusive int32 cumsum of num_tiles_hit)."""
    cum_tiles_hit = torch.cumsum(num_tiles_hit, dim=0, dtype=torch.int32)
    num_intersects = cum_tiles_hit[-1].item()
    return num_intersects, cum_tiles_hit


def sort_isect_pairs(isect_ids: Tensor, gaussian_ids: Tensor,
                     key_bits: int = 64) -> Tuple[Tensor, Tensor]:
    """Stable on-device LSD radix sort of (isect_ids, gaussian_ids) by isect_ids.

    Replaces `torch.sort(isect_ids)` + `torch.gather` of utils.bin_and_sort_gaussians; the
    order of equal keys is the input order (torch.sort gives no such guarantee)."""
    isect_ids = isect_ids.contiguous()
    gaussian_ids = gaussian_ids.to(torch.int32).contiguous()
    _lib.check_device("sort_isect_pairs", isect_ids, gaussian_ids)
    return ops().sort_pairs(isect_ids, gaussian_ids, int(key_bits))


def bin_and_sort_gaussians(num_points: int, num_intersects: int, xys: Tensor, depths: Tensor,
                           radii: Tensor, cum_tiles_hit: Tensor,
                           tile_bounds: Tuple[int, int, int]):
    """(isect_ids, gaussian_ids, isect_ids_sorted, gaussian_ids_sorted, tile_bins).

    tile_bins has max(num_intersects, tiles) rows (gsplat 0.1.2.1: num_intersects rows)."""
    isect_ids, gaussian_ids = map_gaussian_to_intersects(
        num_points, num_intersects, xys, depths, radii, cum_tiles_hit, tile_bounds)
    T = int(tile_bounds[0]) * int(tile_bounds[1])
    isect_ids_sorted, gaussian_ids_sorted = sort_isect_pairs(isect_ids, gaussian_ids,
                                                             32 + _bits_for(T))
    tile_bins = get_tile_bin_edges(num_intersects, isect_ids_sorted, tile_bounds)
    return isect_ids, gaussian_ids, isect_ids_sorted, gaussian_ids_sorted, tile_bins
