"""Spherical-harmonics colour evaluation (gsplat 0.1.2.1 `gsplat/sh.py`).

Called by /root/reference/gaussctrl/gc_model.py:200 as
`spherical_harmonics(n, viewdirs, colors_crop)`; kernels in csrc/sh.hip.
"""
from __future__ import annotations

import torch
from torch import Tensor
from torch.autograd import Function

from . import _lib, exchange


def num_sh_bases(degree: int) -> int:
    if degree == 0:
        return 1
    if degree == 1:
        return 4
    if degree == 2:
        return 9
    if degree == 3:
        return 16
    return 25


def deg_from_sh(num_bases: int) -> int:
    if num_bases == 1:
        return 0
    if num_bases == 4:
        return 1
    if num_bases == 9:
        return 2
    if num_bases == 16:
        return 3
    if num_bases == 25:
        return 4
    assert False, "Invalid number of SH bases"


def spherical_harmonics(degrees_to_use: int, viewdirs: Tensor, coeffs: Tensor) -> Tensor:
    """Colours [N,3] from SH coefficients [N,K,3] along view directions [N,3].

    Only the first num_sh_bases(degrees_to_use) bases are evaluated; the direction is
    renormalised in the kernel; no gradient flows to viewdirs (as in gsplat 0.1.2.1).
    """
    assert coeffs.shape[-2] >= num_sh_bases(degrees_to_use)
    return _SphericalHarmonics.apply(degrees_to_use, viewdirs.contiguous(), coeffs.contiguous())


class _SphericalHarmonics(Function):
    @staticmethod
    def forward(ctx, degrees_to_use: int, viewdirs: Tensor, coeffs: Tensor):
        num_points = coeffs.shape[0]
        degree = deg_from_sh(coeffs.shape[-2])
        if coeffs.shape[-1] != 3 or viewdirs.shape != (num_points, 3):
            raise ValueError(f"bad shapes: coeffs {tuple(coeffs.shape)}, "
                             f"viewdirs {tuple(viewdirs.shape)}")
        viewdirs = viewdirs.float().contiguous()
        coeffs = coeffs.float().contiguous()
        dev = _lib.check_device("spherical_harmonics", viewdirs, coeffs)
        ctx.degree = degree
        ctx.degrees_to_use = degrees_to_use
        ctx.save_for_backward(viewdirs)
        ctx.exchange = exchange.active()  # data-parallel SH-gradient exchange, if any
        colors = torch.empty((num_points, 3), device=dev, dtype=torch.float32)
        _lib.call("gsplat_compute_sh_forward", num_points, degree, int(degrees_to_use),
                  _lib.ptr(viewdirs), _lib.ptr(coeffs), _lib.ptr(colors), _lib.stream(dev))
        return colors

    @staticmethod
    def backward(ctx, v_colors: Tensor):
        (viewdirs,) = ctx.saved_tensors
        num_points = v_colors.shape[0]
        K = num_sh_bases(ctx.degree)
        dev = viewdirs.device
        v_colors = v_colors.float().contiguous()
        if ctx.exchange is not None:
            degree, dtu = ctx.degree, int(ctx.degrees_to_use)
            return None, None, ctx.exchange.reduce(
                v_colors, lambda means, views: sh_backward_views(degree, dtu, means, views))
        v_coeffs = torch.empty((num_points, K, 3), device=dev, dtype=torch.float32)
        _lib.call("gsplat_compute_sh_backward", num_points, ctx.degree, int(ctx.degrees_to_use),
                  _lib.ptr(viewdirs), _lib.ptr(v_colors), _lib.ptr(v_coeffs), _lib.stream(dev))
        return None, None, v_coeffs


def sh_backward_views(degree: int, degrees_to_use: int, means: Tensor, views: Tensor) -> Tensor:
    """sum_r Y(means - campos_r) (x) v_colors_r over the gathered view records
    views [R, >= 3N + 3] = [v_colors_r (3N) | campos_r (3) | ...]  (exchange.ShViewExchange)."""
    n = means.shape[0]
    means = means.float().contiguous()
    views = views.float().contiguous()
    dev = _lib.check_device("sh_backward_views", means, views)
    K = num_sh_bases(degree)
    v_coeffs = torch.empty((n, K, 3), device=dev, dtype=torch.float32)
    _lib.call("gsplat_compute_sh_backward_views", n, degree, int(degrees_to_use), views.shape[0],
              _lib.ptr(means), _lib.ptr(views), views.shape[1], _lib.ptr(v_coeffs),
              _lib.stream(dev))
    return v_coeffs
