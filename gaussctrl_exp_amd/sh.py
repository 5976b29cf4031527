"""Spherical-harmonics colour evaluation (gsplat 0.1.2.1 `gsplat/sh.py`).

Called by /root/reference/gaussctrl/gc_model.py:200 as
`spherical_harmonics(n, viewdirs, colors_crop)`; kernels in csrc/sh.hip.
"""
from __future__ import annotations

import os

import torch
from torch import Tensor
from torch.autograd import Function

from . import _lib, exchange
from .ops import ops


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

    When `coeffs` is the caller's cat((features_dc[:, None], features_rest), 1) of two leaf
    parameters -- gc_model.py:172 and splatfacto -- the gradient goes straight to those two
    parameters as contiguous tensors (gsplat_compute_sh_backward_split) instead of through
    cat's backward, whose strided views cost AccumulateGrad two full layout copies (~100 us
    per step at 1M Gaussians).  Values are identical; only coeffs itself sees no gradient
    (it is an intermediate nobody reads).  GSPLAT_MI355X_SH_CAT_BYPASS=0 turns this off.
    """
    assert coeffs.shape[-2] >= num_sh_bases(degrees_to_use)
    leaves = _cat_leaves(coeffs) if _CAT_BYPASS and torch.is_grad_enabled() else None
    if leaves is not None:
        return _SphericalHarmonicsSplit.apply(degrees_to_use, viewdirs.contiguous(),
                                              coeffs.detach().contiguous(), *leaves)
    return _SphericalHarmonics.apply(degrees_to_use, viewdirs.contiguous(), coeffs.contiguous())


_CAT_BYPASS = os.environ.get("GSPLAT_MI355X_SH_CAT_BYPASS", "1") != "0"


def _cat_leaves(coeffs: Tensor):
    """(features_dc, features_rest) when coeffs = cat((dc[:, None, :], rest), dim=1) of two fp32
    contiguous leaf tensors that require grad (the autograd graph shows CatBackward0 over
    UnsqueezeBackward0(1) of dc's AccumulateGrad and rest's AccumulateGrad); else None."""
    fn = coeffs.grad_fn
    if fn is None or type(fn).__name__ != "CatBackward0":
        return None
    if getattr(fn, "_saved_dim", None) not in (1, -2) or len(fn.next_functions) != 2:
        return None
    (f0, _), (f1, _) = fn.next_functions
    if f0 is None or f1 is None or type(f0).__name__ != "UnsqueezeBackward0" or \
            getattr(f0, "_saved_dim", None) not in (1, -2) or len(f0.next_functions) != 1:
        return None
    a0 = f0.next_functions[0][0]
    if a0 is None or type(a0).__name__ != "AccumulateGrad" or \
            type(f1).__name__ != "AccumulateGrad":
        return None
    dc, rest = a0.variable, f1.variable
    n, K = coeffs.shape[0], coeffs.shape[1]
    ok = (dc.shape == (n, 3) and rest.shape == (n, K - 1, 3) and coeffs.shape[2] == 3 and
          all(t.dtype == torch.float32 and t.is_contiguous() and t.requires_grad and
              t.device == coeffs.device for t in (dc, rest)))
    return (dc, rest) if ok else None


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
        _lib.check_device("spherical_harmonics", viewdirs, coeffs)
        ctx.degree = degree
        ctx.degrees_to_use = degrees_to_use
        ctx.save_for_backward(viewdirs)
        ctx.exchange = exchange.active()  # data-parallel SH-gradient exchange, if any
        return ops().sh_fwd(degree, int(degrees_to_use), viewdirs, coeffs)

    @staticmethod
    def backward(ctx, v_colors: Tensor):
        (viewdirs,) = ctx.saved_tensors
        v_colors = v_colors.float().contiguous()
        if ctx.exchange is not None:
            degree, dtu = ctx.degree, int(ctx.degrees_to_use)
            return None, None, ctx.exchange.reduce(
                v_colors, lambda means, views: sh_backward_views(degree, dtu, means, views))
        return None, None, ops().sh_bwd(ctx.degree, int(ctx.degrees_to_use), viewdirs, v_colors)


class _SphericalHarmonicsSplit(Function):
    """_SphericalHarmonics whose coefficient gradient goes to (features_dc, features_rest)."""

    @staticmethod
    def forward(ctx, degrees_to_use: int, viewdirs: Tensor, coeffs: Tensor, features_dc: Tensor,
                features_rest: Tensor):
        colors = _SphericalHarmonics.forward(ctx, degrees_to_use, viewdirs, coeffs)
        return colors

    @staticmethod
    def backward(ctx, v_colors: Tensor):
        (viewdirs,) = ctx.saved_tensors
        n = v_colors.shape[0]
        K = num_sh_bases(ctx.degree)
        dev = viewdirs.device
        v_colors = v_colors.float().contiguous()
        if ctx.exchange is not None:
            from .fused import sh_backward_views_split
            degree, dtu = ctx.degree, int(ctx.degrees_to_use)
            v_dc, v_rest = ctx.exchange.reduce(
                v_colors, lambda means, views: sh_backward_views_split(degree, dtu, means, views))
            return None, None, None, v_dc, v_rest
        v_dc = torch.empty((n, 3), device=dev, dtype=torch.float32)
        v_rest = torch.empty((n, K - 1, 3), device=dev, dtype=torch.float32)
        _lib.call("gsplat_compute_sh_backward_split", n, ctx.degree, int(ctx.degrees_to_use),
                  _lib.ptr(viewdirs), _lib.ptr(v_colors), _lib.ptr(v_dc),
                  _lib.ptr(v_rest) if K > 1 else None, _lib.stream(dev))
        return None, None, None, v_dc, v_rest


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
