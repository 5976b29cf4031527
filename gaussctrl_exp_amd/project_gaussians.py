"""Python bindings for 3D Gaussian projection (gsplat 0.1.2.1 `gsplat/project_gaussians.py`).

Same function name, positional signature, outputs, dtypes and autograd behaviour as the
gsplat 0.1.2.1 API that /root/reference/gaussctrl/gc_model.py:174-188 calls; the kernels
are the gfx950 ones in csrc/project.hip reached through the C ABI.
"""
from __future__ import annotations

import threading

from typing import Tuple

import torch
from torch import Tensor
from torch.autograd import Function

from . import _lib
from .ops import ops


def project_gaussians(
    means3d: Tensor,
    scales: Tensor,
    glob_scale: float,
    quats: Tensor,
    viewmat: Tensor,
    projmat: Tensor,
    fx: float,
    fy: float,
    cx: float,
    cy: float,
    img_height: int,
    img_width: int,
    tile_bounds: Tuple[int, int, int],
    clip_thresh: float = 0.01,
) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """Project 3D Gaussians to 2D.

    Args: means3d [N,3], scales [N,3] (already exp'd), glob_scale, quats [N,4] (w,x,y,z),
    viewmat [3,4] or [4,4] world->camera (first 12 row-major floats used), projmat [4,4]
    (= P @ viewmat), fx, fy, cx, cy, img_height, img_width, tile_bounds (tiles_x, tiles_y, 1),
    clip_thresh (near plane).

    Returns (xys [N,2], depths [N], radii [N] int32, conics [N,3], num_tiles_hit [N] int32,
    cov3d [N,6]); culled Gaussians have radii == 0.  Gradients flow to means3d, scales and
    quats (gsplat 0.1.x returns None for viewmat/projmat).
    """
    out = _ProjectGaussians.apply(
        means3d.contiguous(), scales.contiguous(), glob_scale, quats.contiguous(),
        viewmat.contiguous(), projmat.contiguous(), fx, fy, cx, cy, img_height, img_width,
        tile_bounds, clip_thresh)
    ws1 = getattr(_LAST, "ws1", None)
    if ws1 is not None:
        # the binning's depth-sort inputs, written by the projection kernel: the rasterize call
        # on exactly these (unmodified) outputs bins with gsplat_bin_count_keyed
        _LAST.ws1 = None
        from .rasterize import keyed_workspaces
        keyed_workspaces.put((out[0], out[1], out[2], out[4]), int(tile_bounds[0]),
                             int(tile_bounds[1]), ws1)
    return out


_LAST = threading.local()


def _as_f32(t: Tensor) -> Tensor:
    return t if t.dtype == torch.float32 else t.float()


class _ProjectGaussians(Function):
    """Project 3D Gaussians to 2D (autograd wrapper of the C-ABI project kernels)."""

    @staticmethod
    def forward(ctx, means3d, scales, glob_scale, quats, viewmat, projmat, fx, fy, cx, cy,
                img_height, img_width, tile_bounds, clip_thresh=0.01):
        num_points = means3d.shape[-2]
        if num_points < 1 or means3d.shape[-1] != 3:
            raise ValueError(f"Invalid shape for means3d: {means3d.shape}")
        means3d, scales, quats = _as_f32(means3d), _as_f32(scales), _as_f32(quats)
        viewmat, projmat = _as_f32(viewmat).contiguous(), _as_f32(projmat).contiguous()
        if viewmat.numel() < 12 or projmat.numel() != 16:
            raise ValueError("viewmat must hold >= 12 floats ([3,4] or [4,4]), projmat [4,4]")
        dev = _lib.check_device("project_gaussians", means3d, scales, quats, viewmat, projmat)
        n = num_points
        cov3d = torch.empty((n, 6), device=dev, dtype=torch.float32)
        xys = torch.empty((n, 2), device=dev, dtype=torch.float32)
        depths = torch.empty((n,), device=dev, dtype=torch.float32)
        radii = torch.empty((n,), device=dev, dtype=torch.int32)
        conics = torch.empty((n, 3), device=dev, dtype=torch.float32)
        num_tiles_hit = torch.empty((n,), device=dev, dtype=torch.int32)
        P = _lib.ptr
        ws1 = torch.empty((_lib.query("gsplat_bin_count_workspace_size", n),), device=dev,
                          dtype=torch.uint8)
        _lib.call("gsplat_project_gaussians_forward_binned", n, P(means3d), P(scales),
                  float(glob_scale), P(quats), P(viewmat), P(projmat), float(fx), float(fy),
                  float(cx), float(cy), int(img_height), int(img_width), int(tile_bounds[0]),
                  int(tile_bounds[1]), float(clip_thresh), P(cov3d), P(xys), P(depths),
                  P(radii), P(conics), P(num_tiles_hit), P(ws1), ws1.numel(), _lib.stream(dev))
        _LAST.ws1 = ws1
        ctx.img_height = img_height
        ctx.img_width = img_width
        ctx.num_points = num_points
        ctx.glob_scale = glob_scale
        ctx.fx, ctx.fy, ctx.cx, ctx.cy = fx, fy, cx, cy
        ctx.save_for_backward(means3d, scales, quats, viewmat, projmat, cov3d, radii, conics)
        ctx.mark_non_differentiable(radii, num_tiles_hit)
        # Outputs nothing consumed (depths, cov3d in the splatfacto caller) reach backward as
        # None instead of autograd-materialised zero tensors (one fill kernel each).
        ctx.set_materialize_grads(False)
        return (xys, depths, radii, conics, num_tiles_hit, cov3d)

    @staticmethod
    def backward(ctx, v_xys, v_depths, v_radii, v_conics, v_num_tiles_hit, v_cov3d):
        means3d, scales, quats, viewmat, projmat, cov3d, radii, conics = ctx.saved_tensors
        n = ctx.num_points
        dev = means3d.device
        v_xys = _as_f32(v_xys).contiguous() if v_xys is not None else \
            torch.zeros((n, 2), device=dev, dtype=torch.float32)
        v_conics = _as_f32(v_conics).contiguous() if v_conics is not None else \
            torch.zeros((n, 3), device=dev, dtype=torch.float32)
        if v_depths is not None:  # NULL = zero depth gradient
            v_depths = _as_f32(v_depths).contiguous()
        v_mean3d, v_scale, v_quat = ops().project_bwd(
            means3d, scales, float(ctx.glob_scale), quats, viewmat, projmat, float(ctx.fx),
            float(ctx.fy), float(ctx.cx), float(ctx.cy), int(ctx.img_height),
            int(ctx.img_width), cov3d, radii, conics, v_xys, v_depths, v_conics)
        # one gradient per input of forward (gsplat 0.1.2.1 returns None for the rest)
        return (v_mean3d, v_scale, None, v_quat, None, None, None, None, None, None, None,
                None, None, None)
