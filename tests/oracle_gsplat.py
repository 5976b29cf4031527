"""CPU emulation of the gsplat 0.1.2.1 API on the C oracle (test infrastructure only).

Each autograd Function calls oracle/oracle.py, so the SAME caller code
(gaussctrl_exp_amd.scene.render, a restatement of gc_model.get_outputs) runs once on the
MI355X kernels and once here, and the two are compared.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import oracle as O  # noqa: E402

from gaussctrl_exp_amd import exchange  # noqa: E402


def _alpha_max():
    from gaussctrl_exp_amd import quirks
    return quirks.backward_alpha_clamp()


def _np(t):
    return t.detach().cpu().numpy()


class _Project(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means, scales, glob_scale, quats, viewmat, projmat, fx, fy, cx, cy, H, W,
                tile_bounds, clip_thresh=0.01):
        out = O.project_forward(_np(means), _np(scales), glob_scale, _np(quats), _np(viewmat),
                                _np(projmat), fx, fy, cx, cy, H, W, tile_bounds, clip_thresh)
        xys, depths, radii, conics, nth, cov3d = [torch.from_numpy(o) for o in out]
        ctx.args = (glob_scale, fx, fy, cx, cy, H, W)
        ctx.save_for_backward(means, scales, quats, viewmat, projmat, cov3d, radii, conics)
        return xys, depths, radii, conics, nth, cov3d

    @staticmethod
    def backward(ctx, v_xys, v_depths, v_radii, v_conics, v_nth, v_cov3d):
        means, scales, quats, viewmat, projmat, cov3d, radii, conics = ctx.saved_tensors
        glob_scale, fx, fy, cx, cy, H, W = ctx.args
        _, _, v_mean, v_scale, v_quat = O.project_backward(
            _np(means), _np(scales), glob_scale, _np(quats), _np(viewmat), _np(projmat), fx, fy,
            cx, cy, H, W, _np(cov3d), _np(radii), _np(conics), _np(v_xys), _np(v_depths),
            _np(v_conics))
        return (torch.from_numpy(v_mean), torch.from_numpy(v_scale), None,
                torch.from_numpy(v_quat)) + (None,) * 10


def project_gaussians(*args):
    return _Project.apply(*args)


class _SH(torch.autograd.Function):
    @staticmethod
    def forward(ctx, deg, viewdirs, coeffs):
        ctx.deg, ctx.K = deg, coeffs.shape[1]
        ctx.exchange = exchange.active()
        ctx.save_for_backward(viewdirs)
        return torch.from_numpy(O.sh_forward(deg, _np(viewdirs), _np(coeffs)))

    @staticmethod
    def backward(ctx, v):
        (viewdirs,) = ctx.saved_tensors
        if ctx.exchange is not None:  # data-parallel SH-gradient exchange (gloo tests)
            deg, K = ctx.deg, ctx.K
            return None, None, ctx.exchange.reduce(v.contiguous(), lambda means, views: (
                torch.from_numpy(O.sh_backward_views(deg, _np(means), _np(views), K))))
        return None, None, torch.from_numpy(O.sh_backward(ctx.deg, _np(viewdirs), _np(v), ctx.K))


def spherical_harmonics(deg, viewdirs, coeffs):
    return _SH.apply(deg, viewdirs, coeffs)


class _Raster(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xys, depths, radii, conics, nth, colors, opacity, H, W, background,
                return_alpha):
        f = O.render_forward(_np(xys), _np(depths), _np(radii), _np(conics), _np(nth),
                             _np(colors), _np(opacity), H, W, _np(background))
        ctx.f = f
        ctx.opacity_shape = opacity.shape
        ctx.save_for_backward(xys, conics, colors, opacity, background)
        img = torch.from_numpy(f["img"])
        if return_alpha:
            return img, torch.from_numpy(f["alpha"].astype(np.float32))
        return img

    @staticmethod
    def backward(ctx, v_img, v_alpha=None):
        xys, conics, colors, opacity, background = ctx.saved_tensors
        if v_alpha is None:
            v_alpha = torch.zeros_like(v_img[..., 0])
        v_xy, v_conic, v_colors, v_opac = O.render_backward(
            ctx.f, _np(xys), _np(conics), _np(colors), _np(opacity), _np(background),
            _np(v_img), _np(v_alpha), alpha_max=_alpha_max())
        return (torch.from_numpy(v_xy), None, None, torch.from_numpy(v_conic), None,
                torch.from_numpy(v_colors), torch.from_numpy(v_opac).reshape(ctx.opacity_shape),
                None, None, None, None)


def rasterize_gaussians(xys, depths, radii, conics, nth, colors, opacity, H, W,
                        background=None, return_alpha=False):
    if background is None:
        background = torch.ones(colors.shape[-1])
    return _Raster.apply(xys, depths, radii, conics, nth, colors, opacity, H, W, background,
                         return_alpha)


def sh_backward_views(degree, degrees_to_use, means, views):
    K = {0: 1, 1: 4, 2: 9, 3: 16, 4: 25}[degree]
    return torch.from_numpy(O.sh_backward_views(degrees_to_use, _np(means), _np(views), K))


class API:
    sh_backward_views = staticmethod(sh_backward_views)
    project_gaussians = staticmethod(project_gaussians)
    spherical_harmonics = staticmethod(spherical_harmonics)
    rasterize_gaussians = staticmethod(rasterize_gaussians)
