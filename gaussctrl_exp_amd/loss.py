"""Fused splatfacto photometric loss on MI355X.

nerfstudio 1.0 splatfacto's get_loss_dict (reached from the reference's training step,
/root/reference/gaussctrl/gc_pipeline.py:477-478) computes

    main_loss = (1 - ssim_lambda) * |gt - pred|.mean()
                + ssim_lambda * (1 - SSIM(gt.permute(2,0,1)[None], pred.permute(2,0,1)[None]))

with pytorch_msssim's SSIM (11x11 Gaussian window sigma 1.5, 'valid' filtering, data range 1,
K = (0.01, 0.03)).  `fused_splatfacto_loss` evaluates it with two HIP kernels (csrc/loss.hip)
instead of ~20 torch ops and 10 MIOpen convolutions; gradients flow to `pred` only.  The torch
restatement it is tested against is train.splatfacto_loss.
"""
from __future__ import annotations

import ctypes

import torch
from torch import Tensor
from torch.autograd import Function

from . import _lib

SSIM_WIN, SSIM_SIGMA = 11, 1.5


def _window_host():
    coords = torch.arange(SSIM_WIN, dtype=torch.float32) - SSIM_WIN // 2
    g = torch.exp(-(coords ** 2) / (2 * SSIM_SIGMA ** 2))
    g = g / g.sum()
    return (ctypes.c_float * SSIM_WIN)(*g.tolist())


_WINDOW = _window_host()


class _FusedL1SSIM(Function):
    @staticmethod
    def forward(ctx, pred: Tensor, gt: Tensor, ssim_lambda: float, clamp_pred: bool = False):
        if pred.dim() != 3 or pred.shape != gt.shape:
            raise ValueError("fused_splatfacto_loss: pred and gt must both be [H, W, C]")
        pred = pred.float().contiguous()
        gt = gt.float().contiguous()
        dev = _lib.check_device("fused_splatfacto_loss", pred, gt)
        H, W, C = pred.shape
        nb = _lib.lib().gsplat_l1_ssim_num_blocks(H, W)
        partials = torch.empty((max(2 * nb, 1),), device=dev, dtype=torch.float32)
        n_maps = 3 * C * max(H - SSIM_WIN + 1, 0) * max(W - SSIM_WIN + 1, 0)
        dmaps = torch.empty((n_maps if ssim_lambda != 0 else 1,), device=dev,
                            dtype=torch.float32)  # (lambda 0: L1 only, no SSIM maps)
        loss = torch.empty((), device=dev, dtype=torch.float32)
        P = _lib.ptr
        _lib.call("gsplat_l1_ssim_forward", H, W, C, P(pred), P(gt), ctypes.cast(_WINDOW,
                  ctypes.c_void_p), float(ssim_lambda), int(bool(clamp_pred)), P(partials),
                  P(dmaps), P(loss), _lib.stream(dev))
        ctx.save_for_backward(pred, gt, dmaps)
        ctx.ssim_lambda = float(ssim_lambda)
        ctx.clamp_pred = int(bool(clamp_pred))
        return loss

    @staticmethod
    def backward(ctx, grad_loss):
        pred, gt, dmaps = ctx.saved_tensors
        H, W, C = pred.shape
        g = grad_loss.float().contiguous()
        v_pred = torch.empty_like(pred)
        P = _lib.ptr
        _lib.call("gsplat_l1_ssim_backward", H, W, C, P(pred), P(gt), ctypes.cast(_WINDOW,
                  ctypes.c_void_p), ctx.ssim_lambda, ctx.clamp_pred, P(dmaps), P(g), P(v_pred),
                  _lib.stream(pred.device))
        return v_pred, None, None, None


def fused_splatfacto_loss(pred: Tensor, gt: Tensor, ssim_lambda: float = 0.2,
                          clamp_pred: bool = False) -> Tensor:
    """(1 - ssim_lambda) * L1 + ssim_lambda * (1 - SSIM) on [H, W, C] images, on the GPU.
    clamp_pred: the loss of torch.clamp(pred, max=1.0) (gc_model.py:222) without materialising
    the clamped image (its forward and backward kernels fold into the loss kernels)."""
    return _FusedL1SSIM.apply(pred, gt, ssim_lambda, clamp_pred)


def fused_splatfacto_loss_and_grad(pred: Tensor, gt: Tensor, ssim_lambda: float = 0.2,
                                   clamp_pred: bool = False):
    """(loss, d loss / d pred) of fused_splatfacto_loss in one call, without an autograd graph
    (the direct training step, fused.render_fused(direct=True)): the same two kernels, the
    backward of a unit loss gradient."""
    from .fused import _DirectCtx, _unit_grad
    ctx = _DirectCtx((True, False, False, False))
    with torch.no_grad():
        loss = _FusedL1SSIM.forward(ctx, pred, gt, ssim_lambda, clamp_pred)
        v_pred = _FusedL1SSIM.backward(ctx, _unit_grad(loss.device))[0]
    return loss, v_pred
