"""Fused L1 + SSIM loss kernel (csrc/loss.hip) vs the torch restatement of
splatfacto's loss (train.splatfacto_loss, pytorch_msssim semantics) evaluated in float64.

Bar: loss within 2e-6 absolute; d loss / d pred per element within 1e-4 of the largest
reference gradient magnitude (fp32 evaluation of E[y^2] - mu^2 style statistics cancels;
the float64 reference is exact to ~1e-12)."""
import pytest
import torch

from gaussctrl_exp_amd.loss import fused_splatfacto_loss
from gaussctrl_exp_amd.train import splatfacto_loss

@pytest.mark.gpu
@pytest.mark.parametrize("H,W,C,seed", [(11, 11, 3, 0), (48, 64, 3, 1), (75, 100, 3, 2),
                                         (128, 96, 1, 3), (33, 17, 4, 4), (270, 481, 3, 5)])
def test_fused_loss_matches_torch(gpu, H, W, C, seed):
    g = torch.Generator().manual_seed(seed)
    gt = torch.rand(H, W, C, generator=g)
    pred = (gt + 0.15 * torch.randn(H, W, C, generator=g)).clamp(0, 1)
    p = pred.to(gpu).requires_grad_()
    loss = fused_splatfacto_loss(p, gt.to(gpu), 0.2)
    loss.backward()
    p64 = pred.double().requires_grad_()
    ref = splatfacto_loss(p64, gt.double())
    ref.backward()
    assert abs(loss.item() - ref.item()) <= 2e-6, (loss.item(), ref.item())
    err = (p.grad.double().cpu() - p64.grad).abs().max().item()
    scale = p64.grad.abs().max().item()
    assert err <= 1e-4 * scale, (err, scale)


@pytest.mark.gpu
def test_fused_loss_upstream_gradient_scales(gpu):
    g = torch.Generator().manual_seed(7)
    gt = torch.rand(40, 40, 3, generator=g).to(gpu)
    pred = torch.rand(40, 40, 3, generator=g).to(gpu)
    p1 = pred.clone().requires_grad_()
    fused_splatfacto_loss(p1, gt).backward()
    p2 = pred.clone().requires_grad_()
    (3.5 * fused_splatfacto_loss(p2, gt)).backward()
    ref = 3.5 * p1.grad
    assert (p2.grad - ref).abs().max().item() <= 1e-6 * ref.abs().max().item()


def test_fused_loss_has_no_cpu_path():
    """CPU tensors raise instead of silently running a torch fallback."""
    with pytest.raises(RuntimeError, match="no CPU path"):
        fused_splatfacto_loss(torch.rand(20, 20, 3), torch.rand(20, 20, 3))


@pytest.mark.gpu
def test_l1_only_unaligned_inputs(gpu):
    """The L1-only kernels' scalar path (inputs not 16-byte aligned: views at an odd offset)
    gives the same loss and gradient as the aligned 16-byte-vector path."""
    g = torch.Generator().manual_seed(7)
    full_p = torch.rand(33 * 17 * 3 + 1, generator=g).to(gpu)
    full_g = torch.rand(33 * 17 * 3 + 1, generator=g).to(gpu)
    outs = []
    for off in (1, None):
        if off:
            p0, g0 = full_p[off:].view(33, 17, 3), full_g[off:].view(33, 17, 3)
        else:
            p0, g0 = full_p[1:].clone().view(33, 17, 3), full_g[1:].clone().view(33, 17, 3)
        p = p0.detach().requires_grad_()
        loss = fused_splatfacto_loss(p, g0, 0.0)
        loss.backward()
        outs.append((loss.item(), p.grad.clone()))
    assert abs(outs[0][0] - outs[1][0]) <= 1e-6 * max(1.0, outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.gpu
def test_fused_loss_rejects_small_images(gpu):
    with pytest.raises(RuntimeError, match="H, W >= 11"):
        fused_splatfacto_loss(torch.rand(10, 20, 3, device=gpu), torch.rand(10, 20, 3, device=gpu))


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,C", [(48, 64, 3), (5, 7, 3), (1080, 1080, 3)])
def test_l1_only_fast_path(gpu, H, W, C):
    """ssim_lambda = 0 takes the L1-only kernels (any image size): loss and gradient equal
    torch's |gt - pred|.mean() (gradient sign(pred - gt) / n, sign(0) = 0)."""
    g = torch.Generator().manual_seed(H)
    gt = torch.rand(H, W, C, generator=g)
    pred = gt.clone()
    pred[: H // 2] += 0.1 * torch.randn(H // 2, W, C, generator=g)  # exact ties elsewhere
    p = pred.to(gpu).requires_grad_()
    loss = fused_splatfacto_loss(p, gt.to(gpu), 0.0)
    loss.backward()
    p64 = pred.double().requires_grad_()
    ref = torch.abs(gt.double() - p64).mean()
    ref.backward()
    assert abs(loss.item() - ref.item()) <= 1e-6 * max(1.0, ref.item())
    torch.testing.assert_close(p.grad.double().cpu(), p64.grad, rtol=1e-6, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("lam", [0.2, 0.0])
@pytest.mark.parametrize("H,W,C,seed", [(48, 64, 3, 1), (270, 481, 3, 5)])
def test_fused_loss_with_folded_clamp(gpu, lam, H, W, C, seed):
    """clamp_pred=True == the loss of torch.clamp(pred, max=1.0) (gc_model.py:222), gradient
    masked exactly where torch's clamp backward masks it (pred > 1)."""
    g = torch.Generator().manual_seed(seed)
    gt = torch.rand(H, W, C, generator=g)
    pred = gt + 0.4 * torch.randn(H, W, C, generator=g)  # ~30 % of values above 1
    pred[0, 0, 0] = 1.0                                   # the boundary passes the gradient
    p = pred.to(gpu).requires_grad_()
    loss = fused_splatfacto_loss(p, gt.to(gpu), lam, clamp_pred=True)
    loss.backward()
    p64 = pred.double().requires_grad_()
    c64 = torch.clamp(p64, max=1.0)
    ref = splatfacto_loss(c64, gt.double()) if lam else torch.abs(gt.double() - c64).mean()
    ref.backward()
    assert abs(loss.item() - ref.item()) <= 2e-6, (loss.item(), ref.item())
    err = (p.grad.double().cpu() - p64.grad).abs().max().item()
    scale = p64.grad.abs().max().item()
    assert err <= 1e-4 * scale, (err, scale)
    assert not p.grad.cpu()[pred > 1].any()
