"""The training step's L1 loss folded into the blend kernels (gsplat_rasterize_forward_clearing_l1
/ gsplat_rasterize_backward_records_l1; fused.render_fused(l1_gt=...), TrainStep(loss="l1")).

Against the same step with the separate loss kernels (csrc/loss.hip, lambda = 0, clamp_pred):
the backward forms each pixel's upstream gradient with exactly l1_only_bwd_kernel's arithmetic,
so every parameter gradient -- and the parameters after the in-backward Adam step -- are
bit-identical under deterministic accumulation, and within the atomic summation order's
rounding with the shipped atomic records; the loss value is the same sum in a different order
(per-wave partials instead of grid-stride blocks, both finished in double): within 1e-6
relative.  Frame sizes cover the strip backward (1080x1080: 4,624 tiles, from 3,584 the
shipped geometry, as at the headline), the 8x8-block backward without (1080x720: 3,060 tiles)
and with the list split (512x384), and a ragged frame (333x201)."""
import numpy as np
import pytest
import torch

from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.camera import synthetic_camera
from gaussctrl_exp_amd.scene import synthetic_scene
from gaussctrl_exp_amd.train import TrainStep

pytestmark = pytest.mark.gpu


def _step(gpu, sc, cam, gt, bg, fuse_l1, adam):
    s = sc.to(gpu)
    t = TrainStep(s, sh_degree=3, loss="l1", render_mode="fused")
    t.fuse_l1 = fuse_l1
    if adam:
        loss = t.step(cam, gt, bg)
        return float(loss), [p.detach().cpu().numpy() for p in s.params()]
    t.zero_grad()
    loss, out = t.forward_backward(cam, gt, bg)
    return float(loss), [p.grad.detach().cpu().numpy() for p in s.params()]


@pytest.mark.parametrize("W,H,n", [(1080, 1080, 400_000), (1080, 720, 300_000),
                                   (512, 384, 60_000), (333, 201, 20_000)])
@pytest.mark.parametrize("adam", [False, True])
@pytest.mark.parametrize("det", [True, False])
def test_fused_l1_equals_loss_kernels(gpu, W, H, n, adam, det):
    if adam and not det:
        pytest.skip("the in-backward Adam is compared bit for bit (deterministic) only")
    sc = synthetic_scene(n, 3, seed=23, scale_lo=0.004, scale_hi=0.03)
    cam = synthetic_camera(W, H).to(gpu)
    gt = torch.rand(H, W, 3, generator=torch.Generator().manual_seed(6)).to(gpu)
    gt[: H // 4] = 1.5  # targets above the clamp: the clamp's gradient mask matters
    bg = torch.tensor([0.9, 1.2, 0.3], device=gpu)  # a background above 1 as well
    prev = _lib.set_deterministic(det)
    try:
        l_ref, ref = _step(gpu, sc, cam, gt, bg, False, adam)
        l_got, got = _step(gpu, sc, cam, gt, bg, True, adam)
    finally:
        _lib.set_deterministic(prev)
    assert abs(l_got - l_ref) <= 1e-6 * abs(l_ref), (l_got, l_ref)
    for name, x, y in zip(("means", "scales", "quats", "opacities", "dc", "rest"), got, ref):
        if not adam:
            assert np.abs(y).max() > 0, name
        if det:
            np.testing.assert_array_equal(x, y, err_msg=name)
        else:  # atomic records: the same terms summed in another order
            np.testing.assert_allclose(x, y, rtol=1e-4, atol=1e-5 * np.abs(y).max(),
                                       err_msg=name)


def test_fused_l1_loss_value(gpu):
    """The loss value against torch on the returned image: mean |clamp(img, 1) - gt|."""
    from gaussctrl_exp_amd.fused import render_fused
    sc = synthetic_scene(50_000, 3, seed=3, scale_lo=0.004, scale_hi=0.03).to(gpu)
    cam = synthetic_camera(640, 480).to(gpu)
    gt = torch.rand(480, 640, 3, generator=torch.Generator().manual_seed(1)).to(gpu)
    bg = torch.tensor([0.5, 1.3, 0.1], device=gpu)
    for _ in range(2):  # the second call bins speculatively
        out = render_fused(sc.requires_grad_(), cam, 3, bg, l1_gt=gt)
        ref = (torch.clamp(out["rgb"].double(), max=1.0) - gt.double()).abs().mean()
        assert abs(float(out["loss"]) - float(ref)) <= 1e-6 * float(ref)
        assert out["loss"].requires_grad and not out["rgb"].requires_grad


@pytest.mark.parametrize("loss_kind", ["l1", "splatfacto"])
@pytest.mark.parametrize("W,H,n", [(1080, 1080, 400_000), (512, 384, 60_000)])
def test_direct_step_equals_autograd(gpu, W, H, n, loss_kind):
    """TrainStep's direct fused step (render_fused(direct=True): forward and backward called
    without an autograd graph; with the L1 + SSIM loss its kernels are called directly too,
    loss.fused_splatfacto_loss_and_grad) against the same step through autograd: the same loss
    and, under deterministic accumulation, bit-identical gradients -- also when they accumulate
    into existing .grad (two steps without zero_grad) and with the in-backward Adam step."""
    from gaussctrl_exp_amd import fused
    sc = synthetic_scene(n, 3, seed=21, scale_lo=0.004, scale_hi=0.03)
    cam = synthetic_camera(W, H).to(gpu)
    gt = torch.rand(H, W, 3, generator=torch.Generator().manual_seed(4)).to(gpu)
    bg = torch.tensor([0.1, 0.7, 0.3], device=gpu)
    prev, prev_direct = _lib.set_deterministic(True), fused.DIRECT_STEP
    res = {}
    try:
        for direct in (True, False):
            fused.DIRECT_STEP = direct
            s = sc.to(gpu)
            t = TrainStep(s, sh_degree=3, loss=loss_kind, render_mode="fused")
            t.zero_grad()
            l1, out = t.forward_backward(cam, gt, bg)
            assert (out["backward"] is not None) == direct
            assert l1.requires_grad != direct
            g1 = [p.grad.detach().clone() for p in s.params()]
            l2, _ = t.forward_backward(cam, gt, bg)  # accumulates
            g2 = [p.grad.detach().cpu().numpy() for p in s.params()]
            t2 = TrainStep(sc.to(gpu), sh_degree=3, loss=loss_kind, render_mode="fused")
            for _ in range(2):
                t2.step(cam, gt, bg)
            res[direct] = (float(l1), [g.cpu().numpy() for g in g1], g2,
                           [p.detach().cpu().numpy() for p in t2.params])
            if direct:  # the direct step's backward runs once
                with pytest.raises(RuntimeError, match="already ran"):
                    out["backward"]()
    finally:
        _lib.set_deterministic(prev)
        fused.DIRECT_STEP = prev_direct
    a, b = res[True], res[False]
    assert a[0] == b[0]
    for x, y in zip(a[1] + a[2] + a[3], b[1] + b[2] + b[3]):
        np.testing.assert_array_equal(x, y)
    assert np.abs(a[1][0]).max() > 0
