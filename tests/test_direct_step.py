"""Host logic of the direct fused training step (fused.render_fused(direct=True), which calls
_FusedRender.forward / backward without an autograd graph).  The numerics -- bit-identical
gradients against the autograd step -- are tests/test_gpu_fused_l1.py's
test_direct_step_equals_autograd; these CPU tests cover when the step is taken and the
context object the static methods share."""
import pytest
import torch

from gaussctrl_exp_amd import fused
from gaussctrl_exp_amd.scene import synthetic_scene


def test_direct_step_ok_needs_contiguous_fp32_leaves(monkeypatch):
    monkeypatch.setattr(fused, "DIRECT_STEP", True)
    sc = synthetic_scene(64, 3, seed=1).requires_grad_()
    assert fused.direct_step_ok(sc)
    monkeypatch.setattr(fused, "DIRECT_STEP", False)  # GSPLAT_MI355X_DIRECT_STEP=0
    assert not fused.direct_step_ok(sc)
    monkeypatch.setattr(fused, "DIRECT_STEP", True)
    # a non-contiguous parameter: the kernels would read a copy, whose gradient only autograd
    # can route back
    q = sc.quats
    sc.quats = torch.nn.Parameter(q.detach().t().contiguous().t())
    assert not sc.quats.is_contiguous()
    assert not fused.direct_step_ok(sc)
    sc.quats = q
    # a non-leaf (e.g. a view of a larger parameter)
    m = sc.means
    sc.means = sc.means * 1.0
    assert not fused.direct_step_ok(sc)
    sc.means = m
    # gradient hooks a caller registered: autograd runs them, the direct step would not
    assert fused.direct_step_ok(sc)
    h = sc.scales.register_hook(lambda g: g)
    assert not fused.direct_step_ok(sc)
    h.remove()
    assert fused.direct_step_ok(sc)
    h = sc.opacities.register_post_accumulate_grad_hook(lambda p: None)
    assert not fused.direct_step_ok(sc)
    h.remove()
    assert fused.direct_step_ok(sc)


def test_direct_ctx_mirrors_the_autograd_context():
    ctx = fused._DirectCtx((True, False) + (False,) * 19)
    assert ctx.needs_input_grad[0] and not any(ctx.needs_input_grad[1:])
    assert ctx.saved_tensors == ()
    a, b = torch.zeros(2), torch.ones(3)
    ctx.save_for_backward(a, None, b)
    assert ctx.saved_tensors[0] is a and ctx.saved_tensors[1] is None and ctx.saved_tensors[2] is b
    ctx.set_materialize_grads(False)
    ctx.mark_non_differentiable(a)
    ctx.meta = (1, 2)  # the forward's own attributes
    assert ctx.meta == (1, 2)


def test_direct_render_rejects_unsupported_calls(monkeypatch):
    sc = synthetic_scene(16, 3, seed=2).requires_grad_()
    with pytest.raises(ValueError, match="direct"):  # the alpha output has no direct backward
        _render(sc, return_alpha=True)
    # without l1_gt the returned image must be the raw one its backward(grad) differentiates
    with pytest.raises(ValueError, match="clamp=False"):
        _render(sc, clamp=True)
    monkeypatch.setattr(fused, "DIRECT_STEP", False)  # not eligible: autograd's step only
    with pytest.raises(ValueError, match="direct"):
        _render(sc)


def _render(sc, **kw):
    """render_fused(direct=True) with a stand-in CPU camera: the refusals come before any
    kernel call."""
    class Cam:
        viewmat = projmat = torch.eye(4)[:3]
        c2w = torch.eye(4)[:3]
        fx = fy = cx = cy = 1.0
        height = width = 8
    fused.render_fused(sc, Cam(), 3, torch.zeros(3), direct=True, **kw)


def test_view_exchange_refuses_an_oversized_table_before_any_collective():
    """ShViewExchange.view checks world x views-per-step against the views kernel's record table
    (exchange.MAX_TABLE) on entry, before the render issues a gather."""
    from gaussctrl_exp_amd import exchange
    x = exchange.ShViewExchange()
    means, campos = torch.zeros(4, 3), torch.zeros(3)
    with x.view(means, campos, 0, exchange.MAX_TABLE):  # world 1: at the limit
        assert exchange.active() is x
    assert exchange.active() is None
    with pytest.raises(ValueError, match="records"):
        with x.view(means, campos, 0, exchange.MAX_TABLE + 1):
            pass
    with pytest.raises(ValueError, match="records"):
        with x.view(means, campos, 0, 0):
            pass
    assert exchange.active() is None
