"""The unchanged caller's path (gc_model.py's glue around the drop-in gsplat API, restated by
scene.render) with the shim's fusions -- projection kernel writing the binning's depth keys
(keyed binning), blend clearing the gradient records (no memset), SH gradient straight to
features_dc / features_rest (no cat backward, no layout copies) -- is bit-identical to the
same path without them (deterministic backward, so runs are comparable bit for bit)."""
import numpy as np
import pytest
import torch

from gaussctrl_exp_amd import _lib, rasterize as R, sh as SH
from gaussctrl_exp_amd.camera import synthetic_camera
from gaussctrl_exp_amd.scene import render, synthetic_scene

pytestmark = pytest.mark.gpu


def _run(gpu, sc, cam, deg):
    s = sc.to(gpu).requires_grad_()
    bg = torch.tensor([0.2, 0.4, 0.6], device=gpu)
    gt = torch.rand(cam.height, cam.width, 3, generator=torch.Generator().manual_seed(3))
    out = render(s, cam.to(gpu), deg, bg)
    ((out["rgb"] - gt.to(gpu)).abs().sum() + 0.1 * out["accumulation"].sum()).backward()
    with torch.no_grad():
        d = render(s, cam.to(gpu), deg, bg, return_depth=True)
    return [out["rgb"], out["accumulation"], d["depth"]] + [p.grad for p in s.params()]


@pytest.mark.parametrize("size", [(128, 96, 4000, 3), (512, 512, 30000, 3), (96, 64, 3000, 0)])
def test_caller_path_fusions_are_exact(gpu, size, monkeypatch, hooks):
    W, H, n, deg = size
    sc = synthetic_scene(n, max(deg, 0), seed=5, scale_lo=0.005, scale_hi=0.05)
    cam = synthetic_camera(W, H)
    prev = _lib.set_deterministic(True)
    try:
        hits0 = R.keyed_workspaces.cache.hits
        fused = [t.detach().cpu() for t in _run(gpu, sc, cam, deg)]
        assert R.keyed_workspaces.cache.hits == hits0 + 2  # keyed binning (train + eval render)
        monkeypatch.setattr(SH, "_CAT_BYPASS", False)
        monkeypatch.setattr(R.keyed_workspaces, "take", lambda *a, **k: None)
        monkeypatch.setattr(_lib.lib(), "gsplat_debug_raster_variant_is_default", lambda: 0)
        plain = [t.detach().cpu() for t in _run(gpu, sc, cam, deg)]
    finally:
        _lib.set_deterministic(prev)
    names = ["rgb", "alpha", "depth", "means", "scales", "quats", "opacities", "dc", "rest"]
    for name, a, b in zip(names, fused, plain):
        assert a.shape == b.shape, name
        np.testing.assert_array_equal(a.numpy(), b.numpy(), err_msg=name)


def test_cat_bypass_only_for_the_callers_pattern(gpu):
    """The SH gradient bypass applies only to cat((dc[:, None], rest), 1) of leaf parameters;
    any other coefficient tensor keeps the plain autograd path (and its gradient)."""
    n, K = 300, 16
    dc = torch.randn(n, 3, device=gpu, requires_grad=True)
    rest = torch.randn(n, K - 1, 3, device=gpu, requires_grad=True)
    vd = torch.nn.functional.normalize(torch.randn(n, 3, device=gpu), dim=-1)
    coeffs = torch.cat((dc[:, None, :], rest), 1)
    assert SH._cat_leaves(coeffs) is not None
    assert SH._cat_leaves(torch.cat((rest, dc[:, None, :]), 1)) is None
    assert SH._cat_leaves(coeffs * 1.0) is None
    c2 = coeffs.detach().requires_grad_()
    assert SH._cat_leaves(c2) is None
    out = SH.spherical_harmonics(3, vd, c2)
    out.sum().backward()
    assert c2.grad is not None and c2.grad.shape == (n, K, 3)
    out = SH.spherical_harmonics(3, vd, coeffs)
    out.sum().backward()
    np.testing.assert_array_equal(dc.grad.cpu().numpy(), c2.grad[:, 0].cpu().numpy())
    np.testing.assert_array_equal(rest.grad.cpu().numpy(), c2.grad[:, 1:].cpu().numpy())
