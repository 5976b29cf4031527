"""Deterministic rasterize backward (gsplat_set_deterministic / GSPLAT_MI355X_DETERMINISTIC,
SURVEY.md §5): two runs give bit-identical gradients -- through the gsplat API (caller path),
the fused training render (records) and the list-split backward -- and the gradients still
meet the oracle bar."""
import numpy as np
import pytest
import torch

from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.camera import synthetic_camera
from gaussctrl_exp_amd.fused import render_fused
from gaussctrl_exp_amd.scene import render, synthetic_scene

pytestmark = pytest.mark.gpu


@pytest.fixture
def deterministic():
    prev = _lib.set_deterministic(True)
    assert _lib.lib().gsplat_get_deterministic() == 1
    yield
    _lib.set_deterministic(prev)
    assert _lib.lib().gsplat_get_deterministic() == int(prev)


def _grads(gpu, mode, sc, cam, api=None):
    s = sc.to(gpu).requires_grad_()
    bg = torch.tensor([0.2, 0.4, 0.6], device=gpu)
    gt = torch.rand(cam.height, cam.width, 3, generator=torch.Generator().manual_seed(3))
    if mode == "fused":
        out = render_fused(s, cam.to(gpu), 3, bg, return_alpha=True)
    else:
        out = render(s, cam.to(gpu), 3, bg, api=api)
    ((out["rgb"] - gt.to(gpu)).abs().sum() + 0.1 * out["accumulation"].sum()).backward()
    return [p.grad.detach().cpu().numpy() for p in s.params()]


# 128x96: the plain strip backward; 512x512: 1,024 tiles, the list-split backward
@pytest.mark.parametrize("size", [(128, 96, 4000), (512, 512, 30000)])
@pytest.mark.parametrize("mode", ["caller", "fused"])
def test_two_runs_bit_identical(gpu, deterministic, mode, size):
    W, H, n = size
    sc = synthetic_scene(n, 3, seed=7, scale_lo=0.005, scale_hi=0.05)
    cam = synthetic_camera(W, H)
    a = _grads(gpu, mode, sc, cam)
    b = _grads(gpu, mode, sc, cam)
    for name, x, y in zip(("means", "scales", "quats", "opacities", "dc", "rest"), a, b):
        assert np.abs(x).max() > 0, name
        np.testing.assert_array_equal(x, y, err_msg=name)


def test_deterministic_grads_meet_the_oracle_bar(gpu, deterministic):
    """Raster-level gradients of the deterministic backward vs the oracle (same bar as the
    atomic backward: their fp32 wave totals are summed exactly, so the slack is smaller)."""
    from parity import CaptureAPI, check_raster_level
    sc = synthetic_scene(3000, 3, seed=21, scale_lo=0.01, scale_hi=0.06)
    cam = synthetic_camera(128, 96)
    cap = CaptureAPI()
    _grads(gpu, "caller", sc, cam, api=cap)
    k = cap.cap
    check_raster_level(gpu, k["xys_in"], k["depths"], k["radii"], k["conics_in"], k["nth"],
                       k["colors_in"], k["opacity_in"], k["background"], 96, 128, k["v_img"],
                       k["v_alpha"], cap.raster_grads(sc.num_points))


def test_deterministic_and_atomic_agree(gpu):
    """The two accumulation modes compute the same gradients up to fp32 summation order."""
    sc = synthetic_scene(4000, 3, seed=9, scale_lo=0.005, scale_hi=0.05)
    cam = synthetic_camera(128, 96)
    prev = _lib.set_deterministic(True)
    try:
        d = _grads(gpu, "fused", sc, cam)
    finally:
        _lib.set_deterministic(prev)
    a = _grads(gpu, "fused", sc, cam)
    for x, y in zip(d, a):
        np.testing.assert_allclose(x, y, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("bwd,mode", [(0, "fused"), (1, "caller"), (2, "caller")])
@pytest.mark.parametrize("chunk", [64, 192])
def test_list_split_bit_identical_to_the_full_walk(gpu, deterministic, bwd, mode, chunk):
    """The list-split backward re-walks the positions behind each part with the full walk's
    operations, so every wave's per-Gaussian totals -- and the deterministic mode's exact sums of
    them -- equal the unsplit walk's bit for bit (8x8 blocks, 16x8 strips, and the frame-size
    dispatch through the fused records)."""
    sc = synthetic_scene(30000, 3, seed=5, scale_lo=0.005, scale_hi=0.06)
    cam = synthetic_camera(512, 384)
    _lib.call("gsplat_debug_set_raster_variant", 1, bwd, 0)
    try:
        _lib.call("gsplat_debug_set_chunk", -1)
        full = _grads(gpu, mode, sc, cam)
        _lib.call("gsplat_debug_set_chunk", chunk)
        split = _grads(gpu, mode, sc, cam)
    finally:
        _lib.call("gsplat_debug_set_chunk", 0)
        _lib.call("gsplat_debug_set_raster_variant", 1, 0, 0)
    for name, x, y in zip(("means", "scales", "quats", "opacities", "dc", "rest"), full, split):
        assert np.abs(x).max() > 0, name
        np.testing.assert_array_equal(y, x, err_msg=name)


def test_deterministic_matches_atomic_at_mean_loss_scale(gpu):
    """splatfacto's loss is a mean (L1 + SSIM), so at 512x384 the per-pixel upstream
    gradients are ~1e-6 and the per-wave totals far smaller; the exact-integer sums (units of
    2^-80) must keep them to fp32 accuracy, not quantise them away."""
    sc = synthetic_scene(30000, 3, seed=13, scale_lo=0.005, scale_hi=0.05)
    cam = synthetic_camera(512, 384)
    gt = torch.rand(cam.height, cam.width, 3, generator=torch.Generator().manual_seed(4))

    def grads():
        s = sc.to(gpu).requires_grad_()
        out = render_fused(s, cam.to(gpu), 3, torch.tensor([0.2, 0.4, 0.6], device=gpu))
        (out["rgb"] - gt.to(gpu)).abs().mean().backward()
        return [p.grad.detach().cpu().numpy() for p in s.params()]

    prev = _lib.set_deterministic(True)
    try:
        d = grads()
    finally:
        _lib.set_deterministic(prev)
    a = grads()
    for name, x, y in zip(("means", "scales", "quats", "opacities", "dc", "rest"), d, a):
        scale = np.abs(y).max()
        assert 0 < scale < 1e-2, name  # the mean-loss regime
        assert np.count_nonzero(x) == np.count_nonzero(y), name  # nothing quantised to zero
        np.testing.assert_allclose(x, y, rtol=1e-3, atol=1e-5 * scale, err_msg=name)
