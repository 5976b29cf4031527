"""Eval render on the MI355X: the binning reuse between gc_model's two rasterize calls
(RGB, then depth as colours; gc_model.py:208-236) and the fused RGB+depth pass
(rasterize_gaussians_rgbd).

Both must be invisible in the results: the fused pass and the cached second call give
bit-identical images to two independent calls, and the cache never serves a stale binning
(in-place edits and recycled allocations miss).
"""
import numpy as np
import pytest
import torch

from gaussctrl_exp_amd import rasterize as R
from gaussctrl_exp_amd.camera import synthetic_camera
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.scene import render, synthetic_scene

pytestmark = pytest.mark.gpu


def _projected(gpu, n=20000, W=256, H=192, seed=7):
    sc = synthetic_scene(n, 3, seed=seed, scale_lo=0.005, scale_hi=0.05, device=gpu)
    cam = synthetic_camera(W, H).to(gpu)
    out = project_gaussians(sc.means, torch.exp(sc.scales), 1,
                            sc.quats / sc.quats.norm(dim=-1, keepdim=True), *cam.project_args())
    g = torch.Generator().manual_seed(seed)
    colors = torch.rand(n, 3, generator=g).to(gpu)
    opac = torch.sigmoid(sc.opacities)
    return out, colors, opac, H, W


def _np(t):
    return t.detach().cpu().numpy()


def _two_calls(xys, depths, radii, conics, nth, colors, opac, H, W, bg):
    rgb, alpha = R.rasterize_gaussians(xys, depths, radii, conics, nth, colors, opac, H, W,
                                       background=bg, return_alpha=True)
    d = R.rasterize_gaussians(xys, depths, radii, conics, nth, depths[:, None].repeat(1, 3),
                              opac, H, W, background=torch.zeros(3, device=xys.device))
    return rgb, d[..., 0:1], alpha


def test_fused_rgbd_equals_two_calls(gpu):
    (xys, depths, radii, conics, nth, _), colors, opac, H, W = _projected(gpu)
    bg = torch.tensor([0.2, 0.4, 0.6], device=gpu)
    R._BIN_CACHE.clear()
    rgb, depth, alpha = _two_calls(xys, depths, radii, conics, nth, colors, opac, H, W, bg)
    frgb, fdepth, falpha = R.rasterize_gaussians_rgbd(xys, depths, radii, conics, nth, colors,
                                                      opac, H, W, background=bg)
    assert fdepth.shape == (H, W, 1) and falpha.shape == (H, W)
    assert (_np(alpha) > 0).mean() > 0.5 and _np(depth).max() > 0
    np.testing.assert_array_equal(_np(frgb), _np(rgb))
    np.testing.assert_array_equal(_np(falpha), _np(alpha))
    np.testing.assert_array_equal(_np(fdepth), _np(depth))


def test_second_call_reuses_binning_and_matches(gpu):
    (xys, depths, radii, conics, nth, _), colors, opac, H, W = _projected(gpu)
    bg = torch.zeros(3, device=gpu)
    R._BIN_CACHE.clear()
    h0 = R._BIN_CACHE.hits
    img1 = R.rasterize_gaussians(xys, depths, radii, conics, nth, colors, opac, H, W, bg)
    img2 = R.rasterize_gaussians(xys, depths, radii, conics, nth, colors * 0.5, opac, H, W, bg)
    assert R._BIN_CACHE.hits == h0 + 1
    R._BIN_CACHE.clear()
    ref2 = R.rasterize_gaussians(xys, depths, radii, conics, nth, colors * 0.5, opac, H, W, bg)
    np.testing.assert_array_equal(_np(img2), _np(ref2))
    assert np.abs(_np(img1) - _np(img2)).max() > 0


def test_cache_misses_after_inplace_edit_and_on_recycled_memory(gpu):
    (xys, depths, radii, conics, nth, _), colors, opac, H, W = _projected(gpu)
    bg = torch.zeros(3, device=gpu)
    R._BIN_CACHE.clear()
    R.rasterize_gaussians(xys, depths, radii, conics, nth, colors, opac, H, W, bg)
    h0 = R._BIN_CACHE.hits
    xys.add_(torch.tensor([17.0, -9.0], device=gpu))  # version bump: must re-bin
    moved = R.rasterize_gaussians(xys, depths, radii, conics, nth, colors, opac, H, W, bg)
    assert R._BIN_CACHE.hits == h0
    R._BIN_CACHE.clear()
    ref = R.rasterize_gaussians(xys, depths, radii, conics, nth, colors, opac, H, W, bg)
    np.testing.assert_array_equal(_np(moved), _np(ref))
    # a new tensor (likely on the freed block's address) with different contents
    shifted = (xys + torch.tensor([-30.0, 11.0], device=gpu)).contiguous()
    del xys
    xys2 = shifted.clone()
    del shifted
    h1 = R._BIN_CACHE.hits
    out = R.rasterize_gaussians(xys2, depths, radii, conics, nth, colors, opac, H, W, bg)
    assert R._BIN_CACHE.hits == h1
    R._BIN_CACHE.clear()
    ref = R.rasterize_gaussians(xys2, depths, radii, conics, nth, colors, opac, H, W, bg)
    np.testing.assert_array_equal(_np(out), _np(ref))


def test_render_fused_depth_equals_reference_caller(gpu):
    sc = synthetic_scene(3000, 3, seed=11, scale_lo=0.002, scale_hi=0.01, device=gpu)
    cam = synthetic_camera(320, 240).to(gpu)
    bg = torch.zeros(3, device=gpu)
    with torch.no_grad():
        a = render(sc, cam, 3, bg, return_depth=True)
        b = render(sc, cam, 3, bg, return_depth=True, fused_depth=True)
    for k in ("rgb", "depth", "accumulation"):
        np.testing.assert_array_equal(_np(a[k]), _np(b[k]))
    assert (_np(a["depth"]) == 1000).any() and (_np(a["depth"]) < 1000).any()
