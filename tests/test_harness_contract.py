"""Harness contract: the reference caller's own arguments and outputs (captured from
/root/reference/gaussctrl/gc_model.py by tools/capture_harness.py into tests/golden/) vs
this repo's restatement of the caller (gaussctrl_exp_amd.camera / scene.render).

CPU tests run scene.render on the oracle-backed gsplat emulation, which is exactly what
the capture ran underneath gc_model, so every captured array must be reproduced
bit-for-bit; the GPU test runs the same inputs through the MI355X kernels."""
import os

import numpy as np
import pytest
import torch

from gaussctrl_exp_amd.camera import gc_camera
from gaussctrl_exp_amd.scene import GaussianScene, render

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(mode):
    d = dict(np.load(os.path.join(GOLDEN, f"harness_bear_{mode}.npz")))
    fx, fy, cx, cy, W, H = d["camera"]
    # nerfstudio Cameras hold intrinsics as float32 tensors; gc_model passes .item() of them
    fx, fy, cx, cy = (float(np.float32(v)) for v in (fx, fy, cx, cy))
    cam = gc_camera(torch.from_numpy(d["c2w"]), fx, fy, cx, cy, int(W), int(H))
    scene = GaussianScene(*[torch.from_numpy(d[f"param_{k}"]) for k in
                            ("means", "scales", "quats", "opacities", "features_dc",
                             "features_rest")])
    return d, cam, scene


@pytest.mark.parametrize("mode", ["train", "eval"])
def test_camera_math_matches_gc_model(mode):
    d, cam, scene = _load(mode)
    np.testing.assert_array_equal(cam.viewmat.numpy(), d["proj_viewmat"])
    np.testing.assert_array_equal(cam.projmat.numpy(), d["proj_projmat"])
    assert tuple(cam.tile_bounds) == tuple(d["proj_tile_bounds"])
    assert (cam.height, cam.width) == tuple(d["proj_hw"])
    np.testing.assert_array_equal(np.array([cam.fx, cam.fy, cam.cx, cam.cy]),
                                  d["proj_intrinsics"])
    assert d["proj_viewmat"].shape == (3, 4)  # gc_model passes viewmat[:3, :]


@pytest.mark.parametrize("mode", ["train", "eval"])
def test_render_restatement_matches_gc_model(mode):
    from oracle_gsplat import API
    d, cam, scene = _load(mode)
    sh_n = int(d["sh_degrees_to_use"])
    assert sh_n == min(int(d["step"]) // 1000, 3)  # gc_model.py:199
    out = render(scene, cam, sh_n, torch.from_numpy(d["raster_background"]),
                 return_depth=(mode == "eval"), api=API)
    np.testing.assert_array_equal(out["rgb"].detach().numpy(), d["out_rgb"])
    np.testing.assert_array_equal(out["accumulation"].detach().numpy(), d["out_accumulation"])
    if mode == "eval":
        np.testing.assert_array_equal(out["depth"].detach().numpy(), d["out_depth"])
        assert int(d["raster_calls"]) == 2
    assert d["out_accumulation"].max() > 0.5  # the fixture actually renders something


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["train", "eval"])
def test_gpu_render_matches_gc_model_golden(gpu, mode):
    d, cam, scene = _load(mode)
    out = render(scene.to(gpu), cam.to(gpu), int(d["sh_degrees_to_use"]),
                 torch.from_numpy(d["raster_background"]).to(gpu),
                 return_depth=(mode == "eval"))
    # the rasterizer's inputs as the reference's capture saw them, for the flip explainer
    import oracle as O
    from parity import assert_close_or_flip
    H, W = (int(v) for v in d["proj_hw"])
    tb = tuple(int(v) for v in d["proj_tile_bounds"])[:2]
    fx, fy, cx, cy = (float(v) for v in d["proj_intrinsics"])
    o = O.project_forward(d["param_means"], d["proj_scales_in"], float(d["proj_glob_scale"]),
                          d["proj_quats_in"], d["proj_viewmat"], d["proj_projmat"], fx, fy, cx, cy,
                          H, W, tb)
    f = O.render_forward(o[0], o[1], o[2], o[3], o[4], d["raster_colors_in"],
                         d["raster_opacity_in"], H, W, d["raster_background"])
    flip = dict(xys=o[0], conics=o[3], opacity=d["raster_opacity_in"],
                gids=f["gaussian_ids_sorted"], bins=f["tile_bins"], tbx=tb[0])
    # zero unexplained outliers: every pixel outside the bar must sit on a threshold flip
    # (tests/parity.py near_threshold_pixel); their count is reported
    for name, got in (("rgb", out["rgb"]), ("accumulation", out["accumulation"])):
        assert_close_or_flip(f"{mode} {name}", got.detach().cpu().numpy(), d[f"out_{name}"],
                             **flip)
    if mode == "eval":
        # gc_model.py:230-236: depth = (depth render) / alpha where alpha > 0, else 1000.  The
        # bar applies to the two rendered quantities; through the division it becomes
        # (tol(num) + depth tol(alpha)) / alpha, tol(x) = 1e-5 + 1e-4 |x|
        ref_d, ref_a = d["out_depth"].astype(np.float64), d["out_accumulation"].astype(np.float64)
        num = ref_d * ref_a
        tol_div = np.where(ref_a > 0, (1e-5 + 1e-4 * np.abs(num) + np.abs(ref_d) *
                                       (1e-5 + 1e-4 * ref_a)) / np.maximum(ref_a, 1e-30), 0.0)
        assert_close_or_flip(f"{mode} depth", out["depth"].detach().cpu().numpy(), ref_d,
                             extra=tol_div, **flip)
