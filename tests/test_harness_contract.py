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
    for name, got in (("rgb", out["rgb"]), ("accumulation", out["accumulation"])) + (
            (("depth", out["depth"]),) if mode == "eval" else ()):
        ref = d[f"out_{name}"]
        got = got.detach().cpu().numpy()
        bad = np.abs(got - ref) > 1e-5 + 1e-4 * np.abs(ref)
        assert bad.mean() <= 1e-3, f"{name}: {bad.mean():.2e} out of tolerance"
