"""Lane-slot accounting hook (gsplat_debug_pair_count, bench.py `lane_occupancy`): the counting
instantiations of the shipped blend kernels render the same image and gradients as the shipped
ones, and their counts are consistent (valid pairs <= live pairs <= lane slots, slots a whole
number of wave iterations)."""
import numpy as np
import pytest
import torch

from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.camera import synthetic_camera
from gaussctrl_exp_amd.fused import render_fused
from gaussctrl_exp_amd.scene import synthetic_scene

pytestmark = pytest.mark.gpu


def _run(gpu, sc, cam, counts=None):
    s = sc.to(gpu).requires_grad_()
    bg = torch.tensor([0.2, 0.4, 0.6], device=gpu)
    gt = torch.rand(cam.height, cam.width, 3, generator=torch.Generator().manual_seed(3))
    if counts is not None:
        assert _lib.call("gsplat_debug_pair_count", _lib.ptr(counts)) == 0
    try:
        out = render_fused(s, cam.to(gpu), 3, bg, return_alpha=True)
        ((out["rgb"] - gt.to(gpu)).abs().sum() + 0.1 * out["accumulation"].sum()).backward()
        torch.cuda.synchronize()
    finally:
        if counts is not None:
            _lib.call("gsplat_debug_pair_count", None)
    return out["rgb"].detach().cpu(), [p.grad.detach().cpu().numpy() for p in s.params()]


# 160x128: the plain strip backward; 512x512: 1,024 tiles, the list-split (chunked) kernels
@pytest.mark.parametrize("size", [(160, 128, 6000), (512, 512, 30000)])
def test_pair_count_matches_shipped(size):
    gpu = torch.device("cuda:0")
    W, H, n = size
    sc = synthetic_scene(n, 3, seed=11, scale_lo=0.01, scale_hi=0.05)
    cam = synthetic_camera(W, H)
    img0, g0 = _run(gpu, sc, cam)
    counts = torch.zeros(6, dtype=torch.int64, device=gpu)
    img1, g1 = _run(gpu, sc, cam, counts)
    assert torch.equal(img0, img1)
    for a, b in zip(g1, g0):  # float atomics: summation order only
        tol = 1e-5 * max(1.0, float(np.abs(b).max()))
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=tol)
    c = counts.tolist()
    print("bwd slots/live/valid", c[0:3], "fwd", c[3:6])
    for s, live, valid in (c[0:3], c[3:6]):
        assert s > 0 and s % 128 == 0
        assert 0 < valid <= live <= s
    # counting off again: nothing accumulates
    _run(gpu, sc, cam)
    assert counts.tolist() == c
