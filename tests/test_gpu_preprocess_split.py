"""The fused preprocess in two parts (gsplat_fused_preprocess_forward_part: 1 = activations +
projection + opacity + binning inputs, 2 = the SH colours; the fused render issues part 2 on a
second stream overlapping the binning) against the one-kernel forward
(gsplat_fused_preprocess_forward_binned):

* every output of the two parts bit-identical to the one kernel's (all SH degrees, ragged N,
  a partial last block);
* the fused render + backward with the split on and off: image, alpha and the six gradients
  bit-identical (deterministic mode);
* bad part numbers and missing tensors are rejected.
"""
import numpy as np
import pytest
import torch

from gaussctrl_exp_amd import _lib, fused
from gaussctrl_exp_amd.camera import synthetic_camera
from gaussctrl_exp_amd.fused import render_fused
from gaussctrl_exp_amd.scene import synthetic_scene

pytestmark = pytest.mark.gpu


def _outputs(gpu, n):
    f32 = dict(device=gpu, dtype=torch.float32)
    o = dict(xys=torch.full((n, 2), np.nan, **f32), depths=torch.full((n,), np.nan, **f32),
             radii=torch.full((n,), -5, device=gpu, dtype=torch.int32),
             conics=torch.full((n, 3), np.nan, **f32),
             nth=torch.full((n,), -5, device=gpu, dtype=torch.int32),
             colors=torch.full((n, 3), np.nan, **f32), opac=torch.full((n,), np.nan, **f32))
    o["ws1"] = torch.zeros((_lib.query("gsplat_bin_count_workspace_size", n),), device=gpu,
                           dtype=torch.uint8)
    return o


@pytest.mark.parametrize("n,deg", [(70001, 3), (4097, 1), (12345, 2), (3000, 4), (20000, 0)])
def test_parts_equal_one_kernel(gpu, n, deg):
    sc = synthetic_scene(n, deg, seed=n % 97, scale_lo=0.004, scale_hi=0.05).to(gpu)
    cam = synthetic_camera(640, 480).to(gpu)
    K = (deg + 1) ** 2
    P, st = _lib.ptr, _lib.stream(gpu)
    p = [t.contiguous() for t in sc.params()]
    campos = cam.c2w[..., :3, 3].reshape(3).contiguous().float()
    tbx, tby = cam.tile_bounds[0], cam.tile_bounds[1]
    cam_args = (P(cam.viewmat.contiguous()), P(cam.projmat.contiguous()), P(campos),
                float(cam.fx), float(cam.fy), float(cam.cx), float(cam.cy), cam.height,
                cam.width, tbx, tby, 0.01)
    rest = P(p[5]) if K > 1 else None
    a = _outputs(gpu, n)
    _lib.call("gsplat_fused_preprocess_forward_binned", n, K, deg, *[P(t) for t in p[:5]], rest,
              *cam_args, P(a["xys"]), P(a["depths"]), P(a["radii"]), P(a["conics"]), P(a["nth"]),
              P(a["colors"]), P(a["opac"]), P(a["ws1"]), a["ws1"].numel(), st)
    b = _outputs(gpu, n)
    _lib.call("gsplat_fused_preprocess_forward_part", 2, n, K, deg, P(p[0]), None, None, None,
              P(p[4]), rest, *cam_args, None, None, None, None, None, P(b["colors"]), None, None,
              0, st)
    _lib.call("gsplat_fused_preprocess_forward_part", 1, n, K, deg, *[P(t) for t in p[:5]], rest,
              *cam_args, P(b["xys"]), P(b["depths"]), P(b["radii"]), P(b["conics"]), P(b["nth"]),
              None, P(b["opac"]), P(b["ws1"]), b["ws1"].numel(), st)
    torch.cuda.synchronize()
    for k in ("xys", "depths", "radii", "conics", "nth", "colors", "opac", "ws1"):
        np.testing.assert_array_equal(b[k].cpu().numpy(), a[k].cpu().numpy(), err_msg=k)
    assert (a["radii"] > 0).any()


def test_split_render_bit_identical(gpu):
    sc = synthetic_scene(60000, 3, seed=21, scale_lo=0.004, scale_hi=0.04)
    cam = synthetic_camera(512, 384).to(gpu)
    bg = torch.tensor([0.2, 0.1, 0.3], device=gpu)
    g = torch.Generator().manual_seed(2)
    v_img = torch.rand(384, 512, 3, generator=g).to(gpu)
    outs = {}
    prev_det = _lib.set_deterministic(True)
    prev = fused.SPLIT_COLOURS, fused.SPLIT_COLOURS_MIN_TILES
    fused.SPLIT_COLOURS_MIN_TILES = 0  # (a small frame: split regardless of its size)
    try:
        for split in (False, True, False, True):  # (second round: capacity-launched binning)
            fused.SPLIT_COLOURS = split
            s = sc.to(gpu).requires_grad_()
            r = render_fused(s, cam, 3, bg, return_alpha=True)
            ((r["rgb"] * v_img).sum() + r["accumulation"].sum()).backward()
            outs[split] = [r["rgb"].detach().cpu().numpy(),
                           r["accumulation"].detach().cpu().numpy()] + \
                [t.grad.cpu().numpy() for t in s.params()]
    finally:
        fused.SPLIT_COLOURS, fused.SPLIT_COLOURS_MIN_TILES = prev
        _lib.set_deterministic(prev_det)
    for name, x, y in zip(("rgb", "alpha", "means", "scales", "quats", "opacities", "dc", "rest"),
                          outs[True], outs[False]):
        np.testing.assert_array_equal(x, y, err_msg=name)


def test_part_argument_checks(gpu):
    n = 100
    f = torch.zeros(n * 48, device=gpu)
    P, st = _lib.ptr, _lib.stream(gpu)
    args = (n, 16, 3, P(f), None, None, None, P(f), P(f), P(f), P(f), P(f), 1.0, 1.0, 1.0, 1.0,
            64, 64, 4, 4, 0.01)
    for part in (0, 3):
        with pytest.raises(RuntimeError):
            _lib.call("gsplat_fused_preprocess_forward_part", part, *args, None, None, None, None,
                      None, P(f), None, None, 0, st)
    with pytest.raises(RuntimeError):  # part 2 without colours
        _lib.call("gsplat_fused_preprocess_forward_part", 2, *args, None, None, None, None, None,
                  None, None, None, 0, st)
    with pytest.raises(RuntimeError):  # part 1 without a workspace / projection outputs
        _lib.call("gsplat_fused_preprocess_forward_part", 1, *args, None, None, None, None, None,
                  None, None, None, 0, st)
