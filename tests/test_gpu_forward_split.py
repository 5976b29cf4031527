"""The list-split forward of small frames (raster.hip: fwd_plan_kernel, raster_fwd_part_kernel,
raster_fwd_combine_kernel; gsplat_rasterize_forward_clearing* with a plan, below 3,584 tiles).

Against the unsplit forward (gsplat_debug_forward_split 0) on the same binning:

* final_idx -- the integer state the backward walks from -- bit-exact, tile by tile, whatever
  part the pixel's termination falls in (chunks forced down to 64 positions, so most lists are
  cut into many parts and terminations land in re-walked later parts);
* final_T and the image within fp32 rounding of the regrouped transmittance product: relative
  (2K + parts + 8) 2^-24 for K composited factors -- checked at 2e-4 relative for T (K stays
  below ~1,600) and at the parity bar (1e-5 abs + 1e-4 rel) for the image;
* mode 2 (every pixel of a split tile resolved by the exact sequential walk): bit-identical in
  all three outputs, which tests the combine's exact walk and its plumbing;
* tiles of a single part are the plain forward, bit for bit (checked through the unsplit
  frames at the default chunk);
* the training step through it: gradients of a smooth loss within the parity bar of the
  unsplit step, the walk table (tile_last) identical.
"""
import numpy as np
import pytest
import torch

from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.camera import synthetic_camera
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians
from gaussctrl_exp_amd.scene import synthetic_scene

pytestmark = pytest.mark.gpu


def _state(gpu, n, W, H, seed, lo=0.004, hi=0.05, opac_shift=0.0):
    sc = synthetic_scene(n, 0, seed=seed, scale_lo=lo, scale_hi=hi).to(gpu)
    cam = synthetic_camera(W, H).to(gpu)
    with torch.no_grad():
        xys, depths, radii, conics, nth, _ = project_gaussians(
            sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
            *cam.project_args())
        I, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W)
    g = torch.Generator().manual_seed(seed + 1)
    colors = torch.rand(n, 3, generator=g).to(gpu)
    opac = torch.sigmoid(sc.opacities.reshape(-1) + opac_shift).contiguous()
    bg = torch.tensor([0.3, 0.5, 0.7], device=gpu)
    return dict(xys=xys, conics=conics, colors=colors, opac=opac, bg=bg, I=I, gids=gids,
                bins=bins, tb=cam.tile_bounds, H=H, W=W, n=n)


def _forward(gpu, s, chunk, mode):
    """gsplat_rasterize_forward_clearing with a list-split plan of `chunk`: (img, final_T,
    final_idx, tile_last) under forward-split mode `mode`."""
    P = _lib.ptr
    tbx, tby = s["tb"][0], s["tb"][1]
    H, W = s["H"], s["W"]
    f32 = dict(device=gpu, dtype=torch.float32)
    img = torch.full((H, W, 3), float("nan"), **f32)
    fT = torch.full((H, W), float("nan"), **f32)
    fi = torch.full((H, W), -7, device=gpu, dtype=torch.int32)
    rec = torch.empty((_lib.query("gsplat_grad_records_bytes", s["n"]),), device=gpu,
                      dtype=torch.uint8)
    pb = _lib.query("gsplat_rasterize_split_bytes", tbx, tby, s["I"], chunk)
    plan = torch.empty((pb,), device=gpu, dtype=torch.uint8)
    prev = _lib.query("gsplat_debug_forward_split", mode)
    try:
        _lib.call("gsplat_rasterize_forward_clearing", tbx, tby, H, W, P(s["gids"]),
                  P(s["bins"]), P(s["xys"]), P(s["conics"]), P(s["colors"]), P(s["opac"]),
                  P(s["bg"]), P(img), P(fT), P(fi), P(rec), rec.numel(), None, s["I"], chunk,
                  P(plan), pb, _lib.stream(gpu))
        torch.cuda.synchronize()
    finally:
        _lib.query("gsplat_debug_forward_split", prev)
    tile_last = plan[:tbx * tby * 4 * 4].view(torch.int32).clone()
    return img.cpu().numpy(), fT.cpu().numpy(), fi.cpu().numpy(), tile_last.cpu().numpy()


CASES = [  # W, H, N, seed, chunk, opacity shift (denser -> more terminations)
    (512, 512, 30000, 3, 64, 0.0),
    (512, 512, 30000, 3, 256, 0.0),
    (320, 256, 60000, 5, 64, 2.0),
    (333, 201, 20000, 7, 128, 1.0),
    (128, 96, 6000, 9, 64, 3.0),
]


@pytest.mark.parametrize("W,H,n,seed,chunk,shift", CASES)
def test_split_forward_against_unsplit(gpu, W, H, n, seed, chunk, shift):
    s = _state(gpu, n, W, H, seed, opac_shift=shift)
    lens = (s["bins"][:, 1] - s["bins"][:, 0]).cpu().numpy()
    assert (lens > chunk).sum() > 10, "the case must split lists"
    ref = _forward(gpu, s, chunk, 0)
    got = _forward(gpu, s, chunk, 1)
    assert np.isfinite(ref[0]).all() and np.isfinite(got[0]).all()
    np.testing.assert_array_equal(got[2], ref[2], err_msg="final_idx")
    np.testing.assert_array_equal(got[3], ref[3], err_msg="tile_last")
    dT = np.abs(got[1].astype(np.float64) - ref[1])
    assert (dT <= 2e-4 * np.abs(ref[1]) + 1e-9).all(), float((dT / (np.abs(ref[1]) + 1e-9)).max())
    dI = np.abs(got[0].astype(np.float64) - ref[0])
    assert (dI <= 1e-5 + 1e-4 * np.abs(ref[0])).all(), float(dI.max())
    # a real share of pixels saturates (a stopped pixel keeps the T before its stop, > 1e-4:
    # below 1e-3 it is within a few Gaussians of it), so the termination fix-up is exercised
    assert (ref[1] < 1e-3).mean() > 0.01 or shift == 0.0


@pytest.mark.parametrize("W,H,n,seed,chunk,shift", CASES[::2])
def test_split_forward_exact_walk_mode_bit_identical(gpu, W, H, n, seed, chunk, shift):
    s = _state(gpu, n, W, H, seed, opac_shift=shift)
    ref = _forward(gpu, s, chunk, 0)
    got = _forward(gpu, s, chunk, 2)
    for name, a, b in zip(("img", "final_T", "final_idx", "tile_last"), got, ref):
        np.testing.assert_array_equal(a, b, err_msg=name)


def test_split_forward_training_step(gpu):
    """The fused render + a smooth loss + backward with the split forward vs without: the six
    gradients within the parity bar (the backward reads final_T, whose rounding differs)."""
    from gaussctrl_exp_amd.fused import render_fused
    sc = synthetic_scene(40000, 3, seed=11, scale_lo=0.004, scale_hi=0.04)
    cam = synthetic_camera(512, 384).to(gpu)
    gt = torch.rand(384, 512, 3, generator=torch.Generator().manual_seed(4)).to(gpu)
    bg = torch.tensor([0.1, 0.2, 0.3], device=gpu)
    out = {}
    prev_det = _lib.set_deterministic(True)
    try:
        _lib.call("gsplat_debug_set_chunk", 64)
        for mode in (0, 1):
            prev = _lib.query("gsplat_debug_forward_split", mode)
            try:
                s = sc.to(gpu).requires_grad_()
                r = render_fused(s, cam, 3, bg, return_alpha=True)
                ((r["rgb"] - gt) ** 2).sum().backward()
                out[mode] = [p.grad.detach().cpu().numpy().astype(np.float64) for p in s.params()]
            finally:
                _lib.query("gsplat_debug_forward_split", prev)
    finally:
        _lib.call("gsplat_debug_set_chunk", 0)
        _lib.set_deterministic(prev_det)
    for name, a, b in zip(("means", "scales", "quats", "opacities", "dc", "rest"), out[1], out[0]):
        scale = np.abs(b).max()
        assert scale > 0, name
        d = np.abs(a - b)
        assert (d <= 1e-5 * scale + 1e-4 * np.abs(b)).all(), (name, float(d.max()), scale)


def test_split_forward_without_backward(gpu):
    """A render with no backward (torch.no_grad: the c2 forward-only bench) takes the split
    forward alone (negative chunk: no walk table, no backward plan): image and alpha within the
    bar of the unsplit render, the mode-2 exact walks bit-identical."""
    from gaussctrl_exp_amd.fused import render_fused
    sc = synthetic_scene(100000, 0, seed=13, scale_lo=0.004, scale_hi=0.05).to(gpu)
    cam = synthetic_camera(512, 512).to(gpu)
    bg = torch.tensor([0.0, 0.0, 0.0], device=gpu)
    outs = {}
    for mode in (0, 1, 2):
        prev = _lib.query("gsplat_debug_forward_split", mode)
        try:
            with torch.no_grad():
                r = render_fused(sc, cam, 0, bg, return_alpha=True)
            outs[mode] = (r["rgb"].cpu().numpy(), r["accumulation"].cpu().numpy())
        finally:
            _lib.query("gsplat_debug_forward_split", prev)
    for k, name in enumerate(("rgb", "alpha")):
        ref, got = outs[0][k].astype(np.float64), outs[1][k]
        assert (np.abs(got - ref) <= 1e-5 + 1e-4 * np.abs(ref)).all(), name
        np.testing.assert_array_equal(outs[2][k], outs[0][k], err_msg=name)


@pytest.mark.parametrize("div", [2, 4])
def test_split_forward_shorter_parts(gpu, div):
    """Parts shorter than the plan's chunk (gsplat_debug_forward_chunk_div): the forward's own
    part bound and records, same guarantees."""
    s = _state(gpu, 30000, 512, 512, 3)
    prev = _lib.query("gsplat_debug_forward_chunk_div", div)
    try:
        ref = _forward(gpu, s, 256, 0)
        got = _forward(gpu, s, 256, 1)
        exact = _forward(gpu, s, 256, 2)
    finally:
        _lib.query("gsplat_debug_forward_chunk_div", prev)
    np.testing.assert_array_equal(got[2], ref[2], err_msg="final_idx")
    dI = np.abs(got[0].astype(np.float64) - ref[0])
    assert (dI <= 1e-5 + 1e-4 * np.abs(ref[0])).all(), float(dI.max())
    for name, a, b in zip(("img", "final_T", "final_idx", "tile_last"), exact, ref):
        np.testing.assert_array_equal(a, b, err_msg=name)
