"""Speculative binning (rasterize.SpeculativeBinning, gsplat_bin_emit_speculative): the emission
and the whole tile sort launched at a capacity before the host reads the intersection count I,
the blend right behind them.  Checks:

* the ids [0, I) and the tile table equal the synchronous binning's bit for bit -- with the
  capacity a little above I (the steady state), far above it, and BELOW it (overflow: the
  table is left all-zero, nothing is written past the capacity, rebin() then gives the exact
  result);
* scenes the sorted scheme handles and small ones binned by tile buckets (also launched at the
  capacity: each bucket kernel returns at once on an overflow and the table is cleared);
* the fused render through it (second call of a frame shape) equals the first call's
  synchronous path: image, alpha and all six gradients bit-identical (deterministic mode), also
  when the capacity overflows and the render re-bins and re-blends.
"""
import numpy as np
import pytest
import torch

from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd import rasterize as R
from gaussctrl_exp_amd.camera import synthetic_camera
from gaussctrl_exp_amd.fused import render_fused
from gaussctrl_exp_amd.scene import synthetic_scene

pytestmark = pytest.mark.gpu


def _keyed(gpu, sc, cam):
    """The fused preprocess's outputs and the keyed binning workspace it fills."""
    n = sc.num_points
    dev = gpu
    f32 = dict(device=dev, dtype=torch.float32)
    xys, depths = torch.empty((n, 2), **f32), torch.empty((n,), **f32)
    radii = torch.empty((n,), device=dev, dtype=torch.int32)
    conics, nth = torch.empty((n, 3), **f32), torch.empty((n,), device=dev, dtype=torch.int32)
    colors, opac = torch.empty((n, 3), **f32), torch.empty((n,), **f32)
    ws1 = torch.empty((_lib.query("gsplat_bin_count_workspace_size", n),), device=dev,
                      dtype=torch.uint8)
    p = [t.contiguous() for t in sc.to(gpu).params()]
    K = 1 + p[5].shape[1]
    c = cam.to(gpu)
    P = _lib.ptr
    tbx, tby = c.tile_bounds[0], c.tile_bounds[1]
    campos = c.c2w[..., :3, 3].reshape(3).contiguous().float()
    _lib.call("gsplat_fused_preprocess_forward_binned", n, K, 3, *[P(t) for t in p[:5]],
              P(p[5]), P(c.viewmat.contiguous()), P(c.projmat.contiguous()), P(campos),
              float(c.fx), float(c.fy), float(c.cx), float(c.cy), c.height, c.width, tbx, tby,
              0.01, P(xys), P(depths), P(radii), P(conics), P(nth), P(colors), P(opac), P(ws1),
              ws1.numel(), _lib.stream(gpu))
    return xys, depths, radii, nth, ws1, c


def _fresh_ws(ws1):
    return ws1.clone()  # the depth sort consumes its inputs: one copy per binning


@pytest.mark.parametrize("n,W,H", [(200_000, 640, 480), (60_000, 320, 256)])
@pytest.mark.parametrize("cap_scale", [1.125, 3.0, 0.5])
def test_speculative_binning_equals_sync(gpu, n, W, H, cap_scale):
    sc = synthetic_scene(n, 3, seed=11, scale_lo=0.004, scale_hi=0.03)
    xys, depths, radii, nth, ws1, cam = _keyed(gpu, sc, synthetic_camera(W, H))
    I, ids, bins = R.bin_gaussians(xys, depths, radii, nth, H, W, keyed_workspace=_fresh_ws(ws1))
    assert I > 0
    key = (gpu, n, (W + 15) // 16, (H + 15) // 16)
    R._EMIT_CAP[key] = max(1, int(I * cap_scale))
    spec = R.bin_gaussians_speculative(xys, depths, radii, nth, H, W,
                                       keyed_workspace=_fresh_ws(ws1))
    assert spec is not None
    ok = spec.finish()
    assert spec.num_intersects == I
    if ok:
        got_ids, got_bins = spec.ids[:I], spec.tile_bins
    else:
        assert cap_scale < 1
        # overflow: the table was left all-zero (a blend behind it reads empty tiles)
        assert int(spec.tile_bins.abs().sum()) == 0
        got_ids, got_bins = spec.rebin()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got_ids.cpu().numpy(), ids.cpu().numpy())
    np.testing.assert_array_equal(got_bins.cpu().numpy(), bins.cpu().numpy())
    # the next call's capacity follows this I
    assert R._EMIT_CAP[key] == R.emit_capacity(I)


@pytest.mark.parametrize("n,W,H,scale,big,cap_scale", [
    (200_000, 640, 480, 0.03, 0, 1.125),      # 1,024-slot sort tiles
    (200_000, 640, 480, 0.03, 512, 1.125),    # + 512 frame-sized Gaussians at one depth
    (700_000, 1080, 1080, 0.02, 300, 1.125),  # > 4M intersections: 4,096-slot sort tiles
    (700_000, 1080, 1080, 0.02, 300, 0.5),    # overflow: nothing counted, table all-zero
])
def test_emission_counted_first_pass(gpu, hooks, n, W, H, scale, big, cap_scale):
    """The speculative binning's tile sort with its first digit counts accumulated by the
    emission (EmitCounts: LDS histograms of each workgroup's first EC_LT sort tiles, the rest
    straight into the tile-major matrix) equals the same binning with the first pass counted by
    its own launch, and the synchronous binning, bit for bit.  `big` Gaussians as large as the
    frame, all at the same depth, sit next to each other in depth order: their workgroups' slot
    ranges span hundreds of sort tiles, so most of their counts take the global path."""
    sc = synthetic_scene(n, 3, seed=13, scale_lo=0.004, scale_hi=scale)
    if big:
        sc.scales.data[:big] = float(np.log(0.9))  # radius ~ the frame: every tile
        sc.means.data[:big] = 0.0  # one depth, centred (the camera looks down -z from z = 4)
    xys, depths, radii, nth, ws1, cam = _keyed(gpu, sc, synthetic_camera(W, H))
    I, ids, bins = R.bin_gaussians(xys, depths, radii, nth, H, W, keyed_workspace=_fresh_ws(ws1))
    assert I > 0
    T = ((W + 15) // 16) * ((H + 15) // 16)
    if big:
        assert int((nth[:big] == T).sum()) > big // 2  # (most cover the whole frame)
    # the two sort-tile plans, both below the generated first pass (2^24)
    assert (I < (4 << 20)) if n == 200_000 else ((4 << 20) <= I < (1 << 24))
    key = (gpu, n, (W + 15) // 16, (H + 15) // 16)
    got = {}
    for on in (1, 0):
        prev = hooks.gsplat_debug_emit_counts(on)
        try:
            R._EMIT_CAP[key] = max(1, int(I * cap_scale))
            spec = R.bin_gaussians_speculative(xys, depths, radii, nth, H, W,
                                               keyed_workspace=_fresh_ws(ws1))
            ok = spec.finish()
            assert spec.num_intersects == I
            if not ok:
                assert cap_scale < 1 and int(spec.tile_bins.abs().sum()) == 0
                continue
            got[on] = (spec.ids[:I].cpu().numpy(), spec.tile_bins.cpu().numpy())
        finally:
            hooks.gsplat_debug_emit_counts(prev)
    if cap_scale < 1:
        return
    for on in (1, 0):
        np.testing.assert_array_equal(got[on][0], ids.cpu().numpy())
        np.testing.assert_array_equal(got[on][1], bins.cpu().numpy())


@pytest.mark.parametrize("case", ["plain", "overflow", "range"])
def test_split_speculative_binning(gpu, case):
    """The speculative binning as two calls (the count phase, a callback, then
    gsplat_bin_emit_speculative -- the fused render's colour part goes out in between): equal
    to the synchronous binning; an overflow and a depth-key range violation found by the count
    call leave the table all-zero and write no id (the emission call checks the count phase's
    violation flag on the device)."""
    n, W, H = 200_000, 640, 480
    sc = synthetic_scene(n, 3, seed=11, scale_lo=0.004, scale_hi=0.03)
    xys, depths, radii, nth, ws1, cam = _keyed(gpu, sc, synthetic_camera(W, H))
    key = (gpu, n, (W + 15) // 16, (H + 15) // 16)
    R._EMIT_CAP.pop(key, None)
    R._KEY_VARY.pop(key, None)
    I, ids, bins = R.bin_gaussians(xys, depths, radii, nth, H, W, keyed_workspace=_fresh_ws(ws1))
    if case == "overflow":
        R._EMIT_CAP[key] = I // 2
    if case == "range":
        R._KEY_VARY[key] = 0xFF  # "only the low byte varies": the upper passes are skipped
    called = []
    spec = R.bin_gaussians_speculative(xys, depths, radii, nth, H, W,
                                       keyed_workspace=_fresh_ws(ws1),
                                       between=lambda: called.append(1))
    assert called == [1]
    ok = spec.finish()
    torch.cuda.synchronize()
    if case == "plain":
        assert ok and spec.num_intersects == I
        np.testing.assert_array_equal(spec.ids[:I].cpu().numpy(), ids.cpu().numpy())
        np.testing.assert_array_equal(spec.tile_bins.cpu().numpy(), bins.cpu().numpy())
    else:
        assert not ok and spec.range_violated == (case == "range")
        assert int(spec.tile_bins.abs().sum()) == 0
    R._EMIT_CAP.pop(key, None)
    R._KEY_VARY.pop(key, None)


def _fused(gpu, sc, cam, gt, bg):
    s = sc.to(gpu).requires_grad_()
    out = render_fused(s, cam.to(gpu), 3, bg, return_alpha=True)
    ((out["rgb"] - gt).abs().sum() + 0.1 * out["accumulation"].sum()).backward()
    return ([out["rgb"].detach().cpu().numpy(), out["accumulation"].detach().cpu().numpy()] +
            [p.grad.detach().cpu().numpy() for p in s.params()], out["num_intersects"])


@pytest.mark.parametrize("W,H,n", [(512, 384, 200_000), (1080, 1080, 400_000)])
@pytest.mark.parametrize("mode", ["plain", "overflow", "range"])
def test_fused_render_speculative_bit_identical(gpu, W, H, n, mode):
    """First call of the frame shape: synchronous binning (it learns the capacity and the depth
    keys' varying bits); the next: speculative (blend launched before the host reads I, the
    depth-sort passes over constant key bytes not launched).  `overflow`: a capacity below I
    forces the re-bin and the second blend; `range`: a depth-key range claimed narrower than it
    is makes the sort skip passes it needs -- the violation is detected on the device and the
    render redoes the preprocess and a full binning.  Bit-identical outputs and gradients
    (deterministic mode)."""
    sc = synthetic_scene(n, 3, seed=17, scale_lo=0.004, scale_hi=0.03)
    cam = synthetic_camera(W, H)
    bg = torch.tensor([0.2, 0.4, 0.6], device=gpu)
    gt = torch.rand(H, W, 3, generator=torch.Generator().manual_seed(2)).to(gpu)
    key = (gpu, n, (W + 15) // 16, (H + 15) // 16)
    prev = _lib.set_deterministic(True)
    try:
        R._EMIT_CAP.pop(key, None)
        R._KEY_VARY.pop(key, None)
        ref, I = _fused(gpu, sc, cam, gt, bg)
        assert key in R._EMIT_CAP and I > 0
        vary = R._KEY_VARY[key]
        assert vary and (vary >> 24) == 0  # depths 2.5-5.5: the top key byte is constant
        if mode == "overflow":
            R._EMIT_CAP[key] = I // 3
        if mode == "range":
            R._KEY_VARY[key] = 0xFF  # "only the low byte varies": passes 1-3 not launched
        got, I2 = _fused(gpu, sc, cam, gt, bg)
        if mode == "range":
            assert R._KEY_VARY[key] == 0xFF | vary  # the violation taught the real range
    finally:
        _lib.set_deterministic(prev)
    assert I2 == I
    names = ("rgb", "alpha", "means", "scales", "quats", "opacities", "dc", "rest")
    for name, x, y in zip(names, got, ref):
        np.testing.assert_array_equal(x, y, err_msg=name)
