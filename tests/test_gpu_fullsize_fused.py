"""The step bench.py times, at BASELINE.json's full sizes (headline 1M @ 1080², c3 bear, c4
garden 2M @ 1080², c5 5M @ 2048²; c2 forward only), through exactly the code bench.py runs:
TrainStep(loss="l1", render_mode="fused").forward_backward (fused.render_fused with the L1 loss
inside the blend), i.e. the kernels of the bench line's `kernels` block:

  gsplat_fused_preprocess_forward_part [2] (SH colours, second stream) + [1] (projection, keys)
  gsplat_bin_speculative       (depth sort + tile sort at the learned capacity, its first pass
                                generated at c5: the second call of the frame shape -- the
                                first one bins synchronously)
  gsplat_rasterize_forward_clearing_l1   (blend + L1 partials + records cleared)
  gsplat_rasterize_backward_records_l1   (L1 upstream formed per pixel, record backward; strip
                                          geometry from 3,584 tiles, 8x8 blocks + list split below)
  gsplat_fused_preprocess_backward       (projection / SH / activation chain rule)

Checked, with zero outliers (tests/parity.py bars):
* projection outputs bit-exact vs the oracle on torch's activations; SH colours vs the oracle;
* the speculative binning bit-exact vs the oracle's stable sort of gsplat's keys;
* the image on sampled tiles vs the oracle's forward, final_idx bit-exact, the loss vs float64;
* the records (raster-level gradients) vs the oracle's rasterize backward on the sampled tiles:
  the ground truth equals the clamped image everywhere else, so the L1 upstream gradient
  sign(clamp(img) - gt) is zero there and the records hold the sampled tiles' sums only;
* the six parameter gradients over ALL N vs the oracle chain (projection + SH VJPs, torch's
  activation derivatives in float64) fed the same raster-level gradients.
"""
import numpy as np
import pytest
import torch

import bench
import oracle as O
from gaussctrl_exp_amd import quirks
from gaussctrl_exp_amd.fused import render_fused
from gaussctrl_exp_amd.train import TrainStep
from parity import assert_close, assert_raster_close, close_frac

pytestmark = pytest.mark.gpu


def _np(t):
    return t.detach().cpu().numpy()


class BenchStep:
    """One view of a bench config stepped as bench.py steps it, intermediates kept."""

    def __init__(self, config, gpu):
        sc, cam = bench.make_workload(config, 0, gpu)
        self.config, self.gpu, self.sc, self.cam = config, gpu, sc, cam.to(gpu)
        c = self.cam
        self.H, self.W, self.tb = c.height, c.width, c.tile_bounds
        self.n = sc.means.shape[0]
        self.K = 1 + sc.features_rest.shape[1]
        self.dtu = {1: 0, 4: 1, 9: 2, 16: 3, 25: 4}[self.K]
        self.bg = torch.tensor([0.3, 0.2, 0.1], device=gpu)
        self.trainer = TrainStep(sc, sh_degree=self.dtu, world_size=1, loss="l1",
                                 render_mode="fused")
        # first call of the frame shape: synchronous binning (learns the capacity / key range);
        # an earlier test in this process may have binned the same shape: forget it
        from gaussctrl_exp_amd import rasterize as R
        key = (gpu, self.n, self.tb[0], self.tb[1])
        for table in (R._EMIT_CAP, R._CAP_WINDOW, R._KEY_VARY):
            table.pop(key, None)
        gt0 = torch.rand(self.H, self.W, 3, generator=torch.Generator().manual_seed(4)).to(gpu)
        self.trainer.zero_grad()
        _, out0 = self.trainer.forward_backward(c, gt0, self.bg)
        assert out0["raster_state"]["binning"] == "sync"
        self.img0 = out0["rgb"].detach().clone()
        T = self.tb[0] * self.tb[1]
        self.tiles = np.random.default_rng(3).choice(
            T, size=min(24 if self.n > 3_000_000 else 48, T), replace=False).astype(np.int32)
        m = np.zeros((self.H, self.W), bool)
        for t in self.tiles:
            y0, x0 = (t // self.tb[0]) * 16, (t % self.tb[0]) * 16
            m[y0:y0 + 16, x0:x0 + 16] = True
        self.mask = m
        # the ground truth: random on the sampled tiles, the clamped image elsewhere (zero L1
        # gradient there)
        gt = torch.clamp(self.img0, max=1.0)
        r = torch.rand(self.H, self.W, 3, generator=torch.Generator().manual_seed(9)).to(gpu)
        mt = torch.from_numpy(m).to(gpu)[..., None]
        self.gt = torch.where(mt, r, gt).contiguous()
        self.trainer.zero_grad()
        self.loss, self.out = self.trainer.forward_backward(c, self.gt, self.bg)
        self.param_grads = [_np(p.grad) for p in sc.params()]
        self.raster_grads = [_np(g) for g in self.out["raster_grads"]()]
        self.inp = {k: _np(v) for k, v in self.out["raster_inputs"].items()}
        st = self.out["raster_state"]
        self.gids, self.bins = _np(st["gaussian_ids_sorted"]), _np(st["tile_bins"])
        self.fT, self.fi = _np(st["final_Ts"]), _np(st["final_idx"])
        self.binning = st["binning"]
        self.img = _np(self.out["rgb"])


@pytest.fixture(scope="module", params=["headline", "c3", "c4", "c5"])
def run(request, gpu, oracle_lib):
    return BenchStep(request.param, gpu)


def _activated(sc):
    """torch's activations on the device (bit-identical to the fused kernel's: test_gpu_fused)
    as float32 numpy."""
    return (_np(torch.exp(sc.scales)), _np(sc.quats / sc.quats.norm(dim=-1, keepdim=True)))


def test_preprocess_outputs(gpu, run):
    c, sc = run.cam, run.sc
    s_act, q_act = _activated(sc)
    o = O.project_forward(_np(sc.means), s_act, 1.0, q_act, _np(c.viewmat), _np(c.projmat),
                          c.fx, c.fy, c.cx, c.cy, run.H, run.W, run.tb)
    for name, r in zip(["xys", "depths", "radii", "conics", "num_tiles_hit"], o[:5]):
        np.testing.assert_array_equal(run.inp[name], r, err_msg=name)
    # SH colours (gc_model.py:196-201): clamp(SH(dirs) + 0.5, min=0), the clamp mask in the sign
    d = _np(sc.means) - _np(c.c2w[:3, 3])
    dirs = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    coeffs = np.concatenate([_np(sc.features_dc)[:, None], _np(sc.features_rest)], 1)
    ref = np.maximum(O.sh_forward(run.dtu, dirs, coeffs) + 0.5, 0.0)
    vis = o[2] > 0
    assert_close("colours (visible)", np.abs(run.inp["colors"][vis]), ref[vis])


def test_speculative_binning_bitexact(gpu, run):
    assert run.binning == "speculative"
    ref = O.bin_and_sort(run.inp["xys"], run.inp["depths"], run.inp["radii"],
                         run.inp["num_tiles_hit"], run.tb)
    assert run.out["num_intersects"] == ref["num_intersects"] > 1 << 20
    np.testing.assert_array_equal(run.gids, ref["gaussian_ids_sorted"])
    np.testing.assert_array_equal(run.bins, ref["tile_bins"])


def test_blend_loss_and_records_on_sampled_tiles(gpu, run):
    inp, bg, mask = run.inp, _np(run.bg), run.mask
    # the same forward as the first (synchronously binned) step: deterministic, bit-identical
    np.testing.assert_array_equal(run.img, _np(run.img0))
    rimg, rT, ridx = O.rasterize_forward(run.tb, run.H, run.W, run.gids, run.bins, inp["xys"],
                                         inp["conics"], np.abs(inp["colors"]), inp["opacity"], bg,
                                         tile_list=run.tiles)
    assert_close("image (sampled tiles)", run.img[mask], rimg[mask])
    assert_close("alpha (sampled tiles)", 1 - run.fT[mask], 1 - rT[mask])
    np.testing.assert_array_equal(run.fi[mask], ridx[mask], err_msg="final_idx")
    gt = _np(run.gt)
    ref_loss = np.abs(np.minimum(run.img.astype(np.float64), 1.0) - gt).mean()
    assert abs(float(run.loss) - ref_loss) <= 1e-6 * ref_loss, (float(run.loss), ref_loss)
    # the L1 loss's upstream gradient (l1_grad1 in raster.hip: sign(clamp(p) - g), masked where
    # the clamp saturates, times d loss / d loss = 1 over 3 H W); zero off the sampled tiles
    p = run.img
    s = np.sign(np.minimum(p, 1.0) - gt) * (p <= 1.0)
    v_img = (np.float32(1.0 / (3.0 * run.H * run.W)) * s).astype(np.float32)
    assert not v_img[~mask].any()
    v_alpha = np.zeros((run.H, run.W), np.float32)
    # (the backward walks from the GPU forward's final state, which matched the oracle's above)
    ref, absum, drift, flip = O.rasterize_backward(
        run.tb, run.H, run.W, run.gids, run.bins, inp["xys"], inp["conics"],
        np.abs(inp["colors"]), inp["opacity"], bg, run.fT, run.fi, v_img, v_alpha,
        alpha_max=quirks.backward_alpha_clamp(), tile_list=run.tiles, return_abs=True,
        return_drift=True, return_flip=True)
    for k, name in enumerate(("v_xy", "v_conic", "v_colors", "v_opacity")):
        assert np.abs(ref[k]).max() > 0, name
        assert_raster_close(f"{run.config} {name}", run.raster_grads[k], ref[k], absum[k],
                            drift[k], flip[k])


def test_fused_backward_chain_all_gaussians(gpu, run):
    """The six parameter gradients of the bench step (all N) vs the oracle chain on the same
    raster-level gradients."""
    v_xy, v_conic, v_colors, v_opac = run.raster_grads
    got = run.param_grads
    sc, c = run.sc, run.cam
    means = _np(sc.means)
    s_act, q_act = _activated(sc)
    vm, pm = _np(c.viewmat), _np(c.projmat)
    o = O.project_forward(means, s_act, 1.0, q_act, vm, pm, c.fx, c.fy, c.cx, c.cy, run.H, run.W,
                          run.tb)
    _, _, v_mean, v_sa, v_qn = O.project_backward(
        means, s_act, 1.0, q_act, vm, pm, c.fx, c.fy, c.cx, c.cy, run.H, run.W, o[5], o[2],
        o[3], v_xy, np.zeros(run.n, np.float32), v_conic)
    vis = o[2] > 0
    d = means - _np(c.c2w[:3, 3])
    dirs = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    coeffs = np.concatenate([_np(sc.features_dc)[:, None], _np(sc.features_rest)], 1)
    # the clamp's backward mask: the kernel keeps it in the colour's sign bit (-0.0 = clamped),
    # which is exactly torch's clamp decision on its SH value (test_gpu_fused: bit-identical)
    passed = ~np.signbit(run.inp["colors"])
    v_sh = np.where(passed & vis[:, None], v_colors, 0).astype(np.float32)
    v_coeffs = O.sh_backward(run.dtu, dirs, v_sh, run.K)
    f64 = lambda a: np.asarray(a, np.float64)
    q = f64(_np(sc.quats))
    qn_norm = np.linalg.norm(q, axis=1, keepdims=True)
    qn = q / qn_norm
    dot = (qn * f64(v_qn)).sum(1, keepdims=True)
    v_quat = (f64(v_qn) - qn * dot) / qn_norm
    # rounding bound of that cancelling difference, per element
    q_slack = 2.0 ** -22 * (np.abs(f64(v_qn)) + np.abs(qn) * np.abs(dot)) / qn_norm
    sig = 1 / (1 + np.exp(-f64(_np(sc.opacities))))
    ref = [f64(v_mean), f64(v_sa) * f64(s_act), v_quat, f64(v_opac) * sig * (1 - sig),
           f64(v_coeffs[:, 0]), f64(v_coeffs[:, 1:])]
    names = ["means", "scales", "quats", "opacities", "features_dc", "features_rest"]
    for k, name in enumerate(names):
        a, b = got[k].reshape(ref[k].shape), ref[k]
        assert np.isfinite(a).all(), name
        assert np.abs(b).max() > 0, name
        mx = assert_close(name, a, b, extra=q_slack if name == "quats" else None)
        print(f"{run.config} {run.n}: {name} max |diff| {mx:.3e}")


def test_c2_forward_full_image(gpu, oracle_lib):
    """c2 (100k @ 512², SH degree 0: sigmoid colours, forward only -- bench.py renders it under
    no_grad): the full image and alpha of the fused forward vs the oracle, zero outliers; the
    second call (speculative binning) included."""
    sc, cam = bench.make_workload("c2", 0, gpu)
    cam = cam.to(gpu)
    bg = torch.tensor([0.3, 0.2, 0.1], device=gpu)
    with torch.no_grad():
        for _ in range(2):
            out = render_fused(sc, cam, 0, bg, return_alpha=True, clamp=False)
    inp = {k: _np(v) for k, v in out["raster_inputs"].items()}
    st = out["raster_state"]
    r = O.render_forward(inp["xys"], inp["depths"], inp["radii"], inp["conics"],
                         inp["num_tiles_hit"], inp["colors"], inp["opacity"], cam.height,
                         cam.width, _np(bg))
    assert r["num_intersects"] == out["num_intersects"] > 0
    np.testing.assert_array_equal(_np(st["gaussian_ids_sorted"]), r["gaussian_ids_sorted"])
    np.testing.assert_array_equal(_np(st["tile_bins"]), r["tile_bins"])
    frac, mx = close_frac(_np(out["rgb"]), r["img"])
    assert frac == 0, (frac, mx)
    assert_close("alpha", 1 - _np(st["final_Ts"]), r["alpha"])
    np.testing.assert_array_equal(_np(st["final_idx"]), r["final_idx"], err_msg="final_idx")
    # colours are sigmoid(features_dc) (gc_model.py:203)
    np.testing.assert_array_equal(inp["colors"], _np(torch.sigmoid(sc.features_dc)))
