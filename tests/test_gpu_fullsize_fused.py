"""The kernels bench.py times, at BASELINE.json's full sizes (headline 1M @ 1080², c3 bear,
c4 garden 2M @ 1080², c5 5M @ 2048²; c2 forward only), driven through the C ABI in exactly
the fused training render's sequence (gaussctrl_exp_amd/fused.py):

  gsplat_fused_preprocess_forward_binned -> gsplat_bin_count_keyed -> gsplat_bin_emit ->
  gsplat_rasterize_forward_clearing -> gsplat_rasterize_backward_records ->
  gsplat_fused_preprocess_backward

Checked, with zero outliers:
* projection outputs bit-exact vs the oracle on torch's activations of the parameters;
* the keyed binning identical to the plain binning of the same outputs (which
  test_gpu_fullsize checks bit-exact against the oracle at these sizes);
* the blend on sampled tiles vs the oracle (image, alpha), and the gradient records cleared;
* the backward's records (raster-level gradients, upstream gradient on the sampled tiles only)
  vs the oracle's rasterize backward on the same forward state (fp32 summation slack);
* with a dense upstream gradient, the fused backward's six parameter gradients over ALL N vs
  the oracle chain (projection + SH VJPs, torch's activation derivatives in float64) fed the
  same records.
"""
import numpy as np
import pytest
import torch

import bench
import oracle as O
from gaussctrl_exp_amd import _lib, quirks
from gaussctrl_exp_amd.rasterize import bin_gaussians
from parity import assert_close, assert_raster_close, close_frac

pytestmark = pytest.mark.gpu


def _np(t):
    return t.detach().cpu().numpy()


class FusedRun:
    """One view of a bench config through the fused C-ABI sequence, intermediates kept."""

    def __init__(self, config, gpu):
        sc, cam = bench.make_workload(config, 0, gpu)
        self.sc, self.cam, self.gpu, self.config = sc, cam.to(gpu), gpu, config
        c = self.cam
        n = sc.means.shape[0]
        K = 1 + sc.features_rest.shape[1]
        self.n, self.K, self.dtu = n, K, {1: 0, 4: 1, 9: 2, 16: 3, 25: 4}[K]
        H, W = c.height, c.width
        self.H, self.W = H, W
        self.tb = c.tile_bounds
        f = lambda *s: torch.empty(*s, device=gpu)
        self.xys, self.depths, self.conics = f(n, 2), f(n), f(n, 3)
        self.colors, self.opac = f(n, 3), f(n)
        self.radii = torch.empty(n, device=gpu, dtype=torch.int32)
        self.nth = torch.empty(n, device=gpu, dtype=torch.int32)
        self.campos = c.c2w[:3, 3].contiguous()
        P, st = _lib.ptr, _lib.stream(gpu)
        ws1 = torch.empty((_lib.query("gsplat_bin_count_workspace_size", n),), device=gpu,
                          dtype=torch.uint8)
        _lib.call("gsplat_fused_preprocess_forward_binned", n, K, self.dtu, P(sc.means),
                  P(sc.scales), P(sc.quats), P(sc.opacities), P(sc.features_dc),
                  P(sc.features_rest) if K > 1 else None, P(c.viewmat), P(c.projmat),
                  P(self.campos), c.fx, c.fy, c.cx, c.cy, H, W, self.tb[0], self.tb[1], 0.01,
                  P(self.xys), P(self.depths), P(self.radii), P(self.conics), P(self.nth),
                  P(self.colors), P(self.opac), P(ws1), ws1.numel(), st)
        self.I, self.gids, self.bins = bin_gaussians(self.xys, self.depths, self.radii, self.nth,
                                                     H, W, keyed_workspace=ws1)
        self.rec = torch.full((_lib.query("gsplat_grad_records_bytes", n),), 0x7F, device=gpu,
                              dtype=torch.uint8)
        self.chunk = _lib.query("gsplat_rasterize_chunk_size", self.tb[0], self.tb[1], self.I)
        self.plan = torch.empty((max(_lib.query("gsplat_rasterize_split_bytes", self.tb[0],
                                                self.tb[1], self.I, self.chunk), 1),),
                                device=gpu, dtype=torch.uint8)
        self.bg = torch.tensor([0.3, 0.2, 0.1], device=gpu)

    def forward(self):
        """The clearing blend; returns (img, final_Ts, final_idx)."""
        P, st, gpu = _lib.ptr, _lib.stream(self.gpu), self.gpu
        H, W = self.H, self.W
        img = torch.empty(H, W, 3, device=gpu)
        fT = torch.empty(H, W, device=gpu)
        fi = torch.empty(H, W, device=gpu, dtype=torch.int32)
        vis_only = self.radii if int((self.radii > 0).sum()) < 0.9 * self.n else None
        _lib.call("gsplat_rasterize_forward_clearing", self.tb[0], self.tb[1], H, W, P(self.gids),
                  P(self.bins), P(self.xys), P(self.conics), P(self.colors), P(self.opac),
                  P(self.bg), P(img), P(fT), P(fi), P(self.rec), self.rec.numel(), P(vis_only),
                  self.I, self.chunk, P(self.plan), self.plan.numel() if self.chunk > 0 else 0, st)
        self.fT, self.fi = fT, fi
        return img, fT, fi

    def backward(self, v_img, v_alpha, final_Ts=None, final_idx=None):
        """The record backward from the forward's state (or the given final_Ts / final_idx)."""
        P, st = _lib.ptr, _lib.stream(self.gpu)
        self.v_img, self.v_alpha = v_img.to(self.gpu).contiguous(), v_alpha.to(self.gpu).contiguous()
        fT = self.fT if final_Ts is None else final_Ts
        fi = self.fi if final_idx is None else final_idx
        _lib.call("gsplat_rasterize_backward_records", self.tb[0], self.tb[1], self.H, self.W,
                  self.n, P(self.gids), P(self.bins), P(self.xys), P(self.conics),
                  P(self.colors), P(self.opac), P(self.bg), P(fT), P(fi),
                  P(self.v_img), P(self.v_alpha), quirks.backward_alpha_clamp(), self.I,
                  self.chunk, P(self.plan), self.plan.numel() if self.chunk > 0 else 0,
                  # the walk table the forward filled: only for its own final state
                  int(final_idx is None and self.chunk > 0), P(self.rec), self.rec.numel(), st)

    def raster_grads(self):
        """The records (pixel moments) -> gsplat's four raster gradients (the split kernel)."""
        P, n = _lib.ptr, self.n
        out = [torch.empty(n, k, device=self.gpu) for k in (2, 3, 3, 1)]
        _lib.call("gsplat_grad_records_split", n, P(self.rec), self.rec.numel(), P(self.conics),
                  P(self.opac), *[P(t) for t in out], _lib.stream(self.gpu))
        vis = self.radii[:, None] > 0
        return tuple(_np(torch.where(vis, t, torch.zeros_like(t))) for t in out)

    def param_grads(self):
        P, st, gpu, n, K, sc, c = _lib.ptr, _lib.stream(self.gpu), self.gpu, self.n, self.K, \
            self.sc, self.cam
        f = lambda *s: torch.empty(*s, device=gpu)
        out = [f(n, 3), f(n, 3), f(n, 4), f(n, 1), f(n, 3), f(n, K - 1, 3)]
        _lib.call("gsplat_fused_preprocess_backward", n, K, self.dtu, P(sc.means), P(sc.scales),
                  P(sc.quats), P(c.viewmat), P(c.projmat), P(self.campos), c.fx, c.fy, c.cx,
                  c.cy, self.H, self.W, P(self.radii), P(self.conics), P(self.colors),
                  P(self.opac), P(self.rec), *[P(t) for t in out[:5]],
                  P(out[5]) if K > 1 else None, None, st)
        return [_np(t) for t in out]


@pytest.fixture(scope="module", params=["headline", "c3", "c4", "c5"])
def run(request, gpu, oracle_lib):
    return FusedRun(request.param, gpu)


def _activated(sc):
    """torch's activations on the device (bit-identical to the fused kernel's: test_gpu_fused)
    as float32 numpy."""
    return (_np(torch.exp(sc.scales)), _np(sc.quats / sc.quats.norm(dim=-1, keepdim=True)))


def _tiles(run, count, seed=3):
    T = run.tb[0] * run.tb[1]
    return np.random.default_rng(seed).choice(T, size=min(count, T), replace=False).astype(np.int32)


def _mask(run, tiles):
    m = np.zeros((run.H, run.W), bool)
    for t in tiles:
        y0, x0 = (t // run.tb[0]) * 16, (t % run.tb[0]) * 16
        m[y0:y0 + 16, x0:x0 + 16] = True
    return m


def test_preprocess_and_keyed_binning(gpu, run):
    c, sc = run.cam, run.sc
    s_act, q_act = _activated(sc)
    o = O.project_forward(_np(sc.means), s_act, 1.0, q_act, _np(c.viewmat), _np(c.projmat),
                          c.fx, c.fy, c.cx, c.cy, run.H, run.W, run.tb)
    for name, g, r in zip(["xys", "depths", "radii", "conics", "num_tiles_hit"],
                          [run.xys, run.depths, run.radii, run.conics, run.nth], o[:5]):
        np.testing.assert_array_equal(_np(g), r, err_msg=name)
    I, gids, bins = bin_gaussians(run.xys, run.depths, run.radii, run.nth, run.H, run.W)
    assert I == run.I == int(o[4].astype(np.int64).sum()) > 1 << 20
    assert torch.equal(gids, run.gids) and torch.equal(bins, run.bins)


def test_blend_and_records_on_sampled_tiles(gpu, run):
    tiles = _tiles(run, 24 if run.n > 3_000_000 else 48)
    mask = _mask(run, tiles)
    img, fT, fi = run.forward()
    assert int(run.rec.view(-1, 64)[run.radii > 0].count_nonzero()) == 0  # records cleared
    xys, conics, colors, opac = (_np(t) for t in (run.xys, run.conics, run.colors, run.opac))
    bg = _np(run.bg)
    rimg, rT, ridx = O.rasterize_forward(run.tb, run.H, run.W, _np(run.gids), _np(run.bins), xys,
                                         conics, colors, opac, bg, tile_list=tiles)
    assert_close("image (sampled tiles)", _np(img)[mask], rimg[mask])
    assert_close("alpha (sampled tiles)", 1 - _np(fT)[mask], 1 - rT[mask])
    # final_idx: the integer forward state the backward walks from, bit-exact
    np.testing.assert_array_equal(_np(fi)[mask], ridx[mask], err_msg="final_idx")
    gen = torch.Generator().manual_seed(9)
    m = torch.from_numpy(mask)
    v_img = torch.randn(run.H, run.W, 3, generator=gen) * m[..., None]
    v_alpha = torch.randn(run.H, run.W, generator=gen) * m
    run.backward(v_img, v_alpha)
    got = run.raster_grads()
    ref, absum, drift, flip = O.rasterize_backward(
        run.tb, run.H, run.W, _np(run.gids), _np(run.bins), xys, conics, colors, opac, bg,
        _np(fT), _np(fi), v_img.numpy(), v_alpha.numpy(), alpha_max=quirks.backward_alpha_clamp(),
        tile_list=tiles, return_abs=True, return_drift=True, return_flip=True)
    for k, name in enumerate(("v_xy", "v_conic", "v_colors", "v_opacity")):
        assert np.abs(ref[k]).max() > 0
        assert_raster_close(f"{run.config} {name}", got[k], ref[k], absum[k], drift[k], flip[k])
    # the same backward fed the ORACLE's forward state (its final_Ts / final_idx; zero outside the
    # sampled tiles, where the upstream gradient is zero too) instead of the GPU's
    run.rec.fill_(0)
    fT_o = torch.from_numpy(np.ascontiguousarray(rT)).to(gpu)
    fi_o = torch.from_numpy(np.ascontiguousarray(ridx)).to(gpu)
    run.backward(v_img, v_alpha, final_Ts=fT_o, final_idx=fi_o)
    got_o = run.raster_grads()
    ref_o, absum_o, drift_o, flip_o = O.rasterize_backward(
        run.tb, run.H, run.W, _np(run.gids), _np(run.bins), xys, conics, colors, opac, bg, rT,
        ridx, v_img.numpy(), v_alpha.numpy(), alpha_max=quirks.backward_alpha_clamp(),
        tile_list=tiles, return_abs=True, return_drift=True, return_flip=True)
    for k, name in enumerate(("v_xy", "v_conic", "v_colors", "v_opacity")):
        assert_raster_close(f"{run.config} {name} (oracle forward state)", got_o[k], ref_o[k],
                            absum_o[k], drift_o[k], flip_o[k])


def test_fused_backward_chain_all_gaussians(gpu, run):
    """Dense upstream gradient; the fused backward's six gradients (all N) vs the oracle chain
    on the same raster-level gradients."""
    run.forward()
    gen = torch.Generator().manual_seed(11)
    run.backward(torch.randn(run.H, run.W, 3, generator=gen) * 0.1,
                 torch.randn(run.H, run.W, generator=gen) * 0.1)
    v_xy, v_conic, v_colors, v_opac = run.raster_grads()
    got = run.param_grads()
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
    # SH (gc_model.py:196-201): colours = clamp(SH(dirs) + 0.5, min=0); no viewdir gradient
    d = means - _np(run.campos)
    dirs = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    coeffs = np.concatenate([_np(sc.features_dc)[:, None], _np(sc.features_rest)], 1)
    # the clamp's backward mask: the kernel keeps it in the colour's sign bit (-0.0 = clamped),
    # which is exactly torch's clamp decision on its SH value (test_gpu_fused: bit-identical)
    passed = ~np.signbit(_np(run.colors))
    v_sh = np.where(passed & vis[:, None], v_colors, 0).astype(np.float32)
    v_coeffs = O.sh_backward(run.dtu, dirs, v_sh, run.K)
    # activation derivatives (torch's formulas), float64
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
        print(f"{run.n}: {name} max |diff| {mx:.3e}")


def test_c2_forward_full_image(gpu, oracle_lib):
    """c2 (100k @ 512², SH degree 0: sigmoid colours, forward only): the full image and alpha
    of the fused forward vs the oracle, zero outliers."""
    run = FusedRun("c2", gpu)
    img, fT, fi = run.forward()
    r = O.render_forward(_np(run.xys), _np(run.depths), _np(run.radii), _np(run.conics),
                         _np(run.nth), _np(run.colors), _np(run.opac), run.H, run.W,
                         _np(run.bg))
    assert r["num_intersects"] == run.I > 0
    np.testing.assert_array_equal(_np(run.gids), r["gaussian_ids_sorted"])
    np.testing.assert_array_equal(_np(run.bins), r["tile_bins"])
    frac, mx = close_frac(_np(img), r["img"])
    assert frac == 0, (frac, mx)
    assert_close("alpha", 1 - _np(fT), r["alpha"])
    np.testing.assert_array_equal(_np(fi), r["final_idx"], err_msg="final_idx")
    # colours are sigmoid(features_dc) (gc_model.py:203)
    np.testing.assert_array_equal(_np(run.colors), _np(torch.sigmoid(run.sc.features_dc)))
