"""Shared parity machinery of the GPU tests (test infrastructure only).

The bar (BASELINE.json north_star): every rendered value and gradient within
1e-5 abs + 1e-4 rel of the oracle, with NO outliers.  Two error sources are accounted for
explicitly instead of by an outlier allowance:

* fp32 summation order.  A rasterizer gradient is a sum over pixels; gsplat (float atomics)
  and this rasterizer (wave totals + atomics) add its terms in some fp32 order, the oracle in
  double.  The difference is bounded by ~ count * 2^-24 * sum|terms|; the oracle returns
  sum|terms| per element and the bar adds 2^-20 * sum|terms| (raster level only).
* Transmittance recovery.  The backward recovers each Gaussian's T by dividing T_final back
  through every later Gaussian of the tile's list -- gsplat with fp32 division, this rasterizer
  with the hardware reciprocal (1 ulp) -- so recovered T's drift apart by up to ~L ulps for a
  list of length L (the list-split backward restarts T from the forward's checkpoints instead,
  which is within the same bound).  The bar adds L_max * 2^-23 * sum|terms|, L_max the longest
  list among the tiles that contribute (recovery_drift).
* Propagation of that slack.  End to end, the parameter gradients are the projection / SH /
  activation VJPs of the raster-level gradients.  The end-to-end check therefore splits in two:
  (1) the GPU's raster-level gradients (captured at the rasterizer's inputs) vs the oracle's
  raster backward on the same forward state, with the slack above; (2) the GPU's parameter
  gradients vs the oracle-backed caller fed with THOSE raster-level gradients (injected), so the
  rest of the chain is compared without the summation-order noise, again with zero outliers.
"""
from __future__ import annotations

import numpy as np
import torch

import oracle as O
import oracle_gsplat as OG
from gaussctrl_exp_amd import _lib, quirks
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians, rasterize_gaussians
from gaussctrl_exp_amd.sh import spherical_harmonics

ATOL, RTOL = 1e-5, 1e-4


def np_(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


def close_frac(a, b, atol=ATOL, rtol=RTOL, abs_sum=None, extra=None):
    """(fraction of elements with |a - b| > atol + rtol |b| [+ 2^-20 abs_sum] [+ extra], max
    |a - b|).  NaN counts as out of tolerance."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    tol = atol + rtol * np.abs(b)
    if abs_sum is not None:
        tol = tol + np.asarray(abs_sum, np.float64).reshape(b.shape) * 2.0 ** -20
    if extra is not None:
        tol = tol + np.asarray(extra, np.float64).reshape(b.shape)
    bad = ~(np.abs(a - b) <= tol)
    return (bad.mean() if bad.size else 0.0), (np.abs(a - b).max() if a.size else 0.0)


def assert_close(name, a, b, **kw):
    frac, mx = close_frac(a, b, **kw)
    assert frac == 0.0, f"{name}: {frac:.2e} of elements out of tolerance (max |diff| {mx:.3e})"
    return mx


class CaptureAPI:
    """The MI355X gsplat API, with the gradient-carrying rasterize call's inputs, upstream
    gradients (v_img, v_alpha) and raster-level gradients (into xys, conics, colors, opacity)
    captured as numpy arrays after backward."""

    def __init__(self):
        self.cap = {}
        self.project_gaussians = project_gaussians
        self.spherical_harmonics = spherical_harmonics

    def rasterize_gaussians(self, xys, depths, radii, conics, nth, colors, opacity, H, W,
                            background=None, return_alpha=False):
        out = rasterize_gaussians(xys, depths, radii, conics, nth, colors, opacity, H, W,
                                  background=background, return_alpha=return_alpha)
        if not torch.is_grad_enabled() or not colors.requires_grad:
            return out
        c = self.cap
        c.update(xys_in=np_(xys), depths=np_(depths), radii=np_(radii), conics_in=np_(conics),
                 nth=np_(nth), colors_in=np_(colors), opacity_in=np_(opacity).reshape(-1),
                 background=np_(background), H=H, W=W)

        def grab(key):
            def hook(g):
                if g is not None:  # an output the loss does not use may see an undefined grad
                    c[key] = np_(g)
            return hook
        for key, t in (("xys", xys), ("conics", conics), ("colors", colors),
                       ("opacity", opacity)):
            if t.requires_grad:
                t.register_hook(grab(key))
        img, alpha = out if return_alpha else (out, None)
        img.register_hook(grab("v_img"))
        if alpha is not None:
            alpha.register_hook(grab("v_alpha"))
        return out

    def raster_grads(self, n):
        c = self.cap
        z = lambda *s: np.zeros(s, np.float32)
        return [c.get("xys", z(n, 2)), c.get("conics", z(n, 3)), c.get("colors", z(n, 3)),
                c.get("opacity", z(n, 1))]


def injected_api(raster_grads):
    """The oracle-backed gsplat API whose rasterize backward returns the given raster-level
    gradients (v_xy, v_conic, v_colors, v_opacity) instead of its own: the projection, SH and
    caller-glue backward of the oracle chain run on exactly the GPU's raster gradients."""
    inj = [torch.from_numpy(np.ascontiguousarray(g, np.float32)) for g in raster_grads]

    class _RasterInjected(torch.autograd.Function):
        forward = staticmethod(OG._Raster.forward)

        @staticmethod
        def backward(ctx, v_img, v_alpha=None):
            return (inj[0].reshape(-1, 2), None, None, inj[1].reshape(-1, 3), None,
                    inj[2].reshape(-1, 3), inj[3].reshape(ctx.opacity_shape), None, None, None,
                    None)

    class API:
        project_gaussians = staticmethod(OG.project_gaussians)
        spherical_harmonics = staticmethod(OG.spherical_harmonics)
        sh_backward_views = staticmethod(OG.sh_backward_views)

        @staticmethod
        def rasterize_gaussians(xys, depths, radii, conics, nth, colors, opacity, H, W,
                                background=None, return_alpha=False):
            if background is None:
                background = torch.ones(colors.shape[-1])
            return _RasterInjected.apply(xys, depths, radii, conics, nth, colors, opacity, H, W,
                                         background, return_alpha)
    return API


def gpu_forward_state(gpu, xys, depths, radii, conics, nth, colors, opacity, background, H, W):
    """final_Ts / final_idx / image of the MI355X forward (plain entry) on the given inputs,
    plus the binning -- the state the backward ran from."""
    d = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).to(gpu, dt)
    xys_d, dep_d, conics_d = d(xys), d(depths), d(conics)
    radii_d, nth_d = d(radii, torch.int32), d(nth, torch.int32)
    col_d, op_d, bg_d = d(colors), d(np.asarray(opacity).reshape(-1)), d(background)
    I, gids, bins = bin_gaussians(xys_d, dep_d, radii_d, nth_d, H, W)
    tb = ((W + 15) // 16, (H + 15) // 16)
    out = torch.empty(H, W, 3, device=gpu)
    fT = torch.empty(H, W, device=gpu)
    fi = torch.empty(H, W, device=gpu, dtype=torch.int32)
    P = _lib.ptr
    _lib.call("gsplat_rasterize_forward", tb[0], tb[1], H, W, 3, P(gids), P(bins), P(xys_d),
              P(conics_d), P(col_d), P(op_d), P(bg_d), P(out), P(fT), P(fi), _lib.stream(gpu))
    return dict(I=I, gids=np_(gids), bins=np_(bins), img=np_(out), final_Ts=np_(fT),
                final_idx=np_(fi), tile_bounds=tb)


def recovery_drift(bins, tile_list=None) -> float:
    """L_max * 2^-23: the relative transmittance-recovery drift bound (module docstring) for the
    longest list among `tile_list` (default: all tiles) of tile_bins `bins`."""
    b = np.asarray(bins)
    if tile_list is not None:
        b = b[np.asarray(tile_list)]
    return float((b[:, 1] - b[:, 0]).max()) * 2.0 ** -23 if b.size else 0.0


def check_raster_level(gpu, xys, depths, radii, conics, nth, colors, opacity, background, H, W,
                       v_img, v_alpha, got, tile_list=None, label=""):
    """The GPU's raster-level gradients `got` (v_xy, v_conic, v_colors, v_opacity) vs the
    oracle's rasterize backward on the GPU's own forward state, zero outliers under the bar plus
    the fp32 summation slack and the transmittance-recovery drift (module docstring).
    Returns the max |diff| per field."""
    st = gpu_forward_state(gpu, xys, depths, radii, conics, nth, colors, opacity, background, H,
                           W)
    if v_alpha is None or np.asarray(v_alpha).dtype == object:
        v_alpha = np.zeros((H, W), np.float32)
    ref, absum = O.rasterize_backward(st["tile_bounds"], H, W, st["gids"], st["bins"], xys,
                                      conics, colors, np.asarray(opacity).reshape(-1),
                                      background, st["final_Ts"], st["final_idx"], v_img,
                                      v_alpha, alpha_max=quirks.backward_alpha_clamp(),
                                      tile_list=tile_list, return_abs=True)
    drift = recovery_drift(st["bins"], tile_list)
    mx = {}
    for k, name in enumerate(("v_xy", "v_conic", "v_colors", "v_opacity")):
        a = np.asarray(got[k], np.float64).reshape(ref[k].shape)
        mx[name] = assert_close(f"{label}{name}", a, ref[k], abs_sum=absum[k],
                                extra=drift * np.asarray(absum[k], np.float64))
    return mx
