"""Shared parity machinery of the GPU tests (test infrastructure only).

The bar (BASELINE.json north_star): every rendered value and gradient within
1e-5 abs + 1e-4 rel of the oracle, with NO outliers.  Two error sources are accounted for
explicitly instead of by an outlier allowance:

* fp32 summation order.  A rasterizer gradient is a sum over pixels; gsplat (float atomics)
  and this rasterizer (wave totals + atomics) add its terms in some fp32 order, the oracle in
  double.  The difference is bounded by ~ count * 2^-24 * sum|terms|; the oracle returns
  sum|terms| per element and the bar adds 2^-20 * sum|terms| (raster level only).
* Transmittance recovery.  The backward recovers each Gaussian's T by dividing T_final back
  through every later composited Gaussian of the pixel -- gsplat with fp32 division, this
  rasterizer with the hardware reciprocal (1 ulp) -- so at the n-th division the recovered T's
  drift apart by up to ~n ulps (the list-split backward's parts re-walk the positions behind
  them with exactly the full walk's operations, so they add no drift of their own).  Per term,
  not per tile: the oracle returns
  sum over the pixel-Gaussian terms of n * |term| (with v_alpha's components in absolute value,
  since their errors need not cancel when v_alpha does), and the bar adds 2^-23 times that
  (drift_slack).  Each check reports its worst |diff| / allowed ratio (worst_ratio).
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


def worst_ratio(a, b, atol=ATOL, rtol=RTOL, abs_sum=None, extra=None):
    """max over elements of |a - b| / allowed (the bar of close_frac): how much of the slack
    the worst element uses (< 1 passes)."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    tol = atol + rtol * np.abs(b)
    if abs_sum is not None:
        tol = tol + np.asarray(abs_sum, np.float64).reshape(b.shape) * 2.0 ** -20
    if extra is not None:
        tol = tol + np.asarray(extra, np.float64).reshape(b.shape)
    return float((np.abs(a - b) / tol).max()) if a.size else 0.0


def _worst_detail(a, b, atol=ATOL, rtol=RTOL, abs_sum=None, extra=None):
    a, b = np.asarray(a, np.float64).reshape(-1), np.asarray(b, np.float64).reshape(-1)
    s = (np.asarray(abs_sum, np.float64).reshape(-1) * 2.0 ** -20 if abs_sum is not None
         else np.zeros_like(b))
    e = np.asarray(extra, np.float64).reshape(-1) if extra is not None else np.zeros_like(b)
    tol = atol + rtol * np.abs(b) + s + e
    i = int(np.nanargmax(np.abs(a - b) / tol))
    return (f"worst element {i}: got {a[i]:.9g} ref {b[i]:.9g} |diff| {abs(a[i] - b[i]):.3e} "
            f"allowed {tol[i]:.3e} (abs_sum term {s[i]:.3e}, extra {e[i]:.3e})")


def assert_close(name, a, b, **kw):
    frac, mx = close_frac(a, b, **kw)
    assert frac == 0.0, (f"{name}: {frac:.2e} of elements out of tolerance (max |diff| "
                         f"{mx:.3e}); {_worst_detail(a, b, **kw)}")
    print(f"[parity] {name}: max |diff| {mx:.3e}, worst diff/allowed {worst_ratio(a, b, **kw):.3f}")
    return mx


def drift_slack(drift_sum):
    """The transmittance-recovery slack of each element: 2^-23 * the oracle's drift sum."""
    return np.asarray(drift_sum, np.float64) * 2.0 ** -23


def assert_raster_close(name, a, b, abs_sum, drift_sum, flip_sum):
    """A raster-level gradient vs the oracle's: the bar + fp32 summation slack + per-term
    recovery drift, plus -- for the elements that need it -- what the oracle's threshold-flip
    sum allows (decisions within 1e-5 of alpha = 1/255 or sigma = 0 that another fp32
    implementation may take the other way, gsplat_oracle.c).  Reports how many elements used
    the flip allowance; zero elements outside both."""
    b = np.asarray(b, np.float64).reshape(np.shape(a))
    drift = drift_slack(drift_sum).reshape(b.shape)
    flip = np.asarray(flip_sum, np.float64).reshape(b.shape)
    frac, _ = close_frac(a, b, abs_sum=abs_sum, extra=drift)
    mx = assert_close(name, a, b, abs_sum=abs_sum, extra=drift + flip)
    if frac:
        print(f"[parity] {name}: {int(round(frac * b.size))} elements within a threshold-flip "
              f"allowance only")
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
    ref, absum, drift, flip = O.rasterize_backward(
        st["tile_bounds"], H, W, st["gids"], st["bins"], xys, conics, colors,
        np.asarray(opacity).reshape(-1), background, st["final_Ts"], st["final_idx"], v_img,
        v_alpha, alpha_max=quirks.backward_alpha_clamp(), tile_list=tile_list, return_abs=True,
        return_drift=True, return_flip=True)
    mx = {}
    for k, name in enumerate(("v_xy", "v_conic", "v_colors", "v_opacity")):
        a = np.asarray(got[k], np.float64).reshape(ref[k].shape)
        mx[name] = assert_raster_close(f"{label}{name}", a, ref[k], absum[k], drift[k], flip[k])
    return mx


def near_threshold_pixel(i, j, xys, conics, opacity, gids, bins, tbx, alpha_max=0.999,
                         rel=1e-5):
    """True if the oracle's front-to-back walk of pixel (i, j) (gsplat's forward, SURVEY A9, in
    float32 as oracle/gsplat_oracle.c evaluates it) meets a decision within `rel` of its
    threshold: sigma >= 0 with |sigma| tiny, alpha within rel of 1/255, or T (1 - alpha) within
    rel of 1e-4.  Two fp32 implementations whose sigma / exp round differently (the GPU:
    fma-ordered sigma and the hardware exp2, as gsplat's __expf; the oracle: expf) may decide
    such a Gaussian differently -- a 'threshold flip', which changes the pixel by about that
    Gaussian's alpha T colour and is the only mismatch the bar allows to be explained rather
    than bounded."""
    f = np.float32
    t = (i // 16) * tbx + j // 16
    T = f(1.0)
    for k in range(int(bins[t][0]), int(bins[t][1])):
        g = int(gids[k])
        a, b, c = (f(v) for v in conics[g])
        dx, dy = f(xys[g][0]) - f(j), f(xys[g][1]) - f(i)
        sigma = f(0.5) * (a * dx * dx + c * dy * dy) + b * dx * dy
        alpha = min(f(alpha_max), f(opacity[g]) * np.exp(-sigma, dtype=np.float32))
        if abs(float(sigma)) <= 1e-6 and float(alpha) >= 1 / 255:
            return True
        if abs(float(alpha) * 255.0 - 1.0) <= rel:
            return True
        if sigma < 0 or alpha < f(1.0 / 255.0):
            continue
        nT = T * (f(1.0) - alpha)
        if abs(float(nT) / 1e-4 - 1.0) <= rel:
            return True
        if nT <= f(1e-4):
            break
        T = nT
    return False


def assert_close_or_flip(name, img, ref, xys, conics, opacity, gids, bins, tbx, **kw):
    """assert_close on an [H, W, C] image, except that a pixel whose every out-of-bar channel
    lies on a threshold flip of the oracle's walk (near_threshold_pixel) is counted and reported
    instead of failing; returns the number of such pixels."""
    img, ref = np.asarray(img, np.float64), np.asarray(ref, np.float64)
    tol = ATOL + RTOL * np.abs(ref)
    if kw.get("extra") is not None:
        tol = tol + np.asarray(kw["extra"], np.float64).reshape(ref.shape)
    bad = ~(np.abs(img - ref) <= tol)
    pix = np.argwhere(bad.reshape(ref.shape[0], ref.shape[1], -1).any(-1))
    unexplained = [(int(i), int(j)) for i, j in pix
                   if not near_threshold_pixel(i, j, xys, conics, np.asarray(opacity).reshape(-1),
                                               gids, bins, tbx)]
    assert not unexplained, (f"{name}: {len(unexplained)} pixels out of tolerance without a "
                             f"threshold flip, e.g. {unexplained[:5]}; "
                             f"{_worst_detail(img, ref, **kw)}")
    print(f"[parity] {name}: {len(pix)} pixels differ by a threshold flip, 0 unexplained")
    return len(pix)
