"""Fused training render: the reference caller's glue and gsplat's three calls in four HIP
kernel groups (csrc/preprocess.hip, binning.hip, raster.hip).

GaussCtrlModel.get_outputs (/root/reference/gaussctrl/gc_model.py:158-222) turns the raw
splatfacto parameters into gsplat's inputs with ~10 torch ops -- cat of the SH features
(:172), exp(scales) (:177), quats / |quats| (:178), viewdirs (:197-198), SH + clamp (:200-201)
or sigmoid(dc) (:203), sigmoid(opacities) (:215) -- then calls project_gaussians (:174),
spherical_harmonics (:200) and rasterize_gaussians (:208) and clamps the image (:222).
`render_fused` computes the same image and the same six parameter gradients with

  forward:  gsplat_fused_preprocess_forward_part [1] (activations + projection + the
            binning's depth keys and records) with [2] (SH + clamp) on a second stream from
            3,584 tiles (else gsplat_fused_preprocess_forward_binned, one kernel) ->
            gsplat_bin_speculative (depth sort + tile sort launched at the capacity learned
            from the frame shape's earlier calls: no host read of the intersection count before
            the blend; the first call: gsplat_bin_count_keyed_ex / gsplat_bin_emit) ->
            gsplat_rasterize_forward_clearing(_l1) (the blend, which also zeroes the
            backward's per-Gaussian gradient records and, with the L1 loss, sums it)
  backward: gsplat_rasterize_backward_records(_l1) -> gsplat_fused_preprocess_backward(_adam)
            (projection VJP + SH backward + the activations' chain rule, one kernel)

so none of the glue's elementwise kernels, reductions, the cat, its backward's strided copies
or the caller's `radii.sum() == 0` host sync remain.  Results equal the unchanged-caller path
(scene.render) within fp32 rounding of the activations; tests/test_gpu_fused.py holds both
against the CPU oracle.  The unchanged caller (gc_model.py through the gsplat shim) is still
the drop-in; this is the framework's own training step (TrainStep(render_mode="fused")).
"""
from __future__ import annotations

import ctypes
import os
import weakref
from typing import Optional

import torch
from torch import Tensor
from torch.autograd import Function

from . import _lib, exchange, quirks
from .camera import GCCamera
from .rasterize import (BLOCK_X, BLOCK_Y, SPEC_STATS, bin_gaussians, bin_gaussians_speculative,
                        speculative_capacity, last_num_visible)

_DEG_OF_BASES = {1: 0, 4: 1, 9: 2, 16: 3, 25: 4}

# How the last forward binned: "speculative" (capacity-launched, no host read), "host" (the
# scheme needs I on the host first) or "sync" (first call of the frame shape)
LAST_BINNING = {"mode": None}
# the preprocess's SH-colour part on a second stream, overlapping the binning
# (gsplat_fused_preprocess_forward_part); GSPLAT_MI355X_SPLIT_COLOURS=0: one kernel (A/B runs)
SPLIT_COLOURS = os.environ.get("GSPLAT_MI355X_SPLIT_COLOURS", "1") != "0"
SPLIT_COLOURS_MIN_TILES = 3584  # (the blend kernels' small-frame threshold as well)
_SIDE = {}


def _side_stream(dev) -> torch.cuda.Stream:
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return s


class _FusedRender(Function):
    @staticmethod
    def forward(ctx, means, scales, quats, opacities, features_dc, features_rest, viewmat,
                projmat, campos, fx, fy, cx, cy, H, W, degrees_to_use, background,
                return_alpha, aux, adam=None, l1_gt=None):
        # l1_gt [H,W,3]: the render returns (loss, image) instead -- loss = mean |clamp(image,
        # max=1) - l1_gt| (splatfacto's L1 with ssim_lambda 0 on gc_model.py:222's clamped
        # image) computed by the blend, whose backward forms the image gradient per pixel
        # (gsplat_rasterize_forward_clearing_l1 / _backward_records_l1): no loss kernels
        n = means.shape[0]
        K = 1 + features_rest.shape[1]
        if K not in _DEG_OF_BASES or features_dc.shape != (n, 3) or \
                features_rest.shape[-1] != 3 or means.shape != (n, 3):
            raise ValueError("render_fused: bad parameter shapes")
        if not 0 <= degrees_to_use <= _DEG_OF_BASES[K]:
            raise ValueError(f"render_fused: degrees_to_use {degrees_to_use} > layout degree")
        dev = _lib.check_device("render_fused", means, scales, quats, opacities, features_dc,
                                features_rest, viewmat, projmat, campos, background)
        H, W = int(H), int(W)
        tbx, tby = (W + BLOCK_X - 1) // BLOCK_X, (H + BLOCK_Y - 1) // BLOCK_Y
        f32 = dict(device=dev, dtype=torch.float32)
        # the seven per-Gaussian outputs carved from one allocation (12 words per Gaussian: one
        # caching-allocator call instead of seven, ~1.5 us of host time each -- the small frames'
        # step is bound by the host path)
        slab = torch.empty((12 * n,), **f32)
        xys, depths = slab[:2 * n].view(n, 2), slab[2 * n:3 * n]
        radii = slab[3 * n:4 * n].view(torch.int32)
        conics = slab[4 * n:7 * n].view(n, 3)
        nth = slab[7 * n:8 * n].view(torch.int32)
        colors, opac = slab[8 * n:11 * n].view(n, 3), slab[11 * n:12 * n]
        # (needs_input_grad ignores the caller's grad mode: a render under torch.no_grad -- the
        # forward-only bench step, an eval render -- keeps no records, plan or walk table)
        need_grad = any(ctx.needs_input_grad[:6]) and aux.get("grad_mode", True)
        rec = torch.empty((max(_lib.query("gsplat_grad_records_bytes", n), 1),), device=dev,
                          dtype=torch.uint8) if need_grad else None
        P, st = _lib.ptr, _lib.stream(dev)
        # the preprocess kernel also writes the binning's depth-sort inputs into its workspace
        ws1 = torch.empty((max(_lib.query("gsplat_bin_count_workspace_size", n), 1),),
                          device=dev, dtype=torch.uint8)
        cam_args = (P(viewmat), P(projmat), P(campos), float(fx), float(fy), float(cx),
                    float(cy), H, W, tbx, tby, 0.01)
        # (frames from SPLIT_COLOURS_MIN_TILES tiles: on small frames the second stream's
        # event work costs the host more than the overlap saves -- c3 step 0.371 -> 0.402 ms)
        split_colours = K > 1 and SPLIT_COLOURS and tbx * tby >= SPLIT_COLOURS_MIN_TILES

        def preprocess():
            """The preprocess; with split_colours its SH-colour part goes out on a second
            stream (joined before the blend, join_colours) and overlaps the binning."""
            if not split_colours:
                _lib.call("gsplat_fused_preprocess_forward_binned", n, K, int(degrees_to_use),
                          P(means), P(scales), P(quats), P(opacities), P(features_dc),
                          P(features_rest) if K > 1 else None, *cam_args, P(xys), P(depths),
                          P(radii), P(conics), P(nth), P(colors), P(opac), P(ws1), ws1.numel(),
                          st)
                return
            colours_part()
            _lib.call("gsplat_fused_preprocess_forward_part", 1, n, K, int(degrees_to_use),
                      P(means), P(scales), P(quats), P(opacities), P(features_dc),
                      P(features_rest), *cam_args, P(xys), P(depths), P(radii), P(conics),
                      P(nth), None, P(opac), P(ws1), ws1.numel(), st)

        joined = [True]  # the step's stream has waited for the latest colour part

        def colours_part():
            cur = torch.cuda.current_stream(dev)
            side = _side_stream(dev)
            side.wait_stream(cur)
            joined[0] = False
            _lib.call("gsplat_fused_preprocess_forward_part", 2, n, K, int(degrees_to_use),
                      P(means), None, None, None, P(features_dc), P(features_rest), *cam_args,
                      None, None, None, None, None, P(colors), None, None, 0, side.cuda_stream)

        def join_colours():
            # once per colour part: a second cross-stream wait (the blend joins, then the end of
            # the forward would again) costs the device a barrier packet for nothing
            if split_colours and not joined[0]:
                torch.cuda.current_stream(dev).wait_stream(_side_stream(dev))
                joined[0] = True
        # every output and scratch buffer of the forward is allocated before the first launch,
        # so the preprocess, the binning and the blend go out back to back (the host's work
        # between them left the GPU idle: ~24 us before the blend at c3)
        visible_hint = last_num_visible(dev)
        chunk, plan = 0, None
        if l1_gt is not None:
            if l1_gt.shape != (H, W, 3) or return_alpha:
                raise ValueError("render_fused: the L1 loss needs gt [H, W, 3] and no alpha")
            l1_gt = _contig_f32(l1_gt)
            l1_part = torch.empty((_lib.query("gsplat_rasterize_l1_partials_bytes", tbx, tby)
                                   // 4,), **f32)
            loss = torch.empty((), **f32)
        # (image, final T and final index: one allocation too)
        pix = torch.empty((5 * H * W,), **f32)
        out_img = pix[:3 * H * W].view(H, W, 3)
        final_Ts = pix[3 * H * W:4 * H * W].view(H, W)
        final_idx = pix[4 * H * W:].view(torch.int32).view(H, W)

        def plan_for(layout_i):
            """(chunk, plan buffer) of the list-split plan laid out for layout_i intersections."""
            c = _lib.query("gsplat_rasterize_chunk_size", tbx, tby, layout_i)
            if not need_grad or c == 0:  # (the plan is the backward's)
                return 0, None
            return c, torch.empty((_lib.query("gsplat_rasterize_split_bytes", tbx, tby,
                                              layout_i, c),), device=dev, dtype=torch.uint8)
        # the speculative binning's layout is its capacity, known now
        spec_cap = speculative_capacity(n, H, W, dev)
        prepared = (spec_cap, plan_for(spec_cap)) if spec_cap > 0 else None

        preprocess()
        # data-parallel view exchange: this view's sparse-record bitmap and the ranks' visible
        # counts (async all-gather), as soon as radii exist (exchange.ShViewExchange.plan)
        xchg = exchange.active() if K > 1 and need_grad and adam is None else None
        if xchg is not None:
            xchg.plan(n, radii, st)
        # The binning's emission and tile sort are launched at this frame shape's capacity
        # without the host read of I (rasterize.SpeculativeBinning), the blend right behind
        # them; the host reads I only then, while the GPU works, and re-bins on an overflow.
        spec = bin_gaussians_speculative(xys, depths, radii, nth, H, W, keyed_workspace=ws1)
        LAST_BINNING["mode"] = "sync" if spec is None else (
            "speculative" if spec.slot is not None else "host")
        SPEC_STATS["sync" if spec is None else "speculative"] += 1
        if spec is None:  # first call of this frame shape (or nothing to bin)
            num_intersects, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W,
                                                       keyed_workspace=ws1)
            layout_i = num_intersects
        else:
            num_intersects, gids, bins = None, spec.ids, spec.tile_bins
            layout_i = spec.layout_intersects

        def blend(gids, bins, layout_i):
            """The blend (it also clears the gradient records the backward accumulates into and
            fills the list-split plan, whose layout follows layout_i)."""
            nonlocal chunk, plan
            join_colours()
            if prepared is not None and prepared[0] == layout_i:
                chunk, plan = prepared[1]
            else:
                chunk, plan = plan_for(layout_i)
            args = (tbx, tby, H, W, P(gids), P(bins), P(xys), P(conics), P(colors), P(opac),
                    P(background), P(out_img), P(final_Ts), P(final_idx), P(rec),
                    rec.numel() if rec is not None else 0,
                    # skip culled Gaussians' records when many are culled (real scenes);
                    # at ~all visible the radii loads cost more than the stores they save
                    P(radii) if rec is not None and visible_hint < 0.9 * n else None,
                    layout_i, chunk, P(plan), plan.numel() if plan is not None else 0)
            if l1_gt is None:
                _lib.call("gsplat_rasterize_forward_clearing", *args, st)
            else:
                _lib.call("gsplat_rasterize_forward_clearing_l1", *args, P(l1_gt), 1, P(l1_part),
                          4 * l1_part.numel(), P(loss), st)

        if spec is not None:
            blend(gids, bins, layout_i)
            if not spec.finish():
                SPEC_STATS["range" if spec.range_violated else "overflow"] += 1
                if spec.range_violated:
                    # a depth digit the sort assumed constant varied: the sort consumed its
                    # keys, so the (deterministic) preprocess writes them again; full binning
                    preprocess()
                    num_intersects, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W,
                                                               keyed_workspace=ws1)
                    layout_i = num_intersects
                else:  # I > capacity: the blend saw empty tiles; bin and blend again
                    gids, bins = spec.rebin()
                    layout_i = spec.layout_intersects
                    num_intersects = spec.num_intersects
                if num_intersects >= 1:
                    blend(gids, bins, layout_i)
            else:
                num_intersects = spec.num_intersects
                gids = gids[:num_intersects]
        elif num_intersects >= 1:
            blend(gids, bins, layout_i)
        # the colours are saved for the backward and returned in aux: the side-stream kernel
        # must have finished even when no blend ran (nothing visible) to join it
        join_colours()
        if num_intersects < 1:
            # nothing visible: the background (the caller returns it at gc_model.py:189-190),
            # and every gradient is zero
            out_img = torch.ones(H, W, 3, **f32) * background
            final_Ts = torch.ones(H, W, **f32)
            final_idx = torch.zeros(H, W, device=dev, dtype=torch.int32)
            if rec is not None:
                rec.zero_()
            chunk, plan = 0, None
            if l1_gt is not None:  # (the blend did not run: the background's loss)
                from .loss import fused_splatfacto_loss
                with torch.no_grad():
                    loss = fused_splatfacto_loss(out_img, l1_gt, 0.0, True)
        ctx.meta = (n, K, int(degrees_to_use), float(fx), float(fy), float(cx), float(cy), H, W,
                    tbx, tby, num_intersects, chunk, layout_i)
        ctx.plan, ctx.rec = plan, rec
        ctx.opac_shape = opacities.shape
        ctx.exchange = xchg
        # data-parallel: all-reduce the four non-SH gradients from inside the backward (one flat
        # buffer, overlapping the SH views kernel) when autograd will hand them over as the
        # parameters' .grad (no gradient to accumulate into)
        ctx.early = ctx.exchange is not None and all(
            t.is_leaf and t.grad is None for t in (means, scales, quats, opacities))
        if adam is not None:
            if ctx.exchange is not None:
                raise ValueError("render_fused: the in-backward Adam step is single-GPU only")
            for p, q in zip(adam["params"], (means, scales, quats, opacities, features_dc,
                                             features_rest)):
                if p.data_ptr() != q.data_ptr():
                    raise ValueError("render_fused: in-backward Adam needs the parameters "
                                     "themselves (contiguous fp32), not copies")
        ctx.adam = adam
        ctx.save_for_backward(means, scales, quats, opacities, features_dc, features_rest,
                              viewmat, projmat, campos,
                              background, xys, radii, conics, colors, opac, gids, bins, final_Ts,
                              final_idx)
        ctx.set_materialize_grads(False)
        ctx.l1 = (out_img, l1_gt) if l1_gt is not None else None
        aux.update(xys=xys, radii=radii, depths=depths, num_intersects=num_intersects,
                   records=rec, num_points=n, conics=conics, colors=colors, opacity=opac,
                   num_tiles_hit=nth, gaussian_ids_sorted=gids, tile_bins=bins,
                   final_Ts=final_Ts, final_idx=final_idx, binning=LAST_BINNING["mode"])
        if l1_gt is not None:
            ctx.mark_non_differentiable(out_img)
            return loss, out_img
        if return_alpha:
            return out_img, 1 - final_Ts
        return out_img

    @staticmethod
    def backward(ctx, v_img, v_alpha=None):
        (means, scales, quats, opacities, features_dc, features_rest, viewmat, projmat, campos,
         background, xys, radii, conics, colors, opac, gids, bins, final_Ts,
         final_idx) = ctx.saved_tensors
        n, K, dtu, fx, fy, cx, cy, H, W, tbx, tby, I, chunk, layout_i = ctx.meta
        dev = means.device
        P, st = _lib.ptr, _lib.stream(dev)
        rec = ctx.rec
        if ctx.l1 is not None:  # (loss, image): v_img is the loss's gradient, v_alpha unused
            g_loss, v_img, v_alpha = v_img, None, None
            if I >= 1 and g_loss is not None:
                pred, gt = ctx.l1
                _lib.call("gsplat_rasterize_backward_records_l1", tbx, tby, H, W, n, P(gids),
                          P(bins), P(xys), P(conics), P(colors), P(opac), P(background),
                          P(final_Ts), P(final_idx), P(pred), P(gt), 1,
                          P(g_loss.float().contiguous()), quirks.backward_alpha_clamp(),
                          layout_i if chunk > 0 else I, chunk, P(ctx.plan),
                          ctx.plan.numel() if ctx.plan is not None else 0,
                          int(ctx.plan is not None), P(rec), rec.numel(), st)
        elif I >= 1 and (v_img is not None or v_alpha is not None):
            v_img = v_img.float().contiguous() if v_img is not None else \
                torch.zeros((H, W, 3), device=dev, dtype=torch.float32)
            if v_alpha is not None:
                v_alpha = v_alpha.float().contiguous()
            _lib.call("gsplat_rasterize_backward_records", tbx, tby, H, W, n, P(gids), P(bins),
                      P(xys), P(conics), P(colors), P(opac), P(background), P(final_Ts),
                      P(final_idx), P(v_img), P(v_alpha), quirks.backward_alpha_clamp(),
                      layout_i if chunk > 0 else I, chunk,
                      P(ctx.plan), ctx.plan.numel() if ctx.plan is not None else 0,
                      int(ctx.plan is not None), P(rec), rec.numel(), st)
        if ctx.adam is not None:
            # Adam inside the backward: parameters (and moments) updated in place, no gradients
            a = ctx.adam
            cast = ctypes.cast
            head = (n, K, dtu, P(means), P(scales), P(quats), P(opacities), P(features_dc),
                    P(features_rest) if K > 1 else None, P(viewmat), P(projmat), P(campos),
                    fx, fy, cx, cy, H, W, P(radii), P(conics), P(colors), P(opac), P(rec),
                    cast(a["exp_avgs"], ctypes.c_void_p), cast(a["exp_avg_sqs"], ctypes.c_void_p))
            tail = (float(a["betas"][0]), float(a["betas"][1]), float(a["eps"]), st)
            _lib.call("gsplat_fused_preprocess_backward_adam", *head,
                      cast(a["lrs"], ctypes.c_void_p), int(a["step"]), *tail)
            return (None,) * 21
        f32 = dict(device=dev, dtype=torch.float32)
        xchg = ctx.exchange
        if xchg is not None and rec is not None:
            return _exchange_backward(ctx, xchg, rec, st)
        v_means = torch.empty((n, 3), **f32)
        v_scales = torch.empty((n, 3), **f32)
        v_quats = torch.empty((n, 4), **f32)
        v_opac = torch.empty((n, 1), **f32)
        v_dc = torch.empty((n, 3), **f32)
        v_rest = torch.empty((n, K - 1, 3), **f32)
        _lib.call("gsplat_fused_preprocess_backward", n, K, dtu, P(means), P(scales), P(quats),
                  P(viewmat), P(projmat), P(campos), fx, fy, cx, cy, H, W, P(radii), P(conics),
                  P(colors), P(opac), P(rec), P(v_means), P(v_scales), P(v_quats), P(v_opac),
                  P(v_dc), P(v_rest) if K > 1 else None, None, st)
        return (v_means, v_scales, v_quats, v_opac.view(ctx.opac_shape), v_dc, v_rest) + \
            (None,) * 15


def _exchange_backward(ctx, xchg, rec, st):
    """The fused backward under the data-parallel view exchange (exchange.ShViewExchange).  Right
    after the raster backward this view's colour-gradient record is packed from the records and
    its all-gather issued (it overlaps the geometry backward, and -- several views per rank --
    the rank's next views).  The geometry gradients go to one flat buffer [11 N] (summed over
    the rank's views: gsplat_fused_preprocess_backward_accumulate).  The last view of the step
    issues the flat all-reduce (async: it overlaps the views kernel; train.GradExchange waits)
    and evaluates every gathered record; earlier views return no gradient."""
    (means, scales, quats, opacities, features_dc, features_rest, viewmat, projmat, campos,
     background, xys, radii, conics, colors, opac, gids, bins, final_Ts,
     final_idx) = ctx.saved_tensors
    n, K, dtu, fx, fy, cx, cy, H, W = ctx.meta[:9]
    P = _lib.ptr
    dev = means.device
    if not ctx.early and xchg.views_per_step > 1:
        raise RuntimeError("render_fused: several views per rank need the four geometry "
                           "parameters without a .grad (zero_grad before the step's first view)")
    xchg.send_view(n, rec, radii, colors, st)
    first = xchg.geo is None
    if first:
        xchg.geo = torch.empty((11 * n,), device=dev, dtype=torch.float32)
    flat = xchg.geo
    v_means, v_scales = flat[:3 * n].view(n, 3), flat[3 * n:6 * n].view(n, 3)
    v_quats, v_opac = flat[6 * n:10 * n].view(n, 4), flat[10 * n:].view(n, 1)
    v_colors = torch.empty((n, 3), device=dev, dtype=torch.float32)
    head = (n, K, dtu, P(means), P(scales), P(quats), P(viewmat), P(projmat), P(campos), fx, fy,
            cx, cy, H, W, P(radii), P(conics), P(colors), P(opac), P(rec), P(v_means),
            P(v_scales), P(v_quats), P(v_opac))
    if first:
        _lib.call("gsplat_fused_preprocess_backward", *head, None, None, P(v_colors), st)
    else:
        _lib.call("gsplat_fused_preprocess_backward_accumulate", *head, P(v_colors), st)
    if not xchg.last_view:
        return (None,) * 21
    xchg.geo = None
    if ctx.early:  # (else autograd accumulates into existing grads: GradExchange reduces them)
        xchg.all_reduce_early(flat, {p.data_ptr(): g.data_ptr() for p, g in zip(
            (means, scales, quats, opacities), (v_means, v_scales, v_quats, v_opac))})
    v_dc, v_rest = xchg.reduce_views(_DEG_OF_BASES[K], dtu)
    return (v_means, v_scales, v_quats, v_opac.view(ctx.opac_shape), v_dc, v_rest) + \
        (None,) * 15


def sh_backward_views_split(degree: int, degrees_to_use: int, means: Tensor, views: Tensor):
    """(v_features_dc [N,3], v_features_rest [N,K-1,3]) = sum_r Y(means - campos_r) (x)
    v_colors_r over the gathered view records (exchange.ShViewExchange)."""
    n = means.shape[0]
    means = means.float().contiguous()
    views = views.float().contiguous()
    dev = _lib.check_device("sh_backward_views_split", means, views)
    K = {0: 1, 1: 4, 2: 9, 3: 16, 4: 25}[degree]
    v_dc = torch.empty((n, 3), device=dev, dtype=torch.float32)
    v_rest = torch.empty((n, K - 1, 3), device=dev, dtype=torch.float32)
    _lib.call("gsplat_compute_sh_backward_views_split", n, degree, int(degrees_to_use),
              views.shape[0], _lib.ptr(means), _lib.ptr(views), views.shape[1], _lib.ptr(v_dc),
              _lib.ptr(v_rest) if K > 1 else None, _lib.stream(dev))
    return v_dc, v_rest


def _contig_f32(t: Tensor) -> Tensor:
    return t if (t.dtype == torch.float32 and t.is_contiguous()) else t.float().contiguous()


# The camera centre c2w[:3, 3] is a strided column: contiguous, it is a copy kernel (and ~30 us
# of host time) per render.  One cached copy per camera pose, reused while the very same c2w
# tensor (weak reference) is unmodified (version counter) -- as rasterize.py's binning cache.
_CAMPOS = [None, -1, None]


def _campos(cam: GCCamera) -> Tensor:
    c2w = cam.c2w
    ref, version, t = _CAMPOS
    if ref is not None and ref() is c2w and version == c2w._version:
        return t
    t = _contig_f32(c2w[..., :3, 3].reshape(3))
    _CAMPOS[:] = [weakref.ref(c2w), c2w._version, t]
    return t


class _DirectCtx:
    """The context _FusedRender.forward / backward read and write, for a training step that
    calls the two back to back without an autograd graph (render_fused(direct=True)): the same
    kernels and gradients, without Function.apply, the saved-tensor bookkeeping, the engine's
    hand-off to its device thread and AccumulateGrad -- ~100 us of host time per step, which is
    what bounds the small frames' step (c3: host 0.41 ms per step against 0.26 ms of kernels,
    tools/host_timeline.py)."""

    def __init__(self, needs_input_grad):
        self.needs_input_grad = needs_input_grad
        self.saved_tensors = ()

    def save_for_backward(self, *tensors):
        self.saved_tensors = tensors

    def set_materialize_grads(self, value):
        pass

    def mark_non_differentiable(self, *tensors):
        pass


# the training step calls the fused forward and backward directly (TrainStep); "0": through
# autograd (A/B runs)
DIRECT_STEP = os.environ.get("GSPLAT_MI355X_DIRECT_STEP", "1") != "0"
_UNIT = {}


def _unit_grad(dev) -> Tensor:
    """A kept scalar 1.0: the loss's own gradient (autograd's seed is a fill kernel per step)."""
    t = _UNIT.get(dev)
    if t is None:
        t = _UNIT[dev] = torch.ones((), device=dev, dtype=torch.float32)
    return t


def _has_grad_hooks(t: Tensor) -> bool:
    """A gradient hook a caller registered on the parameter (register_hook /
    register_post_accumulate_grad_hook): autograd runs it, the direct step would not."""
    return bool(getattr(t, "_backward_hooks", None)) or \
        bool(getattr(t, "_post_accumulate_grad_hooks", None))


def direct_step_ok(scene) -> bool:
    """render_fused(direct=True) takes the parameters' gradients itself: it needs them as the
    contiguous fp32 leaves the kernels read (no copy for autograd to route a gradient through),
    and no gradient hooks on them (the direct step assigns .grad without running hooks, so a
    hooked parameter takes the autograd path)."""
    return DIRECT_STEP and all(
        t.is_leaf and t.dtype == torch.float32 and t.is_contiguous() and not _has_grad_hooks(t)
        for t in (scene.means, scene.scales, scene.quats, scene.opacities, scene.features_dc,
                  scene.features_rest))


def render_fused(scene, cam: GCCamera, sh_degree_to_use: int, background: Tensor,
                 return_alpha: bool = False, clamp: bool = True, adam=None,
                 l1_gt: Optional[Tensor] = None, direct: bool = False):
    """scene.render's training output (gc_model.py:158-222) through the fused kernels.

    Returns dict(rgb [H,W,3] (clamped at 1 as gc_model.py:222 -- or, clamp=False, the raw
    image for a loss that applies the clamp itself: loss.fused_splatfacto_loss(clamp_pred=True)),
    accumulation [H,W,1] or None,
    xys [N,2] and radii [N] (detached), xys_grad: callable returning v_xy [N,2] after
    backward -- what splatfacto's densification reads from `xys.grad`).
    adam: optim.FusedAdam.fused_spec(params) of the six parameters -- the backward then takes
    that Adam step itself (gsplat_fused_preprocess_backward_adam: parameters updated in place,
    no .grad); single-GPU only.
    l1_gt [H,W,3]: also return "loss" = mean |clamp(rgb, max=1) - l1_gt| (the training step's
    L1, splatfacto's loss at ssim_lambda 0), computed by the blend kernel; the loss is the
    differentiable output (its backward forms the image gradient inside the rasterizer
    backward) and "rgb" is the detached raw image (clamp ignored).
    direct (direct_step_ok(scene), no alpha): no autograd graph -- the outputs are detached and
    "backward" is a callable that runs the fused backward once and accumulates the six
    gradients into the parameters' .grad as autograd's backward would (TrainStep's step): of
    d loss / d loss = 1 (or its argument) with l1_gt, else of its argument, d image [H,W,3]
    (loss.fused_splatfacto_loss_and_grad)."""
    # the caller's grad mode (inside Function.forward it is always off); the direct step runs
    # its forward under no_grad but does take a backward
    aux = {"grad_mode": bool(direct) or torch.is_grad_enabled()}
    args = [_contig_f32(scene.means), _contig_f32(scene.scales), _contig_f32(scene.quats),
            _contig_f32(scene.opacities), _contig_f32(scene.features_dc),
            _contig_f32(scene.features_rest), _contig_f32(cam.viewmat), _contig_f32(cam.projmat),
            _campos(cam), cam.fx, cam.fy, cam.cx, cam.cy, cam.height, cam.width,
            int(sh_degree_to_use), _contig_f32(background), bool(return_alpha), aux, adam,
            l1_gt]
    backward = None
    if direct:
        if return_alpha or not direct_step_ok(scene):
            raise ValueError("render_fused(direct=True) needs contiguous fp32 leaf parameters "
                             "without gradient hooks (direct_step_ok) and no alpha output")
        if l1_gt is None and clamp:
            # the returned image would be clamp(rgb, max=1) while backward(grad) feeds grad to the
            # rasterizer as the raw image's gradient, dropping the clamp's zero-gradient mask
            raise ValueError("render_fused(direct=True) without l1_gt returns the raw image: "
                             "pass clamp=False (and apply the clamp in the loss)")
        params = args[:6]
        ctx = _DirectCtx(tuple(t.requires_grad for t in params) + (False,) * 15)
        with torch.no_grad():
            out = _FusedRender.forward(ctx, *args)

        def backward(grad: Optional[Tensor] = None):
            """The step's backward (once): d loss -> the parameters' .grad (accumulated)."""
            nonlocal ctx
            if ctx is None:
                raise RuntimeError("render_fused(direct=True): backward already ran")
            c, ctx = ctx, None
            if not any(c.needs_input_grad[:6]):
                return
            if l1_gt is not None:  # d loss: 1 unless given
                g = _unit_grad(out[0].device) if grad is None else grad
            elif grad is None:
                raise ValueError("render_fused(direct=True) without l1_gt: backward needs the "
                                 "image gradient")
            else:  # d image
                g = grad
            with torch.no_grad():
                grads = _FusedRender.backward(c, g, None)
                for p, gp in zip(params, grads[:6]):
                    if gp is None or not p.requires_grad:
                        continue
                    if p.grad is None:
                        p.grad = gp
                    else:
                        p.grad += gp
    elif not torch.is_grad_enabled():
        # no graph is recorded anyway: the forward without Function.apply's bookkeeping (~10 us
        # of host time; the forward-only bench step and eval renders are host-bound at c2)
        out = _FusedRender.forward(_DirectCtx((False,) * 21), *args)
    else:
        out = _FusedRender.apply(*args)
    loss = None
    if l1_gt is not None:
        loss, img = out
        alpha, rgb, clamp = None, img, False
    else:
        img, alpha = (out if return_alpha else (out, None))
        rgb = torch.clamp(img, max=1.0) if clamp else img

    def split_records():
        """The records (pixel moments, include/gsplat_mi355x.h) -> gsplat's four rasterize
        gradients by gsplat_grad_records_split; zero for culled Gaussians."""
        rec = aux.get("records")
        if rec is None:
            return None
        n, dev = aux["num_points"], rec.device
        out = [torch.empty(n, k, device=dev) for k in (2, 3, 3, 1)]
        P = _lib.ptr
        _lib.call("gsplat_grad_records_split", n, P(rec), rec.numel(), P(aux["conics"]),
                  P(aux["opacity"]), *[P(t) for t in out], _lib.stream(dev))
        vis = aux["radii"][:, None] > 0
        return [torch.where(vis, t, torch.zeros_like(t)) for t in out]

    def xys_grad() -> Optional[Tensor]:
        g = split_records()
        return None if g is None else g[0]

    def raster_grads():
        """After backward: the rasterizer-level gradients in gsplat's convention -- v_xy [N,2],
        v_conic [N,3] (v_conic.y per the CONIC_HALF quirk), v_colors [N,3], v_opacity [N,1] --
        i.e. what gsplat's rasterize_gaussians backward returns for this render; zero for
        culled Gaussians.  None without records (no gradient requested)."""
        g = split_records()
        return None if g is None else tuple(g)

    return {"rgb": rgb, "clamped": bool(clamp), "loss": loss, "backward": backward,
            "accumulation": alpha[..., None] if alpha is not None else None,
            "xys": aux["xys"], "radii": aux["radii"], "xys_grad": xys_grad,
            "raster_grads": raster_grads,
            # the rasterizer's inputs as the fused preprocess wrote them (the colours carry
            # the clamp mask in their sign bit: -0.0, which no rasterizer sum can see)
            "raster_inputs": {k: aux[k] for k in ("xys", "depths", "radii", "conics",
                                                   "num_tiles_hit", "colors", "opacity")},
            # the binning and the blend's final state, as the backward consumes them (tests)
            "raster_state": {k: aux[k] for k in ("gaussian_ids_sorted", "tile_bins", "final_Ts",
                                                  "final_idx", "binning")},
            "num_intersects": aux["num_intersects"]}


@torch.no_grad()
def render_fused_eval(scene, cam: GCCamera, sh_degree_to_use: int, background: Tensor):
    """The eval render of gc_model.get_outputs (gc_model.py:158-238: RGB, alpha and the depth
    image of the second rasterize call, depth / alpha with 1000 where alpha == 0) from one
    fused preprocess kernel, one binning and one RGB+depth traversal
    (gsplat_rasterize_forward_rgbd).  Bit-identical to scene.render(..., return_depth=True,
    fused_depth=True), whose inputs the caller's torch glue prepares.  Used by the eval /
    render_reverse path (gc_pipeline.py:228, gc_render.py:196-203)."""
    n = scene.means.shape[0]
    params = [_contig_f32(t) for t in (scene.means, scene.scales, scene.quats, scene.opacities,
                                       scene.features_dc, scene.features_rest)]
    K = 1 + params[5].shape[1]
    if K not in _DEG_OF_BASES or not 0 <= sh_degree_to_use <= _DEG_OF_BASES[K]:
        raise ValueError("render_fused_eval: bad SH layout / degree")
    viewmat, projmat = _contig_f32(cam.viewmat), _contig_f32(cam.projmat)
    campos, background = _contig_f32(cam.c2w[..., :3, 3].reshape(3)), _contig_f32(background)
    dev = _lib.check_device("render_fused_eval", *params, viewmat, projmat, campos, background)
    H, W = cam.height, cam.width
    tbx, tby = (W + BLOCK_X - 1) // BLOCK_X, (H + BLOCK_Y - 1) // BLOCK_Y
    f32 = dict(device=dev, dtype=torch.float32)
    xys, depths, conics = torch.empty((n, 2), **f32), torch.empty((n,), **f32), \
        torch.empty((n, 3), **f32)
    colors, opac = torch.empty((n, 3), **f32), torch.empty((n,), **f32)
    radii = torch.empty((n,), device=dev, dtype=torch.int32)
    nth = torch.empty((n,), device=dev, dtype=torch.int32)
    P, st = _lib.ptr, _lib.stream(dev)
    ws1 = torch.empty((max(_lib.query("gsplat_bin_count_workspace_size", n), 1),), device=dev,
                      dtype=torch.uint8)
    _lib.call("gsplat_fused_preprocess_forward_binned", n, K, int(sh_degree_to_use),
              *[P(t) for t in params[:5]], P(params[5]) if K > 1 else None, P(viewmat),
              P(projmat), P(campos), float(cam.fx), float(cam.fy), float(cam.cx), float(cam.cy),
              H, W, tbx, tby, 0.01, P(xys), P(depths), P(radii), P(conics), P(nth), P(colors),
              P(opac), P(ws1), ws1.numel(), st)
    num_intersects, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W,
                                               keyed_workspace=ws1)
    if num_intersects < 1:  # nothing visible: the caller's early return (gc_model.py:189-190)
        return {"rgb": background.repeat(H, W, 1), "depth": None, "accumulation": None,
                "xys": xys, "radii": radii}
    out_img = torch.empty((H, W, 3), **f32)
    depth_im = torch.empty((H, W, 1), **f32)
    final_Ts = torch.empty((H, W), **f32)
    final_idx = torch.empty((H, W), device=dev, dtype=torch.int32)
    _lib.call("gsplat_rasterize_forward_rgbd", tbx, tby, H, W, P(gids), P(bins), P(xys),
              P(conics), P(colors), P(depths), P(opac), P(background), P(out_img), P(depth_im),
              P(final_Ts), P(final_idx), st)
    alpha = (1 - final_Ts)[..., None]
    rgb = torch.clamp(out_img, max=1.0)
    depth_im[alpha > 0] = depth_im[alpha > 0] / alpha[alpha > 0]
    depth_im[alpha == 0] = 1000
    return {"rgb": rgb, "depth": depth_im, "accumulation": alpha, "xys": xys, "radii": radii}
