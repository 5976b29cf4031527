"""Data-parallel gradient exchange for one-view-per-GPU training.

Every rank renders its own camera against the same replicated Gaussians, and the optimiser
needs the sum of the per-view gradients on every rank.  Of the 236 B of gradient per
Gaussian, 192 B are the SH coefficient gradient, and for one view that block is the
rank-1 product

    v_coeffs[i, k, c] = Y_k(means[i] - campos) * v_colors[i, c]

(gsplat 0.1.2.1 sh.cuh backward; viewdirs = means - camera centre, gc_model.py:197-200).
The means are replicated, so a view's whole SH gradient is determined by its v_colors
(12 B per Gaussian) and its camera centre.  `ShViewExchange` therefore all-gathers
[v_colors | campos] from every rank (one RCCL all-gather) and evaluates
sum_r Y(means - campos_r) (x) v_colors_r with one HIP kernel
(gsplat_compute_sh_backward_views).  It sums in view order, so every rank produces
bit-identical coefficient gradients and the replicas stay in sync.  At 8 ranks each GPU
receives 7 x 12 B per Gaussian instead of ring-all-reducing 192 B (2 x 7/8 x 192 B moved).
The other 44 B per Gaussian (means, scales, quats, opacities) are still all-reduced
(train.GradExchange).

Validity: the exchange assumes the SH coefficients reach the loss only through
`spherical_harmonics` -- true for the splatfacto / GaussCtrl caller (gc_model.py:190-204),
where features_dc / features_rest are concatenated and used nowhere else.  A caller that
adds another term on the coefficients (a regulariser, say) must use the plain all-reduce
(TrainStep(grad_exchange="allreduce")).
"""
from __future__ import annotations

import contextlib
from typing import Callable, Optional

import torch
import torch.distributed as dist

_ACTIVE: Optional["ShViewExchange"] = None


def active() -> Optional["ShViewExchange"]:
    """The exchange a spherical_harmonics call made now should use in its backward."""
    return _ACTIVE


class ShViewExchange:
    def __init__(self, group=None):
        self.group = group
        self.means: Optional[torch.Tensor] = None
        self.campos: Optional[torch.Tensor] = None
        self.handled = False  # set when this step's SH gradient went through the exchange
        # the fused render's early all-reduce of the other four gradients (one flat buffer):
        # (async work, {param data_ptr: expected grad data_ptr})
        self.early = None
        self.early_steps = 0  # steps that took the early all-reduce (tests)

    @contextlib.contextmanager
    def view(self, means: torch.Tensor, campos: torch.Tensor):
        # (set before the render, so a rank whose render never reaches spherical_harmonics
        #  can still take part in the step's exchange: TrainStep._null_sh_exchange)
        """Scope of one rank's render: SH calls inside it exchange their gradients."""
        global _ACTIVE
        prev = _ACTIVE
        self.means = means.detach()
        self.campos = campos.detach().reshape(3).to(torch.float32)
        _ACTIVE = self
        try:
            yield self
        finally:
            _ACTIVE = prev

    def reset(self):
        self.handled = False
        self.early = None

    def gather(self, v_colors: torch.Tensor) -> torch.Tensor:
        """All ranks' [v_colors (3N floats) | campos (3) | pad] records, [world, 3N + 4]."""
        n = v_colors.shape[0]
        rec = torch.cat([v_colors.reshape(-1).float(), self.campos.to(v_colors.device),
                         torch.zeros(1, device=v_colors.device)])
        world = dist.get_world_size(self.group)
        out = torch.empty((world * (3 * n + 4),), device=v_colors.device, dtype=torch.float32)
        dist.all_gather_into_tensor(out, rec, group=self.group)
        return out.view(world, 3 * n + 4)

    def start_gather(self, send: torch.Tensor):
        """Issue (async) the all-gather of this rank's packed record send [3N + 4] (v_colors |
        campos | 0: gsplat_exchange_pack_colors, right after the raster backward) and return
        the pending (work, out) for reduce(gathered=...): the gather then overlaps the rest of
        the backward instead of following it."""
        world = dist.get_world_size(self.group)
        out = torch.empty((world * send.numel(),), device=send.device, dtype=torch.float32)
        work = dist.all_gather_into_tensor(out, send, group=self.group, async_op=True)
        return work, out

    def reduce(self, v_colors: Optional[torch.Tensor],
               views_backward: Callable[[torch.Tensor, torch.Tensor], torch.Tensor],
               early_flat: Optional[torch.Tensor] = None, early_map=None, gathered=None):
        """Summed coefficient gradient of all ranks' views.  `views_backward(means, views)`
        evaluates sum_r Y(means - campos_r) (x) v_colors_r from the gathered records.

        early_flat: the fused render's means/scales/quats/opacity gradients in one buffer.
        Its all-reduce is issued (async) between the all-gather and the views kernel, so the
        kernel runs while RCCL moves those 44 B per Gaussian; train.GradExchange then skips
        the four parameters (early_map: which gradient storage each parameter must hold) and
        waits for it."""
        if gathered is None:
            views = self.gather(v_colors)
        self.handled = True
        if early_flat is not None:
            self.early = (dist.all_reduce(early_flat, op=dist.ReduceOp.SUM, group=self.group,
                                          async_op=True), dict(early_map))
            self.early_steps += 1
        if gathered is not None:  # (start_gather: in flight since the raster backward)
            work, out = gathered
            work.wait()
            views = out.view(dist.get_world_size(self.group), -1)
        return views_backward(self.means, views)
