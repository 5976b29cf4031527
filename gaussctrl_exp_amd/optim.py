"""Fused multi-tensor Adam for the Gaussian parameter groups.

The reference trains the six splatfacto parameter groups with torch.optim.Adam
(/root/reference/gaussctrl/gc_config.py:58-87, eps 1e-15; stepped at gc_trainer.py:281,298).
`FusedAdam` keeps torch.optim.Adam's `param_groups` / `step()` interface (one parameter per
group, per-group `lr` read at every step, so learning-rate schedules keep working) and takes
the step with ONE HIP launch over every group (csrc/adam.hip) instead of torch's ~6 foreach
passes.  Semantics: torch.optim.Adam(foreach=True), no weight decay, no amsgrad.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List

import torch

from . import _lib


class FusedAdam:
    def __init__(self, groups: List[Dict], betas=(0.9, 0.999), eps: float = 1e-8):
        self.param_groups = []
        for g in groups:
            params = list(g["params"])
            if len(params) != 1:
                raise ValueError("FusedAdam: one parameter tensor per group")
            p = params[0]
            if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
                raise RuntimeError("FusedAdam: parameters must be contiguous fp32 ROCm tensors "
                                   "(no CPU path)")
            d = dict(g)
            d["params"] = params
            self.param_groups.append(d)
        if len(self.param_groups) > 8:
            raise ValueError("FusedAdam: at most 8 parameter groups per launch")
        self.betas = (float(betas[0]), float(betas[1]))
        self.eps = float(eps)
        self.state = {}
        self.step_count = 0

    def _buffers(self, p):
        st = self.state.get(p)
        if st is None:
            st = self.state[p] = {"exp_avg": torch.zeros_like(p),
                                  "exp_avg_sq": torch.zeros_like(p)}
        return st

    @torch.no_grad()
    def step(self, names=None, advance: bool = True):
        """One Adam update of every group with a gradient -- or only of the groups named in
        `names`, so that a caller can update some groups while other gradients are still
        being reduced (TrainStep).  `advance=False` reuses the current step count: the
        groups of one optimisation step split over several calls share their bias
        correction, exactly as one call would."""
        live = [(g, g["params"][0]) for g in self.param_groups if g["params"][0].grad is not None
                and (names is None or g.get("name") in names)]
        if advance:
            self.step_count += 1
        if not live:
            return
        n = len(live)
        P, G, M, V = (ctypes.c_void_p * n)(), (ctypes.c_void_p * n)(), (ctypes.c_void_p * n)(), \
            (ctypes.c_void_p * n)()
        numel, lrs = (ctypes.c_int64 * n)(), (ctypes.c_float * n)()
        for k, (g, p) in enumerate(live):
            grad = p.grad
            if not grad.is_contiguous() or grad.dtype != torch.float32:
                grad = p.grad = grad.float().contiguous()
            st = self._buffers(p)
            P[k], G[k] = p.data_ptr(), grad.data_ptr()
            M[k], V[k] = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
            numel[k], lrs[k] = p.numel(), float(g["lr"])
        cast = ctypes.cast
        _lib.call("gsplat_adam_step", n, cast(P, ctypes.c_void_p), cast(G, ctypes.c_void_p),
                  cast(M, ctypes.c_void_p), cast(V, ctypes.c_void_p),
                  cast(numel, ctypes.c_void_p), cast(lrs, ctypes.c_void_p), self.step_count,
                  self.betas[0], self.betas[1], self.eps, _lib.stream(live[0][1].device))

    def fused_spec(self, params):
        """The state a kernel needs to take this optimiser's next step itself
        (gsplat_fused_preprocess_backward_adam): host arrays of the exp_avg / exp_avg_sq
        pointers and learning rates of `params` (in that order, each the only parameter of its
        group), the step number after increment, betas and eps.  Advances the step count --
        the caller must run the kernel exactly once."""
        by_param = {id(g["params"][0]): g for g in self.param_groups}
        n = len(params)
        M, V = (ctypes.c_void_p * n)(), (ctypes.c_void_p * n)()
        lrs = (ctypes.c_float * n)()
        for k, p in enumerate(params):
            g = by_param.get(id(p))
            if g is None:
                raise ValueError("fused_spec: parameter not managed by this optimiser")
            st = self._buffers(p)
            M[k], V[k] = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
            lrs[k] = float(g["lr"])
        self.step_count += 1
        return {"exp_avgs": M, "exp_avg_sqs": V, "lrs": lrs, "step": self.step_count,
                "betas": self.betas, "eps": self.eps, "params": list(params)}

    def next_step_groups(self, params):
        """[(param, exp_avg, exp_avg_sq, lr)] of `params` for the NEXT step, whose number is
        step_count + 1, without advancing the count: for a kernel that updates these groups
        itself inside this step (exchange.ShViewExchange: the SH-feature groups inside the
        multi-view table kernel) while step(names=<the others>) then advances to the same step
        number for the rest."""
        by_param = {id(g["params"][0]): g for g in self.param_groups}
        out = []
        for p in params:
            g = by_param.get(id(p))
            if g is None:
                raise ValueError("next_step_groups: parameter not managed by this optimiser")
            st = self._buffers(p)
            out.append((p, st["exp_avg"], st["exp_avg_sq"], float(g["lr"])))
        return out

    def zero_grad(self, set_to_none: bool = True):
        for g in self.param_groups:
            p = g["params"][0]
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()
