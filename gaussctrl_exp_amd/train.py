"""Multi-view data-parallel training step (one camera per GPU, RCCL gradient all-reduce).

The reference trains one camera per iteration on one device
(gaussctrl/gc_datamanager.py:213-235 -> gc_pipeline.py:469-480 -> gc_trainer.py:258-301):
render (gc_model.get_outputs) -> splatfacto loss 0.8*L1 + 0.2*(1-SSIM) -> backward ->
Adam over the six Gaussian parameter groups (gc_config.py:58-87).  Here each rank renders
its own camera of a multi-view batch against a replica of the parameters; the per-view
losses sum, so the gradients ([N x 59] fp32, 236 B/Gaussian) are summed across ranks over
RCCL/xGMI, after which every rank takes the identical Adam step.  GradExchange does the
summing: the 192 B/Gaussian SH-coefficient gradient through exchange.ShViewExchange
(all-gather of each view's 12 B/Gaussian colour gradient + camera centre, summed by one HIP
kernel on every rank), the other 44 B/Gaussian by one async all-reduce per parameter
tensor, issued as soon as autograd finishes it.  grad_exchange="allreduce" all-reduces
every tensor instead.
"""
from __future__ import annotations

import math
import os
from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F

from .camera import GCCamera
from .exchange import ShViewExchange
from .fused import direct_step_ok, render_fused
from .scene import PARAM_NAMES, GaussianScene, render

# gc_config.py:58-87 (Adam, eps 1e-15); xyz decays 1.6e-4 -> 1.6e-6 over 30k steps.
GROUP_LR = {"means": 1.6e-4, "features_dc": 0.0025, "features_rest": 0.0025 / 20,
            "opacities": 0.05, "scales": 0.005, "quats": 0.001}
XYZ_LR_FINAL, XYZ_MAX_STEPS = 1.6e-6, 30000
SSIM_LAMBDA = 0.2  # splatfacto SplatfactoModelConfig.ssim_lambda


def _gauss_window(size=11, sigma=1.5, device="cpu"):
    coords = torch.arange(size, dtype=torch.float32, device=device) - size // 2
    g = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
    return g / g.sum()


def ssim(x, y, data_range=1.0, win_size=11, sigma=1.5, k1=0.01, k2=0.03):
    """pytorch_msssim.ssim semantics (separable Gaussian window, 'valid' convolution,
    size_average): x, y [B,C,H,W]."""
    C = x.shape[1]
    w = _gauss_window(win_size, sigma, x.device).to(x.dtype)  # pytorch_msssim: win.to(X.dtype)

    def filt(t):
        t = F.conv2d(t, w.view(1, 1, 1, -1).expand(C, 1, 1, -1), groups=C)
        return F.conv2d(t, w.view(1, 1, -1, 1).expand(C, 1, -1, 1), groups=C)

    c1, c2 = (k1 * data_range) ** 2, (k2 * data_range) ** 2
    mu1, mu2 = filt(x), filt(y)
    s11 = filt(x * x) - mu1 * mu1
    s22 = filt(y * y) - mu2 * mu2
    s12 = filt(x * y) - mu1 * mu2
    cs = (2 * s12 + c2) / (s11 + s22 + c2)
    m = ((2 * mu1 * mu2 + c1) / (mu1 * mu1 + mu2 * mu2 + c1)) * cs
    return m.flatten(2).mean(-1).mean()


def splatfacto_loss(pred, gt):
    """0.8 * L1 + 0.2 * (1 - SSIM) on [H,W,3] images (nerfstudio splatfacto get_loss_dict)."""
    l1 = torch.abs(gt - pred).mean()
    sim = 1 - ssim(gt.permute(2, 0, 1)[None], pred.permute(2, 0, 1)[None])
    return (1 - SSIM_LAMBDA) * l1 + SSIM_LAMBDA * sim


SH_GROUPS = ("features_dc", "features_rest")


def FusedAdamType():
    from .optim import FusedAdam
    return FusedAdam


class GradExchange:
    """Sums every parameter's gradient over the data-parallel ranks (RCCL over xGMI).

    After backward, one async all-reduce per parameter tensor in a fixed (parameter) order,
    then one wait: every rank issues the same collective sequence whatever its own graph
    looked like -- a rank whose view saw no Gaussians (the caller's early background return,
    gc_model.py:189-190) contributes zero gradients instead of skipping collectives and
    hanging the others.  The gradients are reduced in place (the tensors autograd produced:
    no flat bucket to zero-fill and accumulate into).  With an ShViewExchange (`sh`), the
    SH-coefficient parameters (`sh_params`) are skipped in a step whose SH backward already
    produced the all-rank sum through the exchange."""

    def __init__(self, params: List[torch.Tensor], group=None,
                 sh: Optional[ShViewExchange] = None, sh_params=()):
        self.params = list(params)
        self.group = group
        self.sh = sh
        self.sh_ids = {id(p) for p in sh_params}

    def start(self):
        """Issue this step's all-reduces (async); returns the handles for finish()."""
        works = []
        early = self.sh.early if self.sh is not None else None
        if early is not None:
            works.append(early[0])
        for p in self.params:
            if self.sh is not None and self.sh.handled and id(p) in self.sh_ids:
                continue  # already summed over the ranks by the SH view exchange
            if early is not None and p.data_ptr() in early[1]:
                # all-reduced in place by the fused backward (exchange.ShViewExchange.reduce):
                # autograd must have kept that buffer as the gradient
                if p.grad is None or p.grad.data_ptr() != early[1][p.data_ptr()]:
                    raise RuntimeError("GradExchange: a gradient the fused backward all-reduced "
                                       "early is not the parameter's .grad (was it accumulated "
                                       "into an existing gradient?)")
                continue
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            works.append(dist.all_reduce(p.grad, op=dist.ReduceOp.SUM, group=self.group,
                                         async_op=True))
        return works

    def finish(self, works):
        for w in works:
            w.wait()
        if self.sh is not None:
            self.sh.reset()

    def sh_done(self) -> bool:
        """True when the SH-coefficient gradients are already the all-rank sums."""
        return self.sh is not None and self.sh.handled

    def wait(self):
        self.finish(self.start())


class TrainStep:
    """render -> loss -> backward -> [all-reduce] -> Adam, on this rank's camera."""

    def __init__(self, scene: GaussianScene, sh_degree: int = 3, world_size: int = 1,
                 loss: str = "splatfacto", group=None, api=None,
                 grad_exchange: str = "sh_views", render_mode: str = "caller",
                 fuse_adam: bool = True, sparse_exchange: str = "auto"):
        if render_mode not in ("caller", "fused"):
            raise ValueError(f"render_mode must be 'caller' or 'fused', not {render_mode}")
        if render_mode == "fused" and (api is not None or not scene.means.is_cuda):
            raise ValueError("render_mode='fused' runs the MI355X kernels only (no api override, "
                             "ROCm tensors)")
        # "caller": scene.render, the reference caller's torch glue around the gsplat API
        # (gc_model.py:158-238, what gc_model.py runs through the drop-in); "fused": the same
        # step with that glue inside the HIP kernels (fused.render_fused)
        self.render_mode = render_mode
        # single-GPU fused steps take the Adam update inside the backward kernel
        # (gsplat_fused_preprocess_backward_adam): no gradient tensors are written or re-read
        self.fuse_adam = bool(fuse_adam) and render_mode == "fused" and world_size == 1
        # N > 1: the SH-feature groups' Adam step fused into the multi-view SH table kernel
        # (GSPLAT_MI355X_FUSE_SH_ADAM=0: the table kernel's gradients + the multi-tensor Adam)
        self.fuse_sh_adam = bool(fuse_adam) and world_size > 1 and os.environ.get(
            "GSPLAT_MI355X_FUSE_SH_ADAM", "1") != "0"
        # the fused render computes an L1 loss inside its blend kernels (loss="l1"); off:
        # the separate loss kernels (GSPLAT_MI355X_FUSE_L1=0, A/B runs)
        self.fuse_l1 = render_mode == "fused" and os.environ.get("GSPLAT_MI355X_FUSE_L1",
                                                                 "1") != "0"
        self.scene = scene.requires_grad_()
        self.params = scene.params()
        self.world_size = world_size
        if grad_exchange not in ("sh_views", "allreduce"):
            raise ValueError(f"grad_exchange must be 'sh_views' or 'allreduce', not {grad_exchange}")
        # sparse_exchange: "auto" sends only the visible Gaussians' colour gradients when that
        # record is clearly smaller (exchange.py); "on" / "off" force it (tests)
        self.sh_exchange = ShViewExchange(group, sparse=sparse_exchange) if world_size > 1 and \
            grad_exchange == "sh_views" else None
        self.grad_sync = GradExchange(
            self.params, group, sh=self.sh_exchange,
            sh_params=(scene.features_dc, scene.features_rest)) if world_size > 1 else None
        self.group = group
        self.sh_degree = sh_degree
        self.loss_kind = loss
        self.api = api  # gsplat implementation override (tests: CPU-oracle emulation)
        groups = [{"params": [getattr(scene, k)], "lr": GROUP_LR[k], "name": k}
                  for k in PARAM_NAMES]
        if api is None and scene.means.is_cuda:
            from .optim import FusedAdam
            self.opt = FusedAdam(groups, eps=1e-15)  # csrc/adam.hip, one launch per step
        else:  # CPU-oracle emulation (tests): torch's Adam, same semantics
            self.opt = torch.optim.Adam(groups, eps=1e-15, foreach=True)
        self.step_count = 0

    def _xyz_lr(self):
        t = min(self.step_count / XYZ_MAX_STEPS, 1.0)
        return math.exp(math.log(GROUP_LR["means"]) * (1 - t) + math.log(XYZ_LR_FINAL) * t)

    def loss(self, pred, gt, clamp_pred: bool = False):
        """Photometric loss of the rendered image.  clamp_pred: `pred` is the raw render and the
        loss applies the caller's clamp(max=1) itself (gc_model.py:222) -- folded into the HIP
        loss kernels, so the clamped image is never materialised."""
        fused = self.api is None and pred.is_cuda
        if clamp_pred and not (fused and self.loss_kind in ("l1", "splatfacto")):
            pred, clamp_pred = torch.clamp(pred, max=1.0), False
        if self.loss_kind == "l1":
            if fused:  # csrc/loss.hip, ssim_lambda = 0 fast path
                from .loss import fused_splatfacto_loss
                return fused_splatfacto_loss(pred, gt, 0.0, clamp_pred)
            return torch.abs(gt - pred).mean()
        if self.loss_kind == "splatfacto_torch" or not fused:
            return splatfacto_loss(pred, gt)  # torch restatement (CPU-emulation tests)
        from .loss import fused_splatfacto_loss
        return fused_splatfacto_loss(pred, gt, SSIM_LAMBDA, clamp_pred)

    def zero_grad(self):
        for p in self.params:
            p.grad = None
        if self.sh_exchange is not None:
            self.sh_exchange.reset()

    def sync_grads(self):
        """Wait for this step's gradient all-reduces (no-op on one rank)."""
        if self.grad_sync is not None:
            self.grad_sync.wait()

    def flat_grad(self) -> torch.Tensor:
        return torch.cat([p.grad.reshape(-1) for p in self.params])

    def _render(self, cam: GCCamera, background: torch.Tensor, adam=None, gt=None):
        if self.render_mode == "fused":  # raw image: the loss applies the clamp
            # the L1 loss folded into the blend kernels (fused.render_fused l1_gt) unless
            # fuse_l1 is off; with it, the forward and backward are called directly (no
            # autograd graph: out["backward"], fused.direct_step_ok)
            l1 = gt if (self.loss_kind == "l1" and self.fuse_l1 and gt is not None) else None
            # (the direct step's loss: the fused L1 in the blend, or the fused L1 + SSIM kernels
            # called directly as well, forward_backward)
            direct = gt is not None and (l1 is not None or self.loss_kind == "splatfacto") and \
                direct_step_ok(self.scene)
            return render_fused(self.scene, cam, self.sh_degree, background, clamp=False,
                                adam=adam, l1_gt=l1, direct=direct)
        return render(self.scene, cam, self.sh_degree, background, api=self.api)

    def forward_backward(self, cam: GCCamera, gt: torch.Tensor, background: torch.Tensor,
                         adam=None, view: int = 0, of: int = 1):
        """Render, loss and backward of one view -- view `view` of this rank's `of` views this
        step (forward_backward_views)."""
        if self.sh_exchange is not None:
            with self.sh_exchange.view(self.scene.means, cam.c2w[..., :3, 3], view, of):
                out = self._render(cam, background, gt=gt)
        else:
            out = self._render(cam, background, adam=adam, gt=gt)
        loss = out.get("loss")
        direct = out.get("backward")
        if direct is not None:  # the fused render's direct step (no autograd graph)
            if loss is None:  # the L1 + SSIM loss kernels, called directly as well
                from .loss import fused_splatfacto_loss_and_grad
                loss, v_img = fused_splatfacto_loss_and_grad(out["rgb"], gt, SSIM_LAMBDA,
                                                             not out.get("clamped", True))
                direct(v_img)
            else:  # the L1 loss inside the blend
                direct()
            return loss, out
        if loss is None:
            loss = self.loss(out["rgb"], gt, clamp_pred=not out.get("clamped", True))
        if loss.requires_grad:
            # a kept ones() seed: autograd's own seed is a fill kernel per step
            seed = getattr(self, "_seed", None)
            if seed is None or seed.device != loss.device or seed.dtype != loss.dtype or \
                    seed.shape != loss.shape:
                seed = self._seed = torch.ones_like(loss)
            loss.backward(seed)
        elif self.sh_exchange is not None and self.scene.features_rest.shape[1] > 0:
            # no Gaussian in view (the caller returned the background): no local gradient,
            # but the other ranks' SH exchange still needs this rank's (zero) record
            self._null_sh_exchange()
        return loss, out

    def forward_backward_views(self, cams: List[GCCamera], gts: List[torch.Tensor],
                               background: torch.Tensor):
        """Several views per rank in one step (gradients summed over this rank's views and
        all ranks'): with the fused render under the view exchange, each view's record
        all-gather stays in flight while the next view renders, and only the last view's
        exchange is exposed (exchange.py).  Returns the summed loss."""
        if len(cams) != len(gts) or not cams:
            raise ValueError("forward_backward_views: one ground truth per camera")
        if len(cams) > 1 and self.sh_exchange is not None and self.render_mode != "fused":
            raise ValueError("forward_backward_views: several views per rank under the view "
                             "exchange need render_mode='fused'")
        total = 0.0
        for k, (cam, gt) in enumerate(zip(cams, gts)):
            loss, _ = self.forward_backward(cam, gt, background, view=k, of=len(cams))
            total = total + loss.detach()
        return total

    def _null_sh_exchange(self):
        sc = self.scene
        n, K = sc.num_points, sc.features_rest.shape[1] + 1
        degree = {1: 0, 4: 1, 9: 2, 16: 3, 25: 4}[K]
        zeros = torch.zeros(n, 3, device=sc.means.device)
        if self.api is None:
            from .sh import sh_backward_views
            fn = lambda means, views: sh_backward_views(degree, self.sh_degree, means, views)
        else:
            fn = lambda means, views: self.api.sh_backward_views(degree, self.sh_degree, means,
                                                                 views)
        v = self.sh_exchange.reduce(zeros, fn)
        sc.features_dc.grad = v[:, 0, :].contiguous()
        sc.features_rest.grad = v[:, 1:, :].contiguous()

    def step(self, cam, gt, background: Optional[torch.Tensor] = None,
             optimizer: bool = True):
        """One training step (gc_trainer.py:258-301 / gc_pipeline.py:469-480): render, the
        splatfacto loss, backward, gradient exchange (N > 1) and Adam.  cam / gt may be lists:
        several views per rank, their gradients summed (forward_backward_views)."""
        multi = isinstance(cam, (list, tuple))
        if background is None:
            background = torch.rand(3, device=(gt[0] if multi else gt).device)
        if optimizer:
            for g in self.opt.param_groups:
                if g["name"] == "means":
                    g["lr"] = self._xyz_lr()
        if optimizer and not multi and self.fuse_adam and isinstance(self.opt, FusedAdamType()) and \
                all(p.dtype == torch.float32 and p.is_contiguous() for p in self.params):
            # the backward takes the Adam step (one kernel instead of gradient tensors + step)
            self.zero_grad()
            spec = self.opt.fused_spec(self.params)
            loss, out = self.forward_backward(cam, gt, background, adam=spec)
            self.step_count += 1
            return loss
        self.zero_grad()
        xc = self.sh_exchange
        if optimizer and xc is not None and self.fuse_sh_adam and \
                isinstance(self.opt, FusedAdamType()):
            # N > 1: the SH-feature groups' Adam step inside the multi-view table kernel
            # (exchange.reduce_views; gsplat_compute_sh_backward_view_table_adam) at the step
            # number the other groups' step below advances to
            xc.adam = {"groups": self.opt.next_step_groups(
                [self.scene.features_dc, self.scene.features_rest]),
                "step": self.opt.step_count + 1, "betas": self.opt.betas, "eps": self.opt.eps}
        if multi:
            loss = self.forward_backward_views(list(cam), list(gt), background)
        else:
            loss, out = self.forward_backward(cam, gt, background)
        if not optimizer:
            self.sync_grads()
            return loss
        gs = self.grad_sync
        if gs is not None and xc is not None and xc.adam_applied:
            # the SH groups are updated; the geometry all-reduce overlapped the table kernel
            gs.wait()
            self.opt.step(names=[n for n in PARAM_NAMES if n not in SH_GROUPS])
            self.step_count += 1
            return loss
        if xc is not None:
            xc.adam = None  # (not consumed: the caller path / degree-0 steps sum gradients)
        if gs is not None and gs.sh_done() and isinstance(self.opt, FusedAdamType()):
            # the SH-feature gradients (81 % of the update's bytes) are final: update them
            # while the other groups' all-reduces are in flight, then the rest
            works = gs.start()
            self.opt.step(names=SH_GROUPS)
            gs.finish(works)
            self.opt.step(names=[n for n in PARAM_NAMES if n not in SH_GROUPS], advance=False)
        else:
            self.sync_grads()
            self.opt.step()
        self.step_count += 1
        return loss
