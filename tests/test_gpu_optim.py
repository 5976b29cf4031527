"""Fused multi-tensor Adam (csrc/adam.hip) vs torch.optim.Adam(foreach=True)
with the reference's group learning rates (gc_config.py:58-87, eps 1e-15), over several steps
with a changing learning rate.  Bar: parameters within 1e-6 relative + 1e-7 absolute of
torch after 5 steps (fp32; the two differ only by fma contraction)."""
import pytest
import torch

from gaussctrl_exp_amd.optim import FusedAdam
from gaussctrl_exp_amd.train import GROUP_LR

SHAPES = {"means": (1000, 3), "scales": (1000, 3), "quats": (1000, 4), "opacities": (1000, 1),
          "features_dc": (1000, 3), "features_rest": (1001, 15, 3)}


@pytest.mark.gpu
def test_fused_adam_matches_torch(gpu):
    gen = torch.Generator().manual_seed(0)
    init = {k: torch.randn(*s, generator=gen) for k, s in SHAPES.items()}
    grads = [{k: torch.randn(*s, generator=gen) * 1e-3 for k, s in SHAPES.items()}
             for _ in range(5)]
    a = {k: v.clone().to(gpu).requires_grad_() for k, v in init.items()}
    b = {k: v.clone().to(gpu).requires_grad_() for k, v in init.items()}
    oa = FusedAdam([{"params": [a[k]], "lr": GROUP_LR[k], "name": k} for k in SHAPES], eps=1e-15)
    ob = torch.optim.Adam([{"params": [b[k]], "lr": GROUP_LR[k], "name": k} for k in SHAPES],
                          eps=1e-15, foreach=True)
    for step, gr in enumerate(grads):
        for opt, prm in ((oa, a), (ob, b)):
            for g in opt.param_groups:
                if g["name"] == "means":
                    g["lr"] = GROUP_LR["means"] * 0.9 ** step
            for k in SHAPES:
                prm[k].grad = gr[k].to(gpu)
            opt.step()
    for k in SHAPES:
        torch.testing.assert_close(a[k].detach(), b[k].detach(), rtol=1e-6, atol=1e-7,
                                   msg=lambda m: f"{k}: {m}")


def test_fused_adam_has_no_cpu_path():
    p = torch.zeros(4, requires_grad=True)
    with pytest.raises(RuntimeError, match="no CPU path"):
        FusedAdam([{"params": [p], "lr": 1e-3}])
