"""Same-process A/B of the work-ordered record backward (gsplat_debug_bwd_order: the shortest
P % of tiles by forward walk dispatched last) on the whole fused bench step and on the backward
kernel alone (HIP events around gsplat_rasterize_backward_records via timing.timed_calls).
CFGS (default "headline c4 c5"), PCTS (default "0 20 34 50")."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
import bench
from gaussctrl_exp_amd import _lib, timing
from gaussctrl_exp_amd.train import TrainStep

dev = torch.device("cuda:0")
L = _lib.lib()
pcts = [int(x) for x in os.environ.get("PCTS", "0 20 34 50").split()]
for cfg in os.environ.get("CFGS", "headline c4 c5").split():
    N, W, H, deg, *_ = bench.CONFIGS[cfg]
    scene, cam = bench.make_workload(cfg, 0, dev)
    cam = cam.to(dev)
    gt = torch.rand(cam.height, cam.width, 3, generator=torch.Generator().manual_seed(1)).to(dev)
    bg = torch.zeros(3, device=dev)
    tr = TrainStep(scene, sh_degree=deg, world_size=1, loss="l1", render_mode="fused")

    def step():
        tr.zero_grad()
        tr.forward_backward(cam, gt, bg)

    ref = None
    res = {p: ([], []) for p in pcts}
    for rnd in range(4):
        for p in pcts:
            L.gsplat_debug_bwd_order(p)
            for _ in range(3):
                step()
            if rnd == 0:
                g = torch.cat([t.grad.flatten() for t in tr.params])
                if ref is None:
                    ref = g.clone()
                else:
                    d = ((g - ref).abs() / (1e-6 + ref.abs().max())).max().item()
                    assert d < 1e-4, (p, d)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                step()
            e1.record(); torch.cuda.synchronize()
            res[p][0].append(e0.elapsed_time(e1) / 20)
            with timing.timed_calls() as tm:
                for _ in range(10):
                    step()
                s = tm.summary()
            res[p][1].append(s["gsplat_rasterize_backward_records"][1])
    L.gsplat_debug_bwd_order(0)
    print(f"{cfg}:", flush=True)
    for p in pcts:
        print(f"  late {p:2d}%: step {np.median(res[p][0]):.4f} ms  bwd {np.median(res[p][1]):.4f} ms",
              flush=True)
