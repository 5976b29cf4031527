"""Step time with the emission pre-launched before the host's read of I vs launched after it
(rasterize.PRELAUNCH_EMISSION), alternating blocks of bench.py's step in one process (CFGS env:
comma-separated configs; median ms per step over the blocks)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from gaussctrl_exp_amd import rasterize as R  # noqa: E402
from gaussctrl_exp_amd.fused import render_fused  # noqa: E402
from gaussctrl_exp_amd.train import TrainStep  # noqa: E402

dev = torch.device("cuda:0")
for cfg in os.environ.get("CFGS", "headline,c3,c2").split(","):
    N, W, H, deg, *_ = bench.CONFIGS[cfg]
    scene, cam = bench.make_workload(cfg, 0, dev)
    cam = cam.to(dev)
    gt = torch.rand(cam.height, cam.width, 3, generator=torch.Generator().manual_seed(1)).to(dev)
    bg = torch.zeros(3, device=dev)
    t = TrainStep(scene, sh_degree=deg, world_size=1, loss="l1", render_mode="fused")
    fwd_only = cfg in bench.FORWARD_ONLY

    def step():
        if fwd_only:
            with torch.no_grad():
                render_fused(scene, cam, deg, bg)
            return
        t.zero_grad()
        t.forward_backward(cam, gt, bg)

    res = {True: [], False: []}
    for _ in range(10):
        step()
    for rnd in range(8):
        for on in (True, False) if rnd % 2 == 0 else (False, True):
            R.PRELAUNCH_EMISSION = on
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(30):
                step()
            torch.cuda.synchronize()
            res[on].append((time.perf_counter() - t0) / 30 * 1e3)
    R.PRELAUNCH_EMISSION = True
    a, b = np.median(res[True]), np.median(res[False])
    print(f"{cfg}: ms/step prelaunched {a:.4f}  after the host read {b:.4f}  ({(b / a - 1) * 100:+.1f} %)"
          f"  blocks {np.round(res[True], 4).tolist()} / {np.round(res[False], 4).tolist()}",
          flush=True)
