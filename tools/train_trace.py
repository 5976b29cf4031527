"""The bench's full train step (splatfacto 0.8 L1 + 0.2 SSIM loss, backward, Adam) alone, for a
kernel trace: `rocprofv3 --kernel-trace -d DIR -o run -- python3 tools/train_trace.py`, then
tools/step_timeline.py DIR/run_results.db fused_fwd_proj_kernel 5.  CFG selects the config
(default headline), STEPS the traced steps (default 30, after 40 untimed ones)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

import bench
from gaussctrl_exp_amd.train import TrainStep

cfg = os.environ.get("CFG", "headline")
steps = int(os.environ.get("STEPS", "30"))
N, W, H, deg, lo, hi, seed, _real, desc = bench.CONFIGS[cfg]
dev = torch.device("cuda:0")
scene, cam = bench.make_workload(cfg, 0, dev)
cam = cam.to(dev)
gt = torch.rand(cam.height, cam.width, 3, generator=torch.Generator().manual_seed(1000)).to(dev)
tr = TrainStep(scene, sh_degree=deg, world_size=1, loss="l1", render_mode="fused")
tr.loss_kind = "splatfacto"
for _ in range(40):
    tr.step(cam, gt)
torch.cuda.synchronize()
for _ in range(steps):
    tr.step(cam, gt)
torch.cuda.synchronize()
print(f"{cfg}: {steps} train steps traced")
