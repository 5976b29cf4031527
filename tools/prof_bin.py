"""Binning only, headline scene, for rocprofv3 --kernel-trace --stats."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import bench
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians
from gaussctrl_exp_amd.scene import synthetic_scene

cfg = os.environ.get("CFG", "headline")
N, W, H, deg, lo, hi, seed, _real, desc = bench.CONFIGS[cfg]
dev = torch.device("cuda:0")
sc = synthetic_scene(N, deg, seed=seed, scale_lo=lo, scale_hi=hi, device=dev)
cam = bench.view_camera(W, H, 0).to(dev)
with torch.no_grad():
    xys, depths, radii, conics, nth, _ = project_gaussians(
        sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
        *cam.project_args())
    for _ in range(10):
        I, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W)
    torch.cuda.synchronize()
print("I", I)
