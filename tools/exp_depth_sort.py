"""Depth-sort scheme A/B inside the binning (gsplat_debug_depth_sort_wide): bin_count time
per call with the three 11-bit passes vs four 8-bit passes, same scene (CFG, default headline).
Run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians

cfg = os.environ.get("CFG", "headline")
dev = torch.device("cuda:0")
sc, cam = bench.make_workload(cfg, 0, dev)
cam = cam.to(dev)
with torch.no_grad():
    xys, depths, radii, conics, nth, _ = project_gaussians(
        sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
        *cam.project_args())
for wide in (1, 0, 1, 0):
    _lib.call("gsplat_debug_depth_sort_wide", wide)
    for _ in range(3):
        bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
    e.record(); torch.cuda.synchronize()
    print(f"{cfg} wide={wide}: bin_gaussians {s.elapsed_time(e) / 20:.4f} ms", flush=True)
_lib.call("gsplat_debug_depth_sort_wide", 0)
