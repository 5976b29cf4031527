"""Binning schemes A/B (gsplat_debug_binning_scheme): bit-exact agreement of
gaussian_ids_sorted / tile_bins between tile bucketing and the sorted scheme, and the time of
bin_gaussians (both phases and the host read of I) per config."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians

dev = torch.device("cuda:0")
for cfg in os.environ.get("CFGS", "headline,c4,c3,c2,c5").split(","):
    sc, cam = bench.make_workload(cfg, 0, dev)
    cam = cam.to(dev)
    H, W = cam.height, cam.width
    with torch.no_grad():
        xys, depths, radii, conics, nth, _ = project_gaussians(
            sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
            *cam.project_args())
    out = {}
    times = {0: [], 1: []}
    for rnd in range(6):
        for scheme in [int(x) for x in os.environ.get("SCHEMES", "1,0").split(",")]:
            _lib.call("gsplat_debug_binning_scheme", scheme | (int(os.environ.get("BKDBG", "0")) << 1 if scheme else 0))
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            r = bin_gaussians(xys, depths, radii, nth, H, W)
            e.record()
            torch.cuda.synchronize()
            times[scheme].append(s.elapsed_time(e))
            out[scheme] = r
    _lib.call("gsplat_debug_binning_scheme", 1)
    if len(out) < 2:
        continue
    (I1, g1, b1), (I0, g0, b0) = out[1], out[0]
    same = I1 == I0 and torch.equal(g1, g0) and torch.equal(b1, b0)
    lens = (b0[:, 1] - b0[:, 0]).cpu()
    print(f"{cfg}: I={I0} tiles={b0.shape[0]} max list {int(lens.max())} | bit-exact {same} | "
          f"bucket {np.median(times[1][1:]):.4f} ms  sorted {np.median(times[0][1:]):.4f} ms",
          flush=True)
    if not same:
        print("  I", I1, I0, "gids diff", (g1 != g0).sum().item() if g1.shape == g0.shape else "shape",
              "bins diff", (b1 != b0).sum().item())
