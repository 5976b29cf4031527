"""Workload statistics of the headline raster (per-tile list lengths and traversal depths)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians
from gaussctrl_exp_amd.scene import synthetic_scene

cfg = sys.argv[1] if len(sys.argv) > 1 else "headline"
N, W, H, deg, lo, hi, seed, _real, desc = bench.CONFIGS[cfg]
dev = torch.device("cuda:0")
sc = synthetic_scene(N, deg, seed=seed, scale_lo=lo, scale_hi=hi, device=dev)
cam = bench.view_camera(W, H, 0).to(dev)
with torch.no_grad():
    xys, depths, radii, conics, nth, _ = project_gaussians(
        sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
        *cam.project_args())
    I, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W)
    tb = cam.tile_bounds
    colors = torch.rand(N, 3, device=dev)
    opac = torch.sigmoid(sc.opacities).contiguous()
    out = torch.empty(H, W, 3, device=dev); fT = torch.empty(H, W, device=dev)
    fi = torch.empty(H, W, device=dev, dtype=torch.int32)
    P = _lib.ptr
    _lib.call("gsplat_rasterize_forward", tb[0], tb[1], H, W, 3, P(gids), P(bins), P(xys),
              P(conics), P(colors), P(opac), P(torch.zeros(3, device=dev)), P(out), P(fT), P(fi),
              _lib.stream(dev))
    torch.cuda.synchronize()
b = bins.cpu().numpy(); cnt = b[:, 1] - b[:, 0]
fi = fi.cpu().numpy(); fT = fT.cpu().numpy()
T = tb[0] * tb[1]
tile_of = (np.arange(H)[:, None] // 16) * tb[0] + (np.arange(W)[None, :] // 16)
depth = (fi - b[tile_of, 0] + 1).clip(0)
maxdepth = np.zeros(T); np.maximum.at(maxdepth, tile_of.ravel(), depth.ravel())
unterm = np.zeros(T); np.maximum.at(unterm, tile_of.ravel(), (fT > 1e-3).ravel().astype(float))
fwd_iters = np.where(unterm > 0, cnt, maxdepth + 1)
print(f"{cfg}: N={N} I={I} T={T} vis={(radii>0).sum().item()}")
print(f"tile count: mean {cnt.mean():.0f} p50 {np.median(cnt):.0f} p90 {np.percentile(cnt,90):.0f} max {cnt.max()}")
print(f"bwd iters/tile (max final_idx depth): mean {maxdepth.mean():.0f} max {maxdepth.max():.0f} sum {maxdepth.sum():.3e}")
print(f"fwd iters/tile (est): mean {fwd_iters.mean():.0f} sum {fwd_iters.sum():.3e}; tiles with unterminated px {unterm.mean():.2f}")
print(f"pixel depth: mean {depth.mean():.0f}; alpha mean {1-fT.mean():.3f}")
