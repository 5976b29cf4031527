"""Phase timestamps of the bucket binning's MSD tile-sort kernel (headline)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians
dev = torch.device("cuda:0")
sc, cam = bench.make_workload(os.environ.get("CFG", "headline"), 0, dev)
cam = cam.to(dev)
with torch.no_grad():
    xys, depths, radii, conics, nth, _ = project_gaussians(
        sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
        *cam.project_args())
_lib.call("gsplat_debug_binning_scheme", 1)
for _ in range(3):
    bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
T = cam.tile_bounds[0] * cam.tile_bounds[1]
buf = torch.zeros((T + 1) * 8, dtype=torch.int64, device=dev)
_lib.call("gsplat_debug_sort_timing", _lib.ptr(buf), 1)
bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
torch.cuda.synchronize()
_lib.call("gsplat_debug_sort_timing", None, 0)
L = buf.view(-1, 8).cpu().numpy()
L = L[L[:, 6] > 0]
t0 = L[:, 0].min()
print("tiles logged", len(L), "span us", (L[:, 6].max() - t0) / 100)
d = np.diff(L[:, :7], axis=1) / 100.0
for k, name in enumerate(["load+gather", "minmax", "hist", "scan", "scatter", "rank+write"]):
    print(f"  {name:12s} mean {d[:, k].mean():7.2f} us  p90 {np.percentile(d[:, k], 90):7.2f}")
st = (L[:, 0] - t0) / 100.0
print("  per-WG total mean", ((L[:, 6] - L[:, 0]) / 100).mean(), "starts p50/p90",
      np.median(st), np.percentile(st, 90))
