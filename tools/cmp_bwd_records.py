"""Compare the raster backward's gradient records field by field between two backward variants
(gsplat_debug_set_raster_variant bwd_pxl; default 3 vs 1) on a bench config: per field, the
fraction of Gaussians whose records differ beyond 1e-4 relative, and a few examples."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
# the gsplat_debug_* switches live in the test library (include/gsplat_mi355x.h "test hooks")
os.environ.setdefault("GSPLAT_MI355X_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                        "..", "gaussctrl_exp_amd",
                                                        "libgsplat_mi355x_hooks.so"))
import numpy as np
import torch
import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians

cfg = os.environ.get("CFG", "c3")
A, B = [int(x) for x in os.environ.get("BWD", "3,1").split(",")]
dev = torch.device("cuda:0")
sc, cam = bench.make_workload(cfg, 0, dev)
cam = cam.to(dev)
N, H, W = sc.num_points, cam.height, cam.width
P, st = _lib.ptr, _lib.stream(dev)
with torch.no_grad():
    xys, depths, radii, conics, nth, _ = project_gaussians(
        sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
        *cam.project_args())
    I, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W)
tb = cam.tile_bounds
torch.manual_seed(0)
colors = torch.rand(N, 3, device=dev)
opac = torch.sigmoid(sc.opacities).contiguous()
bg = torch.rand(3, device=dev)
out = torch.empty(H, W, 3, device=dev); fT = torch.empty(H, W, device=dev)
fi = torch.empty(H, W, device=dev, dtype=torch.int32)
v_out = torch.randn(H, W, 3, device=dev); v_a = torch.randn(H, W, device=dev)
_lib.call("gsplat_rasterize_forward", tb[0], tb[1], H, W, 3, P(gids), P(bins), P(xys),
          P(conics), P(colors), P(opac), P(bg), P(out), P(fT), P(fi), st)
recs = {}
for v in (A, B):
    _lib.call("gsplat_debug_set_raster_variant", 1, v, 0)
    rec = torch.zeros(_lib.query("gsplat_grad_records_bytes", N), dtype=torch.uint8, device=dev)
    _lib.call("gsplat_rasterize_backward_records", tb[0], tb[1], H, W, N, P(gids), P(bins),
              P(xys), P(conics), P(colors), P(opac), P(bg), P(fT), P(fi), P(v_out), P(v_a),
              0.99, I, 0, None, 0, 0, P(rec), rec.numel(), st)
    torch.cuda.synchronize()
    recs[v] = rec.view(torch.float32).view(N, 16)[:, :9].cpu().numpy().astype(np.float64)
_lib.call("gsplat_debug_set_raster_variant", 1, 0, 0)
a, b = recs[A], recs[B]
names = ["Sx", "Sy", "Sxx", "Sxy", "Syy", "r", "g", "b", "S0"]
touched = np.abs(b).sum(1) > 0
print(f"{cfg}: N={N} I={I} touched={touched.sum()}")
for k, nm in enumerate(names):
    d = np.abs(a[:, k] - b[:, k])
    bad = d > 1e-4 * (np.abs(b[:, k]) + np.abs(b).max(1) * 1e-3) + 1e-6
    idx = np.nonzero(bad)[0]
    print(f"{nm}: bad {bad.mean():.3e} ({len(idx)})", [(int(i), round(a[i, k], 5), round(b[i, k], 5)) for i in idx[:4]])
if len(idx):
    g = int(idx[0])
    print("example Gaussian", g, "xy", xys[g].tolist(), "radius", int(radii[g]), "conic", conics[g].tolist())
