"""A/B of raster backward variants (gsplat_debug_set_raster_variant; default: the shipped 8x8
block backward vs the 16x8-strip kernel): gradient agreement and interleaved timing, on a
bench config (CFG)."""
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

cfg = os.environ.get("CFG", "headline")
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
wsz = _lib.query("gsplat_rasterize_backward_workspace_size", N, 3)
ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
amax = float(os.environ.get("AMAX", "0.99"))

def fwd():
    _lib.call("gsplat_rasterize_forward", tb[0], tb[1], H, W, 3, P(gids), P(bins), P(xys),
              P(conics), P(colors), P(opac), P(bg), P(out), P(fT), P(fi), st)

def bwd(g):
    _lib.call("gsplat_rasterize_backward", tb[0], tb[1], H, W, 3, N, P(gids), P(bins), P(xys),
              P(conics), P(colors), P(opac), P(bg), P(fT), P(fi), P(v_out), P(v_a), amax,
              *[P(x) for x in g], P(ws), wsz, st)

def timeit(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps

# VARIANTS="fwd_pxl:bwd_pxl:flags,..." (gsplat_debug_set_raster_variant) or FLAGS (bwd_pxl 2)
if os.environ.get("VARIANTS"):
    variants = [tuple(int(v) for v in x.split(":")) for x in os.environ["VARIANTS"].split(",")]
else:
    variants = [(1, int(x), 0) for x in os.environ.get("BWD", "1,2").split(",")]
fwd(); torch.cuda.synchronize()
grads = {}
for f in variants:
    _lib.call("gsplat_debug_set_raster_variant", *f)
    g = [torch.zeros(N, k, device=dev) for k in (2, 3, 3, 1)]
    bwd(g); torch.cuda.synchronize()
    grads[f] = g
ref = grads[variants[-1]]
for f in variants[:-1]:
    for name, a, b in zip(("v_xy", "v_conic", "v_rgb", "v_opac"), grads[f], ref):
        d = (a - b).abs()
        scale = b.abs().max().item()
        bad = (d > 1e-5 + 1e-4 * b.abs()).float().mean().item()
        print(f"flags {f} vs {variants[-1]} {name}: max|d| {d.max().item():.3e} "
              f"(max|g| {scale:.3e}) frac>tol {bad:.2e} finite {torch.isfinite(a).all().item()}")
res = {f: [] for f in variants}
for rnd in range(5):
    for f in variants:
        _lib.call("gsplat_debug_set_raster_variant", *f)
        g = grads[f]
        res[f].append(timeit(lambda: bwd(g)))
_lib.call("gsplat_debug_set_raster_variant", 1, 0, 0)
print(f"{cfg}: N={N} I={I} tiles={tb[0]*tb[1]}")
for f in variants:
    print(f"bwd variant={f}: {np.median(res[f]):.4f} ms  (rounds {np.round(res[f], 4).tolist()})")
