"""Interleaved A/B timing of raster forward/backward variants on the headline scene
(HIP events on the launch stream; median over rounds; one process)."""
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
from gaussctrl_exp_amd.scene import synthetic_scene

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
colors = torch.rand(N, 3, device=dev)
opac = torch.sigmoid(sc.opacities).contiguous()
bg = torch.zeros(3, device=dev)
out = torch.empty(H, W, 3, device=dev); fT = torch.empty(H, W, device=dev)
fi = torch.empty(H, W, device=dev, dtype=torch.int32)
v_out = torch.randn(H, W, 3, device=dev); v_a = torch.randn(H, W, device=dev)
g = [torch.empty(N, k, device=dev) for k in (2, 3, 3, 1)]
wsz = _lib.query("gsplat_rasterize_backward_workspace_size", N, 3)
ws = torch.empty(wsz, dtype=torch.uint8, device=dev)

def fwd():
    _lib.call("gsplat_rasterize_forward", tb[0], tb[1], H, W, 3, P(gids), P(bins), P(xys),
              P(conics), P(colors), P(opac), P(bg), P(out), P(fT), P(fi), st)

def bwd():
    _lib.call("gsplat_rasterize_backward", tb[0], tb[1], H, W, 3, N, P(gids), P(bins), P(xys),
              P(conics), P(colors), P(opac), P(bg), P(fT), P(fi), P(v_out), P(v_a), 0.99,
              *[P(x) for x in g], P(ws), wsz, st)

def timeit(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps

# VARIANTS="fwd_pxl,bwd_pxl,flags;..." (default: the shipped one and a few ablations)
variants = [tuple(int(x) for x in v.split(",")) for v in os.environ.get(
    "VARIANTS", "1,2,0;1,2,1;1,2,64;1,4,0;1,2,32;2,2,0").split(";")]
res = {v: {"fwd": [], "bwd": []} for v in variants}
for rnd in range(5):
    for v in variants:
        _lib.call("gsplat_debug_set_raster_variant", *v)
        fwd(); torch.cuda.synchronize()
        res[v]["fwd"].append(timeit(fwd))
        res[v]["bwd"].append(timeit(bwd))
_lib.call("gsplat_debug_set_raster_variant", 1, 2, 0)
print(f"{cfg}: I={I}")
for v in variants:
    print(f"fwd_pxl={v[0]} bwd_pxl={v[1]} flags={v[2]}: fwd {np.median(res[v]['fwd']):.3f} ms"
          f"  bwd {np.median(res[v]['bwd']):.3f} ms")
