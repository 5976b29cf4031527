"""Binning scheme A/B per config (same process): bin_gaussians per call (events around 20
calls) with the shipped dispatch, the depth sort + tile sort forced, and the tile buckets
forced (gsplat_debug_binning_scheme -1 / 0 / 1); outputs must stay identical.  CFGS env
(default "c2 c3 headline")."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
# the gsplat_debug_* switches live in the test library (include/gsplat_mi355x.h "test hooks")
os.environ.setdefault("GSPLAT_MI355X_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                        "..", "gaussctrl_exp_amd",
                                                        "libgsplat_mi355x_hooks.so"))
import torch
import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians

dev = torch.device("cuda:0")
OPTS = {"shipped": [], "sorted": [("gsplat_debug_binning_scheme", 0, -1)],
        "bucket": [("gsplat_debug_binning_scheme", 1, -1)]}
for cfg in os.environ.get("CFGS", "c2 c3 headline").split():
    sc, cam = bench.make_workload(cfg, 0, dev)
    cam = cam.to(dev)
    with torch.no_grad():
        xys, depths, radii, conics, nth, _ = project_gaussians(
            sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
            *cam.project_args())
    del sc
    ref = None
    for name, sets in OPTS.items():
        for fn, on, _ in sets:
            getattr(_lib.lib(), fn)(on)
        for _ in range(3):
            out = bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
        if ref is None:
            ref = out
        same = out[0] == ref[0] and torch.equal(out[1], ref[1]) and torch.equal(out[2], ref[2])
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
        e.record()
        torch.cuda.synchronize()
        for fn, _, off in sets:
            getattr(_lib.lib(), fn)(off)
        print(f"{cfg} {name:9s}: bin_gaussians {s.elapsed_time(e) / 20:.4f} ms, identical {same}",
              flush=True)
