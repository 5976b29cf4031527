"""bin_gaussians ms per call under binning switches, same process, interleaved rounds:
depth sort 4 x 8-bit vs 3 x 11-bit digits (gsplat_debug_depth_sort_wide) x keys per thread
(gsplat_debug_sort_items; 0 = automatic).  CFGS (default "c2 c3 headline")."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians

dev = torch.device("cuda:0")
L = _lib.lib()
# (depth_sort_wide, sort_items, depth_key_range): SETTINGS env "w:i:r,..." overrides
SETTINGS = [tuple(int(v) for v in x.split(":")) for x in os.environ["SETTINGS"].split(",")] \
    if os.environ.get("SETTINGS") else [(w, it, 1) for w in (0, 1) for it in (0, 8, 16)]
for cfg in os.environ.get("CFGS", "c2 c3 headline").split():
    sc, cam = bench.make_workload(cfg, 0, dev)
    cam = cam.to(dev)
    with torch.no_grad():
        xys, depths, radii, nth, = (lambda o: (o[0], o[1], o[2], o[4]))(project_gaussians(
            sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
            *cam.project_args()))
    del sc
    ref = None
    res = {s: [] for s in SETTINGS}
    for rnd in range(4):
        for s in SETTINGS:
            L.gsplat_debug_depth_sort_wide(s[0])
            _lib.call("gsplat_debug_sort_items", s[1])
            L.gsplat_debug_depth_key_range(s[2])
            out = bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
            if ref is None:
                ref = out
            elif rnd == 0:
                assert out[0] == ref[0] and torch.equal(out[1], ref[1]) and torch.equal(out[2], ref[2])
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
            e1.record(); torch.cuda.synchronize()
            res[s].append(e0.elapsed_time(e1) / 20)
    L.gsplat_debug_depth_sort_wide(0)
    _lib.call("gsplat_debug_sort_items", 0)
    L.gsplat_debug_depth_key_range(1)
    print(f"{cfg}: I={ref[0]}", flush=True)
    for s in SETTINGS:
        print(f"  wide={s[0]} items={s[1]} key_range={s[2]}: {np.median(res[s]):.4f} ms",
              flush=True)
