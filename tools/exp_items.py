"""bin_gaussians time vs keys per thread of the radix-sort passes (CFG env config)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from gaussctrl_exp_amd import _lib  # noqa: E402
from gaussctrl_exp_amd.project_gaussians import project_gaussians  # noqa: E402
from gaussctrl_exp_amd.rasterize import bin_gaussians  # noqa: E402

cfg = os.environ.get("CFG", "headline")
dev = torch.device("cuda:0")
sc, cam = bench.make_workload(cfg, 0, dev)
cam = cam.to(dev)
with torch.no_grad():
    xys, depths, radii, conics, nth, _ = project_gaussians(
        sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
        *cam.project_args())
res = {}
ref = None
for rnd in range(3):
    for it in (0, 4, 8, 16):
        _lib.call("gsplat_debug_sort_items", it)
        I, g, b = bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
        if ref is None:
            ref = (g.clone(), b.clone())
        assert torch.equal(g, ref[0]) and torch.equal(b, ref[1])
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
        e.record()
        torch.cuda.synchronize()
        res.setdefault(it, []).append(s.elapsed_time(e) / 10 * 1e3)
_lib.call("gsplat_debug_sort_items", 0)
print(f"{cfg}: I={I}  " + "  ".join(f"items {k or 'auto'}: {np.median(v):.1f} us"
                                     for k, v in res.items()))
