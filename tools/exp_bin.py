"""Device time of the two binning phases per radix-sort scheme (1 = reduce-then-scan, 0 =
one-sweep look-back) for several configurations (HIP events, median of 5 rounds x 20 calls)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch

import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.project_gaussians import project_gaussians

dev = torch.device("cuda:0")
P = _lib.ptr


def timeit(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for cfg in os.environ.get("CFGS", "c2,c3,headline").split(","):
    sc, cam = bench.make_workload(cfg, 0, dev)
    cam = cam.to(dev)
    H, W = cam.height, cam.width
    tbx, tby = cam.tile_bounds[:2]
    with torch.no_grad():
        xys, depths, radii, conics, nth, _ = project_gaussians(
            sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
            *cam.project_args())
    n = sc.num_points
    st = _lib.stream(dev)
    ws1 = torch.empty(_lib.query("gsplat_bin_count_workspace_size", n), device=dev,
                      dtype=torch.uint8)
    counts = torch.empty(2, device=dev, dtype=torch.int32)

    def count():
        _lib.call("gsplat_bin_count", n, P(xys), P(depths), P(radii), P(nth), tbx, tby, P(counts),
                  P(ws1), ws1.numel(), st)

    count()
    I = int(counts[1].item())
    ws2 = torch.empty(_lib.query("gsplat_bin_emit_workspace_size", I), device=dev,
                      dtype=torch.uint8)
    gids = torch.empty(I, device=dev, dtype=torch.int32)
    bins = torch.empty(tbx * tby, 2, device=dev, dtype=torch.int32)

    def emit():
        _lib.call("gsplat_bin_emit", n, I, tbx, tby, P(gids), P(bins), P(ws1), ws1.numel(),
                  P(ws2), ws2.numel(), st)

    res = {}
    for scheme in (1, 0):
        _lib.call("gsplat_debug_sort_scheme", scheme)
        res[scheme] = ([], [])
        for _ in range(5):
            count()
            emit()
            torch.cuda.synchronize()
            res[scheme][0].append(timeit(count))
            res[scheme][1].append(timeit(emit))
    _lib.call("gsplat_debug_sort_scheme", 1)
    print(f"{cfg}: N={n} I={I}  " + "  ".join(
        f"scheme {s}: count {np.median(r[0]):.1f} us emit {np.median(r[1]):.1f} us"
        for s, r in res.items()), flush=True)
