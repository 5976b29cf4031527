"""Binning switch A/B (same scene, same process): bin_gaussians time per call with the depth
sort compacting the culled Gaussians away or not (gsplat_debug_compact_depth_sort) and the tile
sort's first LSD pass generated from the allotments or run over emitted pairs
(gsplat_debug_emit_pass0).
CFGS (default "headline c4 c5").  Run under rocprofv3 --kernel-trace --stats for the split."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians

dev = torch.device("cuda:0")
L = _lib.lib()
for cfg in os.environ.get("CFGS", "headline c4 c5").split():
    sc, cam = bench.make_workload(cfg, 0, dev)
    cam = cam.to(dev)
    with torch.no_grad():
        xys, depths, radii, conics, nth, _ = project_gaussians(
            sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
            *cam.project_args())
    del sc
    for items in [int(x) for x in os.environ.get("ITEMS_LIST", "").split()]:
        # keys per thread of every radix pass (0 = automatic: 4 below 4M keys, 16 above)
        _lib.call("gsplat_debug_sort_items", items)
        for _ in range(3):
            bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
        e.record()
        torch.cuda.synchronize()
        print(f"{cfg} sort_items={items}: bin_gaussians {s.elapsed_time(e) / 20:.4f} ms",
              flush=True)
    _lib.call("gsplat_debug_sort_items", 0)
    for rng in [int(x) for x in os.environ.get("RANGE_LIST", "").split()]:
        # depth passes whose digit is constant only copy (2: always, 1: auto) or rank (0)
        L.gsplat_debug_depth_key_range(rng)
        for _ in range(3):
            bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
        e.record()
        torch.cuda.synchronize()
        print(f"{cfg} key_range={rng}: bin_gaussians {s.elapsed_time(e) / 20:.4f} ms", flush=True)
    L.gsplat_debug_depth_key_range(1)
    for rep in range(int(os.environ.get("REPS", "2"))):
        for compact in (1, 0):
            for gen in (2, 0):
                L.gsplat_debug_compact_depth_sort(compact)
                L.gsplat_debug_emit_pass0(gen)
                for _ in range(3):
                    bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
                e.record()
                torch.cuda.synchronize()
                print(f"{cfg} compact={compact} gen_pass0={gen}: bin_gaussians "
                      f"{s.elapsed_time(e) / 20:.4f} ms", flush=True)
    L.gsplat_debug_compact_depth_sort(1)
    L.gsplat_debug_emit_pass0(1)
    del xys, depths, radii, conics, nth
    torch.cuda.empty_cache()
