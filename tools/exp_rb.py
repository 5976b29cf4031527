"""Region-binning plan sweep (gsplat_tune_rb: target workgroups, regions per axis, mapping):
times the whole speculative binning (gsplat_bin_speculative, HIP events) per setting on a
bench config's first view.  Usage: exp_rb.py <config> [wgs,regs,map | scheme=S ...]
(scheme=S: gsplat_debug_binning_scheme -- -1 shipped, 0 tile sort, 2 region binning)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from gaussctrl_exp_amd import _lib  # noqa: E402
from gaussctrl_exp_amd import rasterize as R  # noqa: E402


def main():
    cfg = sys.argv[1]
    settings = [s if s.startswith("scheme=") else tuple(int(x) for x in s.split(","))
                for s in sys.argv[2:]] or [(-1, -1, -1)]
    dev = torch.device("cuda:0")
    sc, cam = bench.make_workload(cfg, 0, dev)
    cam = cam.to(dev)
    n = sc.num_points
    p = [t.contiguous() for t in sc.params()]
    K = 1 + p[5].shape[1]
    f32 = dict(device=dev, dtype=torch.float32)
    xys, depths = torch.empty((n, 2), **f32), torch.empty((n,), **f32)
    radii = torch.empty((n,), device=dev, dtype=torch.int32)
    conics, nth = torch.empty((n, 3), **f32), torch.empty((n,), device=dev, dtype=torch.int32)
    colors, opac = torch.empty((n, 3), **f32), torch.empty((n,), **f32)
    ws1 = torch.empty((_lib.query("gsplat_bin_count_workspace_size", n),), device=dev,
                      dtype=torch.uint8)
    P = _lib.ptr
    tbx, tby = cam.tile_bounds[0], cam.tile_bounds[1]
    campos = cam.c2w[..., :3, 3].reshape(3).contiguous().float()
    _lib.call("gsplat_fused_preprocess_forward_binned", n, K, 3, *[P(t) for t in p[:5]],
              P(p[5]), P(cam.viewmat.contiguous()), P(cam.projmat.contiguous()), P(campos),
              float(cam.fx), float(cam.fy), float(cam.cx), float(cam.cy), cam.height,
              cam.width, tbx, tby, 0.01, P(xys), P(depths), P(radii), P(conics), P(nth),
              P(colors), P(opac), P(ws1), ws1.numel(), _lib.stream(dev))
    I, ids, bins = R.bin_gaussians(xys, depths, radii, nth, cam.height, cam.width,
                                   keyed_workspace=ws1.clone())
    ref_ids, ref_bins = ids.cpu(), bins.cpu()
    L = _lib.lib()
    for s in settings:
        if isinstance(s, str):
            L.gsplat_debug_binning_scheme(int(s.split("=")[1]))
            L.gsplat_tune_rb(-1, -1, -1)
        else:
            L.gsplat_debug_binning_scheme(2)  # (the plan knobs are the region binning's)
            L.gsplat_tune_rb(*s)
        times = []
        for it in range(25):
            w = ws1.clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            spec = R.bin_gaussians_speculative(xys, depths, radii, nth, cam.height, cam.width,
                                               keyed_workspace=w)
            e1.record()
            ok = spec.finish()
            torch.cuda.synchronize()
            assert ok
            if it >= 5:
                times.append(e0.elapsed_time(e1))
            if it == 0 and (isinstance(s, str) or s[2] < 10):  # (map >= 10: timing-only ablations, wrong output)
                assert torch.equal(spec.ids[:I].cpu(), ref_ids) and \
                    torch.equal(spec.tile_bins.cpu(), ref_bins), s
        times.sort()
        print(f"{cfg} {s}: bin_speculative median {times[len(times) // 2]:.4f} "
              f"min {times[0]:.4f} ms (I={I})", flush=True)
    L.gsplat_tune_rb(-1, -1, -1)
    L.gsplat_debug_binning_scheme(-1)


if __name__ == "__main__":
    with _lib.hooks():  # (gsplat_tune_rb: the test library)
        main()
