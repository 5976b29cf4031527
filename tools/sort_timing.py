"""Per-workgroup phase timing of the one-sweep radix-sort passes on the headline binning
(gsplat_debug_sort_timing hook).  Phases: ticket+hist scan, key load, rank+publish,
look-back, scatter+write.  Times in us (s_memrealtime: 100 MHz)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians
from gaussctrl_exp_amd.scene import synthetic_scene

N, W, H, deg, lo, hi, seed, _real, desc = bench.CONFIGS[os.environ.get("CFG", "headline")]
dev = torch.device("cuda:0")
sc = synthetic_scene(N, deg, seed=seed, scale_lo=lo, scale_hi=hi, device=dev)
cam = bench.view_camera(W, H, 0).to(dev)
with torch.no_grad():
    xys, depths, radii, conics, nth, _ = project_gaussians(
        sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
        *cam.project_args())
    for _ in range(5):
        I, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W)
    def nblk(n):
        items = 16 if n >= (4 << 20) else 4
        return (n + 256 * items - 1) // (256 * items)
    nb_d = nblk(N)
    nb_t = nblk(I)
    scheme = int(os.environ.get("SCHEME", "1"))
    for sch in (0, 1):
        _lib.call("gsplat_debug_sort_scheme", sch)
        for _ in range(3):
            bin_gaussians(xys, depths, radii, nth, H, W)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            bin_gaussians(xys, depths, radii, nth, H, W)
        e1.record()
        torch.cuda.synchronize()
        print(f"scheme {'reduce-then-scan' if sch else 'one-sweep'}: bin_gaussians "
              f"{e0.elapsed_time(e1) / 20 * 1e3:.1f} us/call (incl. host sync)")
    _lib.call("gsplat_debug_sort_scheme", scheme)
    buf = torch.zeros(8 * (4 * nb_d + 2 * nb_t), dtype=torch.int64, device=dev)
    _lib.call("gsplat_debug_sort_timing", _lib.ptr(buf), 6)
    I2, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W)
    torch.cuda.synchronize()
    _lib.call("gsplat_debug_sort_timing", None, 0)
t = buf.cpu().numpy().astype(np.float64) / 100.0  # us
off = 0
names = ["ticket", "load", "rank", "cnt-scan", "lds-scatter", "lookback", "write"]
for k, nb in enumerate([nb_d] * 4 + [nb_t] * 2):
    a = t[off: off + 8 * nb].reshape(nb, 8)
    off += 8 * nb
    d = np.diff(a, axis=1)
    span = a[:, 7].max() - a[:, 0].min()
    st = a[:, 0] - a[:, 0].min()
    print(f"pass {k} ({'depth' if k < 4 else 'tile'}, {nb} WGs): span {span:.1f} us; start spread "
          f"p50 {np.median(st):.1f} max {st.max():.1f}; per-WG total p50 "
          f"{np.median(a[:,7]-a[:,0]):.1f}")
    print("   " + "  ".join(f"{nm} p50 {np.median(d[:, i]):5.2f} p90 {np.percentile(d[:, i], 90):5.2f}"
                           for i, nm in enumerate(names)))
