"""Backward lane utilisation on the headline raster: for sampled tiles, wave iterations after
the strip cull (touches_rect, restated in torch) vs pixel-Gaussian pairs that are valid
(idx <= final_idx, sigma >= 0, alpha >= 1/255).  Also the forward's iterations."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians
from gaussctrl_exp_amd.scene import synthetic_scene

cfg = sys.argv[1] if len(sys.argv) > 1 else "headline"
N, W, H, deg, lo, hi, seed, _real, desc = bench.CONFIGS[cfg]
dev = torch.device("cuda:0")
sc = synthetic_scene(N, deg, seed=seed, scale_lo=lo, scale_hi=hi, device=dev)
cam = bench.view_camera(W, H, 0).to(dev)
with torch.no_grad():
    xys, depths, radii, conics, nth, _ = project_gaussians(
        sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
        *cam.project_args())
    I, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W)
    tb = cam.tile_bounds
    colors = torch.rand(N, 3, device=dev)
    opac = torch.sigmoid(sc.opacities).contiguous()
    out = torch.empty(H, W, 3, device=dev); fT = torch.empty(H, W, device=dev)
    fi = torch.empty(H, W, device=dev, dtype=torch.int32)
    P = _lib.ptr
    _lib.call("gsplat_rasterize_forward", tb[0], tb[1], H, W, 3, P(gids), P(bins), P(xys),
              P(conics), P(colors), P(opac), P(torch.zeros(3, device=dev)), P(out), P(fT), P(fi),
              _lib.stream(dev))
    torch.cuda.synchronize()

    def touches(gx, gy, a, b, c, o, rx0, rx1, ry0, ry1):
        dx = gx - torch.clamp(gx, rx0, rx1); dy = gy - torch.clamp(gy, ry0, ry1)
        d2 = dx * dx + dy * dy
        hm, hd = 0.5 * (a + c), 0.5 * (a - c)
        lmax = hm + torch.sqrt(hd * hd + b * b); det = a * c - b * b
        lmin = det / lmax
        keep = ~(0.25 * lmin * d2 > torch.log(255 * o) + 0.01)
        keep |= ~((det > 0) & (lmax > 0))
        return keep & (o >= 1 / 255)

    def touches_exact(gx, gy, a, b, c, o, rx0, rx1, ry0, ry1):
        """min over the rectangle of sigma (exact for a PSD conic), culled with a margin."""
        dx0, dx1 = gx - rx1, gx - rx0
        dy0, dy1 = gy - ry1, gy - ry0
        inside = (dx0 <= 0) & (dx1 >= 0) & (dy0 <= 0) & (dy1 >= 0)
        def q(dx, dy):
            return a * dx * dx + 2 * b * dx * dy + c * dy * dy
        best = torch.full_like(gx, float("inf"))
        for dxe in (dx0, dx1):
            dys = torch.clamp(-b * dxe / c, dy0, dy1)
            best = torch.minimum(best, q(dxe, dys))
        for dye in (dy0, dy1):
            dxs = torch.clamp(-b * dye / a, dx0, dx1)
            best = torch.minimum(best, q(dxs, dye))
        smin = torch.where(inside, torch.zeros_like(best), 0.5 * best)
        keep = ~(smin * 0.999 - 1e-3 > torch.log(255 * o))
        keep |= ~((a * c - b * b > 0) & (a > 0))
        return keep & (o >= 1 / 255)

    rng = np.random.default_rng(0)
    T = tb[0] * tb[1]
    sample = rng.choice(T, 256, replace=False)
    tot = {k: 0.0 for k in ("pairs_valid", "fwd_pairs", "list")}
    b = bins.cpu().numpy()
    for t in sample:
        s, e = int(b[t, 0]), int(b[t, 1])
        if e <= s:
            continue
        tx, ty = t % tb[0], t // tb[0]
        g = gids[s:e].long()
        idx = torch.arange(s, e, device=dev)
        gx, gy = xys[g, 0], xys[g, 1]
        a, bb, c = conics[g, 0], conics[g, 1], conics[g, 2]
        o = opac[g, 0]
        ys = torch.arange(ty * 16, min(ty * 16 + 16, H), device=dev)
        xs = torch.arange(tx * 16, min(tx * 16 + 16, W), device=dev)
        py, px = torch.meshgrid(ys.float(), xs.float(), indexing="ij")
        dx = gx[:, None, None] - px; dy = gy[:, None, None] - py
        sig = 0.5 * (a[:, None, None] * dx * dx + c[:, None, None] * dy * dy) + bb[:, None, None] * dx * dy
        al = torch.clamp(o[:, None, None] * torch.exp(-sig), max=0.999)
        fin = fi[ty * 16: ty * 16 + len(ys), tx * 16: tx * 16 + len(xs)]
        v = (sig >= 0) & (al >= 1 / 255)
        tot["fwd_pairs"] += (v & (idx[:, None, None] <= fin + 1)).sum().item()
        tot["pairs_valid"] += (v & (idx[:, None, None] <= fin)).sum().item()
        tot["list"] += e - s
        # sub-wave groups: a wave footprint (W x R) split into 4 groups of 16 lanes that each
        # walk their own culled list (iterations per wave = the longest of the 4 lists)
        for (wc, wr), (gc, gr) in (((16, 8), (8, 4)), ((8, 8), (4, 4)), ((16, 8), (16, 2))):
            key = f"grouped_{wc}x{wr}_by_{gc}x{gr}"
            for c0 in range(tx * 16, min(tx * 16 + 16, W), wc):
                for r0 in range(ty * 16, min(ty * 16 + 16, H), wr):
                    longest = 0
                    for sc0 in range(c0, min(c0 + wc, W), gc):
                        sc1 = min(sc0 + gc - 1, W - 1)
                        for sr0 in range(r0, min(r0 + wr, H), gr):
                            sr1 = min(sr0 + gr - 1, H - 1)
                            mf = fin[sr0 - ty * 16: sr1 - ty * 16 + 1,
                                     sc0 - tx * 16: sc1 - tx * 16 + 1].max().item()
                            k = touches_exact(gx, gy, a, bb, c, o, float(sc0), float(sc1),
                                              float(sr0), float(sr1))
                            longest = max(longest, (k & (idx <= mf)).sum().item())
                    tot[key] = tot.get(key, 0) + longest
        # wave footprints (cols, rows): strips of the full tile width and 8x8 blocks
        for cols, rows in ((16, 8), (16, 4), (16, 16), (8, 8), (8, 16)):
            for c0 in range(tx * 16, min(tx * 16 + 16, W), cols):
                c1 = min(c0 + cols - 1, W - 1)
                for r0 in range(ty * 16, min(ty * 16 + 16, H), rows):
                    r1 = min(r0 + rows - 1, H - 1)
                    mf = fin[r0 - ty * 16: r1 - ty * 16 + 1, c0 - tx * 16: c1 - tx * 16 + 1].max().item()
                    for name, fn in (("cons", touches), ("exact", touches_exact)):
                        k = fn(gx, gy, a, bb, c, o, float(c0), float(c1), float(r0), float(r1))
                        key = f"{name}_{cols}x{rows}"
                        tot[key] = tot.get(key, 0) + (k & (idx <= mf)).sum().item()
                        if name == "exact":  # iterations with >= 1 valid pair in the wave
                            sub = v[:, r0 - ty * 16: r1 - ty * 16 + 1, c0 - tx * 16: c1 - tx * 16 + 1]
                            fsub = fin[r0 - ty * 16: r1 - ty * 16 + 1, c0 - tx * 16: c1 - tx * 16 + 1]
                            live = (sub & (idx[:, None, None] <= fsub)).flatten(1).any(1)
                            lk = f"live_{cols}x{rows}"
                            tot[lk] = tot.get(lk, 0) + (k & (idx <= mf) & live).sum().item()
    n = len(sample)
    print({k: round(v / n, 1) for k, v in tot.items()})
    for k in sorted(t for t in tot if t.startswith("grouped")):
        print(f"{k}: wave iters/tile {tot[k] / n:7.1f}")
    for cols, rows in ((16, 8), (16, 4), (16, 16), (8, 8), (8, 16)):
        for name in ("cons", "exact"):
            key = f"{name}_{cols}x{rows}"
            pix = cols * rows
            print(f"{name:5s} {cols}x{rows}: wave iters/tile {tot[key]/n:7.1f}; lane util "
                  f"{tot['pairs_valid'] / (tot[key] * pix):.3f}")
        lk = f"live_{cols}x{rows}"
        print(f"      {cols}x{rows}: iterations with a valid pair: "
              f"{tot[lk] / tot[f'exact_{cols}x{rows}']:.3f} of the exact-cull iterations")
