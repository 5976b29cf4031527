"""Where the blend kernels' lane slots go (headline or another bench config).

For sampled tiles and each wave footprint (8x8 forward blocks, 16x8 backward strips): the
exact-cull candidates a wave iterates over (touches_rect restated in torch, up to the
footprint's last contributing list position), and how the (candidate, pixel) slots split into
valid pairs (sigma >= 0, alpha >= 1/255, position <= the pixel's final index), spatial misses
(alpha < 1/255 or sigma < 0 at a live pixel) and terminated pixels (position past the pixel's
final index).  Also the iteration count of a per-lane candidate walk: per 64-candidate batch,
the wave runs as long as its busiest lane (max over pixels of that pixel's valid candidates
in the batch)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch

import bench
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians

cfg = sys.argv[1] if len(sys.argv) > 1 else "headline"
NS = int(sys.argv[2]) if len(sys.argv) > 2 else 128
N, W, H, deg, lo, hi, seed, _real, desc = bench.CONFIGS[cfg]
dev = torch.device("cuda:0")
sc, cam = bench.make_workload(cfg, 0, dev)
cam = cam.to(dev)
with torch.no_grad():
    xys, depths, radii, conics, nth, _ = project_gaussians(
        sc.means, torch.exp(sc.scales), 1, sc.quats / sc.quats.norm(dim=-1, keepdim=True),
        *cam.project_args())
    I, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W)
    tb = cam.tile_bounds
    colors = torch.rand(N, 3, device=dev)
    opac = torch.sigmoid(sc.opacities).contiguous()
    out = torch.empty(H, W, 3, device=dev)
    fT = torch.empty(H, W, device=dev)
    fi = torch.empty(H, W, device=dev, dtype=torch.int32)
    P = _lib.ptr
    _lib.call("gsplat_rasterize_forward", tb[0], tb[1], H, W, 3, P(gids), P(bins), P(xys),
              P(conics), P(colors), P(opac), P(torch.zeros(3, device=dev)), P(out), P(fT),
              P(fi), _lib.stream(dev))
    torch.cuda.synchronize()

    def touches_exact(gx, gy, a, b, c, o, rx0, rx1, ry0, ry1):
        dx0, dx1 = gx - rx1, gx - rx0
        dy0, dy1 = gy - ry1, gy - ry0
        inside = (dx0 <= 0) & (dx1 >= 0) & (dy0 <= 0) & (dy1 >= 0)

        def q(dx, dy):
            return a * dx * dx + 2 * b * dx * dy + c * dy * dy
        best = torch.full_like(gx, float("inf"))
        for dxe in (dx0, dx1):
            best = torch.minimum(best, q(dxe, torch.clamp(-b * dxe / c, dy0, dy1)))
        for dye in (dy0, dy1):
            best = torch.minimum(best, q(torch.clamp(-b * dye / a, dx0, dx1), dye))
        smin = torch.where(inside, torch.zeros_like(best), 0.5 * best)
        keep = ~(smin * 0.999 - 1e-3 > torch.log(255 * o))
        keep |= ~((a * c - b * b > 0) & (a > 0))
        return keep & (o >= 1 / 255)

    rng = np.random.default_rng(0)
    T = tb[0] * tb[1]
    b = bins.cpu().numpy()
    nonempty = np.nonzero(b[:, 1] > b[:, 0])[0]
    sample = rng.choice(nonempty, min(NS, len(nonempty)), replace=False)
    acc = {}

    def add(k, v):
        acc[k] = acc.get(k, 0.0) + float(v)
    for t in sample:
        s, e = int(b[t, 0]), int(b[t, 1])
        tx, ty = t % tb[0], t // tb[0]
        g = gids[s:e].long()
        idx = torch.arange(s, e, device=dev)
        gx, gy = xys[g, 0], xys[g, 1]
        a, bb, c = conics[g, 0], conics[g, 1], conics[g, 2]
        o = opac[g, 0]
        ys = torch.arange(ty * 16, min(ty * 16 + 16, H), device=dev)
        xs = torch.arange(tx * 16, min(tx * 16 + 16, W), device=dev)
        py, px = torch.meshgrid(ys.float(), xs.float(), indexing="ij")
        dx = gx[:, None, None] - px
        dy = gy[:, None, None] - py
        sig = 0.5 * (a[:, None, None] * dx * dx + c[:, None, None] * dy * dy) + \
            bb[:, None, None] * dx * dy
        al = torch.clamp(o[:, None, None] * torch.exp(-sig), max=0.999)
        fin = fi[ty * 16: ty * 16 + len(ys), tx * 16: tx * 16 + len(xs)]
        sp = (sig >= 0) & (al >= 1 / 255)
        live = idx[:, None, None] <= fin
        add("list", e - s)
        add("tile_last", (fin.max() - s + 1).item())
        add("valid_bwd", (sp & live).sum())
        add("valid_fwd", (sp & (idx[:, None, None] <= fin + 1)).sum())
        add("pixels", len(ys) * len(xs))
        for (cols, rows, name, extra) in ((8, 8, "fwd8x8", 1), (16, 8, "bwd16x8", 0),
                                         (8, 8, "bwd8x8", 0), (16, 16, "bwd16x16", 0),
                                         (8, 4, "bwd8x4", 0)):
            for c0 in range(tx * 16, min(tx * 16 + 16, W), cols):
                c1 = min(c0 + cols - 1, W - 1)
                for r0 in range(ty * 16, min(ty * 16 + 16, H), rows):
                    r1 = min(r0 + rows - 1, H - 1)
                    fs = fin[r0 - ty * 16: r1 - ty * 16 + 1, c0 - tx * 16: c1 - tx * 16 + 1]
                    mf = fs.max().item() + extra
                    k = touches_exact(gx, gy, a, bb, c, o, float(c0), float(c1), float(r0),
                                      float(r1)) & (idx <= mf)
                    ncand = int(k.sum())
                    sub_sp = sp[:, r0 - ty * 16: r1 - ty * 16 + 1, c0 - tx * 16: c1 - tx * 16 + 1]
                    sub_live = idx[:, None, None] <= fs + extra
                    kk = k[:, None, None]
                    add(name + "_cand", ncand)
                    add(name + "_slots", ncand * cols * rows)
                    add(name + "_valid", (kk & sub_sp & sub_live).sum())
                    add(name + "_miss", (kk & ~sub_sp & sub_live).sum())
                    add(name + "_term", (kk & ~sub_live).sum())
                    # per-lane walk: candidates in compaction order, batches of 64
                    v = (sub_sp & sub_live)[k].flatten(1)  # [cand, pixels]
                    it = 0
                    for b0 in range(0, ncand, 64):
                        it += int(v[b0:b0 + 64].sum(0).max()) if v.shape[0] else 0
                    add(name + "_lane_walk_iters", it)
        # active-rectangle cull for the 16x8 backward strips: the strip walks its list from its
        # last contributing position down in 64-position batches; in a batch whose lowest
        # position is p0 only pixels with final index >= p0 can use any of its Gaussians, so the
        # batch's candidates could be culled against the bounding box of those pixels
        for c0 in range(tx * 16, min(tx * 16 + 16, W), 16):
            c1 = min(c0 + 15, W - 1)
            for r0 in range(ty * 16, min(ty * 16 + 16, H), 8):
                r1 = min(r0 + 7, H - 1)
                fs = fin[r0 - ty * 16: r1 - ty * 16 + 1, c0 - tx * 16: c1 - tx * 16 + 1]
                last = int(fs.max().item())
                kept = 0
                bhi = last
                while bhi >= s:
                    p0 = max(bhi - 63, s)
                    act = (fs >= p0).nonzero()
                    if len(act):
                        ar0 = float(r0 + act[:, 0].min().item())
                        ar1 = float(r0 + act[:, 0].max().item())
                        ac0 = float(c0 + act[:, 1].min().item())
                        ac1 = float(c0 + act[:, 1].max().item())
                        sl = slice(p0 - s, bhi - s + 1)
                        kept += int(touches_exact(gx[sl], gy[sl], a[sl], bb[sl], c[sl], o[sl],
                                                  ac0, ac1, ar0, ar1).sum())
                    bhi -= 64
                add("active_cand", kept)
        # two-queue strip backward: a 16x8 strip whose lanes hold a pixel of the top 16x4 half
        # (.x) and one of the bottom half (.y); each half walks its own candidate queue, so a
        # 64-position batch takes max(top, bottom) iterations instead of |top u bottom|
        for c0 in range(tx * 16, min(tx * 16 + 16, W), 16):
            c1 = min(c0 + 15, W - 1)
            for r0 in range(ty * 16, min(ty * 16 + 16, H), 8):
                halves = []
                for h0 in (r0, r0 + 4):
                    h1 = min(h0 + 3, H - 1)
                    if h0 > H - 1:
                        halves.append(torch.zeros(e - s, dtype=torch.bool, device=dev))
                        continue
                    fs = fin[h0 - ty * 16: h1 - ty * 16 + 1, c0 - tx * 16: c1 - tx * 16 + 1]
                    halves.append(touches_exact(gx, gy, a, bb, c, o, float(c0), float(c1),
                                                float(h0), float(h1)) & (idx <= fs.max()))
                top, bot = halves
                it2 = 0
                for b0 in range(0, e - s, 64):
                    it2 += max(int(top[b0:b0 + 64].sum()), int(bot[b0:b0 + 64].sum()))
                add("dual_iters", it2)
                add("dual_union", int((top | bot).sum()))
    n = len(sample)
    print(f"config {cfg}: {n} sampled tiles; per tile:")
    print(f"  active-rectangle strips: candidates/tile {acc['active_cand'] / n:7.1f}")
    print(f"  two-queue strips: iterations/tile {acc['dual_iters'] / n:7.1f} "
          f"(union of the halves' candidates {acc['dual_union'] / n:7.1f})")
    for k in ("list", "tile_last", "valid_bwd", "valid_fwd"):
        print(f"  {k:12s} {acc[k] / n:9.1f}")
    for name in ("fwd8x8", "bwd16x16", "bwd16x8", "bwd8x8", "bwd8x4"):
        sl = acc[name + "_slots"]
        print(f"  {name:9s} cand/tile {acc[name + '_cand'] / n:7.1f}  slots: valid "
              f"{acc[name + '_valid'] / sl:.3f} miss {acc[name + '_miss'] / sl:.3f} "
              f"term {acc[name + '_term'] / sl:.3f}  lane-walk iters/tile "
              f"{acc[name + '_lane_walk_iters'] / n:7.1f}")
