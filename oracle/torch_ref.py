"""Pure-PyTorch differentiable restatement of the gsplat 0.1.2.1 forward pass.

TEST INFRASTRUCTURE ONLY (tests/ and bench.py cpu_baseline).  Parity vs real gsplat:
"parity unpinned" (see oracle/gsplat_oracle.c header).

Purpose: the C oracle's backward is a restatement of gsplat's *hand-written* VJPs
(backward.cu / helpers.cuh).  This module re-derives those gradients with torch
autograd from the forward math alone, so the hand VJPs are checked against calculus.
gsplat 0.1.x's VJPs deviate from the exact derivative in three documented places
(SURVEY.md Appendix A); `quirks=True` reproduces each deviation with a
straight-through construction so autograd yields exactly what gsplat's VJP computes:

  A5  project_pix_vjp drops the derivative of the perspective divide 1/(w+1e-6)
      -> rw is detached.
  A6  project_cov3d_ewa_vjp recomputes t WITHOUT the 1.3*tan_fov clamp
      -> T = T_unclamped + (T_clamped - T_unclamped).detach().
  A8  quat_to_rotmat_vjp ignores the normalisation Jacobian -> the norm is detached.

The remaining quirk, the 0.99 alpha clamp in rasterize backward (A10), is not the
gradient of any forward; tests keep opacity*exp(-sigma) < 0.99 where they compare
against autograd.  `rasterize` is the naive per-pixel CPU rasterizer (loop over
depth-ordered Gaussians, vectorised over pixels).
"""
from __future__ import annotations

import torch

BLOCK = 16


def _f32(x):
    """gsplat's float literal (0.3f, 1e-6f, SH_C1 ...) as the double it converts to: the
    float64 restatement then differs from the float64 oracle by rounding only."""
    return float(torch.tensor(x, dtype=torch.float32))


_EWA, _LIM, _EIG, _EPS_W = _f32(0.3), _f32(1.3), _f32(0.1), _f32(1e-6)
_AMAX, _AMIN, _TMIN = _f32(0.999), _f32(1.0 / 255.0), _f32(1e-4)


def _quirk_flags(quirks):
    """(A5, A6, A8) straight-throughs from quirks: a bool switches all three; an int is the
    library's GSPLAT_QUIRK_* mask, whose EWA_UNCLAMPED bit (4) selects A6 (A5 and A8 are not
    switchable in the kernels and stay on)."""
    if isinstance(quirks, bool):
        return quirks, quirks, quirks
    return True, bool(int(quirks) & 4), True


def quat_to_rotmat(q, quirks=True):
    n = q.norm(dim=-1, keepdim=True)
    if quirks:
        n = n.detach()
    q = q / n
    w, x, y, z = q.unbind(-1)
    R = torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y),
    ], dim=-1)
    return R.reshape(q.shape[:-1] + (3, 3))


def cov3d_full(scales, glob_scale, quats, quirks=True):
    R = quat_to_rotmat(quats, quirks)
    M = R * (glob_scale * scales)[..., None, :]
    return M @ M.transpose(-1, -2)


def project(means, scales, glob_scale, quats, viewmat, projmat, fx, fy, cx, cy, H, W,
            tile_bounds, clip_thresh=0.01, quirks=True):
    """Returns xys, depths, radii, conics, num_tiles_hit, cov3d (gsplat layout) plus the
    visibility mask.  Culled entries are zero, like gsplat's zero-initialised outputs."""
    q5, q6, q8 = _quirk_flags(quirks)
    dt = means.dtype
    vm = viewmat.reshape(-1)[:12].reshape(3, 4).to(dt)
    Pm = projmat.reshape(4, 4).to(dt)
    Wr, tv = vm[:, :3], vm[:, 3]
    t = means @ Wr.T + tv
    V = cov3d_full(scales, glob_scale, quats, q8)
    tan_fovx = 0.5 * W / fx
    tan_fovy = 0.5 * H / fy
    lim_x, lim_y = _LIM * tan_fovx, _LIM * tan_fovy
    tz = t[:, 2]
    txc = tz * torch.clamp(t[:, 0] / tz, -lim_x, lim_x)
    tyc = tz * torch.clamp(t[:, 1] / tz, -lim_y, lim_y)

    def jac(tx, ty):
        z0 = torch.zeros_like(tz)
        return torch.stack([
            torch.stack([fx / tz, z0, -fx * tx / tz ** 2], -1),
            torch.stack([z0, fy / tz, -fy * ty / tz ** 2], -1)], -2)

    Jc = jac(txc, tyc)
    if q6:
        Ju = jac(t[:, 0], t[:, 1])
        J = Ju + (Jc - Ju).detach()
    else:
        J = Jc
    T = J @ Wr
    cov2 = T @ V @ T.transpose(-1, -2)
    a = cov2[:, 0, 0] + _EWA
    b = cov2[:, 1, 0]
    c = cov2[:, 1, 1] + _EWA
    det = a * c - b * b
    conic = torch.stack([c / det, -b / det, a / det], -1)
    with torch.no_grad():
        bb = 0.5 * (a + c)
        v1 = bb + torch.sqrt(torch.clamp(bb * bb - det, min=_EIG))
        v2 = bb - torch.sqrt(torch.clamp(bb * bb - det, min=_EIG))
        radius = torch.ceil(3 * torch.sqrt(torch.maximum(v1, v2)))
    ph = torch.cat([means, torch.ones_like(means[:, :1])], -1) @ Pm.T
    rw = 1.0 / (ph[:, 3] + _EPS_W)
    if q5:
        rw = rw.detach()
    xy = torch.stack([0.5 * W * ph[:, 0] * rw + cx - 0.5, 0.5 * H * ph[:, 1] * rw + cy - 0.5],
                     -1)
    with torch.no_grad():
        tcx, tcy = xy[:, 0] / BLOCK, xy[:, 1] / BLOCK
        tr = radius / BLOCK
        tbx, tby = tile_bounds[0], tile_bounds[1]
        tminx = torch.clamp(torch.trunc(tcx - tr), 0, tbx)
        tmaxx = torch.clamp(torch.trunc(tcx + tr + 1), 0, tbx)
        tminy = torch.clamp(torch.trunc(tcy - tr), 0, tby)
        tmaxy = torch.clamp(torch.trunc(tcy + tr + 1), 0, tby)
        area = (tmaxx - tminx) * (tmaxy - tminy)
        vis = (tz > clip_thresh) & (det != 0) & (area > 0)
    m = vis.to(dt)[:, None]
    cov3d = torch.stack([V[:, 0, 0], V[:, 1, 0], V[:, 2, 0], V[:, 1, 1], V[:, 2, 1], V[:, 2, 2]],
                        -1)
    radii = torch.where(vis, radius, torch.zeros_like(radius)).to(torch.int32)
    nth = torch.where(vis, area, torch.zeros_like(area)).to(torch.int32)
    depths = tz * m[:, 0]
    return dict(xys=xy * m, depths=depths, radii=radii, conics=conic * m, num_tiles_hit=nth,
                cov3d=cov3d * (tz > clip_thresh).to(dt)[:, None], visible=vis,
                tile_min=(tminx, tminy), tile_max=(tmaxx, tmaxy))


SH_C0 = _f32(0.28209479177387814)
SH_C1 = _f32(0.4886025119029199)
SH_C2 = [_f32(c) for c in [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792,
         0.5462742152960396]]
SH_C3 = [_f32(c) for c in [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
         -0.4570457994644658, 1.445305721320277, -0.5900435899266435]]
SH_C4 = [_f32(c) for c in [2.5033429417967046, -1.7701307697799304, 0.9461746957575601, -0.6690465435572892,
         0.10578554691520431, -0.6690465435572892, 0.47308734787878004, -1.7701307697799304,
         0.6258357354491761]]


def sh_basis(degree, dirs):
    out = [torch.full_like(dirs[:, 0], SH_C0)]
    if degree >= 1:
        d = dirs / dirs.norm(dim=-1, keepdim=True)
        x, y, z = d.unbind(-1)
        xx, xy, xz, yy, yz, zz = x * x, x * y, x * z, y * y, y * z, z * z
        out += [-SH_C1 * y, SH_C1 * z, -SH_C1 * x]
        if degree >= 2:
            out += [SH_C2[0] * xy, SH_C2[1] * yz, SH_C2[2] * (2 * zz - xx - yy), SH_C2[3] * xz,
                    SH_C2[4] * (xx - yy)]
        if degree >= 3:
            out += [SH_C3[0] * y * (3 * xx - yy), SH_C3[1] * xy * z,
                    SH_C3[2] * y * (4 * zz - xx - yy), SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy),
                    SH_C3[4] * x * (4 * zz - xx - yy), SH_C3[5] * z * (xx - yy),
                    SH_C3[6] * x * (xx - 3 * yy)]
        if degree >= 4:
            out += [SH_C4[0] * xy * (xx - yy), SH_C4[1] * yz * (3 * xx - yy),
                    SH_C4[2] * xy * (7 * zz - 1), SH_C4[3] * yz * (7 * zz - 3),
                    SH_C4[4] * (zz * (35 * zz - 30) + 3), SH_C4[5] * xz * (7 * zz - 3),
                    SH_C4[6] * (xx - yy) * (7 * zz - 1), SH_C4[7] * xz * (xx - 3 * yy),
                    SH_C4[8] * (xx * (xx - 3 * yy) - yy * (3 * xx - yy))]
    return torch.stack(out, -1)


def spherical_harmonics(degrees_to_use, viewdirs, coeffs):
    """Viewdirs carry no gradient in gsplat (sh.py backward returns None for them)."""
    b = sh_basis(degrees_to_use, viewdirs.detach())
    nb = b.shape[-1]
    return (b[:, :, None] * coeffs[:, :nb, :]).sum(1)


def rasterize(xys, depths, radii, conics, num_tiles_hit, colors, opacity, H, W, background,
              tile_min=None, tile_max=None):
    """Naive per-pixel front-to-back compositing with gsplat 0.1.x rules.

    Returns (img [H,W,C], alpha [H,W]).  Gaussians are visited in (depth, id) order,
    which is each tile's sorted order; a pixel sees a Gaussian only if its tile lies in
    the Gaussian's tile bbox (recomputed from xys/radii like map_gaussian_to_intersects).
    """
    dt = colors.dtype
    C = colors.shape[1]
    tbx, tby = (W + BLOCK - 1) // BLOCK, (H + BLOCK - 1) // BLOCK
    iy, ix = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    px, py = ix.reshape(-1).to(dt), iy.reshape(-1).to(dt)
    ptx, pty = ix.reshape(-1) // BLOCK, iy.reshape(-1) // BLOCK
    with torch.no_grad():
        vis = radii > 0
        ids = torch.nonzero(vis).reshape(-1)
        order = torch.argsort(depths.detach()[ids].float(), stable=True)
        ids = ids[order]
        x32 = xys.detach().float()
        r32 = radii.float()
        tminx = torch.clamp(torch.trunc(x32[:, 0] / BLOCK - r32 / BLOCK), 0, tbx).long()
        tmaxx = torch.clamp(torch.trunc(x32[:, 0] / BLOCK + r32 / BLOCK + 1), 0, tbx).long()
        tminy = torch.clamp(torch.trunc(x32[:, 1] / BLOCK - r32 / BLOCK), 0, tby).long()
        tmaxy = torch.clamp(torch.trunc(x32[:, 1] / BLOCK + r32 / BLOCK + 1), 0, tby).long()
    P = H * W
    T = torch.ones(P, dtype=dt)
    done = torch.zeros(P, dtype=torch.bool)
    acc = torch.zeros(P, C, dtype=dt)
    for g in ids.tolist():
        inb = ((ptx >= tminx[g]) & (ptx < tmaxx[g]) & (pty >= tminy[g]) & (pty < tmaxy[g])
               & ~done)
        if not bool(inb.any()):
            continue
        dx = xys[g, 0] - px
        dy = xys[g, 1] - py
        cn = conics[g]
        sigma = 0.5 * (cn[0] * dx * dx + cn[2] * dy * dy) + cn[1] * dx * dy
        alpha = torch.clamp(opacity.reshape(-1)[g] * torch.exp(-sigma), max=_AMAX)
        ok = inb & ~(sigma < 0) & ~(alpha < _AMIN)
        next_T = T * (1 - alpha)
        term = ok & (next_T <= _TMIN)
        done = done | term
        ok = ok & ~term
        okf = ok.to(dt)
        acc = acc + (colors[g][None, :] * (alpha * T)[:, None]) * okf[:, None]
        T = torch.where(ok, next_T, T)
    img = acc + T[:, None] * background.to(dt)[None, :]
    return img.reshape(H, W, C), (1 - T).reshape(H, W)


def bin_and_sort(xys, depths, radii, tile_bounds):
    """gsplat's map_gaussian_to_intersects + sort + get_tile_bin_edges in plain torch (CPU
    baseline; the C oracle is the parity checker).  Key = tile << 32 | depth bits, sorted
    stably (ties by Gaussian id).  Returns (gaussian_ids_sorted [I] int64, tile_bins [T,2])."""
    tbx, tby = int(tile_bounds[0]), int(tile_bounds[1])
    vis = radii > 0
    ids = torch.nonzero(vis).reshape(-1)
    x = xys[ids].float()
    r = radii[ids].float()
    t0x = torch.clamp(torch.trunc(x[:, 0] / BLOCK - r / BLOCK), 0, tbx).long()
    t1x = torch.clamp(torch.trunc(x[:, 0] / BLOCK + r / BLOCK + 1), 0, tbx).long()
    t0y = torch.clamp(torch.trunc(x[:, 1] / BLOCK - r / BLOCK), 0, tby).long()
    t1y = torch.clamp(torch.trunc(x[:, 1] / BLOCK + r / BLOCK + 1), 0, tby).long()
    wx, wy = t1x - t0x, t1y - t0y
    cnt = wx * wy
    keep = cnt > 0
    ids, t0x, t0y, wx, cnt = ids[keep], t0x[keep], t0y[keep], wx[keep], cnt[keep]
    g = torch.repeat_interleave(torch.arange(ids.numel()), cnt)
    start = torch.cumsum(cnt, 0) - cnt
    k = torch.arange(g.numel()) - start[g]
    tile = (t0y[g] + k // wx[g]) * tbx + t0x[g] + k % wx[g]
    dbits = depths[ids].float().contiguous().view(torch.int32).long() & 0xFFFFFFFF
    key = (tile << 32) | dbits[g]
    key, order = torch.sort(key, stable=True)
    gids = ids[g][order]
    tiles_sorted = key >> 32
    T = tbx * tby
    first = torch.searchsorted(tiles_sorted, torch.arange(T))
    last = torch.searchsorted(tiles_sorted, torch.arange(T), right=True)
    return gids, torch.stack([first, last], -1)


def rasterize_tiles(xys, conics, colors, opacity, background, gids_sorted, tile_bins, tiles,
                    tile_bounds, H, W):
    """Per-pixel front-to-back compositing of the listed tiles, vectorised over
    each tile's [list, pixel] pairs: alpha for every pair, the transmittance as a running
    product down the list, gsplat's termination (the first Gaussian with T(1 - alpha) <= 1e-4
    and everything behind it dropped).  Differentiable in xys, conics, colors and opacity.
    Returns [(flat pixel indices, img [p, C], alpha [p])] per tile."""
    out = []
    tbx = int(tile_bounds[0])
    op_all = opacity.reshape(-1)
    for t in tiles:
        ty, tx = divmod(int(t), tbx)
        iy, ix = torch.meshgrid(torch.arange(ty * BLOCK, min(ty * BLOCK + BLOCK, H)),
                                torch.arange(tx * BLOCK, min(tx * BLOCK + BLOCK, W)),
                                indexing="ij")
        px, py = ix.reshape(-1).to(xys.dtype), iy.reshape(-1).to(xys.dtype)
        lo, hi = int(tile_bins[t, 0]), int(tile_bins[t, 1])
        C = colors.shape[1]
        if hi <= lo:
            T = torch.ones_like(px)
            out.append((iy.reshape(-1) * W + ix.reshape(-1),
                        T[:, None] * background[None, :].to(xys.dtype), 1 - T))
            continue
        ids = gids_sorted[lo:hi].long()
        g = xys[ids]
        cn = conics[ids]
        dx = g[:, :1] - px[None, :]
        dy = g[:, 1:2] - py[None, :]
        sigma = 0.5 * (cn[:, :1] * dx * dx + cn[:, 2:3] * dy * dy) + cn[:, 1:2] * dx * dy
        alpha = torch.clamp(op_all[ids][:, None] * torch.exp(-sigma), max=_AMAX)
        ok = (sigma >= 0) & (alpha >= _AMIN)
        a = torch.where(ok, alpha, torch.zeros_like(alpha))
        T_after = torch.cumprod(1 - a, 0)
        T_before = torch.cat([torch.ones_like(T_after[:1]), T_after[:-1]], 0)
        term = ok & (T_after <= _TMIN)
        alive = torch.cumsum(term.to(torch.int32), 0) == 0
        w = a * T_before * alive
        T_fin = torch.prod(torch.where(alive, 1 - a, torch.ones_like(a)), 0)
        img = w.t() @ colors[ids] + T_fin[:, None] * background[None, :].to(xys.dtype)
        out.append((iy.reshape(-1) * W + ix.reshape(-1), img.reshape(-1, C), 1 - T_fin))
    return out


def render_fwd_bwd_sampled(means, scales, quats, opacities, features_dc, features_rest,
                           viewmat, projmat, campos, fx, fy, cx, cy, H, W, sh_degree,
                           n_tiles=64, seed=0, backward=True):
    """The CPU baseline of BASELINE.json / north_star: the whole per-view fwd+bwd render in
    plain PyTorch on the host cores -- gc_model.py's activations (:172-203), projection,
    SH, binning (torch.sort), the naive per-pixel compositing above and the autograd
    backward of all of it -- with the compositing timed on `n_tiles` seeded random tiles and
    extrapolated by the tile count.  Returns (seconds per view, detail dict)."""
    import time
    tb = ((W + BLOCK - 1) // BLOCK, (H + BLOCK - 1) // BLOCK, 1)
    T = tb[0] * tb[1]
    params = [p.detach().clone().requires_grad_() for p in
              (means, scales, quats, opacities, features_dc, features_rest)]
    m, s, q, o, dc, rest = params
    t0 = time.perf_counter()
    pr = project(m, torch.exp(s), 1.0, q / q.norm(dim=-1, keepdim=True), viewmat, projmat,
                 fx, fy, cx, cy, H, W, tb)
    coeffs = torch.cat([dc[:, None], rest], 1)
    if sh_degree > 0:
        vd = m.detach() - campos
        vd = vd / vd.norm(dim=-1, keepdim=True)
        rgb = torch.clamp(spherical_harmonics(sh_degree, vd, coeffs) + 0.5, min=0.0)
    else:
        rgb = torch.sigmoid(dc)
    opac = torch.sigmoid(o)
    with torch.no_grad():
        gids, bins = bin_and_sort(pr["xys"], pr["depths"], pr["radii"], tb)
    t_gauss = time.perf_counter() - t0
    tiles = torch.randperm(T, generator=torch.Generator().manual_seed(seed))[:n_tiles]
    bg = torch.zeros(3, dtype=m.dtype)
    # the compositing's inputs as leaves, so its backward is timed apart from the
    # per-Gaussian VJPs (those run once over all N; the tiles' part is extrapolated)
    mid = [pr["xys"], pr["conics"], rgb, opac]
    leaf = [t.detach().requires_grad_() for t in mid]
    t0 = time.perf_counter()
    outs = rasterize_tiles(*leaf, bg, gids, bins, tiles.tolist(), tb, H, W)
    gen = torch.Generator().manual_seed(seed + 1)
    loss = sum((img * torch.rand(img.shape, generator=gen)).sum() + al.sum()
               for _, img, al in outs)
    t_fwd_tiles = time.perf_counter() - t0
    t_bwd_tiles = t_bwd_gauss = 0.0
    if backward:
        t0 = time.perf_counter()
        loss.backward()
        t_bwd_tiles = time.perf_counter() - t0
        t0 = time.perf_counter()
        torch.autograd.backward(mid, [t.grad for t in leaf])
        t_bwd_gauss = time.perf_counter() - t0
    scale = T / len(tiles)
    total = t_gauss + t_bwd_gauss + (t_fwd_tiles + t_bwd_tiles) * scale
    return total, dict(t_gauss=t_gauss + t_bwd_gauss, t_tiles=t_fwd_tiles + t_bwd_tiles,
                       tiles=len(tiles), scale=scale, intersects=int(gids.numel()),
                       grads=[p.grad for p in params])
