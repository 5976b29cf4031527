"""ctypes/numpy front-end of the C oracle (oracle/gsplat_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product path.  Parity status vs real gsplat 0.1.2.1:
"parity unpinned" (no gsplat source/fixtures exist offline; see gsplat_oracle.c header
and DESIGN.md §Oracle).

Every function mirrors one gsplat 0.1.2.1 `_C` entry point; `render_forward` /
`render_backward` chain them exactly as gsplat's Python wrappers do
(rasterize.py `_RasterizeGaussians`, utils.py `bin_and_sort_gaussians`), which is how
gaussctrl/gc_model.py:174-236 drives them.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
# the same C source built in double (-DORACLE_F64): float64() selects it
_LIB64_PATH = os.path.join(_HERE, "build", "liboracle64.so")
_libs = {}
_f64 = False

f32p = ctypes.POINTER(ctypes.c_float)
f64p = ctypes.POINTER(ctypes.c_double)
i32p = ctypes.POINTER(ctypes.c_int)
i64p = ctypes.POINTER(ctypes.c_int64)


def build(force: bool = False) -> str:
    """Compile the oracle (both precisions) with its Makefile (gcc, -ffp-contract=off)."""
    if force or not (os.path.exists(_LIB_PATH) and os.path.exists(_LIB64_PATH)):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _load(path):
    if path not in _libs:
        build()
        _libs[path] = ctypes.CDLL(path)
    return _libs[path]


def lib():
    return _load(_LIB64_PATH if _f64 else _LIB_PATH)


@contextlib.contextmanager
def float64():
    """Inside: every call runs the double build and takes/returns float64 arrays (the same
    algorithm and float constants; what fp32 rounding contributes is the difference)."""
    global _f64
    prev = _f64
    _f64 = True
    try:
        yield
    finally:
        _f64 = prev


def _dt():
    return np.float64 if _f64 else np.float32


def _r(x):
    return ctypes.c_double(x) if _f64 else ctypes.c_float(x)


def _f(a):
    return np.ascontiguousarray(a, dtype=_dt())


def _p(a):
    if a is None:
        return None
    if a.dtype == np.float32:
        assert not _f64, "float32 array passed to the double oracle"
        return a.ctypes.data_as(f32p)
    if a.dtype == np.float64:
        assert _f64, "float64 array passed to the float oracle"
        return a.ctypes.data_as(f64p)
    if a.dtype == np.int32:
        return a.ctypes.data_as(i32p)
    if a.dtype == np.int64:
        return a.ctypes.data_as(i64p)
    raise TypeError(a.dtype)


# gsplat 0.1.2.1 [VERIFY] behaviours (include/gsplat_mi355x.h GSPLAT_QUIRK_*): same bits as the
# HIP library's gsplat_set_quirks.  ALPHA_099 is applied through alpha_max by the callers.
QUIRK_ALPHA_099, QUIRK_CONIC_HALF, QUIRK_EWA_UNCLAMPED, QUIRKS_ALL = 1, 2, 4, 7


def set_quirks(mask: int) -> None:
    for path in (_LIB_PATH, _LIB64_PATH):
        _load(path).oracle_set_quirks(int(mask))


def get_quirks() -> int:
    return int(lib().oracle_get_quirks())


def backward_alpha_clamp(mask=None) -> float:
    mask = get_quirks() if mask is None else mask
    return 0.99 if mask & QUIRK_ALPHA_099 else 0.999


def num_sh_bases(degree: int) -> int:
    return {0: 1, 1: 4, 2: 9, 3: 16}.get(degree, 25)


def project_forward(means, scales, glob_scale, quats, viewmat, projmat, fx, fy, cx, cy,
                    H, W, tile_bounds, clip_thresh=0.01):
    means, scales, quats = _f(means), _f(scales), _f(quats)
    vm = _f(viewmat).reshape(-1)[:12].copy()
    pm = _f(projmat).reshape(-1)
    n = means.shape[0]
    cov3d = np.zeros((n, 6), _dt())
    xys = np.zeros((n, 2), _dt())
    depths = np.zeros((n,), _dt())
    radii = np.zeros((n,), np.int32)
    conics = np.zeros((n, 3), _dt())
    nth = np.zeros((n,), np.int32)
    lib().oracle_project_forward(
        n, _p(means), _p(scales), _r(glob_scale), _p(quats), _p(vm), _p(pm),
        _r(fx), _r(fy), _r(cx), _r(cy),
        int(H), int(W), int(tile_bounds[0]), int(tile_bounds[1]),
        _r(clip_thresh), _p(cov3d), _p(xys), _p(depths), _p(radii), _p(conics),
        _p(nth))
    return xys, depths, radii, conics, nth, cov3d


def project_backward(means, scales, glob_scale, quats, viewmat, projmat, fx, fy, cx, cy,
                     H, W, cov3d, radii, conics, v_xys, v_depths, v_conics):
    means, scales, quats = _f(means), _f(scales), _f(quats)
    vm = _f(viewmat).reshape(-1)[:12].copy()
    pm = _f(projmat).reshape(-1)
    n = means.shape[0]
    out = [np.zeros((n, k), _dt()) for k in (3, 6, 3, 3, 4)]
    lib().oracle_project_backward(
        n, _p(means), _p(scales), _r(glob_scale), _p(quats), _p(vm), _p(pm),
        _r(fx), _r(fy), _r(cx), _r(cy),
        int(H), int(W), _p(_f(cov3d)), _p(np.ascontiguousarray(radii, np.int32)),
        _p(_f(conics)), _p(_f(v_xys)), _p(_f(v_depths)), _p(_f(v_conics)),
        *[_p(o) for o in out])
    v_cov2d, v_cov3d, v_mean, v_scale, v_quat = out
    return v_cov2d, v_cov3d, v_mean, v_scale, v_quat


def sh_forward(degrees_to_use, viewdirs, coeffs):
    coeffs = _f(coeffs)
    n, K = coeffs.shape[0], coeffs.shape[1]
    degree = {1: 0, 4: 1, 9: 2, 16: 3, 25: 4}[K]
    out = np.zeros((n, 3), _dt())
    lib().oracle_sh_forward(n, degree, int(degrees_to_use), _p(_f(viewdirs)), _p(coeffs),
                            _p(out))
    return out


def sh_backward(degrees_to_use, viewdirs, v_colors, K):
    n = v_colors.shape[0]
    degree = {1: 0, 4: 1, 9: 2, 16: 3, 25: 4}[K]
    out = np.zeros((n, K, 3), _dt())
    lib().oracle_sh_backward(n, degree, int(degrees_to_use), _p(_f(viewdirs)),
                             _p(_f(v_colors)), _p(out))
    return out


def sh_backward_views(degrees_to_use, means, views, K):
    """Multi-view SH backward (data-parallel exchange, include/gsplat_mi355x.h
    gsplat_compute_sh_backward_views): sum over view records r, in order, of
    sh_backward(means - campos_r, v_colors_r); views [R, >= 3N + 3] = [v_colors_r | campos_r]."""
    means = _f(means)
    views = np.asarray(views, _dt())
    n = means.shape[0]
    out = np.zeros((n, K, 3), _dt())
    for r in range(views.shape[0]):
        campos = views[r, 3 * n:3 * n + 3]
        out += sh_backward(degrees_to_use, means - campos[None, :],
                           views[r, :3 * n].reshape(n, 3), K)
    return out


def cov2d_bounds(cov2d):
    cov2d = _f(cov2d)
    n = cov2d.shape[0]
    conics = np.zeros((n, 3), _dt())
    radii = np.zeros((n, 1), _dt())
    lib().oracle_cov2d_bounds(n, _p(cov2d), _p(conics), _p(radii))
    return conics, radii


def map_intersects(xys, depths, radii, cum_tiles_hit, tile_bounds, num_intersects):
    n = xys.shape[0]
    isect = np.zeros((num_intersects,), np.int64)
    gids = np.zeros((num_intersects,), np.int32)
    lib().oracle_map_intersects(n, _p(_f(xys)), _p(_f(depths)),
                                _p(np.ascontiguousarray(radii, np.int32)),
                                _p(np.ascontiguousarray(cum_tiles_hit, np.int32)),
                                int(tile_bounds[0]), int(tile_bounds[1]), _p(isect), _p(gids))
    return isect, gids


def sort_pairs(keys, vals):
    keys = np.ascontiguousarray(keys, np.int64).copy()
    vals = np.ascontiguousarray(vals, np.int32).copy()
    lib().oracle_sort_pairs(ctypes.c_int64(keys.shape[0]), _p(keys), _p(vals))
    return keys, vals


def tile_bin_edges(isect_sorted, rows):
    bins = np.zeros((rows, 2), np.int32)
    lib().oracle_tile_bin_edges(ctypes.c_int64(isect_sorted.shape[0]),
                                _p(np.ascontiguousarray(isect_sorted, np.int64)), _p(bins),
                                ctypes.c_int64(rows))
    return bins


def bin_and_sort(xys, depths, radii, num_tiles_hit, tile_bounds):
    """utils.bin_and_sort_gaussians with tile_bins sized [num_tiles, 2]."""
    cum = np.cumsum(np.asarray(num_tiles_hit, np.int64)).astype(np.int32)
    I = int(cum[-1]) if cum.size else 0
    isect, gids = map_intersects(xys, depths, radii, cum, tile_bounds, I)
    isect_s, gids_s = sort_pairs(isect, gids)
    T = int(tile_bounds[0]) * int(tile_bounds[1])
    bins = tile_bin_edges(isect_s, T)
    return dict(num_intersects=I, cum_tiles_hit=cum, isect_ids=isect, gaussian_ids=gids,
                isect_ids_sorted=isect_s, gaussian_ids_sorted=gids_s, tile_bins=bins)


def rasterize_forward(tile_bounds, H, W, gids_sorted, tile_bins, xys, conics, colors,
                      opacity, background, tile_list=None):
    colors = _f(colors)
    C = colors.shape[1]
    out = np.zeros((H, W, C), _dt())
    final_Ts = np.zeros((H, W), _dt())
    final_idx = np.zeros((H, W), np.int32)
    tl = None if tile_list is None else np.ascontiguousarray(tile_list, np.int32)
    lib().oracle_rasterize_forward(
        int(tile_bounds[0]), int(tile_bounds[1]), int(H), int(W), C,
        _p(np.ascontiguousarray(gids_sorted, np.int32)),
        _p(np.ascontiguousarray(tile_bins, np.int32)), _p(_f(xys)), _p(_f(conics)),
        _p(colors), _p(_f(opacity).reshape(-1)), _p(_f(background)), _p(tl),
        0 if tl is None else tl.shape[0], _p(out), _p(final_Ts), _p(final_idx))
    return out, final_Ts, final_idx


def rasterize_backward(tile_bounds, H, W, gids_sorted, tile_bins, xys, conics, colors,
                       opacity, background, final_Ts, final_idx, v_out, v_out_alpha,
                       alpha_max=0.99, tile_list=None, return_abs=False, return_drift=False,
                       return_flip=False):
    """Returns (v_xy, v_conic, v_colors, v_opacity) [+ abs-sum tuple of the same shapes:
    sum over pixels of |contribution|, the fp32 accumulation-error scale] [+ drift-sum tuple:
    sum over pixels of n_div * |contribution with |v_alpha| componentwise|, the
    transmittance-recovery drift scale (gsplat_oracle.c)] [+ flip-sum tuple: what decisions
    within 1e-5 of their thresholds can change, gsplat_oracle.c]."""
    colors = _f(colors)
    n, C = colors.shape
    v_xy = np.zeros((n, 2), _dt())
    v_conic = np.zeros((n, 3), _dt())
    v_colors = np.zeros((n, C), _dt())
    v_opac = np.zeros((n, 1), _dt())
    tl = None if tile_list is None else np.ascontiguousarray(tile_list, np.int32)
    absum = np.zeros((n, 6 + C), _dt()) if return_abs else None
    drift = np.zeros((n, 6 + C), _dt()) if return_drift else None
    flip = np.zeros((n, 6 + C), _dt()) if return_flip else None
    lib().oracle_rasterize_backward(
        int(tile_bounds[0]), int(tile_bounds[1]), int(H), int(W), C, n,
        _p(np.ascontiguousarray(gids_sorted, np.int32)),
        _p(np.ascontiguousarray(tile_bins, np.int32)), _p(_f(xys)), _p(_f(conics)),
        _p(colors), _p(_f(opacity).reshape(-1)), _p(_f(background)), _p(_f(final_Ts)),
        _p(np.ascontiguousarray(final_idx, np.int32)), _p(_f(v_out)), _p(_f(v_out_alpha)),
        _r(alpha_max), _p(tl), 0 if tl is None else tl.shape[0], _p(v_xy),
        _p(v_conic), _p(v_colors), _p(v_opac), _p(absum), _p(drift), _p(flip))
    split = lambda a: (a[:, 0:2], a[:, 2:5], a[:, 6:], a[:, 5:6])
    out = [(v_xy, v_conic, v_colors, v_opac)]
    if return_abs:
        out.append(split(absum))
    if return_drift:
        out.append(split(drift))
    if return_flip:
        out.append(split(flip))
    return out[0] if len(out) == 1 else tuple(out)


def render_forward(xys, depths, radii, conics, num_tiles_hit, colors, opacity, H, W,
                   background):
    """gsplat 0.1.2.1 `_RasterizeGaussians.forward` (rasterize.py), numpy edition.

    Returns dict(img, alpha, final_Ts, final_idx, gaussian_ids_sorted, tile_bins, ...)."""
    tb = ((W + 15) // 16, (H + 15) // 16, 1)
    b = bin_and_sort(xys, depths, radii, num_tiles_hit, tb)
    C = np.asarray(colors).shape[1]
    if b["num_intersects"] < 1:  # image = background, alpha = 1
        img = np.ones((H, W, C), _dt()) * _f(background)
        final_Ts = np.zeros((H, W), _dt())
        final_idx = np.zeros((H, W), np.int32)
    else:
        img, final_Ts, final_idx = rasterize_forward(
            tb, H, W, b["gaussian_ids_sorted"], b["tile_bins"], xys, conics, colors, opacity,
            background)
    b.update(img=img, alpha=1.0 - final_Ts, final_Ts=final_Ts, final_idx=final_idx,
             tile_bounds=tb)
    return b


def render_backward(fwd, xys, conics, colors, opacity, background, v_img, v_alpha,
                    alpha_max=0.99):
    H, W = fwd["final_Ts"].shape
    n, C = np.asarray(colors).shape
    if fwd["num_intersects"] < 1:
        return (np.zeros((n, 2), _dt()), np.zeros((n, 3), _dt()),
                np.zeros((n, C), _dt()), np.zeros((n, 1), _dt()))
    return rasterize_backward(fwd["tile_bounds"], H, W, fwd["gaussian_ids_sorted"],
                              fwd["tile_bins"], xys, conics, colors, opacity, background,
                              fwd["final_Ts"], fwd["final_idx"], v_img, v_alpha,
                              alpha_max=alpha_max)
