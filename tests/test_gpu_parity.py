"""MI355X kernels (through the C ABI via the gsplat API) vs the CPU oracle.

Bar (north_star): projection outputs, tile counts, intersection keys, sort order and tile
bins bit-exact; images/alpha and every gradient within 1e-5 abs / 1e-4 rel (per element:
|gpu - ref| <= 1e-5 + 1e-4 |ref|), with NO outlier allowance.  The forward blend uses the
hardware exp on the GPU and libm expf on the CPU, so a pixel whose alpha lands within an ulp of
a threshold (1/255, T <= 1e-4) may take the other branch: such a pixel passes only when the
oracle's own walk shows that threshold decision (tests/parity.py: near_threshold_pixel,
flip_sum); every other element must meet the tolerance.
"""
import numpy as np
import pytest
import torch

import oracle as O
from gaussctrl_exp_amd import _lib, quirks
from gaussctrl_exp_amd.camera import synthetic_camera
from gaussctrl_exp_amd.project_gaussians import project_gaussians
from gaussctrl_exp_amd.rasterize import bin_gaussians, rasterize_gaussians
from gaussctrl_exp_amd.scene import render, synthetic_scene
from gaussctrl_exp_amd.sh import spherical_harmonics
from gaussctrl_exp_amd.utils import bin_and_sort_gaussians, compute_cov2d_bounds

pytestmark = pytest.mark.gpu

ATOL, RTOL = 1e-5, 1e-4


def _close_frac(a, b, atol=ATOL, rtol=RTOL, abs_sum=None):
    """Fraction of elements with |a - b| > atol + rtol |b| (+ 2^-20 * sum|terms| when the
    reference's per-element sum of |contributions| is given: the fp32 accumulation error
    any fp32 implementation -- gsplat's atomics included -- incurs on a cancelling sum)."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    tol = atol + rtol * np.abs(b)
    if abs_sum is not None:
        tol = tol + np.asarray(abs_sum, np.float64).reshape(b.shape) * 2.0 ** -20
    bad = ~(np.abs(a - b) <= tol)  # NaN counts as out of tolerance
    return bad.mean() if bad.size else 0.0, (np.abs(a - b).max() if a.size else 0.0)


def _np(t):
    return t.detach().cpu().numpy()


CASES = [
    # (n, W, H, seed, scale_lo, scale_hi, extent)
    (2000, 64, 48, 0, 0.01, 0.08, 1.5),       # ragged image (48 not a tile multiple)
    (5000, 256, 256, 1, 0.005, 0.05, 1.5),
    (20000, 512, 512, 2, 0.003, 0.03, 1.5),
    (3000, 100, 75, 3, 0.02, 0.3, 4.0),       # large Gaussians, some behind the camera
]


def _inputs(n, W, H, seed, lo, hi, ext):
    sc = synthetic_scene(n, 3, seed=seed, scale_lo=lo, scale_hi=hi, extent=ext)
    cam = synthetic_camera(W, H)
    scales = torch.exp(sc.scales)
    quats = sc.quats / sc.quats.norm(dim=-1, keepdim=True)
    return sc, cam, scales, quats


def _project_both(gpu, sc, cam, scales, quats):
    args = (cam.fx, cam.fy, cam.cx, cam.cy, cam.height, cam.width, cam.tile_bounds)
    g = project_gaussians(sc.means.to(gpu), scales.to(gpu), 1, quats.to(gpu),
                          cam.viewmat.to(gpu), cam.projmat.to(gpu), *args)
    o = O.project_forward(sc.means.numpy(), scales.numpy(), 1.0, quats.numpy(),
                          cam.viewmat.numpy(), cam.projmat.numpy(), *args)
    return g, o


@pytest.mark.parametrize("case", CASES)
def test_project_forward_bitexact(gpu, case):
    sc, cam, scales, quats = _inputs(*case)
    g, o = _project_both(gpu, sc, cam, scales, quats)
    names = ["xys", "depths", "radii", "conics", "num_tiles_hit", "cov3d"]
    for name, gt, ot in zip(names, g, o):
        np.testing.assert_array_equal(_np(gt), ot, err_msg=name)
    assert (o[2] > 0).sum() > 0


# quirk masks: gsplat as recalled (all), none, and each [VERIFY] VJP convention alone
@pytest.mark.parametrize("quirk_mask", [7, 0, 2, 4], indirect=True)
@pytest.mark.parametrize("case", CASES)
def test_project_backward(gpu, case, quirk_mask):
    sc, cam, scales, quats = _inputs(*case)
    n = sc.num_points
    gen = torch.Generator().manual_seed(11)
    v_xy, v_d, v_c = torch.randn(n, 2, generator=gen), torch.randn(n, generator=gen), \
        torch.randn(n, 3, generator=gen)
    m, s, q = [t.to(gpu).requires_grad_() for t in (sc.means, scales, quats)]
    args = (cam.fx, cam.fy, cam.cx, cam.cy, cam.height, cam.width, cam.tile_bounds)
    xys, depths, radii, conics, nth, cov3d = project_gaussians(
        m, s, 1, q, cam.viewmat.to(gpu), cam.projmat.to(gpu), *args)
    ((xys * v_xy.to(gpu)).sum() + (depths * v_d.to(gpu)).sum() +
     (conics * v_c.to(gpu)).sum()).backward()
    o = O.project_forward(sc.means.numpy(), scales.numpy(), 1.0, quats.numpy(),
                          cam.viewmat.numpy(), cam.projmat.numpy(), *args)
    ob = O.project_backward(sc.means.numpy(), scales.numpy(), 1.0, quats.numpy(),
                            cam.viewmat.numpy(), cam.projmat.numpy(), cam.fx, cam.fy, cam.cx,
                            cam.cy, cam.height, cam.width, o[5], o[2], o[3], v_xy.numpy(),
                            v_d.numpy(), v_c.numpy())
    for name, gt, ot in (("means", m.grad, ob[2]), ("scales", s.grad, ob[3]),
                         ("quats", q.grad, ob[4])):
        frac, mx = _close_frac(_np(gt), ot)
        assert frac == 0.0, f"{name}: {frac:.2e} of elements out of tolerance (max {mx:.3e})"
    # the C ABI's optional intermediate outputs (v_cov2d, v_cov3d; the wrapper passes NULL)
    # (device copies held in locals: a pointer to a temporary would dangle)
    P = _lib.ptr
    dv = lambda *shape: torch.empty(*shape, device=gpu)
    v_cov2d, v_cov3d, vm, vs, vq = dv(n, 3), dv(n, 6), dv(n, 3), dv(n, 3), dv(n, 4)
    d_view, d_proj = cam.viewmat.to(gpu), cam.projmat.to(gpu)
    d_vxy, d_vd, d_vc = v_xy.to(gpu), v_d.to(gpu), v_c.to(gpu)
    _lib.call("gsplat_project_gaussians_backward", n, P(m.detach()), P(s.detach()), 1.0,
              P(q.detach()), P(d_view), P(d_proj), *args[:6], P(cov3d.detach()), P(radii),
              P(conics.detach()), P(d_vxy), P(d_vd), P(d_vc), P(v_cov2d), P(v_cov3d), P(vm),
              P(vs), P(vq), _lib.stream(gpu))
    for name, gt, ot in (("v_cov2d", v_cov2d, ob[0]), ("v_cov3d", v_cov3d, ob[1]),
                         ("means (C ABI)", vm, ob[2])):
        frac, mx = _close_frac(_np(gt), ot)
        assert frac == 0.0, f"{name}: {frac:.2e} of elements out of tolerance (max {mx:.3e})"


@pytest.mark.parametrize("degree,use", [(0, 0), (1, 1), (2, 2), (3, 3), (3, 0), (3, 2),
                                        (4, 4)])
def test_sh(gpu, degree, use):
    gen = torch.Generator().manual_seed(degree * 7 + use)
    for n in (1, 255, 1000, 4097):
        K = (degree + 1) ** 2
        dirs, coeffs = torch.randn(n, 3, generator=gen), torch.randn(n, K, 3, generator=gen)
        v = torch.randn(n, 3, generator=gen)
        c = coeffs.to(gpu).requires_grad_()
        out = spherical_harmonics(use, dirs.to(gpu), c)
        (out * v.to(gpu)).sum().backward()
        ref = O.sh_forward(use, dirs.numpy(), coeffs.numpy())
        vref = O.sh_backward(use, dirs.numpy(), v.numpy(), K)
        frac, mx = _close_frac(_np(out), ref)
        assert frac == 0.0, f"sh fwd n={n}: max err {mx}"
        frac, mx = _close_frac(_np(c.grad), vref)
        assert frac == 0.0, f"sh bwd n={n}: max err {mx}"


def test_sh_unaligned_slab(gpu):
    """Coefficient slabs that do not start 16-byte aligned take the dword copy path."""
    gen = torch.Generator().manual_seed(5)
    base = torch.randn(1 + 300 * 9 * 3, generator=gen)
    coeffs = base[1:].reshape(300, 9, 3)
    dirs = torch.randn(300, 3, generator=gen)
    cg = base.to(gpu)[1:].reshape(300, 9, 3)
    out = spherical_harmonics(2, dirs.to(gpu), cg)
    np.testing.assert_allclose(_np(out), O.sh_forward(2, dirs.numpy(), coeffs.numpy()),
                               rtol=RTOL, atol=ATOL)


# binning dispatch settings (gsplat_debug_binning_scheme): as shipped (by size), the depth sort +
# tile sort (the shipped scheme above 2^17 Gaussians), the small-scene tile buckets
BIN_SETTINGS = {"shipped": -1, "tilesort": 0, "bucket": 1}


@pytest.mark.parametrize("scheme", list(BIN_SETTINGS))
@pytest.mark.parametrize("case", CASES)
def test_binning_fused_bitexact(gpu, case, scheme, hooks):
    """The binning as dispatched for each case and every scheme (after the depth sort: the
    tile sort of depth-ordered pairs; without it: the tile buckets with per-tile LDS sorts):
    bit-exact against the oracle's stable sort of gsplat's keys."""
    sc, cam, scales, quats = _inputs(*case)
    g, o = _project_both(gpu, sc, cam, scales, quats)
    xys, depths, radii, conics, nth, cov3d = g
    L = _lib.lib()
    prev = L.gsplat_debug_binning_scheme(BIN_SETTINGS[scheme])
    try:
        I, gids, bins = bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
    finally:
        L.gsplat_debug_binning_scheme(prev)
    ref = O.bin_and_sort(o[0], o[1], o[2], o[4], cam.tile_bounds)
    assert I == ref["num_intersects"]
    np.testing.assert_array_equal(_np(gids), ref["gaussian_ids_sorted"])
    np.testing.assert_array_equal(_np(bins), ref["tile_bins"])


def test_binning_inconsistent_allotments(gpu, hooks):
    """Caller-supplied num_tiles_hit that disagree with the tile boxes (allotments larger than
    the box are padded with the sentinel tile, smaller ones truncate the box): every scheme
    places the same ids (the sentinel bucket / sort key last), including Gaussians
    whose allotment spans several expansion rounds (one Gaussian over 600 tiles)."""
    sc, cam, scales, quats = _inputs(20000, 512, 512, 2, 0.003, 0.03, 1.5)
    g, _ = _project_both(gpu, sc, cam, scales, quats)
    xys, depths, radii, conics, nth, cov3d = [t.detach() for t in g]
    nth = nth.clone()
    vis = torch.nonzero(radii > 0).flatten()
    nth[vis[::7]] += 3
    nth[vis[1::7]] = torch.clamp(nth[vis[1::7]] - 1, min=1)
    nth[vis[5]] = 600
    out = []
    L = _lib.lib()
    for scheme in ("tilesort", "bucket"):
        prev = L.gsplat_debug_binning_scheme(BIN_SETTINGS[scheme])
        try:
            I, gids, bins = bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
        finally:
            L.gsplat_debug_binning_scheme(prev)
        out.append((I, _np(gids), _np(bins)))
    # (gsplat leaves such slots unwritten, so no oracle output exists for them: the two
    # independent implementations of the padding semantics must agree)
    for o in out[1:]:
        assert o[0] == out[0][0] == int(nth[radii > 0].sum())
        np.testing.assert_array_equal(o[1], out[0][1])
        np.testing.assert_array_equal(o[2], out[0][2])


@pytest.mark.parametrize("scheme", list(BIN_SETTINGS))
def test_binning_prelaunched_emission(gpu, scheme, hooks):
    """The emission pre-launched before the host reads I (gsplat_bin_emit_prelaunch into
    buffers of the last call's capacity, then gsplat_bin_emit_finish): bit-exact vs the oracle
    with no capacity (first call: gsplat_bin_emit), a capacity of exactly I, a larger one, and
    one intersection too few (the pre-launched kernels write nothing and the emission re-runs
    into buffers sized for I) -- for every binning scheme."""
    from gaussctrl_exp_amd import rasterize as R
    sc, cam, scales, quats = _inputs(20000, 512, 512, 2, 0.003, 0.03, 1.5)
    g, o = _project_both(gpu, sc, cam, scales, quats)
    xys, depths, radii, conics, nth, cov3d = [t.detach() for t in g]
    ref = O.bin_and_sort(o[0], o[1], o[2], o[4], cam.tile_bounds)
    n_ref = ref["num_intersects"]
    key = (xys.device, xys.shape[0], cam.tile_bounds[0], cam.tile_bounds[1])
    L = _lib.lib()
    prev = L.gsplat_debug_binning_scheme(BIN_SETTINGS[scheme])
    try:
        for cap in (None, n_ref, n_ref + 1000, n_ref - 1, n_ref):
            if cap is None:
                R._EMIT_CAP.pop(key, None)
            else:
                R._EMIT_CAP[key] = cap
            I, gids, bins = bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
            assert I == n_ref, cap
            np.testing.assert_array_equal(_np(gids), ref["gaussian_ids_sorted"])
            np.testing.assert_array_equal(_np(bins), ref["tile_bins"])
    finally:
        L.gsplat_debug_binning_scheme(prev)
        R._EMIT_CAP.pop(key, None)


@pytest.mark.parametrize("scheme", ["shipped", "tilesort"])
def test_binning_generated_first_pass(gpu, scheme, hooks):
    """The tile sort's first pass generated from the depth-ordered allotments (shipped from 2^24
    intersections, forced here from 1): bit-exact vs the oracle for the synchronous binning, a
    pre-launched capacity above I and one below it, a speculative binning, and allotments that
    disagree with the boxes (the sentinel slots, a Gaussian over 600 tiles)."""
    from gaussctrl_exp_amd import rasterize as R
    sc, cam, scales, quats = _inputs(150000, 640, 480, 2, 0.003, 0.03, 1.5)
    g, o = _project_both(gpu, sc, cam, scales, quats)
    xys, depths, radii, conics, nth, cov3d = [t.detach() for t in g]
    ref = O.bin_and_sort(o[0], o[1], o[2], o[4], cam.tile_bounds)
    n_ref = ref["num_intersects"]
    key = (xys.device, xys.shape[0], cam.tile_bounds[0], cam.tile_bounds[1])
    L = _lib.lib()
    prev = (L.gsplat_debug_tile_sort_gen(1),
            L.gsplat_debug_binning_scheme(BIN_SETTINGS[scheme]))
    try:
        for cap in (None, n_ref + 777, n_ref - 1, n_ref):
            if cap is None:
                R._EMIT_CAP.pop(key, None)
            else:
                R._EMIT_CAP[key] = cap
            I, gids, bins = bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
            assert I == n_ref, cap
            np.testing.assert_array_equal(_np(gids), ref["gaussian_ids_sorted"])
            np.testing.assert_array_equal(_np(bins), ref["tile_bins"])
        # the padding semantics: the generated pass against the emitted one
        nth2 = nth.clone()
        vis = torch.nonzero(radii > 0).flatten()
        nth2[vis[::7]] += 3
        nth2[vis[5]] = 600
        R._EMIT_CAP.pop(key, None)
        got = bin_gaussians(xys, depths, radii, nth2, cam.height, cam.width)
        L.gsplat_debug_tile_sort_gen(1 << 40)
        R._EMIT_CAP.pop(key, None)
        want = bin_gaussians(xys, depths, radii, nth2, cam.height, cam.width)
        assert got[0] == want[0] == int(nth2[radii > 0].sum())
        np.testing.assert_array_equal(_np(got[1]), _np(want[1]))
        np.testing.assert_array_equal(_np(got[2]), _np(want[2]))
    finally:
        L.gsplat_debug_tile_sort_gen(prev[0])
        L.gsplat_debug_binning_scheme(prev[1])
        R._EMIT_CAP.pop(key, None)


@pytest.mark.parametrize("fixed", [(0x5A00, 0xFF00), (0x5A0000, 0xFF0000),
                                   (0x5A5A00, 0xFFFF00), (0x0, 0x0)])
def test_binning_depth_key_range(gpu, fixed, hooks):
    """Depth keys whose bytes 1 (and 2) are the same for every visible Gaussian (byte 3 always
    is here): those LSD passes move nothing (gsplat_debug_depth_key_range; the device picks
    every pass's buffers, DevIO), also in the middle of the pass sequence, and with only pass 0
    moving (it then writes the sorted output itself) -- bit-exact vs the oracle with and without
    the shortcut.  The sorted scheme is forced (20k Gaussians would take the tile buckets)."""
    sc, cam, scales, quats = _inputs(20000, 512, 512, 2, 0.003, 0.03, 1.5)
    g, o = _project_both(gpu, sc, cam, scales, quats)
    xys, depths, radii, conics, nth, cov3d = [t.detach() for t in g]
    val, mask = fixed
    bits = np.random.default_rng(7).integers(0, 1 << 23, size=depths.shape[0], dtype=np.uint32)
    bits = (bits & ~np.uint32(mask)) | np.uint32(val) | np.uint32(0x40000000)  # in [2, 4)
    d = bits.view(np.float32)
    ref = O.bin_and_sort(o[0], d, o[2], o[4], cam.tile_bounds)
    L = _lib.lib()
    for on in (2, 0):
        prev = L.gsplat_debug_depth_key_range(on)
        prev_s = L.gsplat_debug_binning_scheme(0)
        try:
            I, gids, bins = bin_gaussians(xys, torch.from_numpy(d).to(gpu), radii, nth,
                                          cam.height, cam.width)
        finally:
            L.gsplat_debug_depth_key_range(prev)
            L.gsplat_debug_binning_scheme(prev_s)
        assert I == ref["num_intersects"]
        np.testing.assert_array_equal(_np(gids), ref["gaussian_ids_sorted"])
        np.testing.assert_array_equal(_np(bins), ref["tile_bins"])


@pytest.mark.parametrize("W,H,tiles", [(4096, 2400, 38400), (4112, 4096, 65792)])
def test_binning_large_tile_grid_bitexact(gpu, W, H, tiles):
    """Large tile grids: 38,400 tiles (16-bit tile keys, two 8-bit sort passes) and 65,792
    (17-bit keys, three passes) -- gsplat takes any image size."""
    case = (3000, W, H, 5, 0.01, 0.2, 1.5)
    sc, cam, scales, quats = _inputs(*case)
    assert cam.tile_bounds[0] * cam.tile_bounds[1] == tiles
    g, o = _project_both(gpu, sc, cam, scales, quats)
    xys, depths, radii, conics, nth, cov3d = g
    I, gids, bins = bin_gaussians(xys, depths, radii, nth, cam.height, cam.width)
    ref = O.bin_and_sort(o[0], o[1], o[2], o[4], cam.tile_bounds)
    assert I == ref["num_intersects"] and I > 0
    np.testing.assert_array_equal(_np(gids), ref["gaussian_ids_sorted"])
    np.testing.assert_array_equal(_np(bins), ref["tile_bins"])


@pytest.mark.parametrize("case", CASES)
def test_binning_utils_bitexact(gpu, case):
    sc, cam, scales, quats = _inputs(*case)
    g, o = _project_both(gpu, sc, cam, scales, quats)
    xys, depths, radii, conics, nth, cov3d = g
    cum = torch.cumsum(nth, 0, dtype=torch.int32)
    I = int(cum[-1].item())
    isect, gid, isect_s, gid_s, bins = bin_and_sort_gaussians(
        sc.num_points, I, xys, depths, radii, cum, cam.tile_bounds)
    ref = O.bin_and_sort(o[0], o[1], o[2], o[4], cam.tile_bounds)
    np.testing.assert_array_equal(_np(isect), ref["isect_ids"])
    np.testing.assert_array_equal(_np(gid), ref["gaussian_ids"])
    np.testing.assert_array_equal(_np(isect_s), ref["isect_ids_sorted"])
    np.testing.assert_array_equal(_np(gid_s), ref["gaussian_ids_sorted"])
    T = cam.tile_bounds[0] * cam.tile_bounds[1]
    np.testing.assert_array_equal(_np(bins)[:T], ref["tile_bins"])
    assert not _np(bins)[T:].any()


def test_cov2d_bounds(gpu):
    gen = torch.Generator().manual_seed(3)
    a = torch.rand(1000, generator=gen) * 10 + 0.1
    c = torch.rand(1000, generator=gen) * 10 + 0.1
    b = (torch.rand(1000, generator=gen) * 2 - 1) * torch.sqrt(a * c) * 0.9
    cov = torch.stack([a, b, c], 1)
    cov[0] = torch.tensor([1.0, 1.0, 1.0])  # det == 0
    conics, radii = compute_cov2d_bounds(cov.to(gpu))
    rc, rr = O.cov2d_bounds(cov.numpy())
    np.testing.assert_array_equal(_np(conics), rc)
    np.testing.assert_array_equal(_np(radii), rr)


def _raster_case(gpu, case, C=3, colors_u8=False):
    sc, cam, scales, quats = _inputs(*case)
    g, o = _project_both(gpu, sc, cam, scales, quats)
    n = sc.num_points
    gen = torch.Generator().manual_seed(case[3] + 50)
    colors = torch.rand(n, C, generator=gen)
    if colors_u8:
        colors = (colors * 255).to(torch.uint8)
    opac = torch.sigmoid(sc.opacities)
    bg = torch.rand(C, generator=gen)
    return sc, cam, g, o, colors, opac, bg


@pytest.mark.parametrize("case", CASES)
def test_raster_forward(gpu, case):
    _check_raster_forward(gpu, case)


def _check_raster_forward(gpu, case):
    sc, cam, g, o, colors, opac, bg = _raster_case(gpu, case)
    xys, depths, radii, conics, nth, cov3d = g
    img, alpha = rasterize_gaussians(xys, depths, radii, conics, nth, colors.to(gpu),
                                     opac.to(gpu), cam.height, cam.width, bg.to(gpu),
                                     return_alpha=True)
    f = O.render_forward(o[0], o[1], o[2], o[3], o[4], colors.numpy(), opac.numpy(),
                         cam.height, cam.width, bg.numpy())
    fi, mi = _close_frac(_np(img), f["img"])
    fa, ma = _close_frac(_np(alpha), f["alpha"])
    assert fi == 0 and fa == 0, (fi, mi, fa, ma)


@pytest.mark.parametrize("quirk_mask", [7, 0], indirect=True)
@pytest.mark.parametrize("case", CASES)
def test_raster_backward(gpu, case, quirk_mask):
    """Backward kernel parity, fed the GPU forward state (final_Ts / final_idx) so a forward
    threshold flip cannot leak into the gradient comparison; under gsplat's quirks and
    without them (0.999 backward clamp, v_conic.y = d loss / d conic.y)."""
    _check_raster_backward(gpu, case)


@pytest.mark.parametrize("quirk_mask", [7, 0], indirect=True)
@pytest.mark.parametrize("bwd", [1, 2])
@pytest.mark.parametrize("case", CASES)
def test_raster_backward_geometries(gpu, case, bwd, quirk_mask, hooks):
    """Both shipped backward geometries on every case, whatever the frame size picks: 8x8 blocks
    (bwd 1, small frames) and 16x8 strips (bwd 2, from 3,584 tiles)."""
    _lib.call("gsplat_debug_set_raster_variant", 1, bwd, 0)
    try:
        _check_raster_backward(gpu, case)
    finally:
        _lib.call("gsplat_debug_set_raster_variant", 1, 0, 0)


# (fwd pixels/lane, bwd geometry, flags): see gsplat_debug_set_raster_variant in
# include/gsplat_mi355x.h -- K << 20 the blend kernels' block order in chunks of K block slots
# per XCD (shipped K = 8; 255 << 20 plain dispatch order).
RASTER_VARIANTS = [(1, 0, 255 << 20), (1, 0, 1 << 20), (1, 0, 3 << 20)]


@pytest.mark.ablation
@pytest.mark.parametrize("variant", RASTER_VARIANTS)
@pytest.mark.parametrize("case", [CASES[0], CASES[1], CASES[3]])
def test_raster_variants(gpu, case, variant, hooks):
    """Every blend-kernel block order reachable through gsplat_debug_set_raster_variant meets the
    same bar as the shipped one."""
    _lib.call("gsplat_debug_set_raster_variant", *variant)
    try:
        _check_raster_forward(gpu, case)
        _check_raster_backward(gpu, case)
    finally:
        _lib.call("gsplat_debug_set_raster_variant", 1, 0, 0)


def _check_raster_backward(gpu, case):
    sc, cam, g, o, colors, opac, bg = _raster_case(gpu, case)
    xys, depths, radii, conics, nth, cov3d = [t.detach() for t in g]
    H, W = cam.height, cam.width
    gen = torch.Generator().manual_seed(77)
    v_img = torch.randn(H, W, 3, generator=gen)
    v_alpha = torch.randn(H, W, generator=gen)
    xy = xys.clone().requires_grad_()
    cn = conics.clone().requires_grad_()
    col = colors.to(gpu).requires_grad_()
    op = opac.to(gpu).requires_grad_()
    img, alpha = rasterize_gaussians(xy, depths, radii, cn, nth, col, op, H, W, bg.to(gpu),
                                     return_alpha=True)
    ((img * v_img.to(gpu)).sum() + (alpha * v_alpha.to(gpu)).sum()).backward()
    # oracle backward on the GPU's forward state
    I, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W)
    from gaussctrl_exp_amd import rasterize as R
    tb = cam.tile_bounds
    out = torch.empty(H, W, 3, device=gpu)
    fT = torch.empty(H, W, device=gpu)
    fi = torch.empty(H, W, device=gpu, dtype=torch.int32)
    bg_d = bg.to(gpu)
    P = _lib.ptr
    _lib.call("gsplat_rasterize_forward", tb[0], tb[1], H, W, 3, P(gids), P(bins), P(xys),
              P(conics), P(col.detach()), P(op.detach()), P(bg_d), P(out), P(fT), P(fi),
              _lib.stream(gpu))
    ref, absum, drift, flip = O.rasterize_backward(
        tb, H, W, _np(gids), _np(bins), _np(xys), _np(conics), colors.numpy(), opac.numpy(),
        bg.numpy(), _np(fT), _np(fi), v_img.numpy(), v_alpha.numpy(),
        alpha_max=quirks.backward_alpha_clamp(), return_abs=True, return_drift=True,
        return_flip=True)
    from parity import assert_raster_close
    for k, (name, gt) in enumerate((("xys", xy.grad), ("conics", cn.grad), ("colors", col.grad),
                                    ("opacity", op.grad))):
        assert_raster_close(name, _np(gt), ref[k], absum[k], drift[k], flip[k])


@pytest.mark.parametrize("bwd", [1, 2])
@pytest.mark.parametrize("chunk", [64, 128, 256])
@pytest.mark.parametrize("case", CASES[1:3])
def test_raster_backward_list_split(gpu, case, chunk, bwd, hooks):
    """The list-split backward (parts of a forced chunk size, each re-walking the positions
    behind it; 8x8 block waves or, bwd 2, 16x8 strips): identical forward, gradients within the
    same bar vs the oracle."""
    _lib.call("gsplat_debug_set_chunk", chunk)
    _lib.call("gsplat_debug_set_raster_variant", 1, bwd, 0)
    try:
        _check_raster_forward(gpu, case)
        _check_raster_backward(gpu, case)
    finally:
        _lib.call("gsplat_debug_set_chunk", 0)
        _lib.call("gsplat_debug_set_raster_variant", 1, 0, 0)


@pytest.mark.parametrize("quirk_mask", [7, 0], indirect=True)
@pytest.mark.parametrize("C", [1, 4, 7])
def test_nd_rasterize(gpu, C, quirk_mask):
    """N-channel rasterize (gsplat nd_rasterize) forward and all four backward gradients vs the
    oracle, under gsplat's quirks and without them (v_conic.y = d loss / d conic.y: ADVICE r2)."""
    case = CASES[1]
    sc, cam, g, o, colors, opac, bg = _raster_case(gpu, case, C=C)
    xys, depths, radii, conics, nth, cov3d = [t.detach() for t in g]
    H, W = cam.height, cam.width
    xy = xys.clone().requires_grad_()
    cn = conics.clone().requires_grad_()
    col = colors.to(gpu).requires_grad_()
    op = opac.to(gpu).requires_grad_()
    img, alpha = rasterize_gaussians(xy, depths, radii, cn, nth, col, op, H, W,
                                     bg.to(gpu), return_alpha=True)
    f = O.render_forward(o[0], o[1], o[2], o[3], o[4], colors.numpy(), opac.numpy(), H, W,
                         bg.numpy())
    fr, mx = _close_frac(_np(img), f["img"])
    assert fr == 0, (fr, mx)
    gen = torch.Generator().manual_seed(8)
    v_img = torch.randn(H, W, C, generator=gen)
    (img * v_img.to(gpu)).sum().backward()
    # the oracle's backward on the oracle's own forward state
    ref, absum, drift, flip = O.rasterize_backward(
        f["tile_bounds"], H, W, f["gaussian_ids_sorted"], f["tile_bins"], o[0], o[3],
        colors.numpy(), opac.numpy(), bg.numpy(), f["final_Ts"], f["final_idx"], v_img.numpy(),
        np.zeros((H, W), np.float32), alpha_max=quirks.backward_alpha_clamp(), return_abs=True,
        return_drift=True, return_flip=True)
    from parity import assert_raster_close
    for k, (name, gt) in enumerate((("xys", xy.grad), ("conics", cn.grad), ("colors", col.grad),
                                    ("opacity", op.grad))):
        assert_raster_close(f"C={C} {name}", _np(gt), ref[k], absum[k], drift[k], flip[k])


def test_uint8_colors(gpu):
    sc, cam, g, o, colors, opac, bg = _raster_case(gpu, CASES[0], colors_u8=True)
    xys, depths, radii, conics, nth, cov3d = g
    img = rasterize_gaussians(xys, depths, radii, conics, nth, colors.to(gpu), opac.to(gpu),
                              cam.height, cam.width, bg.to(gpu))
    f = O.render_forward(o[0], o[1], o[2], o[3], o[4], colors.numpy().astype(np.float32) / 255,
                         opac.numpy(), cam.height, cam.width, bg.numpy())
    assert _close_frac(_np(img), f["img"])[0] == 0


def test_empty_scene(gpu):
    """All Gaussians behind the camera: I = 0 -> background image, alpha = 1,
    zero gradients."""
    sc, cam, scales, quats = _inputs(500, 64, 64, 0, 0.01, 0.05, 1.0)
    means = sc.means.clone()
    means[:, 2] += 10.0  # camera at z=4 looking down -z: everything behind it
    xys, depths, radii, conics, nth, cov3d = project_gaussians(
        means.to(gpu), scales.to(gpu), 1, quats.to(gpu), cam.viewmat.to(gpu),
        cam.projmat.to(gpu), cam.fx, cam.fy, cam.cx, cam.cy, 64, 64, cam.tile_bounds)
    assert int(radii.sum()) == 0
    col = torch.rand(500, 3, device=gpu, requires_grad=True)
    op = torch.rand(500, 1, device=gpu, requires_grad=True)
    bg = torch.tensor([0.1, 0.2, 0.3], device=gpu)
    img, alpha = rasterize_gaussians(xys, depths, radii, conics, nth, col, op, 64, 64, bg,
                                     return_alpha=True)
    assert torch.allclose(img, bg.expand(64, 64, 3))
    assert torch.all(alpha == 1)
    (img.sum() + alpha.sum()).backward()
    assert float(col.grad.abs().sum()) == 0 and float(op.grad.abs().sum()) == 0


def test_single_gaussian_ragged(gpu):
    means = torch.tensor([[0.05, -0.02, 0.0]])
    scales = torch.tensor([[0.05, 0.03, 0.02]])
    quats = torch.tensor([[0.9, 0.1, 0.2, 0.3]])
    quats = quats / quats.norm()
    cam = synthetic_camera(37, 29)
    args = (cam.fx, cam.fy, cam.cx, cam.cy, cam.height, cam.width, cam.tile_bounds)
    g = project_gaussians(means.to(gpu), scales.to(gpu), 1, quats.to(gpu), cam.viewmat.to(gpu),
                          cam.projmat.to(gpu), *args)
    o = O.project_forward(means.numpy(), scales.numpy(), 1.0, quats.numpy(),
                          cam.viewmat.numpy(), cam.projmat.numpy(), *args)
    for gt, ot in zip(g, o):
        np.testing.assert_array_equal(_np(gt), ot)
    col = torch.tensor([[0.2, 0.5, 0.9]])
    op = torch.tensor([[0.8]])
    img = rasterize_gaussians(*g[:5], col.to(gpu), op.to(gpu), 29, 37)
    f = O.render_forward(o[0], o[1], o[2], o[3], o[4], col.numpy(), op.numpy(), 29, 37,
                         np.ones(3, np.float32))
    assert _close_frac(_np(img), f["img"])[0] == 0


@pytest.mark.parametrize("quirk_mask", [7, 0], indirect=True)
def test_end_to_end_render_grads(gpu, quirk_mask):
    """scene.render (gc_model.get_outputs restated) on the GPU vs the same caller code on the
    oracle-backed gsplat emulation -- image, alpha and depth, and all 6 parameter gradients --
    with zero outliers: the raster-level gradients against the oracle's rasterize backward
    (fp32 summation slack), the rest of the chain against the oracle chain fed with those
    raster-level gradients (tests/parity.py)."""
    from parity import CaptureAPI, assert_close, check_raster_level, injected_api
    sc = synthetic_scene(3000, 3, seed=21, scale_lo=0.01, scale_hi=0.06)
    cam = synthetic_camera(128, 96)
    bg = torch.tensor([0.3, 0.6, 0.9])
    gen = torch.Generator().manual_seed(4)
    gt = torch.rand(96, 128, 3, generator=gen)
    cap = CaptureAPI()
    results = {}
    for name, dev, api in (("gpu", gpu, cap), ("ref", torch.device("cpu"), None)):
        if name == "ref":
            api = injected_api(cap.raster_grads(sc.num_points))
        s = sc.to(dev).requires_grad_()
        c = cam.to(dev)
        out = render(s, c, 3, bg.to(dev), api=api)
        # sums, not means: O(1) gradients, so the absolute tolerance cannot hide a wrong one
        loss = (out["rgb"] - gt.to(dev)).abs().sum() + 0.1 * out["accumulation"].sum()
        loss.backward()
        with torch.no_grad():
            dep = render(s, c, 3, bg.to(dev), return_depth=True, api=api)["depth"]
        results[name] = [_np(out["rgb"]), _np(out["accumulation"]), _np(dep)] + \
                        [_np(p.grad) for p in s.params()]
    k = cap.cap
    check_raster_level(gpu, k["xys_in"], k["depths"], k["radii"], k["conics_in"], k["nth"],
                       k["colors_in"], k["opacity_in"], k["background"], 96, 128, k["v_img"],
                       k["v_alpha"], cap.raster_grads(sc.num_points))
    names = ["rgb", "alpha", "depth", "means", "scales", "quats", "opacities", "features_dc",
             "features_rest"]
    for i, name in enumerate(names):
        assert np.abs(results["ref"][i]).max() > 0, name
        mx = assert_close(name, results["gpu"][i], results["ref"][i])
        print(f"{name}: max |diff| {mx:.3e}")
