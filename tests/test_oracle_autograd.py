"""The C oracle's hand-written VJPs (restated from gsplat 0.1.2.1 backward.cu/helpers.cuh)
checked against torch autograd of the forward math (oracle/torch_ref.py, float64).

CPU only.  These pin the oracle before it is trusted as the GPU kernels' checker: gsplat
has no offline fixtures, so calculus is the independent reference; the
documented gsplat 0.1.x deviations are reproduced in torch_ref with
straight-through constructions and exercised here both ways.
"""
import numpy as np
import pytest
import torch

import torch_ref as TR
from gaussctrl_exp_amd.camera import synthetic_camera
from gaussctrl_exp_amd.scene import synthetic_scene


def _setup(n=300, W=64, H=48, seed=0, scale_lo=0.02, scale_hi=0.12, max_opac=0.95):
    sc = synthetic_scene(n, 3, seed=seed, scale_lo=scale_lo, scale_hi=scale_hi, extent=1.2)
    cam = synthetic_camera(W, H)
    scales = torch.exp(sc.scales)
    quats = sc.quats / sc.quats.norm(dim=-1, keepdim=True)
    opac = torch.sigmoid(sc.opacities) * max_opac
    return sc, cam, scales, quats, opac


def test_project_forward_matches_torch(oracle_lib):
    O = oracle_lib
    sc, cam, scales, quats, _ = _setup()
    xys, depths, radii, conics, nth, cov3d = O.project_forward(
        sc.means.numpy(), scales.numpy(), 1.0, quats.numpy(), cam.viewmat.numpy(),
        cam.projmat.numpy(), cam.fx, cam.fy, cam.cx, cam.cy, cam.height, cam.width,
        cam.tile_bounds)
    r = TR.project(sc.means, scales, 1.0, quats, cam.viewmat, cam.projmat, cam.fx, cam.fy, cam.cx,
                   cam.cy, cam.height, cam.width, cam.tile_bounds)
    vis = radii > 0
    assert vis.sum() > 50
    # integer outputs: identical except where float32 rounding differs at a tile boundary
    assert (radii == r["radii"].numpy()).mean() > 0.99
    assert (nth == r["num_tiles_hit"].numpy()).mean() > 0.99
    both = vis & (r["radii"].numpy() > 0)
    np.testing.assert_allclose(xys[both], r["xys"].detach().numpy()[both], rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(depths[both], r["depths"].detach().numpy()[both], rtol=1e-6)
    np.testing.assert_allclose(conics[both], r["conics"].detach().numpy()[both], rtol=2e-4,
                               atol=1e-6)
    np.testing.assert_allclose(cov3d[both], r["cov3d"].detach().numpy()[both], rtol=1e-4,
                               atol=1e-8)


def _wide(sc, scales):
    """x spread to [-3.6, 3.6] at depths 2.8-5.2 (|x/z| up to ~1.3, past the clamp at 0.61) and
    4x larger Gaussians, so some beyond the clamp still reach into the image."""
    sc.means = sc.means * torch.tensor([3.0, 1.0, 1.0])
    return sc, scales * 4


@pytest.fixture
def quirk_mask(oracle_lib, request):
    """Run the oracle under GSPLAT_QUIRK_* mask request.param, restoring the default after."""
    prev = oracle_lib.get_quirks()
    oracle_lib.set_quirks(request.param)
    yield request.param
    oracle_lib.set_quirks(prev)


# all gsplat quirks, none, and each of the switchable VJP conventions alone
@pytest.mark.parametrize("quirk_mask", [7, 0, 2, 4], indirect=True)
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_project_backward_matches_autograd(oracle_lib, seed, quirk_mask):
    O = oracle_lib
    # seed 2: a scene spread sideways, so part of it lies beyond the 1.3 tan_fov clamp
    sc, cam, scales, quats, _ = _setup(seed=seed, n=600 if seed == 2 else 300)
    if seed == 2:
        sc, scales = _wide(sc, scales)
    xys, depths, radii, conics, nth, cov3d = O.project_forward(
        sc.means.numpy(), scales.numpy(), 1.0, quats.numpy(), cam.viewmat.numpy(),
        cam.projmat.numpy(), cam.fx, cam.fy, cam.cx, cam.cy, cam.height, cam.width,
        cam.tile_bounds)
    g = torch.Generator().manual_seed(100 + seed)
    n = sc.num_points
    v_xys = torch.randn(n, 2, generator=g)
    v_depths = torch.randn(n, generator=g)
    v_conics = torch.randn(n, 3, generator=g) * 10
    _, _, v_mean, v_scale, v_quat = O.project_backward(
        sc.means.numpy(), scales.numpy(), 1.0, quats.numpy(), cam.viewmat.numpy(),
        cam.projmat.numpy(), cam.fx, cam.fy, cam.cx, cam.cy, cam.height, cam.width, cov3d,
        radii, conics, v_xys.numpy(), v_depths.numpy(), v_conics.numpy())
    m = sc.means.double().requires_grad_()
    s = scales.double().requires_grad_()
    q = quats.double().requires_grad_()
    r = TR.project(m, s, 1.0, q, cam.viewmat.double(), cam.projmat.double(), cam.fx, cam.fy,
                   cam.cx, cam.cy, cam.height, cam.width, cam.tile_bounds, quirks=quirk_mask)
    # gsplat's v_conic.y is the gradient w.r.t. one off-diagonal of the symmetric conic
    # (SURVEY A7/A10, quirk CONIC_HALF): the parameter gradient is twice it.
    w = torch.tensor([1.0, 2.0 if quirk_mask & 2 else 1.0, 1.0], dtype=torch.float64)
    vis = torch.from_numpy(radii > 0)
    loss = ((v_xys.double() * r["xys"]).sum(1) + v_depths.double() * r["depths"] +
            (v_conics.double() * w * r["conics"]).sum(1))[vis].sum()
    loss.backward()
    rows = np.ones(n, bool)
    if quirk_mask & 4:
        # gsplat's A6 VJP recomputes the Jacobian VALUE without the clamp for every term (also
        # v_cov3d), which is no straight-through of the clamped forward: beyond the clamp it is
        # the gradient of nothing, so only the Gaussians inside are compared with calculus
        t = sc.means.numpy() @ cam.viewmat.numpy()[:3, :3].T + cam.viewmat.numpy()[:3, 3]
        lim = 1.3 * 0.5 * cam.width / cam.fx
        rows = np.abs(t[:, 0] / t[:, 2]) <= lim
        lim = 1.3 * 0.5 * cam.height / cam.fy
        rows &= np.abs(t[:, 1] / t[:, 2]) <= lim
    np.testing.assert_allclose(v_mean[rows], m.grad.numpy()[rows], rtol=2e-3, atol=2e-3)
    np.testing.assert_allclose(v_scale[rows], s.grad.numpy()[rows], rtol=2e-3, atol=2e-3)
    np.testing.assert_allclose(v_quat[rows], q.grad.numpy()[rows], rtol=2e-3, atol=2e-3)


def test_project_quirk_A6_is_real(oracle_lib):
    """The EWA_UNCLAMPED quirk changes the means gradient of Gaussians beyond the clamp (and
    nothing else): both settings are live code paths."""
    O = oracle_lib
    sc, cam, scales, quats, _ = _setup(seed=2, n=600)
    sc, scales = _wide(sc, scales)
    args = (sc.means.numpy(), scales.numpy(), 1.0, quats.numpy(), cam.viewmat.numpy(),
            cam.projmat.numpy(), cam.fx, cam.fy, cam.cx, cam.cy, cam.height, cam.width)
    xys, depths, radii, conics, nth, cov3d = O.project_forward(*args, cam.tile_bounds)
    n = sc.num_points
    g = np.random.default_rng(0)
    vc = (g.standard_normal((n, 3)) * 10).astype(np.float32)
    zero1, zero2 = np.zeros(n, np.float32), np.zeros((n, 2), np.float32)
    prev = O.get_quirks()
    try:
        outs = {}
        for mask in (7, 3):
            O.set_quirks(mask)
            outs[mask] = O.project_backward(*args, cov3d, radii, conics, zero2, zero1, vc)[2]
    finally:
        O.set_quirks(prev)
    t = sc.means.numpy() @ cam.viewmat.numpy()[:3, :3].T + cam.viewmat.numpy()[:3, 3]
    lim = 1.3 * 0.5 * cam.width / cam.fx
    outside = (np.abs(t[:, 0] / t[:, 2]) > lim) & (radii > 0)
    assert outside.sum() >= 5
    diff = np.abs(outs[7] - outs[3]).max(1) > 1e-6
    assert diff[outside].all() and not diff[~outside & (radii > 0)].any()


def test_project_quirk_A5_is_real(oracle_lib):
    """Without the A5 straight-through (exact perspective-divide derivative) the means
    gradient differs: the oracle follows gsplat's dropped term, not calculus."""
    O = oracle_lib
    sc, cam, scales, quats, _ = _setup(seed=3)
    out = O.project_forward(sc.means.numpy(), scales.numpy(), 1.0, quats.numpy(),
                            cam.viewmat.numpy(), cam.projmat.numpy(), cam.fx, cam.fy, cam.cx,
                            cam.cy, cam.height, cam.width, cam.tile_bounds)
    xys, depths, radii, conics, nth, cov3d = out
    n = sc.num_points
    v_xys = np.ones((n, 2), np.float32)
    zero1, zero3 = np.zeros(n, np.float32), np.zeros((n, 3), np.float32)
    _, _, v_mean, _, _ = O.project_backward(
        sc.means.numpy(), scales.numpy(), 1.0, quats.numpy(), cam.viewmat.numpy(),
        cam.projmat.numpy(), cam.fx, cam.fy, cam.cx, cam.cy, cam.height, cam.width, cov3d,
        radii, conics, v_xys, zero1, zero3)
    m = sc.means.double().requires_grad_()
    r = TR.project(m, scales.double(), 1.0, quats.double(), cam.viewmat.double(),
                   cam.projmat.double(), cam.fx, cam.fy, cam.cx, cam.cy, cam.height, cam.width,
                   cam.tile_bounds, quirks=False)
    r["xys"][torch.from_numpy(radii > 0)].sum().backward()
    assert np.abs(v_mean - m.grad.numpy()).max() > 1e-2


@pytest.mark.parametrize("degree,use", [(0, 0), (1, 1), (2, 2), (3, 3), (3, 1), (4, 4), (4, 2)])
def test_sh_matches_autograd(oracle_lib, degree, use):
    O = oracle_lib
    g = torch.Generator().manual_seed(degree * 10 + use)
    n, K = 200, (degree + 1) ** 2
    dirs = torch.randn(n, 3, generator=g)
    coeffs = torch.randn(n, K, 3, generator=g)
    v = torch.randn(n, 3, generator=g)
    out = O.sh_forward(use, dirs.numpy(), coeffs.numpy())
    c = coeffs.double().requires_grad_()
    ref = TR.spherical_harmonics(use, dirs.double(), c)
    np.testing.assert_allclose(out, ref.detach().numpy(), rtol=1e-5, atol=1e-5)
    (ref * v.double()).sum().backward()
    vc = O.sh_backward(use, dirs.numpy(), v.numpy(), K)
    np.testing.assert_allclose(vc, c.grad.numpy(), rtol=1e-5, atol=1e-6)


def _raster_inputs(O, seed=0, n=300, W=64, H=48, **kw):
    sc, cam, scales, quats, opac = _setup(n=n, W=W, H=H, seed=seed, **kw)
    xys, depths, radii, conics, nth, cov3d = O.project_forward(
        sc.means.numpy(), scales.numpy(), 1.0, quats.numpy(), cam.viewmat.numpy(),
        cam.projmat.numpy(), cam.fx, cam.fy, cam.cx, cam.cy, cam.height, cam.width,
        cam.tile_bounds)
    g = torch.Generator().manual_seed(7 + seed)
    colors = torch.rand(n, 3, generator=g).numpy()
    bg = torch.rand(3, generator=g).numpy()
    return dict(xys=xys, depths=depths, radii=radii, conics=conics, nth=nth, colors=colors,
                opac=opac.numpy(), bg=bg, H=H, W=W)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_raster_forward_matches_torch(oracle_lib, seed):
    O = oracle_lib
    d = _raster_inputs(O, seed)
    f = O.render_forward(d["xys"], d["depths"], d["radii"], d["conics"], d["nth"], d["colors"],
                         d["opac"], d["H"], d["W"], d["bg"])
    img, alpha = TR.rasterize(torch.from_numpy(d["xys"]).double(), torch.from_numpy(d["depths"]),
                              torch.from_numpy(d["radii"]),
                              torch.from_numpy(d["conics"]).double(), None,
                              torch.from_numpy(d["colors"]).double(),
                              torch.from_numpy(d["opac"]).double(), d["H"], d["W"],
                              torch.from_numpy(d["bg"]).double())
    assert f["num_intersects"] > 100
    np.testing.assert_allclose(f["img"], img.numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(f["alpha"], alpha.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_raster_backward_matches_autograd(oracle_lib, seed):
    O = oracle_lib
    d = _raster_inputs(O, seed)
    f = O.render_forward(d["xys"], d["depths"], d["radii"], d["conics"], d["nth"], d["colors"],
                         d["opac"], d["H"], d["W"], d["bg"])
    g = torch.Generator().manual_seed(99 + seed)
    v_img = torch.randn(d["H"], d["W"], 3, generator=g)
    v_alpha = torch.randn(d["H"], d["W"], generator=g)
    v_xy, v_conic, v_col, v_op = O.render_backward(f, d["xys"], d["conics"], d["colors"],
                                                   d["opac"], d["bg"], v_img.numpy(),
                                                   v_alpha.numpy())
    xy = torch.from_numpy(d["xys"]).double().requires_grad_()
    cn = torch.from_numpy(d["conics"]).double().requires_grad_()
    col = torch.from_numpy(d["colors"]).double().requires_grad_()
    op = torch.from_numpy(d["opac"]).double().requires_grad_()
    img, alpha = TR.rasterize(xy, torch.from_numpy(d["depths"]), torch.from_numpy(d["radii"]),
                              cn, None, col, op, d["H"], d["W"],
                              torch.from_numpy(d["bg"]).double())
    ((img * v_img.double()).sum() + (alpha * v_alpha.double()).sum()).backward()
    half = np.array([1.0, 0.5, 1.0])  # gsplat v_conic.y = half the parameter gradient
    np.testing.assert_allclose(v_col, col.grad.numpy(), rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(v_op, op.grad.numpy(), rtol=1e-3, atol=2e-3)
    np.testing.assert_allclose(v_xy, xy.grad.numpy(), rtol=1e-3, atol=2e-3)
    np.testing.assert_allclose(v_conic, cn.grad.numpy() * half, rtol=1e-3, atol=2e-3)


def test_binning_matches_stable_sort(oracle_lib):
    """bin_and_sort restated: keys = tile<<32 | depth bits, stable sort, bins = ranges."""
    O = oracle_lib
    d = _raster_inputs(O, 0)
    tb = ((d["W"] + 15) // 16, (d["H"] + 15) // 16, 1)
    b = O.bin_and_sort(d["xys"], d["depths"], d["radii"], d["nth"], tb)
    keys = b["isect_ids"]
    order = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(b["isect_ids_sorted"], keys[order])
    np.testing.assert_array_equal(b["gaussian_ids_sorted"], b["gaussian_ids"][order])
    tiles = b["isect_ids_sorted"] >> 32
    for t in range(tb[0] * tb[1]):
        idx = np.nonzero(tiles == t)[0]
        if idx.size:
            assert tuple(b["tile_bins"][t]) == (idx[0], idx[-1] + 1)
        else:
            assert tuple(b["tile_bins"][t]) == (0, 0)
    # every Gaussian appears num_tiles_hit times
    np.testing.assert_array_equal(np.bincount(b["gaussian_ids"], minlength=len(d["nth"])),
                                  d["nth"])
