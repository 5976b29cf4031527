"""The fused training render (csrc/preprocess.hip via fused.render_fused) against the CPU
oracle and against the unchanged-caller path (scene.render: gc_model.py's torch glue around
the gsplat API).

Bars: given the activated inputs the fused kernel computed (its optional scales_out /
quats_out), the projection outputs, tile counts and therefore the binning are bit-exact with
the oracle; the activations themselves are torch's formulas in fp32 (within 1 ulp of torch's
kernels); images, alpha and all six parameter gradients meet the end-to-end bar of
test_gpu_parity.test_end_to_end_render_grads (per element 1e-5 + 1e-4 |ref|, <= 0.2 % of
elements outside).
"""
import json
import os
import socket

import numpy as np
import pytest
import torch

import oracle as O
from gaussctrl_exp_amd import _lib
from gaussctrl_exp_amd.camera import gc_camera, look_at_c2w, synthetic_camera
from gaussctrl_exp_amd.fused import render_fused
from gaussctrl_exp_amd.scene import render, synthetic_scene

pytestmark = pytest.mark.gpu

ATOL, RTOL = 1e-5, 1e-4
NAMES = ["means", "scales", "quats", "opacities", "features_dc", "features_rest"]
STATS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out",
                     "fused_activation_stats.json")


def _np(t):
    return t.detach().cpu().numpy()


def _bad_frac(a, b, atol=ATOL, rtol=RTOL):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    bad = ~(np.abs(a - b) <= atol + rtol * np.abs(b))  # NaN counts as out of tolerance
    return (bad.mean() if bad.size else 0.0), (np.abs(a - b).max() if a.size else 0.0)


# (n, W, H, sh_degree, degrees_to_use, seed, scale_lo, scale_hi, extent)
CASES = [
    (3000, 128, 96, 3, 3, 21, 0.01, 0.06, 1.5),
    (2000, 64, 48, 3, 1, 0, 0.01, 0.08, 1.5),     # ragged image, fewer bands than stored
    (3000, 100, 75, 3, 3, 3, 0.02, 0.3, 4.0),     # large Gaussians, some behind the camera
    (2500, 96, 64, 0, 0, 5, 0.01, 0.05, 1.5),     # one SH band: sigmoid colours (gc_model:203)
    (2500, 96, 64, 2, 0, 6, 0.01, 0.05, 1.5),     # SH path evaluated at degree 0
    (2500, 80, 64, 4, 4, 7, 0.01, 0.05, 1.5),     # degree 4 (128-thread blocks)
    (20000, 512, 512, 3, 3, 2, 0.003, 0.03, 1.5),  # 1,024 tiles: list-split backward
]


def _scene_cam(case):
    n, W, H, deg, dtu, seed, lo, hi, ext = case
    return synthetic_scene(n, deg, seed=seed, scale_lo=lo, scale_hi=hi, extent=ext), \
        synthetic_camera(W, H)


@pytest.mark.parametrize("case", CASES)
def test_fused_forward_bitexact_given_activations(gpu, case):
    sc, cam = _scene_cam(case)
    n, W, H, deg, dtu = case[:5]
    d = sc.to(gpu)
    c = cam.to(gpu)
    K = d.features_rest.shape[1] + 1
    f = lambda *s: torch.empty(*s, device=gpu)
    xys, depths, conics, colors, opac = f(n, 2), f(n), f(n, 3), f(n, 3), f(n)
    radii = torch.empty(n, device=gpu, dtype=torch.int32)
    nth = torch.empty(n, device=gpu, dtype=torch.int32)
    s_out, q_out = f(n, 3), f(n, 4)
    campos = c.c2w[:3, 3].contiguous()
    P = _lib.ptr
    tb = cam.tile_bounds
    _lib.call("gsplat_fused_preprocess_forward", n, K, dtu, P(d.means), P(d.scales), P(d.quats),
              P(d.opacities), P(d.features_dc), P(d.features_rest) if K > 1 else None,
              P(c.viewmat), P(c.projmat), P(campos), cam.fx, cam.fy, cam.cx, cam.cy, H, W,
              tb[0], tb[1], 0.01, P(xys), P(depths), P(radii), P(conics), P(nth), P(colors),
              P(opac), None, P(s_out), P(q_out), _lib.stream(gpu))
    # activations: torch's formulas in fp32 (record how often they equal torch's kernels)
    t_s = torch.exp(d.scales)
    t_q = d.quats / d.quats.norm(dim=-1, keepdim=True)
    t_o = torch.sigmoid(d.opacities).reshape(-1)
    stats = {}
    for name, mine, ref in (("scales", s_out, t_s), ("quats", q_out, t_q), ("opacity", opac, t_o)):
        a, b = _np(mine).astype(np.float64), _np(ref).astype(np.float64)
        rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-30)
        stats[name] = {"equal_frac": float((a == b).mean()), "max_rel": float(rel.max())}
        # bit-identical to torch's own kernels (exp, the 4-vector norm order, sigmoid)
        assert (a == b).all(), f"{name}: {1 - (a == b).mean():.2e} differ from torch"
    os.makedirs(os.path.dirname(STATS), exist_ok=True)
    with open(STATS, "a") as fh:
        fh.write(json.dumps({"case": list(case), **stats}) + "\n")
    # projection: bit-exact with the oracle on the kernel's own activated inputs
    o = O.project_forward(_np(d.means), _np(s_out), 1.0, _np(q_out), cam.viewmat.numpy(),
                          cam.projmat.numpy(), cam.fx, cam.fy, cam.cx, cam.cy, H, W, tb)
    for name, g, r in zip(["xys", "depths", "radii", "conics", "num_tiles_hit"],
                          [xys, depths, radii, conics, nth], o[:5]):
        np.testing.assert_array_equal(_np(g), r, err_msg=name)
    assert (o[2] > 0).sum() > 0
    # colours: the caller's SH + clamp (or sigmoid) on the oracle
    if K > 1:
        vd = d.means - c.c2w[:3, 3]
        vd = vd / vd.norm(dim=-1, keepdim=True)
        coeffs = torch.cat([d.features_dc[:, None], d.features_rest], 1)
        ref = np.maximum(O.sh_forward(dtu, _np(vd), _np(coeffs)) + 0.5, 0.0)
    else:
        ref = _np(torch.sigmoid(d.features_dc))
    frac, mx = _bad_frac(_np(colors), ref, atol=1e-6, rtol=1e-5)
    assert frac == 0.0, f"colors: {frac:.2e} out of tolerance (max {mx:.3e})"
    # and bit-identical to the unchanged caller's path on the GPU (torch glue + gsplat API)
    from gaussctrl_exp_amd.project_gaussians import project_gaussians
    from gaussctrl_exp_amd.sh import spherical_harmonics
    with torch.no_grad():
        g = project_gaussians(d.means, t_s, 1, t_q, c.viewmat, c.projmat, cam.fx, cam.fy,
                              cam.cx, cam.cy, H, W, tb)
        if K > 1:
            vd = d.means - c.c2w[:3, 3]
            vd = vd / vd.norm(dim=-1, keepdim=True)
            cc = torch.clamp(spherical_harmonics(dtu, vd, torch.cat(
                [d.features_dc[:, None], d.features_rest], 1)) + 0.5, min=0.0)
        else:
            cc = torch.sigmoid(d.features_dc)
    for name, mine, theirs in zip(["xys", "depths", "radii", "conics", "num_tiles_hit",
                                   "colors"], [xys, depths, radii, conics, nth, colors],
                                  list(g[:5]) + [cc]):
        assert torch.equal(mine, theirs), f"{name}: fused != caller path"


@pytest.mark.parametrize("case", [CASES[0], CASES[1], CASES[6]])
def test_forward_clearing_equals_forward_and_clears_records(gpu, case):
    """gsplat_rasterize_forward_clearing: the blend's outputs are those of the plain
    forward, and the record buffer is all zero afterwards whatever it held."""
    from gaussctrl_exp_amd.project_gaussians import project_gaussians
    from gaussctrl_exp_amd.rasterize import bin_gaussians
    sc, cam = _scene_cam(case)
    n, W, H = case[:3]
    d, c = sc.to(gpu), cam.to(gpu)
    tb = cam.tile_bounds
    with torch.no_grad():
        xys, depths, radii, conics, nth, _ = project_gaussians(
            d.means, torch.exp(d.scales), 1, d.quats / d.quats.norm(dim=-1, keepdim=True),
            *c.project_args())
    I, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W)
    assert I > 0
    colors = torch.rand(n, 3, device=gpu)
    opac = torch.rand(n, device=gpu)
    bg = torch.tensor([0.2, 0.4, 0.6], device=gpu)
    P, st = _lib.ptr, _lib.stream(gpu)
    outs = []
    for clear in (False, True):
        img = torch.full((H, W, 3), float("nan"), device=gpu)
        fT = torch.full((H, W), float("nan"), device=gpu)
        fi = torch.full((H, W), -7, device=gpu, dtype=torch.int32)
        if clear:
            rec = torch.full((_lib.query("gsplat_grad_records_bytes", n),), 255, device=gpu,
                             dtype=torch.uint8)
            _lib.call("gsplat_rasterize_forward_clearing", tb[0], tb[1], H, W, P(gids), P(bins),
                      P(xys), P(conics), P(colors), P(opac), P(bg), P(img), P(fT), P(fi),
                      P(rec), rec.numel(), None, 0, 0, None, 0, st)
            torch.cuda.synchronize()
            assert int(rec.count_nonzero()) == 0
            # visible-only clearing: culled Gaussians' records keep their bytes
            rec.fill_(255)
            img2 = torch.empty_like(img)
            _lib.call("gsplat_rasterize_forward_clearing", tb[0], tb[1], H, W, P(gids), P(bins),
                      P(xys), P(conics), P(colors), P(opac), P(bg), P(img2), P(fT), P(fi),
                      P(rec), rec.numel(), P(radii), 0, 0, None, 0, st)
            r = rec.view(n, 64)
            vis = radii > 0
            assert (~vis).any() or n == int(vis.sum())
            assert int(r[vis].count_nonzero()) == 0 and bool((r[~vis] == 255).all())
            assert torch.equal(img2, img)
        else:
            _lib.call("gsplat_rasterize_forward", tb[0], tb[1], H, W, 3, P(gids), P(bins),
                      P(xys), P(conics), P(colors), P(opac), P(bg), P(img), P(fT), P(fi), st)
        outs.append((img, fT, fi))
    for name, a, b in zip(("img", "final_Ts", "final_idx"), *outs):
        assert torch.equal(a, b), name
    with pytest.raises(RuntimeError):  # clear size must be a multiple of 16 bytes
        _lib.call("gsplat_rasterize_forward_clearing", tb[0], tb[1], H, W, P(gids), P(bins),
                  P(xys), P(conics), P(colors), P(opac), P(bg), P(img), P(fT), P(fi),
                  P(rec), 24, None, 0, 0, None, 0, st)


@pytest.mark.parametrize("case", [CASES[0], CASES[1], CASES[6]])
def test_forward_filled_split_plan(gpu, case):
    """The list-split plan's walk table filled by the clearing forward's waves
    (gsplat_rasterize_forward_clearing with a plan) gives every tile the same walk as the
    backward's own split_work_kernel (per-tile maxima equal), and the record backward given
    plan_filled = 1 is bit-identical to plan_filled = 0 in the deterministic mode."""
    from gaussctrl_exp_amd.project_gaussians import project_gaussians
    from gaussctrl_exp_amd.rasterize import bin_gaussians
    sc, cam = _scene_cam(case)
    n, W, H = case[:3]
    d, c = sc.to(gpu), cam.to(gpu)
    tb = cam.tile_bounds
    T = tb[0] * tb[1]
    with torch.no_grad():
        xys, depths, radii, conics, nth, _ = project_gaussians(
            d.means, torch.exp(d.scales), 1, d.quats / d.quats.norm(dim=-1, keepdim=True),
            *c.project_args())
    I, gids, bins = bin_gaussians(xys, depths, radii, nth, H, W)
    assert I > 0
    g = torch.Generator().manual_seed(3)
    colors = torch.rand(n, 3, generator=g).to(gpu)
    opac = torch.rand(n, generator=g).to(gpu)
    bg = torch.tensor([0.2, 0.4, 0.6], device=gpu)
    v_img = torch.randn(H, W, 3, generator=g).to(gpu)
    v_a = torch.randn(H, W, generator=g).to(gpu)
    P, st = _lib.ptr, _lib.stream(gpu)
    chunk = 64  # forced: every case splits
    plan = torch.full((_lib.query("gsplat_rasterize_split_bytes", tb[0], tb[1], I, chunk),), 0xAB,
                      device=gpu, dtype=torch.uint8)
    rec_bytes = _lib.query("gsplat_grad_records_bytes", n)
    img = torch.empty(H, W, 3, device=gpu)
    fT = torch.empty(H, W, device=gpu)
    fi = torch.empty(H, W, device=gpu, dtype=torch.int32)
    prev = _lib.set_deterministic(True)
    try:
        recs, tables = [], []
        for filled in (1, 0):
            rec = torch.full((rec_bytes,), 0x7F, device=gpu, dtype=torch.uint8)
            plan.fill_(0xAB)
            _lib.call("gsplat_rasterize_forward_clearing", tb[0], tb[1], H, W, P(gids), P(bins),
                      P(xys), P(conics), P(colors), P(opac), P(bg), P(img), P(fT), P(fi),
                      P(rec), rec.numel(), None, I, chunk, P(plan), plan.numel(), st)
            if not filled:
                plan.fill_(0xAB)  # the backward derives the table itself
            _lib.call("gsplat_rasterize_backward_records", tb[0], tb[1], H, W, n, P(gids),
                      P(bins), P(xys), P(conics), P(colors), P(opac), P(bg), P(fT), P(fi),
                      P(v_img), P(v_a), 0.99, I, chunk, P(plan), plan.numel(), filled, P(rec),
                      rec.numel(), st)
            torch.cuda.synchronize()
            tables.append(plan[:16 * T].view(torch.int32).view(T, 4).max(dim=1).values.clone())
            recs.append(rec.clone())
    finally:
        _lib.set_deterministic(prev)
    assert torch.equal(tables[0], tables[1])
    assert torch.equal(recs[0], recs[1])
    assert int((tables[0] >= 0).sum()) > 0


@pytest.mark.parametrize("case", [CASES[0], CASES[2], CASES[3], CASES[6]])
def test_binned_forward_and_keyed_count_equal_the_separate_passes(gpu, case):
    """gsplat_fused_preprocess_forward_binned + gsplat_bin_count_keyed: the same projection
    outputs, intersection count, sorted ids and tile bins as the plain forward followed by the
    binning's own depth-key pass (gsplat_bin_count)."""
    from gaussctrl_exp_amd.rasterize import bin_gaussians
    sc, cam = _scene_cam(case)
    n, W, H, deg, dtu = case[:5]
    d, c = sc.to(gpu), cam.to(gpu)
    K = d.features_rest.shape[1] + 1
    tb = cam.tile_bounds
    campos = c.c2w[:3, 3].contiguous()
    P, st = _lib.ptr, _lib.stream(gpu)
    outs = []
    for binned in (False, True):
        f = lambda *s: torch.full(s, float("nan"), device=gpu)
        o = dict(xys=f(n, 2), depths=f(n), conics=f(n, 3), colors=f(n, 3), opac=f(n),
                 radii=torch.full((n,), -5, device=gpu, dtype=torch.int32),
                 nth=torch.full((n,), -5, device=gpu, dtype=torch.int32))
        head = (n, K, dtu, P(d.means), P(d.scales), P(d.quats), P(d.opacities),
                P(d.features_dc), P(d.features_rest) if K > 1 else None, P(c.viewmat),
                P(c.projmat), P(campos), cam.fx, cam.fy, cam.cx, cam.cy, H, W, tb[0], tb[1],
                0.01, P(o["xys"]), P(o["depths"]), P(o["radii"]), P(o["conics"]), P(o["nth"]),
                P(o["colors"]), P(o["opac"]))
        if binned:
            ws = torch.full((_lib.query("gsplat_bin_count_workspace_size", n),), 0xAB,
                            device=gpu, dtype=torch.uint8)
            _lib.call("gsplat_fused_preprocess_forward_binned", *head, P(ws), ws.numel(), st)
            b = bin_gaussians(o["xys"], o["depths"], o["radii"], o["nth"], H, W,
                              keyed_workspace=ws)
        else:
            _lib.call("gsplat_fused_preprocess_forward", *head, None, None, None, st)
            b = bin_gaussians(o["xys"], o["depths"], o["radii"], o["nth"], H, W)
        outs.append((o, b))
    (o0, b0), (o1, b1) = outs
    for k in o0:
        assert torch.equal(o0[k], o1[k]), k
    assert b0[0] == b1[0] > 0
    assert torch.equal(b0[1], b1[1]) and torch.equal(b0[2], b1[2])
    with pytest.raises(RuntimeError):  # a workspace too small for the depth-sort inputs
        _lib.call("gsplat_fused_preprocess_forward_binned", *head, P(ws), 64, st)


def _fused_run(sc, cam, deg, bg, gt, dev):
    """The fused training render + the test loss on the GPU; returns (outputs and gradients,
    the rasterizer-level record of the render: inputs, upstream and raster gradients)."""
    s = sc.to(dev).requires_grad_()
    out = render_fused(s, cam.to(dev), deg, bg.to(dev), return_alpha=True, clamp=False)
    img, acc = out["rgb"], out["accumulation"]
    up = {}
    img.register_hook(lambda g: up.__setitem__("v_img", _np(g)))
    acc.register_hook(lambda g: up.__setitem__("v_alpha", _np(g)[..., 0]))
    rgb = torch.clamp(img, max=1.0)  # gc_model.py:222
    # sums, not means: O(1) gradients, so the absolute tolerance cannot hide a wrong one
    loss = (rgb - gt.to(dev)).abs().sum() + 0.1 * acc.sum()
    loss.backward()
    res = [_np(rgb), _np(acc)] + [_np(p.grad) for p in s.params()]
    raster = {k: _np(v) for k, v in out["raster_inputs"].items()}
    raster.update(up, grads=[_np(g) for g in out["raster_grads"]()], xys_grad=_np(
        out["xys_grad"]()))
    return res, raster


def _ref_run(sc, cam, deg, bg, raster_grads):
    """The unchanged caller (scene.render, gc_model.py's glue) on the oracle-backed gsplat,
    its rasterize backward fed the GPU's raster-level gradients (tests/parity.py)."""
    from parity import injected_api
    s = sc.requires_grad_()
    out = render(s, cam, deg, bg, api=injected_api(raster_grads))
    (out["rgb"].sum() + out["accumulation"].sum()).backward()  # upstream replaced anyway
    return [_np(out["rgb"]), _np(out["accumulation"])] + [_np(p.grad) for p in s.params()]


@pytest.mark.parametrize("case", CASES)
def test_fused_render_grads_match_oracle(gpu, case, quirk_mask):
    """The fused training render (bench.py's step) vs the oracle with zero outliers: its
    rasterizer-level gradients (the backward's records) vs the oracle's rasterize backward on
    the same forward state, and image, alpha and all six parameter gradients vs the oracle
    caller chain fed with those raster gradients."""
    from parity import assert_close, check_raster_level
    sc, cam = _scene_cam(case)
    deg = case[4]
    bg = torch.tensor([0.3, 0.6, 0.9])
    gt = torch.rand(cam.height, cam.width, 3, generator=torch.Generator().manual_seed(4))
    fused, r = _fused_run(sc, cam, deg, bg, gt, gpu)
    check_raster_level(gpu, r["xys"], r["depths"], r["radii"], r["conics"], r["num_tiles_hit"],
                       r["colors"], r["opacity"], bg.numpy(), cam.height, cam.width, r["v_img"],
                       r["v_alpha"], r["grads"])
    ref = _ref_run(sc, cam, deg, bg, r["grads"])
    for i, name in enumerate(["rgb", "alpha"] + NAMES):
        assert np.isfinite(fused[i]).all(), f"{name}: non-finite values"
        if fused[i].size and i >= 2 and not (name == "features_rest" and deg == 0):
            assert np.abs(ref[i]).max() > 1e-3, f"{name}: degenerate reference gradient"
        mx = assert_close(name, fused[i], ref[i])
        print(f"{name}: max |diff| {mx:.3e}")


@pytest.mark.parametrize("quirk_mask", [0], indirect=True)
@pytest.mark.parametrize("case", [CASES[0], CASES[2]])
def test_fused_render_grads_without_quirks(gpu, case, quirk_mask):
    """The fused kernels under the consistent conventions (quirk mask 0: 0.999 backward clamp,
    d loss / d conic.y, the clamped EWA Jacobian; CASES[2] has Gaussians beyond the clamp)."""
    test_fused_render_grads_match_oracle(gpu, case, quirk_mask)


def test_fused_xys_grad_is_the_raster_gradient(gpu):
    """render_fused's xys_grad() (what splatfacto reads from xys.grad) is the raster-level v_xy,
    and the caller path's xys.grad (retain_grad) meets the same oracle bar."""
    from parity import CaptureAPI, check_raster_level
    sc, cam = _scene_cam(CASES[0])
    bg = torch.zeros(3)
    gt = torch.rand(cam.height, cam.width, 3, generator=torch.Generator().manual_seed(1))
    _, r = _fused_run(sc, cam, 3, bg, gt, gpu)
    np.testing.assert_array_equal(r["xys_grad"], r["grads"][0])
    cap = CaptureAPI()
    s2 = sc.to(gpu).requires_grad_()
    ref = render(s2, cam.to(gpu), 3, bg.to(gpu), api=cap)
    (ref["rgb"] - gt.to(gpu)).abs().sum().backward()
    k = cap.cap
    np.testing.assert_array_equal(_np(ref["xys"].grad), k["xys"])
    check_raster_level(gpu, k["xys_in"], k["depths"], k["radii"], k["conics_in"], k["nth"],
                       k["colors_in"], k["opacity_in"], k["background"], cam.height, cam.width,
                       k["v_img"], k.get("v_alpha"), cap.raster_grads(sc.num_points))


def test_fused_empty_view_gives_background_and_zero_grads(gpu):
    sc = synthetic_scene(2000, 3, seed=1).to(gpu).requires_grad_()
    away = gc_camera(look_at_c2w((0.0, 0.0, 4.0), target=(0.0, 0.0, 8.0), up=(0.0, 1.0, 0.0)),
                     200.0, 200.0, 64.0, 48.0, 128, 96).to(gpu)
    bg = torch.tensor([0.2, 0.4, 0.6], device=gpu)
    out = render_fused(sc, away, 3, bg, return_alpha=True)
    assert out["num_intersects"] == 0
    assert torch.equal(out["rgb"], bg.expand(96, 128, 3))
    assert not out["accumulation"].any()
    out["rgb"].sum().backward()
    assert all(p.grad is not None and not p.grad.any() for p in sc.params())


@pytest.mark.parametrize("case", [CASES[0], CASES[6]])
def test_fused_render_under_no_grad_keeps_no_backward_state(gpu, case):
    """A render under torch.no_grad (the forward-only bench step, an eval render) gives the same
    image and alpha bit for bit as one that keeps the backward's state, and keeps none: no
    gradient records, no list-split plan (needs_input_grad alone ignores the grad mode)."""
    n, W, H, deg, dtu, *_ = case
    sc, cam = _scene_cam(case)
    sc = sc.to(gpu).requires_grad_()
    cam = cam.to(gpu)
    bg = torch.tensor([0.1, 0.2, 0.3], device=gpu)
    with torch.no_grad():
        a = render_fused(sc, cam, dtu, bg, return_alpha=True)
    b = render_fused(sc, cam, dtu, bg, return_alpha=True)
    assert torch.equal(a["rgb"], b["rgb"].detach())
    assert torch.equal(a["accumulation"], b["accumulation"].detach())
    assert a["raster_grads"]() is None
    (b["rgb"].sum() + b["accumulation"].sum()).backward()
    assert all(p.grad is not None for p in sc.params())
    assert b["raster_grads"]() is not None


def test_fused_rejects_cpu_tensors():
    sc = synthetic_scene(10)
    with pytest.raises(RuntimeError, match="ROCm device"):
        render_fused(sc, synthetic_camera(32, 32), 3, torch.zeros(3))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_fused_trainstep_exchange_over_rccl_world1(gpu):
    """TrainStep(render_mode="fused") single-rank vs its multi-rank configuration (SH view
    exchange through gsplat_compute_sh_backward_views_split + all-reduces) over RCCL at world
    size 1, and vs the caller-glue TrainStep -- in deterministic mode, so the three runs share
    bit-identical rasterizer gradients and only the chains after them are compared."""
    import torch.distributed as dist
    from gaussctrl_exp_amd.train import TrainStep
    from parity import assert_close

    store = dist.TCPStore("127.0.0.1", _free_port(), 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=gpu)
    prev = _lib.set_deterministic(True)
    try:
        cam = synthetic_camera(256, 192).to(gpu)
        gt = torch.rand(192, 256, 3, generator=torch.Generator().manual_seed(2)).to(gpu)
        bg = torch.tensor([0.2, 0.3, 0.4], device=gpu)
        flats = {}
        for ws, mode in ((1, "fused"), (2, "fused"), (1, "caller")):
            t = TrainStep(synthetic_scene(20000, 3, seed=6, device=gpu), sh_degree=3,
                          world_size=ws, loss="splatfacto", render_mode=mode)
            t.step(cam, gt, background=bg, optimizer=False)
            flats[(ws, mode)] = t.flat_grad().cpu().numpy()
        base = flats[(1, "fused")]
        assert np.abs(base).max() > 0
        assert_close("fused exchange (world 1 as 2 views)", flats[(2, "fused")], base,
                     atol=1e-6, rtol=1e-5)
        mx = assert_close("fused vs caller train step", base, flats[(1, "caller")])
        print(f"fused vs caller: max |diff| {mx:.3e}")
    finally:
        _lib.set_deterministic(prev)
        dist.destroy_process_group()


@pytest.mark.parametrize("deterministic", [True, False])
def test_fused_adam_in_backward_matches_separate_step(gpu, deterministic):
    """TrainStep(render_mode="fused") on one GPU takes the Adam step inside the backward
    kernel; three steps equal the same step with gradient tensors + FusedAdam (same formulas).
    Deterministic mode: bit-identical parameters.  Default mode: the rasterizer's atomic
    summation order differs run to run, and Adam's first steps map a gradient to about
    lr * sign(g), so an element whose gradient is ~0 may move either way -- bounded by 2 lr
    per step: Adam's |update| <= lr (1 - beta1) / sqrt(1 - beta2) = 3.16 lr (Kingma & Ba)."""
    from gaussctrl_exp_amd.train import GROUP_LR, TrainStep
    cam = synthetic_camera(256, 192).to(gpu)
    gt = torch.rand(192, 256, 3, generator=torch.Generator().manual_seed(3)).to(gpu)
    bg = torch.tensor([0.2, 0.3, 0.4], device=gpu)
    params = {}
    prev = _lib.set_deterministic(deterministic)
    try:
        for fuse in (True, False):
            t = TrainStep(synthetic_scene(20000, 3, seed=8, device=gpu), sh_degree=3,
                          loss="splatfacto", render_mode="fused", fuse_adam=fuse)
            for _ in range(3):
                t.step(cam, gt, background=bg)
            assert t.opt.step_count == 3 and t.step_count == 3
            if fuse:
                assert all(p.grad is None for p in t.params)  # gradients never materialised
            params[fuse] = [p.detach().cpu().numpy() for p in t.params]
    finally:
        _lib.set_deterministic(prev)
    for k, (name, a, b) in enumerate(zip(NAMES, params[True], params[False])):
        assert not np.array_equal(b, _np(getattr(synthetic_scene(20000, 3, seed=8), name)))
        if deterministic:
            np.testing.assert_array_equal(a, b, err_msg=name)
        else:
            assert np.abs(a - b).max() <= 3 * 2 * 3.17 * GROUP_LR[name], name


@pytest.mark.parametrize("case", [CASES[0], CASES[2], CASES[3], CASES[6]])
def test_fused_eval_render_bitexact_with_caller(gpu, case):
    """render_fused_eval == scene.render(return_depth=True, fused_depth=True) bit for bit (the
    forward of the fused preprocess is bit-identical to the caller's glue + gsplat calls)."""
    from gaussctrl_exp_amd.fused import render_fused_eval
    sc, cam = _scene_cam(case)
    d, c = sc.to(gpu), cam.to(gpu)
    bg = torch.tensor([0.1, 0.2, 0.3], device=gpu)
    a = render_fused_eval(d, c, case[4], bg)
    with torch.no_grad():
        b = render(d, c, case[4], bg, return_depth=True, fused_depth=True)
    for k in ("rgb", "depth", "accumulation", "xys", "radii"):
        assert torch.equal(a[k], b[k]), k
